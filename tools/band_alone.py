"""One rank's BASELINE config-4 row band (524288 x 524288 split into 8 mpi-horz bands,
src/mpi/mpi-horz-driver.cpp:31-32), filled ALONE on one GPU with its halo row
pre-published from the pinned oracle's fixture (tests/golden/config4_524288_shipped.npz)
-- the per-GPU kernel of the 8-GPU run, timed (and profiled under rocprofv3) without the
chain around it.  Checks the band's last row against the fixture.

  python tools/band_alone.py --rank 7 --sweep vertical|horizontal --reps 5
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import nwhip  # noqa: E402
from conftest import config4_golden  # noqa: E402

N, P, GAP = 524288, 8, -1

ap = argparse.ArgumentParser()
ap.add_argument("--rank", type=int, default=7)
ap.add_argument("--sweep", choices=["vertical", "horizontal"], default="vertical")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--substrips", type=int, default=0)
ap.add_argument("--strip-waves", type=int, default=0)
ap.add_argument("--flags", type=int, default=0)
args = ap.parse_args()

g = config4_golden()
rows, start = nwhip.band_layout(N, P, args.rank)
k0 = int(np.searchsorted(g["rows"], start))
k1 = int(np.searchsorted(g["rows"], start + rows - 1))
assert g["rows"][k1] == start + rows - 1
first = start == 0  # band 0: row 0 is the boundary row (no halo)
assert first or g["rows"][k0] == start
halo, want_last = (None if first else g["full"][k0]), g["full"][k1]
ctx = nwhip.Context(0)
tab = nwhip.Context.alloc_table(N, rows - 1)
d1 = torch.from_numpy(nwhip.synth(1, N)).cuda()
d2 = torch.from_numpy(nwhip.synth(2, N)[start:start + rows - 1].copy()).cuda()
j = np.arange(N + 1, dtype=np.int64)
if not first:
    vals = halo.astype(np.int64) if args.sweep == "vertical" else halo.astype(np.int64) - GAP * (j + start)
size = N + 1 if args.sweep == "vertical" else nwhip.feed_bytes(N) // 8
ts = []
for rep in range(args.reps + 1):
    tag = 3 + rep
    hin = None
    if not first:
        gr = np.full(size, np.int64(tag) << 32, np.int64)
        gr[:N + 1] |= vals & 0xFFFFFFFF
        hin = torch.from_numpy(gr).cuda()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.sweep == "vertical":
        ctx.fill_band(d1, d2, tab, halo_in=hin, tag=tag, row0=start, substrips=args.substrips,
                      strip_waves=args.strip_waves, flags=args.flags)
    else:
        ctx.fill_tband(d1, d2, tab, row0=start, feed_in=hin, tag=tag, flags=args.flags)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
    st = ctx.status()
    assert st == nwhip.NW_OK, (st, ctx.debug_failure())
ok = np.array_equal(tab[rows - 1, :N + 1].cpu().numpy(), want_last)
best = min(ts[1:])
print(f"band {args.rank} ({rows} x {N + 1}) {args.sweep} flags={args.flags}: ms={best:.2f} "
      f"all={[round(t, 2) for t in ts[1:]]} GB/s={4.0 * rows * (N + 1) / (best * 1e6):.0f} last_row_ok={ok}",
      flush=True)
