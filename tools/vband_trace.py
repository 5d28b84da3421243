"""Vertical-strip sweep of one config-4 row band (524288 columns x 65536 rows) at a
capped number of resident strips: kernel time and the per-strip traversal (strip
start -> end, debug trace, s_memrealtime at 100 MHz).

In the vertical sweep band r+1's strip k starts once band r's strip k has reached
its last row, so the per-band delay of the N = 8 pipeline is the traversal of band
r's strips, and the band's own fill time is its throughput term.
Fewer resident strips -> each strip is less throttled by HBM (shorter traversal)
at a possibly longer band time: this prints both per grid size.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--waves", default="256,192,160,128,96,64")
ap.add_argument("--sub", type=int, default=0)
ap.add_argument("--nc", type=int, default=0)
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--save", default="", help="write start/end (us) per strip to <save>_w<waves>.npz")
args = ap.parse_args()
ctx = nwhip.Context(0)
n1, n2 = args.n1, args.n2
s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
tab = nwhip.Context.alloc_table(n1, n2)
cap = (n1 + 1 + 63) // 64
tr = torch.zeros(cap * 24, dtype=torch.int64, device="cuda")
for w in [int(x) for x in args.waves.split(",")]:
    kw = dict(waves=w, flags=args.flags, substrips=args.sub, strip_waves=args.nc, kernel=nwhip.KERNEL_STRIPS)
    ctx.set_trace(None)
    r0 = ctx.fill(s1, s2, tab, (1, 0, -1), **kw)
    r1 = ctx.fill(s1, s2, tab, (1, 0, -1), **kw)
    ctx.set_trace(tr)
    r = ctx.fill(s1, s2, tab, (1, 0, -1), **kw)
    ctx.set_trace(None)
    assert r.status == 0 and r0.status == 0
    ns = r.strips
    t = tr[: ns * 24].view(ns, 24).cpu().numpy().astype(np.float64)
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, 1] - t0) / 100.0
    dur = en - st
    first = dur[: min(ns, r.waves)]
    if args.save:
        np.savez(f"{args.save}_w{r.waves}.npz", start=st, end=en, wait=t[:, 3] / 100.0, kernel_ms=r.kernel_ms,
                 waves=r.waves,
                 substrips=r.substrips, strip_waves=r.strip_waves, n1=n1, n2=n2)
    print(f"waves={r.waves} C={r.substrips} NC={r.strip_waves} strips={ns} kernel_ms untraced "
          f"{min(r0.kernel_ms, r1.kernel_ms):.3f} traced {r.kernel_ms:.3f} span_us {en.max():.0f}", flush=True)
    print(f"   traversal us: strip0 {dur[0]:.0f}  first pass med {np.median(first):.0f} max {first.max():.0f}  "
          f"all med {np.median(dur):.0f} p90 {np.percentile(dur, 90):.0f} max {dur.max():.0f}  "
          f"-> ns/row strip0 {dur[0] / (n2 + 1) * 1e3:.1f} med {np.median(dur) / (n2 + 1) * 1e3:.1f}", flush=True)
    print(f"   start lag us: med {np.median(np.diff(st)):.2f}; GB/s {4.0 * (n1 + 1) * (n2 + 1) / r.kernel_ms / 1e6:.0f}",
          flush=True)
