"""Per-strip timeline of P row bands filled together on one GPU in horizontal strips
(nw_bands.LocalTBands: band r-1's last row feeds band r's first strip column by
column).  Prints, per band, when its first / last strip started and ended and the
strips' durations (s_memrealtime, 100 MHz, one clock for the whole device) -- to
see which strip paces the chain across the band boundary."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nw_bands  # noqa: E402
import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--P", type=int, default=2)
ap.add_argument("--plain-reps", type=int, default=3, help="untraced fills timed first (events and wall)")
args = ap.parse_args()
lb = nw_bands.LocalTBands(args.n1, args.n2, args.P)
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, args.n2)).cuda()
lb.fill(s1, s2)
import time  # noqa: E402
for _ in range(args.plain_reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    a.record()
    lb.fill(s1, s2)
    b.record()
    torch.cuda.synchronize()
    print(f"untraced fill: events {a.elapsed_time(b):.3f} ms, wall {(time.perf_counter() - w0) * 1e3:.3f} ms", flush=True)
trs = []
for r, (rows, _) in enumerate(lb.layout):
    ns = -(-rows // 256) + 1
    tr = torch.zeros(ns * 24, dtype=torch.int64, device="cuda")
    lb.ctxs[r].set_trace(tr)
    trs.append((tr, ns))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
score = lb.fill(s1, s2)
e1.record()
torch.cuda.synchronize()
print(f"P={args.P} {args.n1}x{args.n2} ms={e0.elapsed_time(e1):.3f} score={score}")
ts = []
for r, (tr, ns) in enumerate(trs):
    lb.ctxs[r].set_trace(None)
    t = tr.view(ns, 24).cpu().numpy().astype(np.float64)
    t = t[t[:, 0] > 0]
    ts.append(t)
t0 = min(t[:, 0].min() for t in ts)
for r, t in enumerate(ts):
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
    dur = en - st
    print(f"band {r}: {t.shape[0]} strips; first start {st.min():.0f} us, last start {st.max():.0f}; "
          f"ends {en.min():.0f} .. {en.max():.0f}; duration first {dur[0]:.0f} med {np.median(dur):.0f} "
          f"last {dur[-1]:.0f} max {dur.max():.0f} us; start lag med {np.median(np.diff(st)):.2f} us; "
          f"feed waits med {np.median(t[:, 2]):.0f} (us {np.median(t[:, 3]) / 100:.0f}) strip0 {t[0, 2]:.0f} "
          f"(us {t[0, 3] / 100:.0f}); ring wait (last wave) med {np.median(t[:, 12]) / 100:.0f} "
          f"last strip {t[-1, 12] / 100:.0f} us", flush=True)
    for q in [0, 1, t.shape[0] - 2, t.shape[0] - 1]:
        print(f"   strip {q}: start {st[q]:.0f} end {en[q]:.0f} dur {dur[q]:.0f} slow {t[q, 2]:.0f} "
              f"wait {t[q, 3] / 100:.0f} ringwait {t[q, 11] / 100:.0f}/{t[q, 12] / 100:.0f}")
lb.close()
