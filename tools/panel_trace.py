"""Per-panel timeline of one row-scan panel fill (debug trace, s_memrealtime at
100 MHz): ramp (start offsets), duration, and the time the first / last compute
wave of each panel spent waiting for ring space (its store wave) and for its left
values (the previous panel's granules / the previous wave)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=262144)
ap.add_argument("--shape", default="4:4")
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--kernel", type=int, default=2)
args = ap.parse_args()
c, nw = (int(x) for x in args.shape.split(":"))
ctx = nwhip.Context(0)
n = args.n
s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
tab = nwhip.Context.alloc_table(n, n)
W = nwhip.trace_words()
tr = torch.zeros(((n + 64) // 64 + 8) * W, dtype=torch.int64, device="cuda")
kw = dict(substrips=c, strip_waves=nw, kernel=args.kernel, flags=args.flags)
ctx.fill(s1, s2, tab, **kw)
ctx.set_trace(tr)
r = ctx.fill(s1, s2, tab, **kw)
ctx.set_trace(None)
ns = r.strips
t = tr[: ns * W].view(ns, W).cpu().numpy().astype(np.float64)
t0 = t[:, 0].min()
st = (t[:, 0] - t0) / 100.0  # us
en = (t[:, 1] - t0) / 100.0
dur = en - st
print(f"n={n} shape={c}:{nw} kernel={r.kernel} flags={args.flags} panels={ns} workers={r.waves} "
      f"kernel_ms={r.kernel_ms:.3f} score={r.score}")
print(f"  start offsets (us): p1 {st[1]:.1f}  p{ns // 2} {st[ns // 2]:.1f}  last {st[-1]:.1f}; "
      f"median hop {np.median(np.diff(st)):.2f} us")
print(f"  duration (ms): min {dur.min() / 1e3:.2f} med {np.median(dur) / 1e3:.2f} max {dur.max() / 1e3:.2f}; "
      f"end of last {en.max() / 1e3:.2f}")
for col, nm in ((11, "wave 0 ring wait"), (3, "wave 0 feed wait"), (12, "last wave ring wait"),
                (13, "last wave feed wait")):
    f = t[:, col] / 100.0 / np.maximum(dur, 1e-9)
    print(f"  {nm:22s} fraction of panel time: med {np.median(f):.3f} p10 {np.percentile(f, 10):.3f} "
          f"p90 {np.percentile(f, 90):.3f}  (panel 0: {f[0]:.3f})")
print(f"  slow feed waits per panel: med {np.median(t[:, 2]):.0f}")
