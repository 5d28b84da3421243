"""Smith-Waterman fill time per strip / panel shape (device-resident, 64k x 64k by default).
--shapes C:NC for strips, pC:NW for the panel kernel (nw_rows.hip)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--shapes", default="4:1,2:2,1:4,2:1,p4:1,p2:2,p1:4,p4:2,p2:4,p4:4")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--flags", type=int, default=0, help="nw_params.flags (1: table stores to a scratch tile)")
args = ap.parse_args()
ctx = nwhip.Context(0)
n = args.n
s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
tab = nwhip.Context.alloc_table(n, n)
for sh in args.shapes.split(","):
    kern = nwhip.KERNEL_PANELS if sh.startswith("p") else nwhip.KERNEL_STRIPS
    c, nc = (int(x) for x in sh.lstrip("p").split(":"))
    kw = dict(substrips=c, strip_waves=nc, mode=nwhip.MODE_SW, kernel=kern, flags=args.flags)
    ctx.fill(s1, s2, tab, (1, -1, -1), **kw)
    ts = [ctx.fill(s1, s2, tab, (1, -1, -1), **kw).kernel_ms for _ in range(args.reps)]
    r = ctx.fill(s1, s2, tab, (1, -1, -1), **kw)
    print(f"SW {n}x{n} {'panels' if kern == nwhip.KERNEL_PANELS else 'strips'} C={c} NC={nc} flags={args.flags} ms={min(ts):.3f} GCUPS={n * n / (min(ts) * 1e6):.1f} score={r.score}", flush=True)
