"""Smith-Waterman strip-kernel timing for the config-5 attribution:
an n2 x n1 SW fill (default 65536 x 256 = strip 0 ALONE: one (2,2) strip, its
compute and store waves, no chain, no other strip's HBM traffic) or the config-5
square, with nw_params.flags (513 = timing only + no store waves: the compute waves
alone).  Prints ms per fill and ns per row (the strip's pace) over --reps fills."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=256)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--shape", default="2,2")
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
c, nc = (int(x) for x in args.shape.split(","))
ctx = nwhip.Context(0)
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, args.n2)).cuda()
tab = nwhip.Context.alloc_table(args.n1, args.n2)
kw = dict(substrips=c, strip_waves=nc, mode=nwhip.MODE_SW, kernel=nwhip.KERNEL_STRIPS, flags=args.flags)
ctx.fill(s1, s2, tab, (1, -1, -1), **kw)
ts = [ctx.fill(s1, s2, tab, (1, -1, -1), **kw).kernel_ms for _ in range(args.reps)]
ms = min(ts)
print(f"SW {args.n2}x{args.n1} ({c},{nc}) flags={args.flags} ms={ms:.3f} ns/row={ms * 1e6 / (args.n2 + 1):.2f} "
      f"all={[round(t, 3) for t in ts]}", flush=True)
