"""Device-resident fill time of an n1 x n2 table per strip shape (the row-band
geometry of the multi-GPU bench is 524288 x 65536 per GPU: wide and short, so
the strip-to-strip hop, not the store rate, can bound it)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--shapes", default="4:1,2:2,1:4,2:1")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--kernel", type=int, default=0, help="0 auto, 1 strips, 2 panels")
ap.add_argument("--flags", type=int, default=0, help="nw_params.flags (513 = 0x201: timing only + no store waves, the compute pace)")
args = ap.parse_args()
ctx = nwhip.Context(0)
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, args.n2)).cuda()
tab = nwhip.Context.alloc_table(args.n1, args.n2)
for sh in args.shapes.split(","):
    c, nc = (int(x) for x in sh.split(":"))
    ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=args.kernel, flags=args.flags)
    ts = [ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=args.kernel, flags=args.flags).kernel_ms for _ in range(args.reps)]
    ms = min(ts)
    print(f"{args.n1}x{args.n2} kernel={args.kernel} flags={args.flags} C={c} NC={nc} ms={ms:.3f} GCUPS={args.n1 * args.n2 / (ms * 1e6):.1f} "
          f"all={[round(t, 2) for t in ts]}", flush=True)
