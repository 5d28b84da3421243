"""Cost of the block-cyclic decomposition on one GPU: a 524288 x 65536 table (one
GPU's share of config 4) filled as ONE launch of m chained row blocks
(nw_bands.LocalCycleBands with P = 1: the multi-block kernel path, block k+1's
halo = block k's last row through the rank's own halo buffer) against the plain
band fill of the same rows.  m = 1 is the plain fill through the cycle API."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nw_bands  # noqa: E402
import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--blocks", default="1,2,4,8")
ap.add_argument("--shape", default="0:0", help="C:NC (0:0 = the band shape for the block height)")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
c, nc = (int(x) for x in args.shape.split(":"))
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = nwhip.synth(2, args.n2)
ctx = nwhip.Context(0)
tab = nwhip.Context.alloc_table(args.n1, args.n2)
d2 = torch.from_numpy(s2).cuda()
ctx.fill(s1, d2, tab, substrips=c, strip_waves=nc)
ts = [ctx.fill(s1, d2, tab, substrips=c, strip_waves=nc).kernel_ms for _ in range(args.reps)]
r = ctx.fill(s1, d2, tab, substrips=c, strip_waves=nc)
print(f"plain {args.n1}x{args.n2} shape={r.substrips},{r.strip_waves} ms={min(ts):.3f} score={r.score}", flush=True)
del tab
torch.cuda.empty_cache()
for m in (int(x) for x in args.blocks.split(",")):
    lb = nw_bands.LocalCycleBands(args.n1, args.n2, 1, m, substrips=c, strip_waves=nc)
    sc = lb.fill(s1, s2)
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc = lb.fill(s1, s2)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"cycle m={m} h={lb.h} shape={lb.substrips},{lb.strip_waves} ms={min(ts):.3f} (wall, incl. "
          f"side-char copies) score={sc}", flush=True)
    lb.close()
    del lb
    torch.cuda.empty_cache()
