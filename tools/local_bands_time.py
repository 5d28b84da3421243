"""One-process timing of P row bands on one GPU (LocalBands: vertical strips, halo
buffers; LocalTBands: horizontal strips, feed buffers) -- both through fine-grained
link buffers in local memory, each band on 1/P of the workers."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nw_bands  # noqa: E402
import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", type=int, default=65536)
ap.add_argument("--P", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--only", choices=["vertical", "horizontal"], default=None)
args = ap.parse_args()
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, args.n2)).cuda()
for name, cls in (("vertical", nw_bands.LocalBands), ("horizontal", nw_bands.LocalTBands)):
    if args.only not in (None, name):
        continue
    lb = cls(args.n1, args.n2, args.P)
    lb.fill(s1, s2)
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        score = lb.fill(s1, s2)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"{name} {args.n1}x{args.n2} P={args.P} ms={min(ts):.2f} all={[round(t, 2) for t in ts]} score={score}", flush=True)
    lb.close()
    del lb
    torch.cuda.empty_cache()
