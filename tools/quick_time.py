"""Quick device-resident timing of the fill at a few sizes / worker counts."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="32768,65536")
ap.add_argument("--waves", default="0")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--sub", default="0")
args = ap.parse_args()
ctx = nwhip.Context(0)
for n in [int(x) for x in args.sizes.split(",")]:
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    for w, k in [(int(x), int(y)) for x in args.waves.split(",") for y in args.sub.split(",")]:
        ctx.fill(s1, s2, tab, waves=w, flags=args.flags, substrips=k)  # warmup
        ts = []
        for _ in range(args.reps):
            r = ctx.fill(s1, s2, tab, waves=w, flags=args.flags, substrips=k)
            ts.append(r.kernel_ms)
        ms = min(ts)
        gcups = n * n / (ms * 1e6)
        print(f"n={n} K={r.substrips} waves={r.waves} strips={r.strips} ms={ms:.3f} (all {[round(t,3) for t in ts]}) "
              f"GCUPS={gcups:.1f} store_GBps={4*(n+1)*(n+1)/(ms*1e6):.1f} score={r.score} status={r.status}",
              flush=True)
    del tab
    torch.cuda.empty_cache()
