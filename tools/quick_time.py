"""Quick device-resident timing of the fill at a few sizes / strip shapes / worker
counts / row pitches.

  --shapes C:NC,...   columns per lane : compute waves per strip (0:0 = auto)
  --pitches P,...     row pitch in int32 (0 = nw_table_pitch)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="32768,65536")
ap.add_argument("--waves", default="0")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--shapes", default="0:0")
ap.add_argument("--pitches", default="0")
ap.add_argument("--kernel", type=int, default=0, help="0 auto, 1 strips, 2 panels")
args = ap.parse_args()
ctx = nwhip.Context(0)
shapes = [tuple(int(v) for v in x.split(":")) for x in args.shapes.split(",")]
for n in [int(x) for x in args.sizes.split(",")]:
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    for pitch in [int(x) for x in args.pitches.split(",")]:
        tab = nwhip.Context.alloc_table(n, n, pitch=pitch)
        for w in [int(x) for x in args.waves.split(",")]:
            for c, nc in shapes:
                kw = dict(waves=w, flags=args.flags, substrips=c, strip_waves=nc, kernel=args.kernel)
                ctx.fill(s1, s2, tab, **kw)  # warmup
                ts = []
                for _ in range(args.reps):
                    r = ctx.fill(s1, s2, tab, **kw)
                    ts.append(r.kernel_ms)
                ms = min(ts)
                gcups = n * n / (ms * 1e6)
                print(f"n={n} pitch={tab.shape[1]} C={r.substrips} NC={r.strip_waves} "
                      f"kernel={r.kernel} waves={r.waves} strips={r.strips} ms={ms:.3f} "
                      f"(all {[round(t, 3) for t in ts]}) GCUPS={gcups:.1f} "
                      f"store_GBps={4 * (n + 1) * (n + 1) / (ms * 1e6):.1f} score={r.score} "
                      f"status={r.status}", flush=True)
        del tab
        torch.cuda.empty_cache()
