"""Device-resident fill time of one row band (n1 columns x n2 rows below the
boundary row) in horizontal strips (nw_fill_tband_async: 256-row strips along the
columns) against the vertical-strip fill of the same table -- the per-GPU
geometry of the multi-GPU row-band bench is 524288 x 65536.  Prints ms and the
per-column pace of the horizontal sweep, T / (n1 + (strips - 1) * 64)."""
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--flags", type=int, default=0, help="nw_params.flags (513 = 0x201: timing only + no store waves, the compute pace)")
ap.add_argument("--shape", default="4,1", help="horizontal strip shape C,NC: 4,1 or 2,2")
ap.add_argument("--dense", action="store_true", help="NW_TBAND_DENSE_POLLS (follower polls with s_sleep 1)")
ap.add_argument("--vertical", default="4:1,2:2", help="vertical-strip shapes to time beside it ('' = none)")
args = ap.parse_args()
SC, SNC = (int(x) for x in args.shape.split(","))
ctx = nwhip.Context(0)
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, args.n2)).cuda()
tab = nwhip.Context.alloc_table(args.n1, args.n2)
st = torch.cuda.current_stream()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


tag = [0]


def tband():
    tag[0] += 1
    ctx.fill_tband(s1, s2, tab, tag=tag[0], flags=args.flags, substrips=SC, strip_waves=SNC, dense_polls=args.dense)


timed(tband)
ts = [timed(tband) for _ in range(args.reps)]
assert ctx.status() == nwhip.NW_OK
ms = min(ts)
strips = -(-args.n2 // 256)
pace = ms * 1e6 / (args.n1 + (strips - 1) * 64)
score = int(tab[args.n2, args.n1].item())
print(f"horizontal ({SC},{SNC}) {args.n1}x{args.n2} flags={args.flags} ms={ms:.3f} GCUPS={args.n1 * args.n2 / (ms * 1e6):.1f} "
      f"pace={pace:.1f}ns/col score={score} all={[round(t, 2) for t in ts]}", flush=True)
for sh in [x for x in args.vertical.split(",") if x]:
    c, nc = (int(x) for x in sh.split(":"))
    ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=1, flags=args.flags)
    ts = [ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=1, flags=args.flags).kernel_ms
          for _ in range(args.reps)]
    print(f"vertical {args.n1}x{args.n2} C={c} NC={nc} ms={min(ts):.3f} score={int(tab[args.n2, args.n1].item())} "
          f"all={[round(t, 2) for t in ts]}", flush=True)
