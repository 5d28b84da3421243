"""Per-step cost of the fill kernel: one strip (n1 = 64*C - 1 columns) over many
rows, alone on the device -- the wave's serial speed with no hand-off waits and
no store contention.  Prints ns/row and shader cycles per step (2.39 GHz)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=131072)
ap.add_argument("--shapes", default="4:1,2:1,1:1,2:2,1:2,1:4")
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--tag", default="")
args = ap.parse_args()
ctx = nwhip.Context(0)
n2 = args.rows
s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
for c, nc in [tuple(int(v) for v in x.split(":")) for x in args.shapes.split(",")]:
    n1 = 64 * c * nc  # one strip: columns 1 .. n1 (column 0 is the boundary)
    s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
    tab = nwhip.Context.alloc_table(n1, n2)
    kw = dict(substrips=c, strip_waves=nc, flags=args.flags)
    ctx.fill(s1, s2, tab, **kw)
    ms = min(ctx.fill(s1, s2, tab, **kw).kernel_ms for _ in range(3))
    ns = ms * 1e6 / n2
    print(f"{args.tag} C={c} NC={nc} rows={n2} ms={ms:.3f} ns/row={ns:.2f} "
          f"cyc/step={ns * 2.39:.1f} cyc/cell-per-wave={ns * 2.39 / (64 * c):.3f} "
          f"cells/ns={64 * c * nc / ns:.2f}", flush=True)
    del tab
