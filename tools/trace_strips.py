"""Per-strip timeline of one fill (debug trace: s_memrealtime at 100 MHz)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=32768)
ap.add_argument("--n1", type=int, default=0, help="columns (default: --n, a square); e.g. 256 = one strip alone")
ap.add_argument("--waves", default="0")
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--sub", type=int, default=0)
ap.add_argument("--nc", type=int, default=0)
ap.add_argument("--save", default="")
ap.add_argument("--sw", action="store_true", help="Smith-Waterman mode, scheme (1,-1,-1)")
args = ap.parse_args()
ctx = nwhip.Context(0)
n = args.n
n1 = args.n1 or n
s1 = torch.from_numpy(nwhip.synth(1, n1)).cuda()
s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
tab = nwhip.Context.alloc_table(n1, n)
nstrips = max(2, (n1 + 1 + 63) // 64)
tr = torch.zeros(nstrips * 24, dtype=torch.int64, device="cuda")
for w in [int(x) for x in args.waves.split(",")]:
    ctx.set_trace(None)
    kw = dict(waves=w, flags=args.flags, substrips=args.sub, strip_waves=args.nc)
    if args.sw:
        kw.update(mode=nwhip.MODE_SW, kernel=nwhip.KERNEL_STRIPS)
    sch = (1, -1, -1) if args.sw else (1, 0, -1)
    r0 = ctx.fill(s1, s2, tab, sch, **kw)
    ctx.set_trace(tr)
    r = ctx.fill(s1, s2, tab, sch, **kw)
    nstrips = r.strips
    ctx.set_trace(None)
    t = tr[: nstrips * 24].view(nstrips, 24).cpu().numpy().astype(np.float64)
    if args.save:
        np.save(f"{args.save}_w{w}_k{r.substrips}.npy", t)
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0   # us
    en = (t[:, 1] - t0) / 100.0
    dur = en - st
    lag = np.diff(st)
    # hop lag: time strip p reached the middle (quarter) of the table after strip p-1 did
    for col, nm in ((5, "mid"), (4, "quarter")):
        tm = t[:, col]
        ok = (tm[1:] > 0) & (tm[:-1] > 0)
        hop = (tm[1:] - tm[:-1])[ok] / 100.0
        if hop.size:
            pq = np.percentile(hop, [10, 50, 90])
            w = r.waves
            later = hop[w:] if hop.size > w else hop
            print(f"  hop lag at {nm} (us): mean {hop.mean():.2f} p10 {pq[0]:.2f} med {pq[1]:.2f} p90 {pq[2]:.2f} "
                  f"p99 {np.percentile(hop, 99):.2f} max {hop.max():.1f}; "
                  f"first pass med {np.median(hop[:w]):.2f}; later med {np.median(later):.2f}")
    # hand-off visibility: producer p-1 starts iteration nblocks/2+1 (publishes
    # block nblocks/2 chunk 0 14 steps later) -> consumer p sees that chunk
    ok = (t[1:, 9] > 0) & (t[:-1, 8] > 0)
    vis = (t[1:, 9] - t[:-1, 8])[ok] / 100.0
    waited = (t[1:, 10] > 0)[ok]
    if vis.size:
        pr = lambda a: f"p10 {np.percentile(a, 10):.2f} med {np.median(a):.2f} p90 {np.percentile(a, 90):.2f} (n={a.size})"
        print(f"  block mid chunk 0: consumer saw it - producer published (us): all {pr(vis)}")
        if waited.any():
            print(f"     consumers that waited for it: {pr(vis[waited])}; waited from publish-x: "
                  f"{pr(((t[1:, 10] - t[:-1, 8])[ok][waited]) / 100.0)}")
    busy = (dur - t[:, 3] / 100.0).sum()
    print(f"  sum(strip time - wait) / (waves * span) = {busy / (r.waves * en.max()):.3f}; "
          f"sum(wait) / (waves*span) = {t[:, 3].sum() / 100.0 / (r.waves * en.max()):.3f}")
    print(f"n={n} C={r.substrips} NC={r.strip_waves} waves={r.waves} strips={r.strips} kernel_ms={r.kernel_ms:.3f} (untraced {r0.kernel_ms:.3f}) "
          f"span_us={en.max():.0f}")
    clk = (t[:, 7] - t[:, 6]) / np.maximum(t[:, 1] - t[:, 0], 1) * 100e6 / 1e9
    print(f"  effective shader clock GHz per strip: strip0 {clk[0]:.3f} p10 {np.percentile(clk, 10):.3f} "
          f"med {np.median(clk):.3f} p90 {np.percentile(clk, 90):.3f}")
    busy_row = (dur - t[:, 3] / 100.0) / n * 1000.0
    print(f"  busy ns/row: strip0 {busy_row[0]:.2f} med {np.median(busy_row):.2f} p90 {np.percentile(busy_row, 90):.2f}")
    print(f"  strip duration us: min {dur.min():.0f} med {np.median(dur):.0f} max {dur.max():.0f}"
          f"  -> per row {np.median(dur)/n*1000:.2f} ns")
    if lag.size:
        print(f"  start lag us: med {np.median(lag):.2f} p10 {np.percentile(lag,10):.2f} p90 {np.percentile(lag,90):.2f}")
    print(f"  slow waits/strip: med {np.median(t[:,2]):.0f} max {t[:,2].max():.0f}; wait us/strip med "
          f"{np.median(t[:,3])/100:.0f} max {t[:,3].max()/100:.0f}")
    print(f"  ring back-pressure us/strip: first wave med {np.median(t[:,11])/100:.0f} "
          f"(strip0 {t[0,11]/100:.0f}); last wave med {np.median(t[:,12])/100:.0f} "
          f"(strip0 {t[0,12]/100:.0f}); last wave feed wait med {np.median(t[:,13])/100:.0f}")
    cyc = (t[:, 7] - t[:, 6])
    print(f"  cycles/step inside run_iter: first wave strip0 {t[0,14]/n:.1f} med {np.median(t[:,14])/n:.1f}; "
          f"last wave strip0 {t[0,15]/n:.1f} med {np.median(t[:,15])/n:.1f}; whole strip med {np.median(cyc)/n:.1f}")
    for q in sorted({min(x, nstrips - 1) for x in [0, 1, 2, nstrips // 4, nstrips // 4 + 1, nstrips // 2, nstrips - 2, nstrips - 1]}):
        print(f"   strip {q}: start {st[q]:.1f} end {en[q]:.1f} dur {dur[q]:.1f} slow {t[q,2]:.0f} wait {t[q,3]/100:.1f} "
              f"ringwait first {t[q,11]/100:.0f} last {t[q,12]/100:.0f} lastfeed {t[q,13]/100:.0f} "
              f"run_iter cyc/step first {t[q,14]/n:.1f} last {t[q,15]/n:.1f} "
              f"store wave cyc/row wait {t[q,16]/n:.1f} read {t[q,17]/n:.1f} store {t[q,18]/n:.1f}")
