"""Per-strip timeline of one horizontal-strip band fill (nw_fill_tband_async with
the debug trace): the lag between adjacent strips at a quarter / the middle of
the sweep (the hop), strip durations, feed waits -- s_memrealtime at 100 MHz."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nwhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n1", type=int, default=524288)
ap.add_argument("--n2", default="16384,65536")
ap.add_argument("--shape", default="4,1", help="horizontal strip shape C,NC: 4,1 or 2,2")
ap.add_argument("--dense", action="store_true", help="NW_TBAND_DENSE_POLLS (follower polls with s_sleep 1)")
args = ap.parse_args()
SC, SNC = (int(x) for x in args.shape.split(","))
ctx = nwhip.Context(0)
s1 = torch.from_numpy(nwhip.synth(1, args.n1)).cuda()
for n2 in [int(x) for x in args.n2.split(",")]:
    s2 = torch.from_numpy(nwhip.synth(2, n2)).cuda()
    tab = nwhip.Context.alloc_table(args.n1, n2)
    nstrips = -(-n2 // 256)
    tr = torch.zeros(nstrips * 24, dtype=torch.int64, device="cuda")
    ctx.fill_tband(s1, s2, tab, tag=1, substrips=SC, strip_waves=SNC, dense_polls=args.dense)
    ctx.set_trace(tr)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ctx.fill_tband(s1, s2, tab, tag=2, substrips=SC, strip_waves=SNC, dense_polls=args.dense)
    e1.record()
    torch.cuda.synchronize()
    ctx.set_trace(None)
    t = tr.view(nstrips, 24).cpu().numpy().astype(np.float64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
    print(f"({SC},{SNC}) {args.n1}x{n2} strips={nstrips} ms={e0.elapsed_time(e1):.3f} span_us={en.max():.0f}")
    for col, nm in ((4, "quarter"), (5, "mid")):
        hop = np.diff(t[:, col]) / 100.0
        print(f"  hop at {nm} (us): med {np.median(hop):.2f} p10 {np.percentile(hop, 10):.2f} "
              f"p90 {np.percentile(hop, 90):.2f} max {hop.max():.1f}; first 8 {np.round(hop[:8], 2).tolist()}")
    print(f"  start lag (us): med {np.median(np.diff(st)):.2f}; first 8 {np.round(np.diff(st)[:8], 2).tolist()}")
    dur = en - st
    print(f"  strip duration (us): first {dur[0]:.0f} med {np.median(dur):.0f} max {dur.max():.0f}; "
          f"end of last {en[-1]:.0f}")
    # the chain accumulates the MEAN strip-to-strip lag, rare stalls included: the end
    # lags, and where the largest ones arose (a stall shifts every strip below it)
    lag = np.diff(en)
    hq, hm = np.diff(t[:, 4]) / 100.0, np.diff(t[:, 5]) / 100.0
    print(f"  end lag (us): mean {lag.mean():.2f} (= (end of last - end of first) / {nstrips - 1}) med "
          f"{np.median(lag):.2f} p99 {np.percentile(lag, 99):.1f} max {lag.max():.1f}; lags > 50 us: "
          f"{int((lag > 50).sum())}, their sum {lag[lag > 50].sum():.0f} us")
    for k in np.argsort(-np.maximum(np.maximum(lag, hq), hm))[:6]:
        s = k + 1
        print(f"   strip {s}: end lag {lag[k]:.1f} hop quarter {hq[k]:.1f} mid {hm[k]:.1f} us; feed waits "
              f"{t[s, 2]:.0f} ({t[s, 3] / 100:.0f} us); ring-space wait first/last wave {t[s, 11] / 100:.0f} / "
              f"{t[s, 12] / 100:.0f} us; its producer's ring wait {t[k, 11] / 100:.0f} / {t[k, 12] / 100:.0f} us")
    print(f"  feed waits / strip: med {np.median(t[:, 2]):.0f} max {t[:, 2].max():.0f}; wait us med "
          f"{np.median(t[:, 3]) / 100:.0f} max {t[:, 3].max() / 100:.0f}; ring-space wait us (last wave) med "
          f"{np.median(t[:, 12]) / 100:.0f}", flush=True)
    cyc = t[:, 14] / (args.n1 + 1)
    clk = (t[:, 7] - t[:, 6]) / np.maximum(t[:, 1] - t[:, 0], 1) * 100e6 / 1e9
    print(f"  compute wave cycles per step inside run_iter: strip 0 {cyc[0]:.1f} med {np.median(cyc):.1f} "
          f"p90 {np.percentile(cyc, 90):.1f}; shader clock GHz med {np.median(clk):.3f}")
    if t[:, 20].any():  # feeder wave builds (NW_FEEDER): its stalls
        mx = t[:, 20] / 100.0
        order = np.argsort(-mx)[:6]
        print(f"  feeder: ring-space wait us/strip med {np.median(t[:, 19]) / 100:.0f} max {t[:, 19].max() / 100:.0f}; "
              f"longest no-data streak us med {np.median(mx):.1f} max {mx.max():.0f}; streaks > 100 us: "
              f"{int(t[:, 23].sum())} in {int((t[:, 23] > 0).sum())} strips")
        for q in order:
            print(f"   strip {q}: longest streak {mx[q]:.0f} us waiting for row {int(t[q, 21])}, ended at "
                  f"{(t[q, 22] - t0) / 100.0:.0f} us; strip start {st[q]:.0f} end {en[q]:.0f}; "
                  f"left strip end {en[q - 1] if q > 0 else 0:.0f}", flush=True)
    del tab
    torch.cuda.empty_cache()
