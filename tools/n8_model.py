"""N-GPU row-band pipeline model of config 4 (524288 x 524288, 8 contiguous mpi-horz
bands of 65536 rows, src/mpi/mpi-horz-driver.cpp:31-32), VERTICAL strip sweep,
driven by the per-strip timeline of ONE band filled alone on one MI355X
(tools/vband_trace.py --save: start / end of every strip of a 524288 x 65536 band).

Each GPU runs the band kernel of the trace: a persistent grid of W workers claims the
band's S strips in order.  Strip k of band r may start when
  * a worker of GPU r is free,
  * strip k-1 of band r has started at least h_s earlier (the trace's minimum start lag),
  * band r-1's strip k has reached its last row + L (its halo: the band's last-row
    segment, stored into this GPU's HBM over xGMI; L = 3 us, the guide's loaded
    hand-off),
and it ends no earlier than its own measured duration after its start and h_e after
strip k-1 ended (the trace's minimum end lag: a strip cannot overtake its left
neighbour).  The durations are those of the band alone: contention between the
bands of one node is per GPU (each has its own HBM), so only the shift of a band's
strip starts changes what each strip meets, which the model ignores.

  python tools/n8_model.py profiles/r04m_vband_def_w256.npz [--bands 8] [--n1-ms 44.9]
prints the modelled N-band step time, GCUPS and the ratio to the N = 1 bench.
"""
import argparse
import heapq

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--bands", default="1,2,4,8")
ap.add_argument("--halo-us", type=float, default=3.0)
ap.add_argument("--n1-ms", type=float, default=44.9, help="N = 1 bench step (262144^2) for the ratio")
args = ap.parse_args()

z = np.load(args.trace)
st, en = z["start"], z["end"]
W, n1, n2 = int(z["waves"]), int(z["n1"]), int(z["n2"])
# A strip's duration in the band-alone run includes its waits for its left neighbour
# (all strips of a pass start together there); with the traces that record them
# (`wait`, vband_trace.py since r04) the model uses the work time dur - wait and lets
# the end-lag constraint rebuild the chain -- older traces give a pessimistic model.
dur = en - st
if "wait" in z.files:
    dur = np.maximum(dur - z["wait"], 0.0)
S = dur.size
lag_s = np.diff(st)
lag_e = np.diff(en)
h_s = max(0.0, float(np.percentile(lag_s, 5)))
h_e = max(0.0, float(np.percentile(lag_e, 5)))
print(f"trace {args.trace}: {S} strips, {W} workers, band {n2} x {n1}, alone {en.max() / 1e3:.2f} ms; "
      f"strip {'work' if 'wait' in z.files else 'duration'} med {np.median(dur):.0f} us (strip 0 {dur[0]:.0f}); "
      f"start lag p5 {h_s:.2f} us, "
      f"end lag p5 {h_e:.2f} us")
n1_cells = 262144.0 * 262144.0
g1 = n1_cells / (args.n1_ms * 1e-3) / 1e9
for P in [int(x) for x in args.bands.split(",")]:
    prev_end = None
    t_end = 0.0
    for r in range(P):
        free = [0.0] * W
        heapq.heapify(free)
        s_prev = e_prev = -1e30
        ends = np.empty(S)
        for k in range(S):
            w = heapq.heappop(free)
            s = max(w, s_prev + h_s)
            if prev_end is not None:
                s = max(s, prev_end[k] + args.halo_us)
            e = max(s + dur[k], e_prev + h_e)
            ends[k] = e
            heapq.heappush(free, e)
            s_prev, e_prev = s, e
        prev_end = ends
        t_end = max(t_end, ends.max())
    cells = float(n1) * n2 * P
    g = cells / (t_end * 1e-6) / 1e9
    print(f"  bands {P}: step {t_end / 1e3:.2f} ms, {g:.0f} GCUPS, {g / g1:.2f}x the N = 1 bench "
          f"({g1:.0f} GCUPS at {args.n1_ms} ms)")
