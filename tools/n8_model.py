"""N-GPU row-band critical-path models of config 4 (524288 x 524288, 8 contiguous
mpi-horz bands of 65536 rows, src/mpi/mpi-horz-driver.cpp:31-32).

Two modes.

1. VERTICAL strip sweep from a trace (the original mode):
     python tools/n8_model.py profiles/r04m_vband_def_w256.npz [--bands 8] [--n1-ms 44.9]
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
   Prints the modelled N-band step time, GCUPS and the ratio to the N = 1 bench.

2. KERNEL FAMILIES:
     python tools/n8_model.py --families [--inputs profiles/n8_inputs.json]
   the per-family critical path of one N = 8 fill from per-step, per-hop and per-band
   costs measured alone on one GPU (profiles/n8_inputs.json names the source of every
   number), in three columns: the BARE bound (the isolated compute step of
   tools/ubench/tile_step.hip, the guide's loaded hand-off, the store rate of the
   unchained band), the IN-FILL bound (the compute step each shape actually runs at
   inside the fill, from the traces, and the hand-off measured in them), and where
   one exists the CURRENT design's own model.  Families:
     H(C,NC)  row bands swept in horizontal strips of 64*C*NC rows (nw_fill_tband_async
              builds (4,1)): the chain of S = 8*65536/H strips, strip k+1 trailing
              strip k by a hop h = NC*63 steps of lane skew + (NC-1) LDS hand-offs +
              one memory hand-off; the last strip starts (S-1)*h in and sweeps the
              524288 columns in D >= max(band bytes / store rate, n1 * step):
              T >= D + (S-1)*h.
     V(C,NC)  row bands swept in vertical strips of W = 64*C*NC columns: band 7
              starts no earlier than 7 traversals tau of a band by one strip and then
              stores its 137 GB, and the last strip of band 7 sits behind the chain
              across band 0 and down all 8 bands:
              T >= max(7*tau + bytes/rate, (n1/W - 1)*h + 8*tau).
     P        the row-scan panel kernel (nw_rows.hip) as a vertical sweep:
              T >= 7*tau_panel + bytes/rate, tau_panel = 65536 rows * its row time.
     PH       a row-scan sweep of horizontal strips (no lane skew; not built as a
              band sweep): its leader alone needs n1 * the one-wave 256-row scan step.
"""
import argparse
import heapq
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N1_COLS, BAND_ROWS, NBANDS = 524288, 65536, 8


def band_bytes(n1: int = N1_COLS, rows: int = BAND_ROWS) -> float:
    return 4.0 * (n1 + 1) * (rows + 1)


def target_ms(n1_ms: float, n: int = 262144, big: int = N1_COLS, ratio: float = 6.0) -> float:
    """Per-fill time of the big table that is `ratio` x the N = 1 bench's GCUPS."""
    g1 = n * n / (n1_ms * 1e-3)
    return big * big / (ratio * g1) * 1e3


def hop_us(step_ns: float, nc: int, gran_rows: int, mem_us: float, lds_us: float) -> float:
    """Strip-to-strip lag: NC waves of 63-step lane skew, NC-1 intra-strip LDS hand-offs
    (a published chunk + lds_us), one memory hand-off (a chunk + mem_us)."""
    skew = nc * 63 * step_ns * 1e-3
    lds = (nc - 1) * (gran_rows * step_ns * 1e-3 + lds_us)
    gran = gran_rows * step_ns * 1e-3 + mem_us
    return skew + lds + gran


def family_bounds(inp: dict, which: str) -> list:
    """[(family, geometry, T ms, detail)] for the inputs `which`:
    "bare"   -- each shape's isolated compute step (cycles) with the hop built from its
                parts (hop_us) and the guide's memory hand-off;
    "infill" -- each shape's measured strip-to-strip hop and per-row paces from the
                traces of the fill itself (followers' busy pace for the horizontal
                leader's sweep, strip 0's for a vertical traversal)."""
    rate = inp["store_tbps"] * 1e12
    d_store = band_bytes() / rate * 1e3  # ms: one band's bytes at the store rate
    out = []
    shapes = inp["step_cycles"] if which == "bare" else inp["infill"]
    for key, v in shapes.items():
        c, nc = (int(x) for x in key.split(","))
        if which == "bare":
            step = v / inp["clock_ghz"]  # ns per step = per row of a strip
            h = hop_us(step, nc, inp["gran_rows"], inp["mem_handoff_us"], inp["lds_handoff_us"])
            lead = follow = step
        else:
            h, lead, follow = v["hop_us"], v["leader_ns_per_row"], v["follower_ns_per_row"]
        # horizontal strips
        h_rows = 64 * c * nc
        s = NBANDS * BAND_ROWS // h_rows
        d = max(d_store, N1_COLS * follow * 1e-6)
        t_h = d + (s - 1) * h * 1e-3
        out.append((f"H({c},{nc})", f"{h_rows}-row strips, chain of {s}", t_h,
                    f"D {d:.1f} ms + {s - 1} hops x {h:.2f} us (sweep {follow:.1f} ns/column)"))
        # vertical strips
        w = 64 * c * nc
        tau = BAND_ROWS * lead * 1e-6  # ms: one strip's traversal of a band
        t_store = (NBANDS - 1) * tau + d_store
        t_chain = (N1_COLS // w - 1) * h * 1e-3 + NBANDS * tau
        out.append((f"V({c},{nc})", f"{w}-column strips", max(t_store, t_chain),
                    f"max(7 tau + bytes/rate = {t_store:.1f}, {N1_COLS // w - 1} hops x {h:.2f} us + 8 tau "
                    f"= {t_chain:.1f}) ms, tau {tau:.2f} ms"))
    pr = inp["panel_row_ns"][which]
    tau_p = BAND_ROWS * pr * 1e-6
    out.append(("P", "row-scan panels, vertical", (NBANDS - 1) * tau_p + d_store,
                f"7 x {tau_p:.2f} ms + {d_store:.1f} ms (row {pr:.0f} ns)"))
    ph = inp["scan_step_ns_1wave"][which]
    out.append(("PH", "row-scan, horizontal strips (not built)", max(d_store, N1_COLS * ph * 1e-6),
                f"leader alone: {N1_COLS} columns x {ph:.0f} ns"))
    return out


def families_main(args) -> None:
    with open(args.inputs) as f:
        inp = json.load(f)
    tgt = target_ms(inp["n1_bench_ms"])
    print(f"config 4, N = {NBANDS}: 6x the N = 1 bench ({inp['n1_bench_ms']} ms at 262144^2) needs "
          f"<= {tgt:.2f} ms per fill; 5x <= {target_ms(inp['n1_bench_ms'], ratio=5.0):.2f} ms")
    bare = {f: (geo, t, d) for f, geo, t, d in family_bounds(inp, "bare")}
    infill = {f: (geo, t, d) for f, geo, t, d in family_bounds(inp, "infill")}
    cur = inp.get("current", {})
    print(f"{'family':8} {'geometry':36} {'bare bound':>11} {'in-fill':>9} {'current':>9}")
    for fam, (geo, tb, _) in bare.items():
        ti = infill[fam][1] if fam in infill else float("nan")
        tc = cur.get(fam, {}).get("ms")
        print(f"{fam:8} {geo:36} {tb:9.1f}ms {ti:7.1f}ms {('%7.1fms' % tc) if tc else '      -':>9}"
              f"{'  < 6x line' if tb < tgt else ''}")
    print("\nper family (in-fill inputs):")
    for fam, (geo, t, d) in infill.items():
        print(f"  {fam:8} {t:6.1f} ms  {d}")
    for fam, c in cur.items():
        print(f"  current {fam}: {c['ms']} ms -- {c['how']}")


def vertical_trace_main(args) -> None:
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?", help="vertical-sweep band trace (.npz) for mode 1")
    ap.add_argument("--bands", default="1,2,4,8")
    ap.add_argument("--halo-us", type=float, default=3.0)
    ap.add_argument("--n1-ms", type=float, default=44.9, help="N = 1 bench step (262144^2) for the ratio")
    ap.add_argument("--families", action="store_true", help="mode 2: the per-family critical-path table")
    ap.add_argument("--inputs", default=os.path.join(ROOT, "profiles", "n8_inputs.json"))
    args = ap.parse_args()
    if args.families:
        families_main(args)
    elif args.trace:
        vertical_trace_main(args)
    else:
        ap.error("a trace (mode 1) or --families (mode 2)")


if __name__ == "__main__":
    main()
