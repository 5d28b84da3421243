#!/usr/bin/env python3
"""Strip-shape tuner: the MI355X analogue of the reference's block tuner
(src/common/block-tuner.cpp:26-34 sweeps tile N x M; src/block-tune.sh:3-42 and
src/buf-tune.sh:3-43 drive it over sizes).

Here the knobs are the kernel family (nw_params.kernel: anti-diagonal strips or
row-scan panels) and its shape (C columns per lane, NC chained compute waves;
nw_params.substrips / strip_waves).  Two steps:

  on the GPU box:   python tools/tune.py --measure --out gpurun_out/tune.json
                    times every supported shape at each size class (device-resident
                    fills, min of --reps after a warmup, bit-exact score checked)
  here:             python tools/tune.py --write gpurun_out/tune.json
                    writes fast-needleman-wunsch_amd/csrc/nw_tuned.h (the table that
                    nw_capi.cpp make_shape consults for auto-shaped fills) and
                    tools/tune_table.json (the measurements, committed)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (kernel, C, NC): 1 = strips (nw_fill.hip), 2 = panels (nw_rows.hip)
SHAPES = [(1, 2, 2), (1, 1, 4), (1, 4, 1), (1, 2, 1), (1, 1, 2), (1, 1, 1),
          (2, 4, 4), (2, 2, 4), (2, 4, 2), (2, 4, 1), (2, 2, 2), (2, 1, 4)]
SIZES = [4096, 16384, 32768, 65536, 131072, 262144]
HEADER = os.path.join(ROOT, "fast-needleman-wunsch_amd", "csrc", "nw_tuned.h")


def measure(args):
    sys.path.insert(0, os.path.join(ROOT, "fast-needleman-wunsch_amd"))
    import torch
    import nwhip
    with open(os.path.join(ROOT, "tests", "golden", "synth_scores.json")) as f:
        golden = json.load(f)
    ctx = nwhip.Context(0)
    res = []
    for n in [int(x) for x in args.sizes.split(",")]:
        s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
        s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
        tab = nwhip.Context.alloc_table(n, n)
        want = golden.get(f"{n}:1,0,-1")
        for kernel, c, nc in SHAPES:
            r = ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=kernel)  # warmup (first touch)
            ts = []
            for _ in range(args.reps):
                r = ctx.fill(s1, s2, tab, substrips=c, strip_waves=nc, kernel=kernel)
                ts.append(r.kernel_ms)
            ok = want is None or r.score == want
            e = {"n": n, "kernel": kernel, "c": c, "nc": nc, "ms": min(ts), "all_ms": [round(t, 3) for t in ts],
                 "gcups": n * n / (min(ts) * 1e6), "score_ok": ok}
            print(json.dumps(e), flush=True)
            res.append(e)
        del tab
        torch.cuda.empty_cache()
    ctx.close()
    with open(args.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(0), "results": res}, f, indent=1)


def write(args):
    with open(args.write) as f:
        data = json.load(f)
    best = {}
    for e in data["results"]:
        if not e["score_ok"]:
            continue
        if e["n"] not in best or e["ms"] < best[e["n"]]["ms"]:
            best[e["n"]] = e
    sizes = sorted(best)
    rows = []
    for i, n in enumerate(sizes):
        # the shape measured best at size n applies to tables larger than the
        # previous measured size
        lo = 0.0 if i == 0 else float((sizes[i - 1] + 1) * (n + 1))
        rows.append((lo, best[n].get("kernel", 1), best[n]["c"], best[n]["nc"], n, best[n]["gcups"]))
    lines = ["// nw_tuned.h -- kernel family and shape per table size for auto fills (nw_params",
             "// kernel = substrips = strip_waves = 0).  Written by tools/tune.py from measurements on",
             f"// an MI355X ({data.get('device', '?')}; tools/tune_table.json); entries in increasing",
             "// min_cells, the last one that applies wins.",
             "#pragma once", "", "namespace nw {", "struct TunedShape {",
             "    double min_cells;  // (n1 + 1) * (n2 + 1) at least",
             "    int kernel;        // 1 = strips (nw_fill.hip), 2 = panels (nw_rows.hip)",
             "    int c, nc;         // columns per lane, chained compute waves per strip / panel",
             "};", "constexpr TunedShape kTuned[] = {"]
    for lo, k, c, nc, n, g in rows:
        lines.append(f"    {{{lo:.1f}, {k}, {c}, {nc}}},  // best at {n}^2: {g:.0f} GCUPS")
    lines += ["};", "}  // namespace nw", ""]
    with open(HEADER, "w") as f:
        f.write("\n".join(lines))
    with open(os.path.join(ROOT, "tools", "tune_table.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("\n".join(lines))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--measure", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tune.json"))
    ap.add_argument("--sizes", default=",".join(map(str, SIZES)))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--write", default="")
    args = ap.parse_args()
    if args.measure:
        measure(args)
    elif args.write:
        write(args)
    else:
        ap.error("--measure (GPU box) or --write <json> (here)")


if __name__ == "__main__":
    main()
