#!/usr/bin/env python3
"""Benchmark: GCUPS of the N x N Needleman-Wunsch fill on MI355X.

Metric (BASELINE.json): GCUPS = inner cells n1*n2 / fill seconds, bit-exact score.
A "step" is one complete fill of the table (device-resident: sequences and
table in HBM before the timed region; nothing copied back inside it).

  N = 1 : BASELINE config 3 -- 262144 x 262144 int32 table (275 GB) on one GPU.
  N > 1 : `value` = row bands across ranks (mpi-horz halo contract, BASELINE
          config 4): n1 = 524288 columns and 65536 rows per GPU (weak scaling;
          N = 8 is 512k x 512k), contiguous as mpi-horz lays them out, each band
          swept in horizontal strips of 256 rows; the same bands in the vertical
          strips of the single-table fill, the rows dealt to the GPUs in 2 blocks
          each (block-cyclic) and column bands (mpi-vert: 65536 columns per GPU x
          524288 rows) run after it as `alt_partitions`.  `value` / `ms_per_step`
          are the PER-FILL latency the reference measures (mpi-horz-driver.cpp:38-83:
          earliest rank start -> latest rank end, each timed fill alone); the same
          fills enqueued back to back give `pipelined_ms_per_fill`, reported beside
          it; fast-needleman-wunsch_amd/nw_bands.py, DESIGN.md "Multi-GPU".

Prints ONE JSON line on rank 0 (see README / DESIGN.md for field meanings).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "fast-needleman-wunsch_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=None,
                    help="sequence length, N x N table (default: 262144 for nw, 65536 for sw)")
    ap.add_argument("--scheme", default=None,
                    help="match,mismatch,gap (default: 1,0,-1 for nw = the reference as shipped; "
                         "1,-1,-1 for sw)")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--substrips", type=int, default=0, help="columns per lane C (0 = auto)")
    ap.add_argument("--strip-waves", type=int, default=0,
                    help="chained compute waves per strip NC (0 = auto)")
    ap.add_argument("--band-rows", type=int, default=65536,
                    help="N>1: rows per GPU band (weak scaling; N=8 -> 512k x 512k, config 4)")
    ap.add_argument("--band-cols", type=int, default=524288, help="N>1: table columns n1")
    ap.add_argument("--partition", choices=["rows", "cols"], default="rows",
                    help="N>1: the partition reported as `value`: row bands (mpi-horz, BASELINE "
                         "config 4; default) or column bands (mpi-vert)")
    ap.add_argument("--alt-partition", choices=["rows", "cols", "none"], default=None,
                    help="N>1: the alternate legs (`alt_partitions`; default: contiguous row bands "
                         "and column bands)")
    ap.add_argument("--band-blocks", type=int, default=1,
                    help="N>1 row bands: blocks of rows per GPU, dealt round robin (1 = contiguous "
                         "mpi-horz bands; the block-cyclic alternate leg uses 2)")
    ap.add_argument("--band-sweep", choices=["auto", "horizontal", "vertical"], default="auto",
                    help="N>1 contiguous row bands: swept in horizontal strips of 256 rows along the "
                         "columns (band r+1 starts a strip hop after band r) or in the vertical strips of "
                         "the single-table fill (band r+1 waits for band r's strips to reach its last "
                         "row); auto = horizontal (the shorter chain at N = 8, DESIGN.md section 5); "
                         "the other runs as an alternate leg")
    ap.add_argument("--tband-shape", default=None,
                    help="N>1 horizontal-strip row bands: strip shape 'C,NC', 4,1 or 2,2 (default: "
                         "nw_bands.TBAND_SHAPE)")
    ap.add_argument("--tband-polls", choices=["auto", "dense", "sparse"], default="auto",
                    help="N>1 horizontal-strip row bands: follower polls with s_sleep 1 (dense) or 64 "
                         "(sparse); auto = dense for chains of 512+ strips, i.e. N >= 2 (nw_bands.tband_dense)")
    ap.add_argument("--kernel", type=int, default=0,
                    help="0 auto, 1 anti-diagonal strips, 2 row-scan panels (nw_params.kernel)")
    ap.add_argument("--col-width", type=int, default=65536,
                    help="N>1 column bands: columns per GPU (weak scaling; n1 = N x this)")
    ap.add_argument("--col-rows", type=int, default=524288, help="N>1 column bands: table rows n2")
    ap.add_argument("--share-gpu", action="store_true",
                    help="N>1 rehearsal: every rank on device 0 (co-resident halves)")
    ap.add_argument("--workload", choices=["nw", "sw"], default="nw",
                    help="nw: the headline NW fill (config 3); sw: Smith-Waterman + traceback (config 5)")
    ap.add_argument("--warmup-timeout-ms", type=int, default=5000,
                    help="N>1: watchdog bound of every wait in the warmup launches (fail fast: a halo that "
                         "never arrives ends the run in seconds, naming the band)")
    ap.add_argument("--debug-withhold-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config5", action="store_true",
                    help="N=1: skip the config-5 (Smith-Waterman 64k + traceback) sub-measurement")
    ap.add_argument("--cpu-n", type=int, default=32768, help="CPU baseline sample side")
    args = ap.parse_args()
    # per-workload defaults; values the user passed are never rewritten
    if args.n is None:
        args.n = 65536 if args.workload == "sw" else 262144
    if args.scheme is None:
        args.scheme = "1,-1,-1" if args.workload == "sw" else "1,0,-1"
    return args


def golden_score(n: int, scheme) -> int | None:
    path = os.path.join(ROOT, "tests", "golden", "synth_scores.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        g = json.load(f)
    return g.get(f"{n}:{','.join(str(x) for x in scheme)}")


def _physical_cores() -> int:
    """Distinct (physical id, core id) pairs in /proc/cpuinfo."""
    cores, phys = set(), "0"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    cores.add((phys, line.split(":", 1)[1].strip()))
    except OSError:
        pass
    return len(cores) or (os.cpu_count() or 1)


def cpu_baseline(n: int, scheme):
    """The reference's CPU fills timed on this host in this run:
    serial (src/serial/serial.cpp) on 1 thread and idxarray-mt
    (src/idxarray/idxarray-mt.cpp) on all usable physical cores and on 8 threads,
    OMP_PROC_BIND=close, median of 3 each, on an n x n sample of the bench workload.
    The reference sources compiled unmodified into oracle/_ref ("reference"), or the
    oracle's restatement ("port") when _ref is absent.  Each leg runs in its own
    process (oracle/cpu_baseline.py) so the OpenMP settings reach the runtime."""
    phys = _physical_cores()
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp_env = os.environ.get("OMP_NUM_THREADS")
    usable = min(phys, share, int(omp_env)) if omp_env and omp_env.isdigit() else min(phys, share)
    legs = {}
    for name, fill, threads in [("serial", "serial", 1), ("idxarray_mt_all", "idxarray-mt", usable),
                                ("idxarray_mt_8", "idxarray-mt", 8)]:
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
        out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--fill", fill,
                              "--n", str(n), "--scheme", ",".join(map(str, scheme))],
                             capture_output=True, text=True, env=env, timeout=600)
        if out.returncode != 0:
            legs[name] = {"error": out.stderr[-300:]}
            continue
        legs[name] = json.loads(out.stdout.strip().splitlines()[-1])
    ok = {k: v for k, v in legs.items() if "gcups" in v}
    best = max(ok.values(), key=lambda v: v["gcups"]) if ok else None
    kinds = sorted({v["kind"] for v in ok.values()})
    return {"value": best["gcups"] if best else None, "unit": "GCUPS",
            "cores": best["threads"] if best else None,
            "kind": kinds[0] if len(kinds) == 1 else "mixed",
            "sample": f"{n}x{n} synthetic seeds 1/2, scheme {tuple(scheme)}; value = the fastest leg "
                      f"({best['fill'] if best else '-'}); median of 3 per leg, fill call only "
                      f"(driver.cpp:26-30), OMP_PROC_BIND=close",
            "legs": {k: {kk: v[kk] for kk in ("fill", "kind", "threads", "gcups", "seconds", "score")
                         if kk in v} | ({"error": v["error"]} if "error" in v else {})
                     for k, v in legs.items()},
            "host": _host_cpu(), "physical_cores": phys, "cpu_share": share,
            "omp_num_threads_env": omp_env,
            "all_cores_cap": (f"idxarray_mt_all runs {usable} threads: capped by OMP_NUM_THREADS={omp_env}, "
                              "the CPU share the GPU box grants one GPU's job" if usable < min(phys, share)
                              else f"idxarray_mt_all runs all {usable} usable physical cores")}


def _host_cpu() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(workload: str, kernel: str):
    """HBM bytes per launch of this workload's fill kernel from the committed
    rocprofv3 PMC summary (profiles/pmc_traffic.json: WRITE_SIZE + 2 x FETCH_SIZE,
    the gfx950 correction of MI355X_MICROARCH.md), and where it came from.  Not
    measured in this run: PMC passes are separate rocprofv3 runs
    (tools/profile_round.sh)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    e = d.get(f"{workload}:{kernel}")
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), (f"profiles/pmc_traffic.json [{workload}:{kernel}], "
                                           f"{e.get('round', '?')} {e.get('date', '')}, "
                                           f"kernel {e.get('kernel_name', '?')}").strip()


def run_single(args):
    import torch
    import nwhip

    scheme = tuple(int(x) for x in args.scheme.split(","))
    n = args.n
    torch.cuda.set_device(0)
    ctx = nwhip.Context(0)
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    tab = nwhip.Context.alloc_table(n, n)
    stream = torch.cuda.current_stream()

    kw = dict(waves=args.waves, substrips=args.substrips, strip_waves=args.strip_waves, kernel=args.kernel)
    for _ in range(args.warmup):
        ctx.fill(s1, s2, tab, scheme, sync=False, **kw)
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        ctx.fill(s1, s2, tab, scheme, sync=False, **kw)
        e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    status = ctx.status()
    if status != 0:
        raise RuntimeError(f"fill reported status {status} ({nwhip.strerror(status)})")
    kms = [e0.elapsed_time(e1) for e0, e1 in evs]
    shape = ctx.fill(s1, s2, tab, scheme, **kw)  # (one more fill, untimed: what ran)
    score = int(tab[n, n].item())
    want = golden_score(n, scheme)
    cells = n * n
    value = cells * args.steps / wall / 1e9
    avg_ms = sum(kms) / len(kms)
    table_bytes = 4.0 * (n + 1) * (n + 1)
    achieved = table_bytes / (avg_ms * 1e6)  # GB/s, algorithmic bytes (4 B per cell)
    workload = f"nw_fill_{n}x{n}"
    kname = {1: "strips", 2: "panels"}.get(shape.kernel, "?")
    traffic, traffic_src = pmc_traffic(workload, kname)
    out = {
        "metric": "GCUPS (DP cell updates/s) on NxN NW fill, bit-exact score",
        "value": round(value, 2),
        "unit": "GCUPS",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (i.i.d. uniform {1,2,3,4}, seeds 1/2)",
        "config": {"workload": workload, "n1": n, "n2": n, "scheme": list(scheme),
                   "table_bytes": int(table_bytes), "layout": "row-major int32, pitch "
                   f"{nwhip.table_pitch(n)}", "waves": args.waves or "auto", "parallelism": "single GPU",
                   "kernel": kname,
                   "shape": [shape.substrips, shape.strip_waves]},
        "score": score,
        "score_golden": want,
        "score_ok": (want == score) if want is not None else None,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_ms_avg": round(avg_ms, 3), "bytes_per_launch": int(table_bytes)},
        "kernel": nwhip.version(),
    }
    del tab
    torch.cuda.empty_cache()
    if not args.no_config5:
        # BASELINE config 5 (Smith-Waterman 64k + on-device traceback), timed in the
        # same run so that the driver's bench records it too; not part of `value`
        out["config5"] = measure_sw(65536, (1, -1, -1), max(3, args.steps), max(2, args.warmup))
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_n, scheme)
    print(json.dumps(out), flush=True)


def measure_sw(n: int, scheme, steps: int, warmup: int, substrips: int = 0, strip_waves: int = 0,
               kernel: int = 0) -> dict:
    """BASELINE config 5: Smith-Waterman fill + best cell + on-device traceback of
    the n x n synthetic pair (a step = all three), checked against
    tests/golden/sw_golden.json (the build's CPU restatement: the reference has no
    local alignment, parity unpinned).  Returns the measurement (no JSON printing)."""
    import hashlib
    import torch
    import nwhip
    torch.cuda.set_device(0)
    ctx = nwhip.Context(0)
    s1 = torch.from_numpy(nwhip.synth(1, n)).cuda()
    s2 = torch.from_numpy(nwhip.synth(2, n)).cuda()
    tab = nwhip.Context.alloc_table(n, n)

    def step():
        r = ctx.fill(s1, s2, tab, scheme, substrips=substrips, strip_waves=strip_waves,
                     mode=nwhip.MODE_SW, kernel=kernel)
        al, ops = ctx.sw_traceback(s1, s2, tab, (r.end_i, r.end_j), scheme)
        return r, al, ops

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fills, tbs = [], []
    for _ in range(steps):
        r, al, ops = step()
        if r.status != 0:
            raise RuntimeError(f"SW fill reported status {r.status} ({nwhip.strerror(r.status)})")
        fills.append(r.kernel_ms)
        tbs.append(al.traceback_ms)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpath = os.path.join(ROOT, "tests", "golden", "sw_golden.json")
    g = json.load(open(gpath))["synth"].get(f"{n}:{','.join(map(str, scheme))}") if os.path.exists(gpath) else None
    ok = None
    if g is not None:
        ok = (al.score == g["score"] and [al.end_i, al.end_j] == g["end"] and
              [al.begin_i, al.begin_j] == g["begin"] and hashlib.sha256(ops.tobytes()).hexdigest() == g["ops_sha256"])
    table_bytes = 4.0 * (n + 1) * (n + 1)
    fill_ms = sum(fills) / len(fills)
    kname = {1: "strips", 2: "panels"}.get(r.kernel, "?")
    traffic, traffic_src = pmc_traffic(f"sw_fill_traceback_{n}x{n}", kname)
    out = {"value": round(n * n * steps / wall / 1e9, 2), "unit": "GCUPS", "steps": steps, "warmup": warmup,
           "ms_per_step": round(wall / steps * 1e3, 3), "workload": f"sw_fill_traceback_{n}x{n}",
           "scheme": list(scheme), "kernel": kname, "shape": [r.substrips, r.strip_waves],
           "score": al.score, "end": [al.end_i, al.end_j], "begin": [al.begin_i, al.begin_j],
           "n_ops": int(al.n_ops), "result_ok": ok,
           "fill_ms_avg": round(fill_ms, 3), "traceback_ms_avg": round(sum(tbs) / len(tbs), 3),
           "roofline": {"bound": "hbm", "achieved": round(table_bytes / (fill_ms * 1e6), 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(table_bytes / (fill_ms * 1e6) / HBM_PEAK_GBPS, 4),
                        "traffic": traffic, "traffic_source": traffic_src,
                        "basis": "fill kernel (+ best cell / locate) only, 4 B per cell"}}
    del tab
    ctx.close()
    torch.cuda.empty_cache()
    return out


def run_sw(args):
    """--workload sw: BASELINE config 5 as the line itself (measure_sw)."""
    import nwhip
    scheme = tuple(int(x) for x in args.scheme.split(","))
    m = measure_sw(args.n, scheme, args.steps, args.warmup, args.substrips, args.strip_waves, args.kernel)
    out = {"metric": "GCUPS (DP cell updates/s) on NxN Smith-Waterman fill + on-device traceback",
           "value": m["value"], "unit": "GCUPS", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": m["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "int32", "data": "synthetic (i.i.d. uniform {1,2,3,4}, seeds 1/2)",
           "config": {"workload": m["workload"], "n1": args.n, "n2": args.n, "scheme": list(scheme),
                      "parallelism": "single GPU", "kernel": m["kernel"], "shape": m["shape"]}}
    out.update({k: m[k] for k in ("score", "end", "begin", "n_ops", "result_ok", "fill_ms_avg",
                                  "traceback_ms_avg", "roofline")})
    out["kernel"] = nwhip.version()
    print(json.dumps(out), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus: int, world_env: str | None, ndev: int, share_gpu: bool) -> tuple[str, str]:
    """How bench.py runs for --gpus `gpus` (the program owns its rank setup, as
    mpi-horz-driver.cpp:14-32 does): ("single", ""), ("ranks", "") when a launcher
    already started one process per rank, ("spawn", "") when this process must start
    `gpus` ranks itself, or ("refuse", why).  Pure: ndev = torch.cuda.device_count()
    (which initialises no GPU on this image), world_env = $WORLD_SIZE or None."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least 1"
    if world_env not in (None, ""):
        try:
            world = int(world_env)
        except ValueError:
            return "refuse", f"WORLD_SIZE={world_env!r} is not an integer"
        if world != gpus:
            return "refuse", (f"WORLD_SIZE={world} but --gpus {gpus}: the launcher started a different number "
                              "of ranks than the line would report")
        if world == 1:
            return "single", ""
        if not share_gpu and ndev < world:
            return "refuse", (f"{world} ranks but {ndev} visible GPU(s): one rank per GPU needs {world} "
                              "(--share-gpu rehearses all ranks on device 0)")
        return "ranks", ""
    if gpus == 1:
        return "single", ""
    if ndev < 1:
        return "refuse", "no visible GPU"
    if not share_gpu and ndev < gpus:
        return "refuse", (f"--gpus {gpus} but {ndev} visible GPU(s) (--share-gpu rehearses all ranks on "
                          "device 0)")
    return "spawn", ""


def spawn_ranks(gpus: int) -> int:
    """`python bench.py --gpus N` with no launcher: start N ranks under
    torch.distributed.run as a CHILD process (never an exec: this process has made no
    GPU call, and the ranks make their own), with the rendezvous on 127.0.0.1.  The
    ranks inherit stdout, so rank 0's JSON line is this command's line.  Returns the
    child's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, NW_BENCH_LAUNCHER="self")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if args.workload == "sw":
        run_sw(args)
        return
    import torch
    plan, why = launch_plan(args.gpus, os.environ.get("WORLD_SIZE"), torch.cuda.device_count(), args.share_gpu)
    if plan == "refuse":
        print(f"bench.py: refusing to run: {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus))
    if plan == "ranks":
        import nw_bands  # multi-GPU row bands (+ column bands as the alternate leg)
        nw_bands.cpu_baseline_fn = cpu_baseline
        nw_bands.run_bands(args)
        return
    run_single(args)


if __name__ == "__main__":
    main()
