"""Summarise a tools/profile_lease.sh output directory into profiles/ (round 4 onwards).

Each profiled program ran three times under rocprofv3 (MI355X_MICROARCH.md HBM /
rocprofv3 recipe: a kernel-trace --stats pass and one --pmc pass per counter):
    <name>_kt/    --kernel-trace --stats
    <name>_w/     --pmc WRITE_SIZE
    <name>_f/     --pmc FETCH_SIZE
For every (workload key, kernel-name filter) below the median dispatch duration and
the median WRITE_SIZE + 2 x FETCH_SIZE (KiB; FETCH doubled: the gfx950 wide-read
correction) are written to profiles/pmc_traffic.json, read by bench.py (N = 1 line and
its config5 object) and nw_bands.py (N > 1 lines, per GPU).  The rocprofv3 stats
summaries are copied to profiles/<tag>_<name>_kernel_stats.csv.

Usage: python tools/summarize_r04.py <outdir> <tag>
"""
import csv
import datetime
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(ROOT, "profiles")

# (program name, workload key, kernel-name filter, algorithmic bytes per launch)
JOBS = [
    ("bench", "nw_fill_262144x262144:panels", "nw_fill_panels", 4 * 262145 * 262145),
    ("bench", "sw_fill_traceback_65536x65536:strips", "nw_fill_strips", 4 * 65537 * 65537),
    ("band_v", "nw_fill_rowband_65538x524289:vertical", "nw_fill_strips", 4 * 65538 * 524289),
    ("band_h", "nw_fill_rowband_65538x524289:horizontal", "nw_fill_strips", 4 * 65538 * 524289),
]


def one(pattern):
    f = sorted(glob.glob(os.path.join(src, pattern), recursive=True))
    return f[0] if f else None


def durations(name, filt):
    t = one(f"{name}_kt/**/*kernel_trace.csv")
    if t is None:
        return [], None
    rows = [r for r in csv.DictReader(open(t)) if filt in r["Kernel_Name"]]
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows], \
        (rows[0]["Kernel_Name"][:90] if rows else None)


def counter(name, sub, cname, filt):
    f = one(f"{name}_{sub}/**/*counter_collection.csv")
    if f is None:
        return []
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if filt in r["Kernel_Name"] and r["Counter_Name"] == cname]


tp = os.path.join(dst, "pmc_traffic.json")
d = json.load(open(tp)) if os.path.exists(tp) else {}
for name in sorted({j[0] for j in JOBS}):
    st = one(f"{name}_kt/**/*kernel_stats.csv")
    if st:
        shutil.copy(st, os.path.join(dst, f"{tag}_{name}_kernel_stats.csv"))
for name, key, filt, alg in JOBS:
    durs, kname = durations(name, filt)
    wr, fe = counter(name, "w", "WRITE_SIZE", filt), counter(name, "f", "FETCH_SIZE", filt)
    if not durs or not wr or not fe:
        print(f"{key}: missing ({len(durs)} dispatches, {len(wr)} WRITE, {len(fe)} FETCH)")
        continue
    wbytes, fbytes = statistics.median(wr) * 1024.0, 2.0 * statistics.median(fe) * 1024.0
    d[key] = {"hbm_bytes_per_launch": wbytes + fbytes, "write_bytes": wbytes, "fetch_bytes_x2": fbytes,
              "algorithmic_bytes": alg, "traffic_over_algorithmic": round((wbytes + fbytes) / alg, 4),
              "rocprof_ms_median": round(statistics.median(durs), 4), "rocprof_ms_mean": round(statistics.mean(durs), 4),
              "dispatches": len(durs), "round": tag, "kernel_name": kname,
              "achieved_gbps_median": round(alg / (statistics.median(durs) * 1e6), 1),
              "date": datetime.date.today().isoformat(),
              "units": "WRITE_SIZE, FETCH_SIZE in KiB (x1024); FETCH doubled (gfx950 wide-read correction)"}
    print(key, json.dumps(d[key]))
json.dump(d, open(tp, "w"), indent=1, sort_keys=True)
