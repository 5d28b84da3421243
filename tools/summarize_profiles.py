"""Turn a tools/profile_round.sh output dir into the committed profiles/ files.

  profiles/<round>_kernel_stats.csv   rocprofv3 --stats summary (as written by rocprofv3)
  profiles/<round>_kernel_trace.csv   per-dispatch durations of the fill kernel
  profiles/<round>_pmc.csv            per-dispatch WRITE_SIZE / FETCH_SIZE of the fill kernel
  profiles/<round>_bench.json         the bench line of the same run
  profiles/pmc_traffic.json           {workload: hbm bytes per launch} read by bench.py

HBM bytes per launch (MI355X_MICROARCH.md, HBM): WRITE_SIZE (KiB) is exact for
16-B-per-lane streaming stores (the table flush); FETCH_SIZE (KiB) counts half of the
bytes of wide reads on gfx950 and is doubled here (the fill's reads are 4-8 B per lane
and small: row packs and hand-off granules).
Usage: python tools/summarize_profiles.py <outdir> <round tag, e.g. r01>
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
KERNEL = "nw_fill_"  # nw_fill_strips<...> or nw::rows::nw_fill_panels<...>


def one(pattern):
    f = sorted(glob.glob(os.path.join(src, pattern), recursive=True))
    return f[0] if f else None


stats = one("kt/**/*kernel_stats.csv")
trace = one("kt/**/*kernel_trace.csv")
bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
workload = bench["config"]["workload"]
shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
rows = [r for r in csv.DictReader(open(trace)) if KERNEL in r["Kernel_Name"]]
with open(os.path.join(dst, f"{tag}_kernel_trace.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["dispatch", "kernel", "duration_ms"])
    for r in rows:
        w.writerow([r["Dispatch_Id"], r["Kernel_Name"][:80],
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6])
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]

pmc = {}
for name in ("pmc_w", "pmc_f"):
    f = one(f"{name}/**/*counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        pmc.setdefault(r["Dispatch_Id"] + name, {})[r["Counter_Name"]] = float(r["Counter_Value"])
with open(os.path.join(dst, f"{tag}_pmc.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["dispatch", "counter", "value_KiB"])
    for k, v in sorted(pmc.items()):
        for c, x in v.items():
            w.writerow([k, c, x])
wr = [v["WRITE_SIZE"] for v in pmc.values() if "WRITE_SIZE" in v]
fe = [v["FETCH_SIZE"] for v in pmc.values() if "FETCH_SIZE" in v]
# warmup + timed launches all run the same fill; use the median dispatch
wbytes = statistics.median(wr) * 1024.0
fbytes = 2.0 * statistics.median(fe) * 1024.0
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
tp = os.path.join(dst, "pmc_traffic.json")
d = json.load(open(tp)) if os.path.exists(tp) else {}
key = f"{workload}:{bench['config'].get('kernel', 'strips')}"  # (bench.py pmc_traffic looks it up so)
import datetime  # noqa: E402
d[key] = {"hbm_bytes_per_launch": wbytes + fbytes, "write_bytes": wbytes,
          "fetch_bytes_x2": fbytes, "algorithmic_bytes": bench["roofline"]["bytes_per_launch"],
          "round": tag, "rocprof_fill_ms_median": statistics.median(durs),
          "bench_kernel_ms_avg": bench["roofline"]["kernel_ms_avg"], "kernel_name": rows[0]["Kernel_Name"][:60],
          "date": datetime.date.today().isoformat(),
          "units": "WRITE_SIZE, FETCH_SIZE in KiB (x1024); FETCH doubled (gfx950 wide-read correction)"}
json.dump(d, open(tp, "w"), indent=1, sort_keys=True)
print(json.dumps(d[key], indent=1))
