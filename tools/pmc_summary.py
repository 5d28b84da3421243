"""Summarise rocprofv3 PMC csv passes (fill kernel only, summed over dispatches / #dispatches)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    tot = collections.defaultdict(float)
    nd = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{d}/pmc*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "nw_fill_" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            nd[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(d)
    for c in sorted(tot):
        print(f"  {c:38s} {tot[c] / max(1, len(nd[c])):.4g}")
