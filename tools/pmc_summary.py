"""Summarise rocprofv3 counter CSVs: per-dispatch mean for a kernel name filter."""
import csv, glob, sys, collections
root, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "scan")
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:40s} {sum(v)/len(v):14.4g}  (n={len(v)})")
