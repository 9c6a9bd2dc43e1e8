"""Summarise rocprofv3 counter CSVs: per-dispatch mean for a kernel name filter.
usage: pmc_summary.py ROOT [KERNEL_FILTER] [PASS_DIR_PREFIX]
(every ROOT/<prefix>*/**/*counter_collection.csv; prefix default "p", the
pass directories of tools/pmc.sh; tools/gpu_run.sh pmc uses "sq_")."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "scan"
prefix = sys.argv[3] if len(sys.argv) > 3 else "p"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/{prefix}*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:40s} {sum(v)/len(v):14.4g}  (n={len(v)})")
