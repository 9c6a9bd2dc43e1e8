"""Short per-kernel summary of a rocprofv3 --stats run_kernel_stats.csv."""
import csv, re, sys

for path in sys.argv[1:]:
    print(f"# {path}")
    print(f"{'kernel':48s} {'calls':>7s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
        name = re.sub(r"^at::native::.*?(\w+_kernel).*", r"torch:\1", name)
        print(f"{name[:48]:48s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:10.2f} "
              f"{float(r['MinNs'])/1e3:9.2f} {float(r['MaxNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}")
