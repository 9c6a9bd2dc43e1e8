"""Walk-to-walk gaps of a pipelined C3 bench from a rocprofv3 kernel trace
(tools/gpu_trace.sh): per consecutive pair of rcdc_walk_kernel launches, the
idle time between walk k's end and walk k + 1's start, and which kernels
ended or started inside that window; then the tail after the last walk.

  python tools/walk_gaps.py TRACE.csv
"""
import csv
import sys


def main(path):
    rows = [r for r in csv.DictReader(open(path)) if "rcdc" in r["Kernel_Name"]]
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["k"] = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    rows.sort(key=lambda r: r["s"])
    walks = [r for r in rows if r["k"] == "rcdc_walk_kernel"]
    gaps = []
    for a, b in zip(walks, walks[1:]):
        g = (b["s"] - a["e"]) / 1e3
        inside = [f"{r['k'].replace('rcdc_', '')}[{(r['s'] - a['e']) / 1e3:.0f}..{(r['e'] - a['e']) / 1e3:.0f}]"
                  for r in rows if r is not a and r is not b and r["e"] > a["e"] - 200e3 and r["s"] < b["s"]
                  and "walk_kernel" not in r["k"]]
        gaps.append(g)
        print(f"walk {(a['e'] - a['s']) / 1e3:8.1f} us, gap {g:7.1f} us: {' '.join(inside)}")
    if gaps:
        print(f"mean gap {sum(gaps) / len(gaps):.1f} us over {len(gaps)} pairs")
    last = walks[-1]
    tail = [r for r in rows if r["s"] >= last["s"] and r is not last]
    if tail:
        end = max(r["e"] for r in tail)
        print(f"after the last walk: {(end - last['e']) / 1e3:.1f} us "
              f"({' '.join(r['k'].replace('rcdc_', '') for r in tail)})")


if __name__ == "__main__":
    main(sys.argv[1])
