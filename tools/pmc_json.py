"""profiles/pmc_<workload>.json from a `tools/gpu_run.sh pmc` run: per-launch
FETCH_SIZE / WRITE_SIZE of the dominant kernel (separate rocprofv3 passes),
FETCH converted with the calibration measured for per-lane 64-B bursts
(profiles/r01_pmc_hbm.txt, tools/ubench/stream_pattern mode 3: FETCH_SIZE
reports 0.518 of the bytes read), next to the bench line's lane-hashed bytes.

  python tools/pmc_json.py gpurun_out/pmc/C3 C3 rcdc_walk_kernel "source text"
"""
import csv
import glob
import json
import os
import sys

CAL = 0.5182


def per_launch(root, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


def main():
    root, wl, kernel, source = sys.argv[1:5]
    fetch, n = per_launch(root, "FETCH_SIZE", kernel)
    write, _ = per_launch(root, "WRITE_SIZE", kernel)
    line = json.loads(open(os.path.join(root, f"{wl.lower()}.json")).read().strip().splitlines()[-1])
    r = line["roofline"]
    rd = fetch * 1024 / CAL
    wr = write * 1024
    lane = r.get("lane_hashed_bytes_per_launch") or r.get("lane_hashed_bytes_per_pass")
    out = {
        "kernel": f"{kernel} ({wl})",
        "workload": line["config"]["workload"],
        "source": source,
        "launches": n,
        "fetch_size_kib_per_launch": round(fetch, 1),
        "write_size_kib_per_launch": round(wr / 1024, 1),
        "calibration": {"reported_fraction": CAL,
                        "note": "FETCH_SIZE reports ~1/2 of per-lane 64-B burst reads on gfx950 "
                                "(tools/ubench/stream_pattern mode 3, profiles/r01_pmc_hbm.txt)"},
        "hbm_read_bytes_per_launch": int(rd),
        "hbm_write_bytes_per_launch": int(wr),
        "hbm_bytes_per_launch": int(rd + wr),
        "lane_hashed_bytes_per_launch": lane,
        "read_over_lane_bytes": round(rd / lane, 3) if lane else None,
        "algorithmic_bytes_per_launch": r.get("algorithmic_bytes_per_launch")
        or line["config"].get("rank0_share_gib") and int(line["config"]["rank0_share_gib"] * 2**30),
    }
    json.dump(out, open(os.path.join("profiles", f"pmc_{wl}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
