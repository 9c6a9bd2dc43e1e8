"""Fold an SQ counter summary (tools/walk_sq.sh / gpu_c4_pmc.sh output:
"NAME value (n=launches)" lines, per-launch averages) into a committed
profiles/pmc_<workload>.json as its "sq" object, so bench.py's roofline names
the kernel's real limiter:
  valu_busy          = SQ_ACTIVE_INST_VALU x 4 / 1024 / (GRBM_GUI_ACTIVE / 8)
                       (4 cycles per wave64 VALU op on a 16-lane SIMD, 1024
                       SIMDs on 256 CUs; GRBM_GUI_ACTIVE summed over 8 XCDs)
  valu_per_lane_byte = SQ_INSTS_VALU x 64 / lane-hashed bytes per launch
  lds_per_lane_byte  = SQ_INSTS_LDS x 64 / lane-hashed bytes
  lds_bank_conflicts = SQ_LDS_BANK_CONFLICT

  python tools/pmc_sq_json.py SUMMARY.txt profiles/pmc_C3.json [--lane-bytes N]
"""
import argparse
import json
import re


def parse(path):
    out = {}
    for line in open(path):
        m = re.match(r"\s*([A-Z_0-9]+)\s+([0-9.e+]+)", line)
        if m:
            out[m.group(1)] = float(m.group(2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("pmc_json")
    ap.add_argument("--lane-bytes", type=float, default=None)
    a = ap.parse_args()
    c = parse(a.summary)
    d = json.load(open(a.pmc_json))
    lane = a.lane_bytes or d.get("lane_hashed_bytes_per_launch")
    sq = {"source": a.summary,
          "valu_busy": round(c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8), 3)}
    if lane:
        sq["valu_per_lane_byte"] = round(c["SQ_INSTS_VALU"] * 64 / lane, 3)
        if "SQ_INSTS_LDS" in c:
            sq["lds_per_lane_byte"] = round(c["SQ_INSTS_LDS"] * 64 / lane, 3)
    if "SQ_LDS_BANK_CONFLICT" in c:
        sq["lds_bank_conflicts"] = int(c["SQ_LDS_BANK_CONFLICT"])
    d["sq"] = sq
    json.dump(d, open(a.pmc_json, "w"), indent=1)
    print(json.dumps(sq))


if __name__ == "__main__":
    main()
