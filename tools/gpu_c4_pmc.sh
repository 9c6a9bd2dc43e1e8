#!/bin/bash
# C4 share (1024 files) PMC for rcdc_walk_kernel: the bench line (c4.json),
# FETCH_SIZE and WRITE_SIZE in separate passes (-> profiles/pmc_C4.json via
# tools/pmc_json.py), and two SQ passes (VALU / LDS issue, busy cycles).
# Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-c4pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
B="bench.py --workload C4 --c4-files 1024 --no-cpu-baseline"
timeout -k 10 300 python -u $B --steps 10 --warmup 3 > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for c in FETCH_SIZE WRITE_SIZE "$P1" "$P2"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmc_$n -o run --output-format csv -- python -u $B --steps 3 --warmup 1 --prewarm 0 --no-parity > $OUT/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $OUT/pmc_$n.log; exit 1; }
done
for d in $OUT/pmc_*/; do python - "$d" <<'PY'
import csv,glob,sys,collections
agg=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "rcdc_walk_kernel" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(f"{k:28s} {sum(v)/len(v):16.6g} (n={len(v)})")
PY
done > $OUT/summary.txt
cat $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
