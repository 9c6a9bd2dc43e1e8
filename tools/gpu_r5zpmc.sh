#!/bin/bash
# Round-5 zstd check counters: two rocprofv3 --pmc passes (8 SQ counters
# each) over the device check of 1 GiB of word text; per-kernel averages of
# rcdc_zstd_block_check_kernel into $OUT/sq_summary.txt.
set -o pipefail
OUT=gpurun_out/${1:-r5zpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
for c in "$P1" "$P2"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/sq_$n -o run --output-format csv -- python -u tools/zstd_prof.py --gib 1 --reps 1 --levels 3 --kinds text --check > $OUT/sq_$n.log 2>&1 || { echo "sq $n failed"; tail -5 $OUT/sq_$n.log; exit 1; }
done
for d in $OUT/sq_*/; do python - "$d" <<'PY'
import csv,glob,sys,collections
agg=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "block_check_kernel" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(f"{k:28s} {sum(v)/len(v):16.6g} (n={len(v)})")
PY
done > $OUT/sq_summary.txt
cat $OUT/sq_summary.txt
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
