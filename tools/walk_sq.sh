#!/bin/bash
# SQ counters of rcdc_walk_kernel: two passes of at
# most 8 SQ counters each, on the C3 bench and on a C4 batch.  Output under
# gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-walk_sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for w in C3 C4; do
  extra=""; [ $w = C4 ] && extra="--c4-files 256"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/${w}_p$i -o run --output-format csv -- python -u bench.py --workload $w $extra --steps 3 --warmup 1 --prewarm 0 --no-cpu-baseline --no-parity --no-ingest > $OUT/${w}_p$i.log 2>&1 || exit 1
  done
done
for w in C3 C4; do echo "== $w"; for d in $OUT/${w}_p1 $OUT/${w}_p2; do python - "$d" <<'PY'
import csv,glob,sys,collections
agg=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "rcdc_walk_kernel" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(f"{k:28s} {sum(v)/len(v):16.6g} (n={len(v)})")
PY
done; done > $OUT/summary.txt
cat $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
