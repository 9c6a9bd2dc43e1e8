#!/bin/bash
# Round-5 PMC pass (as round 4's, C3 without the h2h child process): for C4 (1024-file share), C3 and C2 the
# bench line, then FETCH_SIZE and WRITE_SIZE of the dominant kernel in
# separate rocprofv3 passes (-> profiles/pmc_<W>.json via tools/pmc_json.py
# gpurun_out/$1/<W> <W> <kernel> "<source>"); two SQ passes on C4 (C4SQ=C4) and
# C3 (C3SQ=C3).
# Output under gpurun_out/$1/<W>.
set -o pipefail
OUT=gpurun_out/${1:-r5pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
for W in ${WORKLOADS:-C4 C3 C2}; do
  D=$OUT/$W
  mkdir -p $D
  w=$(echo $W | tr A-Z a-z)
  case $W in
    C4) B="bench.py --workload C4 --c4-files 1024 --no-cpu-baseline"; S=10; PS=3 ;;
    C3) B="bench.py --no-cpu-baseline --no-ingest --no-h2h"; S=20; PS=4 ;;
    C2) B="bench.py --workload C2 --no-cpu-baseline"; S=50; PS=10 ;;
  esac
  timeout -k 10 300 python -u $B --steps $S --warmup 3 > $D/$w.json 2> $D/$w.err || { tail $D/$w.err; exit 1; }
  tail -c 400 $D/$w.json
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d $D/pmc_$c -o run --output-format csv -- python -u $B --steps $PS --warmup 1 --prewarm 0 --no-parity > $D/pmc_$c.log 2>&1 || { echo "pmc $W $c failed"; tail -5 $D/pmc_$c.log; exit 1; }
  done
  echo "$W pmc ok"
done
for SQW in $C4SQ $C3SQ; do
  case $SQW in
    C3) D=$OUT/C3; B="bench.py --no-cpu-baseline --no-ingest --no-h2h" ;;
    *) D=$OUT/C4; B="bench.py --workload C4 --c4-files 1024 --no-cpu-baseline" ;;
  esac
  mkdir -p $D
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  for c in "$P1" "$P2"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $c -d $D/sq_$n -o run --output-format csv -- python -u $B --steps 3 --warmup 1 --prewarm 0 --no-parity > $D/sq_$n.log 2>&1 || { echo "sq $n failed"; tail -5 $D/sq_$n.log; exit 1; }
  done
  for d in $D/sq_*/; do python - "$d" <<'PY'
import csv,glob,sys,collections
agg=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "rcdc_walk_kernel" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in agg.items(): print(f"{k:28s} {sum(v)/len(v):16.6g} (n={len(v)})")
PY
  done > $D/sq_summary.txt
  cat $D/sq_summary.txt
done
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
