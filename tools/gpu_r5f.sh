#!/bin/bash
# Round-5 pass F: C3 A/B of the process's hardware queue count (walk k+1's
# cost/sort kernels behind walk k on a shared queue?), a kernel trace at the
# better count, and the native ingest under a kernel + copy trace.
set -o pipefail
OUT=gpurun_out/${1:-r5f}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
B="--steps 20 --warmup 5 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
run() { timeout -k 10 300 env "$@" python -u bench.py $B > $OUT/$N.json 2>> $OUT/ab.err || exit 1; }
for i in 1 2; do
  N=q4_$i run GPU_MAX_HW_QUEUES=4
  N=q8_$i run GPU_MAX_HW_QUEUES=8
  N=q16_$i run GPU_MAX_HW_QUEUES=16
done
python - $OUT <<'PY'
import json, sys, os, glob
for f in sorted(glob.glob(os.path.join(sys.argv[1], "q*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    r = d.get("roofline", {})
    print(os.path.basename(f), d["ms_per_step"], r.get("kernel_us_per_launch"), r.get("chain_us_per_launch"))
PY
T="--steps 10 --warmup 3 --prewarm 0.2 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
export GPU_MAX_HW_QUEUES=16
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr16 -o run --output-format csv -- python -u bench.py $T > $OUT/tr16.json 2>> $OUT/tr.err || exit 1
f=$(find $OUT/tr16 -name "*kernel_trace.csv" | head -1); python tools/walk_gaps.py $f > $OUT/gaps16.txt; rm -rf $OUT/tr16
tail -n 3 $OUT/gaps16.txt
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --reps 1 --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
grep -v "^ingest batch" $OUT/ing_tr.log | tail -n 6
echo done
