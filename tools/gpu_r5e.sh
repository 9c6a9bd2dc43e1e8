#!/bin/bash
# Round-5 pass E: walk + native-ingest tests, C3 A/B of the cost kernel grid
# (16 fat workgroups vs round 4's grid) and of the round-5 switches, kernel
# traces of both, the native ingest e2e with its timeline.
set -o pipefail
OUT=gpurun_out/${1:-r5e}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py tests/test_gpu_native_ingest.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="--steps 20 --warmup 5 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
run() { timeout -k 10 300 env "$@" python -u bench.py $B $XB > $OUT/$N.json 2>> $OUT/ab.err || exit 1; }
for i in 1 2; do
  N=new$i XB= run X=1
  N=oldcost$i XB= run RCDC_COST_BLOCKS=4096
  N=r4$i XB=--no-flush run RCDC_COST_BLOCKS=4096 RCDC_WALK_ZONEFAST=0 RCDC_WALK_KRESET=0
done
python - $OUT <<'PY'
import json, sys, os, glob
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    r = d.get("roofline", {})
    if "kernel_us_per_launch" in r:
        print(os.path.basename(f), d["ms_per_step"], r["kernel_us_per_launch"], r.get("chain_us_per_launch"))
PY
T="--steps 10 --warmup 3 --prewarm 0.2 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_new -o run --output-format csv -- python -u bench.py $T > $OUT/tr_new.json 2>> $OUT/tr.err || exit 1
f=$(find $OUT/tr_new -name "*kernel_trace.csv" | head -1); python tools/walk_gaps.py $f > $OUT/gaps_new.txt; cp $f $OUT/trace_new.csv; rm -rf $OUT/tr_new
tail -n 3 $OUT/gaps_new.txt
RCDC_INGEST_PROF=1 timeout -k 10 500 tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep -v "^ingest batch" $OUT/ing.log | tail -n 8
echo done
