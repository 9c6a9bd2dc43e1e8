#!/bin/bash
# Round-5 pass D: walk + native-ingest tests, per-switch C3 A/B lines (each
# round-5 walk switch off alone, all on, all off), the native ingest e2e with
# its timeline.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r5d}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py tests/test_gpu_native_ingest.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="--steps 20 --warmup 5 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
run() { timeout -k 10 300 env "$@" python -u bench.py $B $XB > $OUT/$N.json 2>> $OUT/ab.err || exit 1; }
for i in 1 2; do
  N=all_on$i XB= run X=1
  N=all_off$i XB=--no-flush run RCDC_WALK_ZONEFAST=0 RCDC_WALK_KRESET=0 RCDC_WALK_SORTAGG=0
  N=no_flush$i XB=--no-flush run X=1
  N=no_zone$i XB= run RCDC_WALK_ZONEFAST=0
  N=no_kreset$i XB= run RCDC_WALK_KRESET=0
  N=no_sortagg$i XB= run RCDC_WALK_SORTAGG=0
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
# kernel traces of both ends, for the walk-to-walk gaps (tools/walk_gaps.py)
T="--steps 10 --warmup 3 --prewarm 0.2 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_on -o run --output-format csv -- python -u bench.py $T > $OUT/tr_on.json 2>> $OUT/tr.err || exit 1
RCDC_WALK_ZONEFAST=0 RCDC_WALK_KRESET=0 RCDC_WALK_SORTAGG=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_off -o run --output-format csv -- python -u bench.py $T --no-flush > $OUT/tr_off.json 2>> $OUT/tr.err || exit 1
for v in on off; do f=$(find $OUT/tr_$v -name "*kernel_trace.csv" | head -1); python tools/walk_gaps.py $f > $OUT/gaps_$v.txt; cp $f $OUT/trace_$v.csv; done
rm -rf $OUT/tr_on $OUT/tr_off
tail -3 $OUT/gaps_on.txt $OUT/gaps_off.txt
RCDC_INGEST_PROF=1 timeout -k 10 500 tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep -v "^ingest batch" $OUT/ing.log | tail -8
echo done
