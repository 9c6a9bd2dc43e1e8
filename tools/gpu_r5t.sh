#!/bin/bash
# Round-5 pass T: the ingest with polled waits (no thread blocked inside a
# HIP synchronisation call) against blocking waits.
set -o pipefail
OUT=gpurun_out/${1:-r5t}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py tests/test_gpu_zstd_check.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --reps 2"
run() { timeout -k 10 300 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; echo " <- $N"; }
N=poll run RCDC_INGEST_PROF=1
N=block run RCDC_INGEST_PROF=1 RCDC_POLL=0 RCDC_INGEST_POLL=0
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
echo done
