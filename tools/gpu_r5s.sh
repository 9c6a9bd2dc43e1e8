#!/bin/bash
# Round-5 pass S: the ingest against the process's hardware queue count
# (a stream sharing a queue with the 60-70 ms chunk-id kernel waits for it).
set -o pipefail
OUT=gpurun_out/${1:-r5s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --reps 2"
run() { timeout -k 10 300 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; echo " <- $N"; }
N=q16 XA="--hw-queues 16" run RCDC_INGEST_PROF=1
N=q32 XA="--hw-queues 32" run RCDC_INGEST_PROF=1
N=q24 XA="--hw-queues 24" run RCDC_INGEST_PROF=1
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --hw-queues 32 --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
echo done
