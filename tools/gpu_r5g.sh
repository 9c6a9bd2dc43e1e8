#!/bin/bash
# Round-5 pass G: native ingest A/B of the copy piece size and HW queues,
# then a kernel + copy trace of the default.
set -o pipefail
OUT=gpurun_out/${1:-r5g}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
run() { timeout -k 10 300 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep -v "^ingest batch" $OUT/$N.log | grep "^run" | tr '\n' ' '; echo " <- $N"; }
N=p64 XA= run RCDC_INGEST_PROF=1
N=r16 XA="--readers 16" run X=1
N=r12h6 XA="--readers 12 --hash-threads 6" run X=1
N=q4 XA="--hw-queues 4" run X=1
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
echo done
