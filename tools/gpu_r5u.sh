#!/bin/bash
# Round-5 pass U: the ingest's stage A timeline in detail (RCDC_INGEST_PROF=2).
set -o pipefail
OUT=gpurun_out/${1:-r5u}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --reps 2 --no-check"
RCDC_ALLOC_LOG=1 RCDC_INGEST_PROF=2 timeout -k 10 300 $I --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -5 $OUT/ing.log; exit 1; }
grep "^run\|ingest batch" $OUT/ing.log | tail -12; grep -c regrow $OUT/ing.log || true
echo done
