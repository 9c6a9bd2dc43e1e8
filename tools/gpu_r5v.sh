#!/bin/bash
# Round-5 pass V: the ingest's host threads (readers / pack-id hashers) and
# the run length.
set -o pipefail
OUT=gpurun_out/${1:-r5v}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 300 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['checks'])"; echo " <- $N"; }
N=f16_r6_h14 XA="--files 16 --readers 6 --hash-threads 14" run RCDC_INGEST_PROF=1
N=f16_r8_h16 XA="--files 16 --readers 8 --hash-threads 16" run RCDC_INGEST_PROF=1
N=f32_r6_h14 XA="--files 32 --readers 6 --hash-threads 14" run RCDC_INGEST_PROF=1
echo done
