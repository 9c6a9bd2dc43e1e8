#!/bin/bash
# Round-5 pass Z4: two hash threads kept for long chunk ids (A/B: none);
# 16, 32 and 64 files.
set -o pipefail
OUT=gpurun_out/${1:-r5z4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 400 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['pcie_bound']['gibs_input'], d['checks'])"; echo " <- $N"; }
N=f16 XA="--files 16" run RCDC_INGEST_PROF=1
N=f32 XA="--files 32" run RCDC_INGEST_PROF=1
N=f32_r0 XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_ID_THREADS=0
N=f32_r4 XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_ID_THREADS=4
N=f64 XA="--files 64 --no-check" run RCDC_INGEST_PROF=1
rm -rf /tmp/rcdc_ing
echo done
