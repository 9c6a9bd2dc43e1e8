#!/bin/bash
# Round-5 pass Z2: the ingest with 4-way SHA-NI pack and long ids (2-way for
# the last batches); A/B: host ids for the last batch only, multi-buffer ids.
set -o pipefail
OUT=gpurun_out/${1:-r5z2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 400 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['pcie_bound']['gibs_input'], d['checks'])"; echo " <- $N"; }
N=f16 XA="--files 16" run RCDC_INGEST_PROF=1
N=f32 XA="--files 32" run RCDC_INGEST_PROF=1
N=f32_mb XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_SHA=mb
N=f32_t1 XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_TAIL_BATCHES=1
N=f64 XA="--files 64 --no-check" run RCDC_INGEST_PROF=1
rm -rf /tmp/rcdc_ing
echo done
