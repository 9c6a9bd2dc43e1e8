#!/bin/bash
# Round-5 pass Y: SHA-extension pack ids for the last four batches once finish is
# known; tail marks (packs landed, last id); 16, 32 and 96 files of 1 GiB.
set -o pipefail
OUT=gpurun_out/${1:-r5y}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 400 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['pcie_bound']['gibs_input'], d['checks'])"; echo " <- $N"; }
N=f16 XA="--files 16" run RCDC_INGEST_PROF=1
N=f32 XA="--files 32" run RCDC_INGEST_PROF=1
N=f96 XA="--files 96 --no-check" run RCDC_INGEST_PROF=1
echo done
