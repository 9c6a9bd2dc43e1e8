#!/bin/bash
# Round-5 pass Z17: the packs' D2H in ~256 MiB groups of whole packs, each
# hashed as soon as it lands: native ingest GPU tests, then 16 / 32 / 64
# files (the D2H group A/B: RCDC_INGEST_D2H_GROUP=1e12, one group a batch).
set -o pipefail
OUT=gpurun_out/${1:-r5z17}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 400 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['pcie_bound']['gibs_input'], d['checks'])"; echo " <- $N"; }
N=f16 XA="--files 16" run RCDC_INGEST_PROF=1
N=f32 XA="--files 32" run RCDC_INGEST_PROF=1
N=f32_one XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_D2H_GROUP=1000000000000
N=f64 XA="--files 64 --no-check" run RCDC_INGEST_PROF=1
rm -rf /tmp/rcdc_ing
echo done
