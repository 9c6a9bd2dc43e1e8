#!/bin/bash
# Round-5 pass Z: host SHA rates (SHA-NI interleaved 1-4 ways, multi-buffer)
# on the box's cores; the ingest with 2-way SHA-NI pack ids and host ids for
# the last two batches, A/B against 1 way and the last batch only.
set -o pipefail
OUT=gpurun_out/${1:-r5z}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
lscpu | grep -i "model name" > $OUT/cpu.txt
timeout -k 10 200 python -u tools/host_sha_rate.py 1 14 > $OUT/sha_rate.json 2> $OUT/sha_rate.err || { tail $OUT/sha_rate.err; exit 1; }
cat $OUT/cpu.txt $OUT/sha_rate.json
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
run() { timeout -k 10 400 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; python -c "import json;d=json.load(open('$OUT/$N.json'));print(' frac', d['frac_of_bound'], d['pcie_bound']['gibs_input'], d['checks'])"; echo " <- $N"; }
N=f16 XA="--files 16" run RCDC_INGEST_PROF=1
N=f32 XA="--files 32" run RCDC_INGEST_PROF=1
N=f32_w1 XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_SHANI_WAYS=1
N=f32_t1 XA="--files 32 --no-check" run RCDC_INGEST_PROF=1 RCDC_INGEST_TAIL_BATCHES=1
N=f64 XA="--files 64 --no-check" run RCDC_INGEST_PROF=1
rm -rf /tmp/rcdc_ing
echo done
