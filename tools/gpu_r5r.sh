#!/bin/bash
# Round-5 pass R: the ingest's batch copies by a shader kernel (DMA queues
# left to the small transfers) A/B; zstd far path with the any-offset probe.
set -o pipefail
OUT=gpurun_out/${1:-r5r}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --reps 2"
run() { timeout -k 10 300 env "$@" $I --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep "^run" $OUT/$N.log | tr '\n' ' '; echo " <- $N"; }
N=dma run RCDC_INGEST_PROF=1
N=k32 run RCDC_INGEST_PROF=1 RCDC_INGEST_KCOPY=32
N=k64 run RCDC_INGEST_PROF=1 RCDC_INGEST_KCOPY=64
N=k128 run RCDC_INGEST_PROF=1 RCDC_INGEST_KCOPY=128
RCDC_INGEST_KCOPY=64 RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
RCDC_ZSTD_DBG=4 timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text,mixed,random --check > $OUT/kinds.txt 2>&1 || { tail -20 $OUT/kinds.txt; exit 1; }
grep -v amdgpu.ids $OUT/kinds.txt | grep -v "^rcdc zstd phases"; grep "^rcdc zstd phases" $OUT/kinds.txt | sed "s/.*far-path/far-path/" | sort | uniq -c
echo done
