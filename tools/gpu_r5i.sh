#!/bin/bash
# Round-5 pass I: zstd far candidates (structured-data gate, 16-byte minimum,
# batched map loads) and the checker's deeper bitstream lookahead; the
# native ingest with copies on blit kernels instead of the DMA engines.
set -o pipefail
OUT=gpurun_out/${1:-r5i}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
RCDC_ZSTD_DBG=8 timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text,mixed,random --check > $OUT/kinds.txt 2>&1 || { tail -20 $OUT/kinds.txt; exit 1; }
grep -v amdgpu.ids $OUT/kinds.txt
RCDC_ZCK_OCC=3 RCDC_ZSTD_DBG=8 timeout -k 10 300 python -u tools/zstd_prof.py --gib 8 --reps 1 --kinds text --check > $OUT/text_occ3.txt 2>&1 || { tail -20 $OUT/text_occ3.txt; exit 1; }
grep -v amdgpu.ids $OUT/text_occ3.txt
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
run() { timeout -k 10 300 env "$@" $I $XA --json $OUT/$N.json > $OUT/$N.log 2>&1 || { tail -5 $OUT/$N.log; exit 1; }; grep -v "^ingest batch" $OUT/$N.log | grep "^run" | tr '\n' ' '; echo " <- $N"; }
N=ing XA= run RCDC_INGEST_PROF=1
N=ing_nosdma XA= run RCDC_INGEST_PROF=1 HSA_ENABLE_SDMA=0
echo done
