#!/bin/bash
# Round-5 pass K: the checker's sequence decode on the scalar unit; the
# ingest's feeder thread (H2D enqueued as soon as a slot is ready).
set -o pipefail
OUT=gpurun_out/${1:-r5k}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py tests/test_gpu_native_ingest.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
RCDC_ZSTD_DBG=8 timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text --check > $OUT/kinds.txt 2>&1 || { tail -20 $OUT/kinds.txt; exit 1; }
grep -v amdgpu.ids $OUT/kinds.txt
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
RCDC_ALLOC_LOG=1 RCDC_INGEST_PROF=1 timeout -k 10 300 $I --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep -c regrow $OUT/ing.log || true
grep "^run" $OUT/ing.log
echo done
