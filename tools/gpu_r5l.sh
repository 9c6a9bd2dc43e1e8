#!/bin/bash
# Round-5 pass L: far candidates with 8-byte keys/verification, used when the
# block's own table fails; the ingest with pre-sized plans, range readers,
# a host-hashed tail batch and single D2H copies.
set -o pipefail
OUT=gpurun_out/${1:-r5l}
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
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
RCDC_INGEST_PROF=1 timeout -k 10 400 $I --files 32 --batch-mib 4096 --json $OUT/ing32_4g.json > $OUT/ing32_4g.log 2>&1 || { tail -20 $OUT/ing32_4g.log; exit 1; }
grep "^run" $OUT/ing32_4g.log
echo done
