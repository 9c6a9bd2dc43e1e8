#!/bin/bash
# Round-5 pass Q: the ingest with H2D and D2H pumps; zstd far map probe of long repeats
#
set -o pipefail
OUT=gpurun_out/${1:-r5q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py tests/test_gpu_zstd.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
RCDC_INGEST_PROF=1 timeout -k 10 300 $I --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep "^run" $OUT/ing.log
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
RCDC_ZSTD_DBG=4 timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text,mixed --check > $OUT/kinds.txt 2>&1 || { tail -20 $OUT/kinds.txt; exit 1; }
grep -v amdgpu.ids $OUT/kinds.txt | grep -v "^rcdc zstd phases"; grep "^rcdc zstd phases" $OUT/kinds.txt | sed "s/.*far-path/far-path/" | sort | uniq -c
echo done
