#!/bin/bash
# Round-5 pass N: the ingest without legacy-default-stream read-backs and
# with synchronous AEAD calls; zstd per-kernel split for CSV and text.
set -o pipefail
OUT=gpurun_out/${1:-r5n}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py tests/test_gpu_aead.py tests/test_gpu_pack.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
RCDC_INGEST_PROF=1 timeout -k 10 300 $I --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep "^run" $OUT/ing.log
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
for k in csv text; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/z$k -o run --output-format csv -- python -u tools/zstd_prof.py --gib 8 --reps 2 --kinds $k > $OUT/z$k.log 2>&1 || { tail -20 $OUT/z$k.log; exit 1; }
f=$(find $OUT/z$k -name "*kernel_stats.csv" | head -1); cp $f $OUT/zstd_${k}_stats.csv; rm -rf $OUT/z$k
python tools/kstats.py $OUT/zstd_${k}_stats.csv | head -8
done
echo done
