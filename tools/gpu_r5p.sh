#!/bin/bash
# Round-5 pass P: the ingest with the chunk-id streams at low priority; zstd
# far-path density A/B (blocks on the far path, GiB/s, ratio).
set -o pipefail
OUT=gpurun_out/${1:-r5p}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
I="tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8"
RCDC_INGEST_PROF=1 timeout -k 10 300 $I --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
grep "^run" $OUT/ing.log
RCDC_INGEST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ting -o run --output-format csv -- $I --reps 1 --no-check --json $OUT/ing_tr.json > $OUT/ing_tr.log 2>&1 || { tail -20 $OUT/ing_tr.log; exit 1; }
for f in $(find $OUT/ting -name "*_trace.csv"); do cp $f $OUT/ing_$(basename $f); done; rm -rf $OUT/ting
for v in "RCDC_ZSTD_FARDENSE=8" "RCDC_ZSTD_FARDENSE=3" "RCDC_ZSTD_FAR=0"; do
  env $v RCDC_ZSTD_DBG=4 timeout -k 10 300 python -u tools/zstd_prof.py --gib 8 --reps 2 --kinds csv,text > $OUT/z_$v.txt 2>&1 || { tail -20 $OUT/z_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/z_$v.txt | grep -v "^rcdc zstd phases" ; grep "^rcdc zstd phases" $OUT/z_$v.txt | tail -2 | sed 's/.*far-path/far-path/'
done
echo done
