#!/bin/bash
# Round-5 pass Z7: far tables staged in LDS for the map kernel, and the far
# candidate in the first round trip when there is no table candidate: zstd
# tests, then per kind: default, RCDC_ZSTD_FARLDS=0, RCDC_ZSTD_DBG=64.
set -o pipefail
OUT=gpurun_out/${1:-r5z7}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
i=0
for e in NONE=1 RCDC_ZSTD_FARLDS=0 RCDC_ZSTD_DBG=64; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds csv,text,code --check > $OUT/v$i.txt 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  echo "== $e"; cat $OUT/v$i.txt
done
echo done
