#!/bin/bash
# Round-5 pass Z18: the zstd check without per-sequence symbol range checks: zstd
# tests, then per kind with phase
# clocks (RCDC_ZSTD_DBG=8) and plain.
set -o pipefail
OUT=gpurun_out/${1:-r5z18}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for d in 8 0; do
  RCDC_ZSTD_DBG=$d timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds text,csv,code --check > $OUT/dbg$d.txt 2> $OUT/dbg$d.err || { tail $OUT/dbg$d.err; exit 1; }
  echo "== dbg $d"; cat $OUT/dbg$d.txt; grep "check phases" $OUT/dbg$d.err > $OUT/phases$d.txt || true; cat $OUT/phases$d.txt
done
echo done
