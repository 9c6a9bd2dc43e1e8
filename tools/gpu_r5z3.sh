#!/bin/bash
# Round-5 pass Z3: the zstd checker with the Huffman / LL-ML union in LDS
# (16 waves per CU by LDS): the zstd GPU tests, then check rates per kind at
# RCDC_ZCK_OCC=2 (12 waves) and 4 (16 waves, 128 VGPRs).
set -o pipefail
OUT=gpurun_out/${1:-r5z3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for o in 2 4; do
  RCDC_ZCK_OCC=$o timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds text,csv,code,mixed --check > $OUT/occ$o.txt 2> $OUT/occ$o.err || { tail $OUT/occ$o.err; exit 1; }
  echo "== occ $o"; cat $OUT/occ$o.txt
done
echo done
