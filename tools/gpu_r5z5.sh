#!/bin/bash
# Round-5 pass Z5: the zstd check's lane compares in 16-byte steps: the check
# tests, then per kind with phase clocks (RCDC_ZSTD_DBG=8: literals,
# sequences, of which placement + compares) at 16-byte steps and at 4-byte
# steps (RCDC_ZSTD_DBG=24) and the wave-cooperative batch compare
# (RCDC_ZSTD_DBG=40; its tests at 32), and the plain rates.
set -o pipefail
OUT=gpurun_out/${1:-r5z5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd_check.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
RCDC_ZSTD_DBG=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd_check.py tests/test_gpu_zstd.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_coop.log 2>&1 || { tail -40 $OUT/tests_coop.log; exit 1; }
tail -2 $OUT/tests_coop.log
for d in 8 24 40 0 32; do
  RCDC_ZSTD_DBG=$d timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds text,csv,code --check > $OUT/dbg$d.txt 2> $OUT/dbg$d.err || { tail $OUT/dbg$d.err; exit 1; }
  echo "== dbg $d"; cat $OUT/dbg$d.txt; grep "check phases" $OUT/dbg$d.err > $OUT/phases$d.txt || true; tail -3 $OUT/phases$d.txt
done
echo done
