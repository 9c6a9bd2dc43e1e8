#!/bin/bash
# Round-5 pass Z16: the far candidate's first 4 bytes loaded in the first
# round trip (the second only where they match): zstd tests, then per kind.
set -o pipefail
OUT=gpurun_out/${1:-r5z16}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds csv,text,code --check > $OUT/kinds.txt 2> $OUT/kinds.err || { tail $OUT/kinds.err; exit 1; }
cat $OUT/kinds.txt
echo done
