#!/bin/bash
# Walk-path A/B pass: the walk parity tests, then the C3 bench line under
# each env setting given (tools/gpu_sweep.sh).  Output under gpurun_out/$1.
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1 || { tail -30 gpurun_out/$OUT/tests.log; exit 1; }
tail -2 gpurun_out/$OUT/tests.log
bash tools/gpu_sweep.sh $OUT/sweep "$@"
