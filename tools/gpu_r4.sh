#!/bin/bash
# Round-4 GPU pass: the given pytest files (-m gpu), then the C4 share
# (serial vs pipelined, trace, sweeps) and the ABI driver.  Output under
# gpurun_out/$1.  TESTS="..." selects the test files (empty: none).
set -o pipefail
OUT=${1:-r4}
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$OUT/tests.log 2>&1 || { tail -40 gpurun_out/$OUT/tests.log; exit 1; }
  tail -3 gpurun_out/$OUT/tests.log
fi
if [ -n "$C4" ]; then
  NOTRACE=$NOTRACE bash tools/gpu_c4.sh $OUT/c4 $C4SWEEP || exit 1
fi
if [ -n "$C4PMC" ]; then
  bash tools/gpu_c4_pmc.sh $OUT/c4pmc || exit 1
fi
if [ -n "$C3SWEEP" ]; then
  BENCH_ARGS="--no-ingest $C3ARGS" bash tools/gpu_sweep.sh $OUT/c3 $C3SWEEP || exit 1
fi
if [ -n "$ABI" ]; then
  timeout -k 10 300 ./tools/abi_e2e --threads 16 --files 64 --file-mib 256 --batch --mixed > gpurun_out/$OUT/abi_e2e.json 2> gpurun_out/$OUT/abi_e2e.err || { tail gpurun_out/$OUT/abi_e2e.err; exit 1; }
  cat gpurun_out/$OUT/abi_e2e.json
fi
if [ -n "$H2H" ]; then
  timeout -k 10 900 python -u tools/ingest_h2h.py $H2H --json gpurun_out/$OUT/h2h.json > gpurun_out/$OUT/h2h.log 2>&1 || { tail -30 gpurun_out/$OUT/h2h.log; exit 1; }
  tail -3 gpurun_out/$OUT/h2h.log
fi
echo done
