#!/bin/bash
# GPU iteration loop: parity tests, then the bench line (and optional rocprof).
# usage: tools/gpu_check.sh TAG [prof]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log
[ $rc -ne 0 ] && exit $rc
if [ "$2" == "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 50 > $OUT/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
fi
exit $rc
