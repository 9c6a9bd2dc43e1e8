#!/bin/bash
# GPU test pass + the default bench line.  Output under gpurun_out/$1.
# $2: pytest selection (default: the whole -m gpu suite).
set -o pipefail
OUT=gpurun_out/${1:-t}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 900 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
if [ -z "$NOBENCH" ]; then
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
tail -c 2500 $OUT/bench.json
fi
echo done
