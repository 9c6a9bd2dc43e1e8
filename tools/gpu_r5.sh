#!/bin/bash
# Round-5 GPU pass: a pytest selection ($2, default the whole -m gpu suite),
# then bench lines (C3 default, C5, C1).  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 1000 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --workload C5 --steps 20 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err || { tail -20 $OUT/c1.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
echo done
