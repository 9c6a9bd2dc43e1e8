#!/bin/bash
# One GPU-box pass: GPU tests, bench lines (C2 default, C3, C5), rocprof
# kernel stats of C2 and C3.  Output under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-round}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err &&
timeout -k 10 400 python -u bench.py --workload C3 --steps 10 --warmup 2 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python -u bench.py --workload C5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python -u bench.py --steps 200 --no-cpu-baseline --no-parity > $O/prof_c2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python -u bench.py --workload C3 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > $O/prof_c3.log 2>&1
