#!/bin/bash
# C5 kernel times (rocprofv3 kernel stats of the C5 bench line).
set -o pipefail
OUT=gpurun_out/${1:-r5c5prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s -o run --output-format csv -- python -u bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 1; }
f=$(find $OUT/s -name "*kernel_stats.csv" | head -1); head -10 "$f" | cut -d, -f1-5
find $OUT -name "*_kernel_trace.csv" -delete
echo done
