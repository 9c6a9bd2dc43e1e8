#!/bin/bash
# Round-end pass: tools/gpu_round.sh (GPU tests, C2/C3/C5 lines, rocprof of
# C2 and C3), smoke(), and rocprof kernel stats of C3 with the blob ids.
set -o pipefail
O=gpurun_out/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_round.sh ${1:-final} &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3sha -o run -- python -u bench.py --workload C3 --steps 5 --warmup 1 --sha256 --sha-steps 3 --no-cpu-baseline --no-parity > $O/c3sha.json 2> $O/c3sha.err
rc=$?
# keep the merge-back under its size cap: per-dispatch traces are large
find $O -name "*_kernel_trace.csv" -delete
exit $rc
