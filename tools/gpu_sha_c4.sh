#!/bin/bash
# C4 bench line + rocprof kernel stats of C3 with the fused blob ids.
set -o pipefail
O=gpurun_out/${1:-c4sha}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3sha -o run -- python -u bench.py --workload C3 --steps 5 --warmup 1 --sha256 --sha-steps 3 --no-cpu-baseline --no-parity > $O/c3sha.json 2> $O/c3sha.err &&
timeout -k 10 600 python -u bench.py --workload C4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err
