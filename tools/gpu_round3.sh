#!/bin/bash
# Round-3 measurement pass (final tree): the default bench line (C3, with the
# ingest object, parity over every stream and the CPU baseline), C2, C5, C1
# and a C4 share; rocprofv3 kernel stats of the default command; FETCH_SIZE /
# WRITE_SIZE passes and an L2 split for the walk kernel; the native ABI
# driver.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r3final}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || exit 1
echo c3 ok
timeout -k 10 200 python -u bench.py --workload C2 --steps 50 --warmup 5 > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 200 python -u bench.py --workload C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err || exit 1
timeout -k 10 300 python -u bench.py --workload C4 --c4-files 1024 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || exit 1
echo lines ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/stats.log 2>&1 || exit 1
echo stats ok
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/pmc_$n -o run --output-format csv -- python -u bench.py --steps 4 --warmup 1 --prewarm 0 --no-cpu-baseline --no-parity --no-ingest > $OUT/pmc_$n.log 2>&1 || exit 1
done
echo pmc ok
RCDC_HOST_PROFILE=1 timeout -k 10 120 tools/abi_e2e --threads 16 --files 64 --file-mib 256 --mixed --batch > $OUT/abi.json 2> $OUT/abi.err || exit 1
find $OUT -name "*_kernel_trace.csv" -delete
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
