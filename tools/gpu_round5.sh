#!/bin/bash
# Round-5 measurement pass on the final tree: the default bench line (C3 with
# the h2h object from the native engine, parity over every stream, the CPU
# baseline), C2, C5, C1 and the C4 share; rocprofv3 kernel stats of the
# default command; the native host-to-host data path at 32 and 16 files
# (checked; the C3 line's h2h object runs 64); zstd per kind with the device
# check; the native ABI driver.
# Output under gpurun_out/$1.  (PMC: tools/gpu_round4_pmc.sh.)
set -o pipefail
OUT=gpurun_out/${1:-r5final}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
echo c3 ok
timeout -k 10 200 python -u bench.py --workload C2 --steps 50 --warmup 5 > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 200 python -u bench.py --workload C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err || exit 1
timeout -k 10 300 python -u bench.py --workload C4 --c4-files 1024 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || exit 1
echo lines ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-h2h > $OUT/stats.log 2>&1 || exit 1
echo stats ok
I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
timeout -k 10 400 $I --files 32 --json $OUT/h2h32.json > $OUT/h2h32.log 2>&1 || { tail -5 $OUT/h2h32.log; exit 1; }
timeout -k 10 400 $I --files 16 --json $OUT/h2h16.json > $OUT/h2h16.log 2>&1 || { tail -5 $OUT/h2h16.log; exit 1; }
rm -rf /tmp/rcdc_ing
echo h2h ok
timeout -k 10 600 python -u tools/zstd_prof.py --gib 8 --reps 3 --levels 3 --kinds random,zeros,mixed,text,csv,code --check > $OUT/zstd_kinds.txt 2> $OUT/zstd.err || { tail $OUT/zstd.err; exit 1; }
echo zstd ok
timeout -k 10 200 tools/abi_e2e --threads 16 --files 64 --file-mib 256 --mixed --batch > $OUT/abi.json 2> $OUT/abi.err || exit 1
find $OUT -name "*_kernel_trace.csv" -delete
echo done
