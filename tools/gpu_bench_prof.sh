#!/bin/bash
# Measurement pass: bench lines (C3 default + ABI e2e, C2, C1), a 2-rank gloo
# rehearsal of the multi-rank path, rocprofv3 kernel stats of the default
# bench command, and PMC passes (one counter per rocprofv3 run) for HBM
# traffic.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --abi-e2e --aead > $OUT/c3.json 2> $OUT/c3.err || exit 1
timeout -k 10 200 python bench.py --workload C2 --steps 50 --warmup 5 > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 200 python bench.py --workload C5 --steps 20 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 200 python bench.py --workload C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err || exit 1
RCDC_BENCH_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --workload C2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c2_gloo2.json 2> $OUT/c2_gloo2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --prewarm 0 --no-cpu-baseline --no-parity > $OUT/pmc_$c.log 2>&1 || exit 1
done
# blob encryption alone: kernel stats and SQ counters (tools/aead_prof.py)
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/aead_stats -o run --output-format csv -- python tools/aead_prof.py --gib 8 --reps 5 > $OUT/aead_stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/aead_pmc -o run --output-format csv -- python tools/aead_prof.py --gib 8 --reps 3 > $OUT/aead_pmc.log 2>&1 || exit 1
echo done
