#!/bin/bash
# Env sweep of the default bench (C3): each line "ENV... -> value ms_per_step".
# usage: gpu_sweep.sh OUT "ENV1=a ENV2=b" "ENV1=c" ...   (BENCH_ARGS extra args)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $(echo $cfg | tr , " ") timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-parity $BENCH_ARGS > $OUT/s$i.json 2> $OUT/s$i.err || { echo "FAIL $cfg"; tail -5 $OUT/s$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/s$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', '->', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('chain_us_per_launch'), r.get('lane_hashed_bytes_per_launch'), r.get('walk_work',{}).get('chk_rounds'))"
done
