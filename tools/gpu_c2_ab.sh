#!/bin/bash
# C2 scan-kernel A/B: env settings given as arguments, one C2 bench line each
# (value, ms per step, scan kernel us, mismatches).  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --workload C2 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/c2_$i.json 2> $OUT/c2_$i.err || { echo "FAIL $cfg"; tail -5 $OUT/c2_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c2_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', '->', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], d['parity']['mismatches'])"
done
