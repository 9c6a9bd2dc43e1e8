#!/bin/bash
# Round-5 pass M: C2 step A/B (pipelined chain, paired 128-B loads) and the
# FETCH_SIZE of the better one.
set -o pipefail
OUT=gpurun_out/${1:-r5m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
B="bench.py --workload C2 --no-cpu-baseline --steps 50 --warmup 3"
run() { timeout -k 10 300 env "$@" python -u $B $XB > $OUT/$N.json 2>> $OUT/c2.err || exit 1; python -c "
import json;d=json.loads(open('$OUT/$N.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$N',d['value'],d['ms_per_step'],r.get('kernel_us_per_launch'),r.get('resolve_us_per_launch'))"; }
for i in 1 2; do
  N=c2_def$i XB= run X=1
  N=c2_pipe$i XB=--pipeline run X=1
  N=c2_pair$i XB= run RCDC_SCAN_VARIANT=31
done
RCDC_SCAN_VARIANT=31 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_pair -o run --output-format csv -- python -u bench.py --workload C2 --no-cpu-baseline --steps 10 --warmup 1 --prewarm 0 --no-parity > $OUT/pmc_pair.log 2>&1 || { tail -5 $OUT/pmc_pair.log; exit 1; }
echo done
