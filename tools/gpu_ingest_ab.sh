#!/bin/bash
# Ingest A/B: the default bench line's ingest object under each env setting
# given (short C3 timed loop, no CPU baseline, no parity).  Output under
# gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/i$i.json 2> $OUT/i$i.err || { echo "FAIL $cfg"; tail -5 $OUT/i$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/i$i.json').read().strip().splitlines()[-1]); g=d['ingest']; print('$cfg', '->', d['value'], d['ms_per_step'], g['gibs_input'], g['ms'])"
done
