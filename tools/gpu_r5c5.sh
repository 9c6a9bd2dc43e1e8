#!/bin/bash
# Round-5 C5 A/B: the C5 line serial (default) and with the pipelined plan
# (--pipeline: run k's chain beside run k + 1's walk), parity on both.
set -o pipefail
OUT=gpurun_out/${1:-r5c5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/serial.json 2> $OUT/serial.err || { tail $OUT/serial.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline --pipeline > $OUT/pipe.json 2> $OUT/pipe.err || { tail $OUT/pipe.err; exit 1; }
for f in serial pipe; do python -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',d['ms_per_step'],d['value'],r.get('kernel_us_per_launch'),r.get('chain_us_per_launch'),r.get('pipelined'),d['parity'])"; done
echo done
