#!/bin/bash
# Round-5 A/B: the walk cost kernel sampling 64 (default) vs 16 words per
# piece (RCDC_COST_SAMPLES), interleaved C3 lines on one box.
set -o pipefail
OUT=gpurun_out/${1:-r5cost}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
for i in 1 2; do
  for n in 64 16; do
    RCDC_COST_SAMPLES=$n timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-h2h --no-ingest > $OUT/s${n}_$i.json 2> $OUT/s${n}_$i.err || { tail $OUT/s${n}_$i.err; exit 1; }
    python -c "
import json;d=json.loads(open('$OUT/s${n}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('s$n run $i',d['ms_per_step'],d['value'],r.get('kernel_us_per_launch'),d['parity']['mismatches'])"
  done
done
echo done
