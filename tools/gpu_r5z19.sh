#!/bin/bash
# Round-5 pass Z19: the walk's assembly split into placement (a workgroup
# per stream) and a grid-wide scatter of the segments: walk / parity / shard
# / bench GPU tests, then the C5, C3 and C4 lines with parity.
set -o pipefail
OUT=gpurun_out/${1:-r5z19}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py tests/test_shard.py tests/test_gpu_bench.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-h2h > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload C4 --c4-files 1024 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
for f in c5 c3 c4; do python -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',d['ms_per_step'],d['value'],r.get('kernel_us_per_launch'),r.get('chain_us_per_launch'),d['parity'].get('mismatches'))"; done
echo done
