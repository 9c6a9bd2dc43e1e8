#!/bin/bash
# Walk-kernel traffic pass: the walk + parity GPU tests, the default C3 bench
# line, then FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) and the L2
# hit/miss split of rcdc_walk_kernel on a short C3 run.  Output under
# gpurun_out/$1; per-dispatch means in $OUT/pmc_summary.txt.
set -o pipefail
OUT=gpurun_out/${1:-walkpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest > $OUT/c3.json 2> $OUT/c3.err || exit 1
python -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('lane_hashed_bytes_per_launch'), d['parity'])"
i=0
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/p$i -o run --output-format csv -- python -u bench.py --steps 4 --warmup 1 --prewarm 0 --no-cpu-baseline --no-parity --no-ingest > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT rcdc_walk_kernel > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
find $OUT -name "*counter_collection.csv" -size +20M -delete
echo done
