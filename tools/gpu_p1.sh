set -o pipefail
OUT=gpurun_out/p1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -m gpu -x -v -k "pipelined" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/serial$i.json 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pipeline > $OUT/pipe$i.json 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --pipeline > $OUT/pipe_parity.json 2>&1 || exit 1
for f in $OUT/*.json; do echo $f; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'], d['roofline'].get('chain_us_per_launch'), d.get('parity'))"; done
