set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3pair
python -c "import torch" || exit 1
cp rustic_core_amd/librcdc.so /tmp/librcdc_std.so
for v in std pair std pair; do
  if [ $v = pair ]; then cp rustic_core_amd/librcdc_pair.so rustic_core_amd/librcdc.so; else cp /tmp/librcdc_std.so rustic_core_amd/librcdc.so; fi
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-ingest > gpurun_out/r3pair/$v.json 2> gpurun_out/r3pair/$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r3pair/$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('lane_hashed_bytes_per_launch'), d['parity']['mismatches'])"
done
cp rustic_core_amd/librcdc_pair.so rustic_core_amd/librcdc.so
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r3pair/p1 -o run --output-format csv -- python -u bench.py --steps 4 --warmup 1 --prewarm 0 --no-cpu-baseline --no-parity --no-ingest > gpurun_out/r3pair/p1.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/r3pair rcdc_walk_kernel
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3pair/tests.log 2>&1; tail -1 gpurun_out/r3pair/tests.log
cp /tmp/librcdc_std.so rustic_core_amd/librcdc.so
