#!/bin/bash
# A/B of prebuilt librcdc variants (rustic_core_amd/librcdc_<v>.so; "std" =
# the default build) on the C3 bench line.  usage: gpu_lib_ab.sh OUT "v[:ENV=..]" ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
cp rustic_core_amd/librcdc.so /tmp/librcdc_std.so
i=0
for spec in "$@"; do
  i=$((i+1))
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
  if [ $v = std ]; then cp /tmp/librcdc_std.so rustic_core_amd/librcdc.so; else cp rustic_core_amd/librcdc_$v.so rustic_core_amd/librcdc.so; fi
  env $envs timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-30} --warmup 5 --no-cpu-baseline --no-ingest > $OUT/l$i.json 2> $OUT/l$i.err || { echo "FAIL $spec"; tail -5 $OUT/l$i.err; cp /tmp/librcdc_std.so rustic_core_amd/librcdc.so; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/l$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$spec', '->', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('chain_us_per_launch'), d['parity']['mismatches'])"
done
cp /tmp/librcdc_std.so rustic_core_amd/librcdc.so
