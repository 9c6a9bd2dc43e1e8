#!/bin/bash
# Drop-in ABI path: stream/batch tests, then tools/abi_e2e (16 threads, 64 x
# 256 MiB mixed files, 16 MiB reads) under variants given as env strings.
# Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-abi}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python -u -m pytest tests/test_abi_concurrency.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
i=0
for v in "$@"; do
  i=$((i+1))
  for rep in 1 2; do
    env $v RCDC_HOST_PROFILE=1 timeout -k 10 120 tools/abi_e2e --threads 16 --files 64 --file-mib 256 --mixed --batch > $OUT/v${i}_$rep.json 2> $OUT/v${i}_$rep.err || exit 1
    echo "$v rep $rep: $(tail -1 $OUT/v${i}_$rep.json | cut -c1-200) | $(grep 'host path' $OUT/v${i}_$rep.err)"
  done
done
echo done
