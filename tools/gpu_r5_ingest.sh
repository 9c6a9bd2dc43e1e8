#!/bin/bash
# Native ingest engine on the GPU: its ctypes tests, then tools/ingest_e2e
# (files on disk -> packs + ids in host memory) at $2 files of 1 GiB.
# Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r5ing}
NF=${2:-16}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
(df -h /tmp; free -g; nproc; cat /proc/cpuinfo | grep -m1 "model name") > $OUT/box.txt 2>&1
python -c "import torch" || exit 1
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_ingest.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
fi
timeout -k 10 500 tools/ingest_e2e --dir /tmp/rcdc_ing --files $NF --file-mib 1024 --readers 8 ${E2EARGS} --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
cat $OUT/ing.log | tail -5
echo done
