#!/bin/bash
# Round-5 pass B: native ingest tests + walk/parity tests, the C3 and C4
# share bench lines, then tools/ingest_e2e at $2 files of 1 GiB.
set -o pipefail
OUT=gpurun_out/${1:-r5b}
NF=${2:-16}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
(df -h /tmp; free -g; nproc; grep -m1 "model name" /proc/cpuinfo) > $OUT/box.txt 2>&1
python -c "import torch" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_native_ingest.py tests/test_gpu_walk.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-ingest > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload C4 --c4-files 1024 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
echo lines ok
timeout -k 10 500 tools/ingest_e2e --dir /tmp/rcdc_ing --files $NF --file-mib 1024 --readers 8 ${E2EARGS} --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
tail -5 $OUT/ing.log
echo done
