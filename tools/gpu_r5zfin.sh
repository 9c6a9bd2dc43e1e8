#!/bin/bash
# Round-5 zstd on the final tree: the zstd GPU tests, then 8 GiB per kind at
# level 3 with the device check (the committed per-kind table).
set -o pipefail
OUT=gpurun_out/${1:-r5zfin}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py tests/test_gpu_native_ingest.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u tools/zstd_prof.py --gib 8 --reps 3 --levels 3 --kinds random,zeros,mixed,text,csv,code --check > $OUT/zstd_kinds.txt 2> $OUT/zstd.err || { tail $OUT/zstd.err; exit 1; }
cat $OUT/zstd_kinds.txt
echo done
