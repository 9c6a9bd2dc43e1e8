#!/bin/bash
# Round-5 pass Z8: the far candidate tried first (RCDC_ZSTD_DBG=128) against
# the table candidate first (default): zstd
# tests, then per kind.
set -o pipefail
OUT=gpurun_out/${1:-r5z8}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
true
true
i=0
for e in NONE=1 RCDC_ZSTD_DBG=128; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds csv,text,code --check > $OUT/v$i.txt 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
  echo "== $e"; cat $OUT/v$i.txt
done
echo done
