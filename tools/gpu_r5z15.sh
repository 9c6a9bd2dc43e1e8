#!/bin/bash
# Round-5 pass Z15: kernel times of the level-3 compressor on CSV rows, with
# and without far candidates (RCDC_ZSTD_FAR=0), after the map kernel's LDS
# tables (rocprofv3 kernel stats of tools/zstd_prof.py).
set -o pipefail
OUT=gpurun_out/${1:-r5z15}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
for v in far nofar; do
  e=NONE=1; [ $v = nofar ] && e=RCDC_ZSTD_FAR=0
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds csv > $OUT/$v.txt 2> $OUT/$v.err || { tail $OUT/$v.err; exit 1; }
  cat $OUT/$v.txt
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1); head -6 "$f" | cut -d, -f1-5
done
find $OUT -name "*_kernel_trace.csv" -delete
echo done
