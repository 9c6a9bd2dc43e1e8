#!/bin/bash
# Round-5 pass Z6: kernel times of the level-3 compressor with far candidates
# on CSV rows and word text (rocprofv3 kernel stats of tools/zstd_prof.py).
set -o pipefail
OUT=gpurun_out/${1:-r5z6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
for k in csv text; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$k -o run --output-format csv -- python -u tools/zstd_prof.py --gib 4 --reps 3 --levels 3 --kinds $k > $OUT/$k.txt 2> $OUT/$k.err || { tail $OUT/$k.err; exit 1; }
  cat $OUT/$k.txt
  f=$(find $OUT/$k -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-8
done
find $OUT -name "*_kernel_trace.csv" -delete
echo done
