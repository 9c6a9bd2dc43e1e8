#!/bin/bash
# Round-5 pass H: zstd far candidates: the zstd tests, per-kind ratio and
# GiB/s with and without far candidates, and a kernel profile.
set -o pipefail
OUT=gpurun_out/${1:-r5h}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_check.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text,mixed,random --check > $OUT/kinds_far.txt 2>&1 || { tail -20 $OUT/kinds_far.txt; exit 1; }
cat $OUT/kinds_far.txt
RCDC_ZSTD_FAR=0 timeout -k 10 400 python -u tools/zstd_prof.py --gib 8 --reps 3 --kinds csv,code,text --check > $OUT/kinds_nofar.txt 2>&1 || { tail -20 $OUT/kinds_nofar.txt; exit 1; }
cat $OUT/kinds_nofar.txt
RCDC_ZSTD_DBG=8 timeout -k 10 300 python -u tools/zstd_prof.py --gib 2 --reps 1 --kinds text,csv,code --check > $OUT/check_phases.txt 2>&1 || { tail -20 $OUT/check_phases.txt; exit 1; }
grep -v "^rcdc zstd phases" $OUT/check_phases.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u tools/zstd_prof.py --gib 8 --reps 2 --kinds csv,text,mixed > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/zstd_kernel_stats.csv; rm -rf $OUT/prof
python tools/kstats.py $OUT/zstd_kernel_stats.csv | head -12
echo done
