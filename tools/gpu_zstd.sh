#!/bin/bash
# zstd ratio / speed pass: the zstd GPU tests, then tools/zstd_prof.py per
# environment setting (A/B knobs: RCDC_ZSTD_HLOG, RCDC_ZSTD_KEY,
# RCDC_ZSTD_REPCHK, ...).  ZENVS="A=1,B=2 C=3" (space-separated settings,
# comma-separated variables); ZARGS for zstd_prof.py.  Output gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-zstd}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
i=0
for e in ${ZENVS:-NONE=1}; do
  i=$((i+1))
  echo "== $e" | tee -a $OUT/prof.txt
  env $(echo $e | tr , ' ') timeout -k 10 600 python -u tools/zstd_prof.py ${ZARGS:---gib 4 --reps 3 --kinds text,csv,code,mixed,random} >> $OUT/prof.txt 2> $OUT/prof_$i.err || { tail $OUT/prof_$i.err; exit 1; }
done
cat $OUT/prof.txt
echo done
