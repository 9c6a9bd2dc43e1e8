#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a command.
# usage: tools/pmc.sh OUTDIR GROUPFILE -- python script.py args...
set -o pipefail
OUT=$1; GROUPS_FILE=$2; shift 3
mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd $ROOT
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done < $GROUPS_FILE
echo done
