#!/bin/bash
# C4 share (1024 files, log-uniform 4-256 MiB, random bytes) on one GPU:
# serial vs pipelined passes, a per-piece walk trace, and the bench line
# under each env setting given as "NAME=VALUE ..." strings (piece-size
# sweeps).  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-c4}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
B="python -u bench.py --workload C4 --c4-files 1024 --steps 10 --warmup 3 --no-cpu-baseline"
summ() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']
print('$2', d['value'], d['ms_per_step'], 'hash', r['hash_ms_per_pass'], 'chain', r['chain_ms_per_pass'],
      'lane', r['lane_hashed_bytes_per_pass'], 'ref', r['ref_hashed_bytes_per_pass'],
      'lane/ref', round(r['lane_hashed_bytes_per_pass']/r['ref_hashed_bytes_per_pass'],4),
      'lane TB/s', round(r['lane_hashed_bytes_per_pass']/r['hash_ms_per_pass']/1e9,3), d.get('parity'))"; }
timeout -k 10 300 $B --no-pipeline > $OUT/serial.json 2> $OUT/serial.err || { tail -20 $OUT/serial.err; exit 1; }
summ $OUT/serial.json serial
timeout -k 10 300 $B > $OUT/pipe.json 2> $OUT/pipe.err || { tail -20 $OUT/pipe.err; exit 1; }
summ $OUT/pipe.json pipelined
if [ -z "$NOTRACE" ]; then
WALK_TRACE_NPZ=$OUT/trace timeout -k 10 300 python -u tools/walk_trace.py c4 1024 > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
cat $OUT/trace.json
fi
i=0
for e in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $(echo $e | tr , " ") $B --no-parity > $OUT/sw$i.json 2> $OUT/sw$i.err || { tail -20 $OUT/sw$i.err; exit 1; }
  summ $OUT/sw$i.json "$e"
done
echo done
