#!/bin/bash
# Round-5 pass C: walk tests on the tree, interleaved A/B C3 lines for the
# round-5 walk switches (A: RCDC_WALK_ZONEFAST/KRESET/SORTAGG=0 + no flush),
# the native ingest e2e with its timeline.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r5c}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="--steps 20 --warmup 5 --no-ingest --no-h2h --no-cpu-baseline --no-parity"
for i in 1 2; do
  RCDC_WALK_ZONEFAST=0 RCDC_WALK_KRESET=0 RCDC_WALK_SORTAGG=0 timeout -k 10 300 python -u bench.py $B --no-flush > $OUT/a$i.json 2>> $OUT/ab.err || exit 1
  timeout -k 10 300 python -u bench.py $B > $OUT/b$i.json 2>> $OUT/ab.err || exit 1
done
python - $OUT <<'PY'
import json, sys, os
for n in ["a1", "b1", "a2", "b2"]:
    d = json.loads(open(os.path.join(sys.argv[1], n + ".json")).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(n, d["ms_per_step"], r["kernel_us_per_launch"], r["lane_hashed_bytes_per_launch"], r.get("chain_us_per_launch"))
PY
RCDC_INGEST_PROF=1 timeout -k 10 500 tools/ingest_e2e --dir /tmp/rcdc_ing --files 16 --file-mib 1024 --readers 8 --json $OUT/ing.json > $OUT/ing.log 2>&1 || { tail -20 $OUT/ing.log; exit 1; }
tail -40 $OUT/ing.log
echo done
