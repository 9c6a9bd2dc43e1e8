#!/bin/bash
# Round-5 closing pass on the final tree: the whole GPU suite, smoke(), zstd
# per kind (8 GiB, level 3, device check) and the driver's own bench command.
set -o pipefail
OUT=gpurun_out/${1:-r5fin2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u tools/zstd_prof.py --gib 8 --reps 3 --levels 3 --kinds random,zeros,mixed,text,csv,code --check > $OUT/zstd_kinds.txt 2> $OUT/zstd.err || { tail $OUT/zstd.err; exit 1; }
cat $OUT/zstd_kinds.txt
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json
echo done
