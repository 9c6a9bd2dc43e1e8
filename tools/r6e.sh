set -o pipefail
OUT=gpurun_out/r6e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/c5_trace.py > $OUT/c5_trace.json 2> $OUT/c5_trace.err || { tail $OUT/c5_trace.err; exit 1; }
cat $OUT/c5_trace.json
timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
tail -c 300 $OUT/c5.json
