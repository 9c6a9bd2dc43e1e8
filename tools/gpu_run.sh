#!/bin/bash
# The GPU passes of a round, one parametrised driver (run through gpurun from
# the repository root).  usage: tools/gpu_run.sh MODE [OUT] ; output under
# gpurun_out/OUT (default: the mode's name).
#
#   tests   the whole -m gpu suite and smoke()
#   final   tests + smoke() + the driver's bench command (C3 line with h2h,
#           parity over every stream, the CPU baseline)
#   lines   bench lines C3 (default command), C2, C5, C1, C4 (1024-file share),
#           rocprofv3 kernel stats of the default command (--no-h2h), the
#           native host-to-host path at 32 and 16 files
#   pmc     for WORKLOADS (default "C4 C3 C2"): the bench line, then FETCH_SIZE
#           and WRITE_SIZE of the dominant kernel in separate rocprofv3 passes
#           (-> profiles/pmc_<W>.json with tools/pmc_json.py); SQ passes on
#           the workloads in SQW (default "C3 C4")
#
# Every GPU step has its own time limit and the steps are chained: the first
# failure ends the script.
set -o pipefail
MODE=${1:?mode}
OUT=gpurun_out/${2:-$MODE}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-$(pwd)}
python -c "import torch" || exit 1

bench_cmd() {  # the bench command of a workload (no CPU baseline, no h2h child)
  case $1 in
    C4) echo "bench.py --workload C4 --c4-files 1024 --no-cpu-baseline" ;;
    C3) echo "bench.py --no-cpu-baseline --no-h2h" ;;
    C2) echo "bench.py --workload C2 --no-cpu-baseline" ;;
    C5) echo "bench.py --workload C5 --no-cpu-baseline" ;;
  esac
}

run_tests() {
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
}

case $MODE in
  tests)
    run_tests ;;
  final)
    run_tests
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json \
      2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
    tail -c 600 $OUT/bench.json ;;
  lines)
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3.json \
      2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
    echo c3 ok
    timeout -k 10 200 python -u bench.py --workload C2 --steps 50 --warmup 5 > $OUT/c2.json 2> $OUT/c2.err || exit 1
    timeout -k 10 200 python -u bench.py --workload C5 --steps 20 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
    timeout -k 10 200 python -u bench.py --workload C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err || exit 1
    timeout -k 10 400 python -u bench.py --workload C4 --c4-files 1024 --steps 10 --warmup 3 \
      --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || exit 1
    echo lines ok
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
      python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-h2h \
      > $OUT/stats.log 2>&1 || exit 1
    echo stats ok
    I="tools/ingest_e2e --dir /tmp/rcdc_ing --file-mib 1024 --reps 2"
    timeout -k 10 400 $I --files 32 --json $OUT/h2h32.json > $OUT/h2h32.log 2>&1 || { tail -5 $OUT/h2h32.log; exit 1; }
    timeout -k 10 400 $I --files 16 --json $OUT/h2h16.json > $OUT/h2h16.log 2>&1 || { tail -5 $OUT/h2h16.log; exit 1; }
    rm -rf /tmp/rcdc_ing
    find $OUT -name "*_kernel_trace.csv" -delete
    echo h2h ok ;;
  pmc)
    for W in ${WORKLOADS:-C4 C3 C2}; do
      D=$OUT/$W; mkdir -p $D
      B=$(bench_cmd $W)
      w=$(echo $W | tr A-Z a-z)  # (tools/pmc_json.py reads $D/<w>.json)
      timeout -k 10 400 python -u $B --steps 10 --warmup 3 > $D/$w.json 2> $D/$w.err || { tail $D/$w.err; exit 1; }
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 240 rocprofv3 --pmc $c -d $D/pmc_$c -o run --output-format csv -- \
          python -u $B --steps 3 --warmup 1 --prewarm 0 --no-parity > $D/pmc_$c.log 2>&1 \
          || { echo "pmc $W $c failed"; tail -5 $D/pmc_$c.log; exit 1; }
      done
      echo "$W pmc ok"
    done
    for W in ${SQW:-C3 C4}; do
      D=$OUT/$W; mkdir -p $D
      B=$(bench_cmd $W)
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
      P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
      for c in "$P1" "$P2"; do
        n=$(echo $c | cut -d' ' -f1)
        timeout -s KILL 240 rocprofv3 --pmc $c -d $D/sq_$n -o run --output-format csv -- \
          python -u $B --steps 3 --warmup 1 --prewarm 0 --no-parity > $D/sq_$n.log 2>&1 \
          || { echo "sq $W $n failed"; tail -5 $D/sq_$n.log; exit 1; }
      done
      python tools/pmc_summary.py $D rcdc_walk_kernel sq_ > $D/sq_summary.txt || exit 1
      cat $D/sq_summary.txt
    done
    find $OUT -name "*counter_collection.csv" -size +20M -delete
    echo done ;;
  *)
    echo "unknown mode $MODE"; exit 2 ;;
esac
