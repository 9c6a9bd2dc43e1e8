set -o pipefail
OUT=gpurun_out/p2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_sweep.sh p2s "RCDC_CHK_BLOCKS=64" "RCDC_CHK_BLOCKS=96" "RCDC_WALK_SEG=1280" "RCDC_WALK_SPLIT=30" "RCDC_WALK_SPLIT=40 RCDC_WALK_PIECE=3145728" "RCDC_CHK_BLOCKS=64"
