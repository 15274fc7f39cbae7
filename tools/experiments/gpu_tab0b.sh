# GPU check of the batch layer-0 table path: kernel / model tests, the C4
# lock-step parity test (every variant), then a same-box A/B at batch 8 / 16
# (default vs QTTS_HIP_TAB0B=0).
#   bash tools/gpu_tab0b.sh <tag>
set -eo pipefail
TAG=${1:-tab0b}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -m gpu -q -x -p no:cacheprovider -k "c4_batch8" \
  --timeout 280 --timeout-method thread > $O/gpu_b8.log 2>&1 || { tail -30 $O/gpu_b8.log; exit 1; }
tail -1 $O/gpu_b8.log
bash tools/gpu_env_ab.sh $TAG "8 16" "-" "QTTS_HIP_TAB0B=0"
echo done
