#!/bin/bash
# One GPU call: kernel / model tests, the batch-8 lock-step parity test, the
# sampler micro-benchmark, then a same-box A/B of the batch chain's L2
# prefetch (QTTS_HIP_L2PF=63 default vs 31 = without bit 32) at batch 8 / 16.
#   bash tools/gpu_b8pf.sh <tag>
set -eo pipefail
TAG=${1:-b8pf}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -m gpu -q -p no:cacheprovider -k "c4_batch8" \
  --timeout 280 --timeout-method thread > $O/gpu_b8.log 2>&1 || { tail -30 $O/gpu_b8.log; exit 1; }
tail -1 $O/gpu_b8.log
timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1 && tail -3 $O/mb_sample.txt
bash tools/gpu_env_ab.sh $TAG "8 16" "-" "QTTS_HIP_L2PF=31"
echo done
