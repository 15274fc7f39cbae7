# same-box A/B (lib_a vs in-tree) at batch 2, 4, 8, 16 + batch GPU tests
set -o pipefail
mkdir -p gpurun_out/ab5
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_full.py tests/test_voice_clone.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "batch" > gpurun_out/ab5/gpu_tests.log 2>&1 || { tail -30 gpurun_out/ab5/gpu_tests.log; exit 1; }
tail -1 gpurun_out/ab5/gpu_tests.log
for b in 8 16 4 2; do
  bash tools/gpu_ab.sh "--batch $b --steps 2 --warmup 1" 1 > gpurun_out/ab5/ab_b$b.txt 2>&1 || exit 1
  cat gpurun_out/ab5/ab_b$b.txt
done
