# GPU tests, then same-box A/B (lib_a vs in-tree) at batch 1 and 8
set -o pipefail
mkdir -p gpurun_out/ab9
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab9/gpu_tests.log 2>&1 || { tail -30 gpurun_out/ab9/gpu_tests.log; exit 1; }
tail -1 gpurun_out/ab9/gpu_tests.log
bash tools/gpu_ab.sh "--steps 3 --warmup 1" 2 > gpurun_out/ab9/ab_b1.txt 2>&1 || exit 1
cat gpurun_out/ab9/ab_b1.txt
bash tools/gpu_ab.sh "--batch 8 --steps 3 --warmup 1" 1 > gpurun_out/ab9/ab_b8.txt 2>&1 || exit 1
cat gpurun_out/ab9/ab_b8.txt
