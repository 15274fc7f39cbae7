# batch-path parity tests, then a same-box A/B of lib_a (QTTS_LIB) vs the in-tree build at batch 8 and 16.
# lib_a: the baseline build, e.g. `git stash; make -C qwen3-tts-c_amd; cp qwen3-tts-c_amd/lib/*.so
# qwen3-tts-c_amd/lib_a/; git stash pop; make -C qwen3-tts-c_amd` (lib_a/ is git-ignored, not gpurun-ignored)
set -o pipefail
mkdir -p gpurun_out/bab
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_full.py tests/test_voice_clone.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/bab/tests.log 2>&1 || { tail -30 gpurun_out/bab/tests.log; exit 1; }
tail -2 gpurun_out/bab/tests.log
bash tools/gpu_ab.sh "--batch 8 --steps 3 --warmup 1" 2 || exit 1
bash tools/gpu_ab.sh "--batch 16 --steps 3 --warmup 1" 2 || exit 1
