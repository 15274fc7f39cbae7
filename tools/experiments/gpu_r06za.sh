#!/bin/bash
# Round 6: k_convb's stage loads unconditional from clamped addresses, then
# masked (lib_a) vs the tree's conditional loads (lib): codec parity on lib_a,
# then batch-8 / batch-1 codec A/B in alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06za
mkdir -p $O
cd $R
QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_long.py -k "codec or conv or snake or 640_frames_vs or vc_c5 or c5_bench" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_a.log 2>&1 || { tail -30 $O/tests_a.log; exit 1; }
tail -1 $O/tests_a.log
for i in 1 2; do
  for v in "" _a; do
    QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 400 python bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/b8$v.$i.json 2> $O/b8$v.$i.err
  done
done
for v in "" _a; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/b1$v.json 2> $O/b1$v.err
done
for f in $O/b8*.json $O/b1*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); dd=d['detail']; print('$f'.split('/')[-1], d['value'], dd.get('codec_ms'))"; done
