#!/bin/bash
# Round 6: k_convb's SnakeBeta parameters through the scalar cache instead of a
# 12 KB LDS copy (lib), and that plus a 128-VGPR bound so two 8-wave
# workgroups of k_convb<7,4> share a CU (lib_a), against HEAD (lib_b):
# codec tests on both new builds, then alternating batch-8 / batch-1 lines.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06p
mkdir -p $O
cd $R
for v in "" _a; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_kernels.py tests/test_gpu_model.py -k "codec or conv or snake" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests$v.log 2>&1 || { tail -30 $O/tests$v.log; exit 1; }
  tail -1 $O/tests$v.log
done
for i in 1 2; do
  for v in _b "" _a; do
    QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 400 python bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/b8$v.$i.json 2> $O/b8$v.$i.err
  done
done
for v in _b "" _a; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/b1$v.json 2> $O/b1$v.err
done
for f in $O/b8*.json $O/b1*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); dd=d['detail']; print('$f'.split('/')[-1], d['value'], dd.get('codec_ms'), dd.get('step_codec_ms'))"; done
