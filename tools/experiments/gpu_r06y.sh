#!/bin/bash
# Round 6: the short attention's K / V rows as unconditional (clamped) loads
# (lib) against HEAD's per-element conditional loads (lib_b): the whole GPU
# suite on lib, k_attn_o phase stamps (lib_s), then batch-1 / batch-8 lines in
# alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06y
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st.json 2> $O/st.err
grep "gm_dbg] O /" $O/st.err | tail -8
for i in 1 2 3; do
  for v in _b ""; do
    QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/b1$v.$i.json 2> $O/b1$v.$i.err
  done
done
for v in _b ""; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib$v/libqwen_tts_amd.so timeout -k 10 400 python bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/b8$v.json 2> $O/b8$v.err
done
for f in $O/b1*.json $O/b8*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['detail'].get('talker_ms'))"; done
