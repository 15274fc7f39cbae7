#!/bin/bash
# Round-5 pass w: the talker GEMVs issue half their weight rows before x is
# staged and the rest after (k_gemvw WS) -- parity, stamps, and a batch-1 A/B
# against the build without it (lib_a), alternating processes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_long.py tests/test_gpu_full.py -k "matvec or bench_workload or greedy_prefix or default_12 or eos" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "passed|failed" $O/tests.log | tail -2
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=5 timeout -k 10 300 python bench.py --batch 1 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b1.json 2> $O/st_b1.err
grep "gm_dbg" $O/st_b1.err | tail -30 | grep -E "launch|x staged|dot done|pf landed"
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['talker_ms'])"; }
for r in 1 2 3 4; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/base_$r.json 2> $O/base_$r.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/ws_$r.json 2> $O/ws_$r.err
  echo "b1 pair $r base $(val $O/base_$r.json) split $(val $O/ws_$r.json)"
done
