#!/bin/bash
# Round 6: the persistent talker layer actually selected (r06j's gate needed
# S % 32 == 0 and never fired): parity with the engine-use counter, phase
# stamps of layers 13 / 14, then an alternating A/B of the bench line.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tengine.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_TENGINE=1 QTTS_HIP_GM_DBG=13 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_te.json 2> $O/st_te.err
grep te_dbg $O/st_te.err | tail -30
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/base_$i.json 2> $O/base_$i.err
  QTTS_HIP_TENGINE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/te_$i.json 2> $O/te_$i.err
done
for f in $O/base_*.json $O/te_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['detail']['talker_ms'])"; done
