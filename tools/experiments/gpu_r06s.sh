#!/bin/bash
# Round 6 pass s (r + the sweeps wait for the local done signal again): the ring engine with consumer-published granules, attention inputs preloaded, batched merge loads: parity, phase
# stamps of layers 13 / 14, alternating A/B against the launch-per-op layer.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06s
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_tengine.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 2 3; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_TENGINE=$m QTTS_HIP_GM_DBG=13 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_te$m.json 2> $O/st_te$m.err
  grep te_dbg $O/st_te$m.err | tail -34
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/base_$i.json 2> $O/base_$i.err
  QTTS_HIP_TENGINE=2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/te2_$i.json 2> $O/te2_$i.err
  QTTS_HIP_TENGINE=3 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/te3_$i.json 2> $O/te3_$i.err
done
for f in $O/base_*.json $O/te*_?.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['detail']['talker_ms'])"; done
