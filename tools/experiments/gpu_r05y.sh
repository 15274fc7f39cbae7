#!/bin/bash
# Round-5 pass y: the split weight issue for the talker's O projection with the
# attention merge in its prologue too (lib_d, QTTS_GW_WS_AM) vs the kept form
# (lib); alternating processes, 4 rounds; then the O-merge tests on lib_d
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['talker_ms'])"; }
for r in 1 2 3 4; do
  line="b1 round $r"
  for v in ws2 d; do
    case $v in ws2) lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so ;; *) lib=$R/qwen3-tts-c_amd/lib_$v/libqwen_tts_amd.so ;; esac
    QTTS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/b1_${v}_$r.json 2> $O/b1_${v}_$r.err
    line="$line | $v $(val $O/b1_${v}_$r.json)"
  done
  echo "$line"
done
QTTS_LIB=$R/qwen3-tts-c_amd/lib_d/libqwen_tts_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_full.py -k "bench_workload or default_12 or hd128" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_d.log 2>&1 || { tail -20 $O/tests_d.log; exit 1; }
tail -1 $O/tests_d.log
