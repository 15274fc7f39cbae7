#!/bin/bash
# Round-5 pass x: batch-1 A/B of the split weight issue in k_gemvw: base
# (lib_a, every row before x), the talker's shapes with half their rows first
# (lib, QTTS_GW_WSD=2), a third first (lib_b, QTTS_GW_WSD=3), and half first
# for every shape incl. the sub-talker's (lib_c, QTTS_GW_WS_ALL); alternating
# processes, 4 rounds
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['talker_ms'])"; }
for r in 1 2 3 4; do
  line="b1 round $r"
  for v in a ws2 b c; do
    case $v in ws2) lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so ;; *) lib=$R/qwen3-tts-c_amd/lib_$v/libqwen_tts_amd.so ;; esac
    QTTS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/b1_${v}_$r.json 2> $O/b1_${v}_$r.err
    line="$line | $v $(val $O/b1_${v}_$r.json)"
  done
  echo "$line"
done
