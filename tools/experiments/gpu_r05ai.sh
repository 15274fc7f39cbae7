#!/bin/bash
# Round-5 pass ai: the talker's split weight issue on the 0.6B (C2, talker
# H 1024): with (lib) vs without (lib_a, QTTS_GW_NO_WS); alternating, 3 rounds
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ai
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['talker_ms'])"; }
for r in 1 2 3; do
  line="c2 round $r"
  for v in nows ws; do
    lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so; [ $v = nows ] && lib=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so
    QTTS_LIB=$lib timeout -k 10 300 python bench.py --preset 0.6b --greedy --no-cpu-baseline --no-profile --steps 8 --warmup 2 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err
    line="$line | $v $(val $O/c2_${v}_$r.json)"
  done
  echo "$line"
done
