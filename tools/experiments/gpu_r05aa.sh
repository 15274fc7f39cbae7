#!/bin/bash
# Round-5 pass aa: batch GEMV, the talker shapes' weight steps before the x
# staging: half (lib, kept) vs a quarter (lib_b, QTTS_GB_SA_DIV=4); alternating
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aa
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['talker_ms'])"; }
for r in 1 2 3; do
  line="b8 round $r"
  for v in half quarter; do
    case $v in half) lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so ;; *) lib=$R/qwen3-tts-c_amd/lib_b/libqwen_tts_amd.so ;; esac
    QTTS_LIB=$lib timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_${v}_$r.json 2> $O/b8_${v}_$r.err
    line="$line | $v $(val $O/b8_${v}_$r.json)"
  done
  echo "$line"
done
