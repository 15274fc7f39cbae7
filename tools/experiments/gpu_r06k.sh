#!/bin/bash
# Round 6: phase stamps of the persistent talker layer (stamp build lib_s,
# QTTS_HIP_TENGINE=1 QTTS_HIP_GM_DBG=13: layers 13 and 14 of the last frame).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06k
mkdir -p $O
cd $R
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_TENGINE=1 QTTS_HIP_GM_DBG=13 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_te.json 2> $O/st_te.err
grep te_dbg $O/st_te.err | tail -30
