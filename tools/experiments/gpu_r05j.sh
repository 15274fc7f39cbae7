#!/bin/bash
# Round-5 pass j: talker stamps at batch 8 (layer 5) and the batch-1 / C2
# profiles of record + bench lines (gpu_round.sh prof).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
mkdir -p $O
cd $R
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=5 timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_tk_b8.json 2> $O/st_tk_b8.err
grep gm_dbg $O/st_tk_b8.err | tail -28
bash tools/gpu_round.sh r05j prof   # (moved to tools/experiments/ after the pass)
