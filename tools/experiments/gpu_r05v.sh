#!/bin/bash
# Round-5 pass v: the talker layer's in-graph period from kernel-start stamps
# (stamp build lib_s, QTTS_HIP_GM_DBG=5: layer 5's q|k|v, O, gate|up, down;
# their launch offsets within the replayed frame), batch 1 and batch 8
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05v
mkdir -p $O
cd $R
for b in 1 8; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=5 timeout -k 10 300 python bench.py --batch $b --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b$b.json 2> $O/st_b$b.err
  echo "== batch $b"; grep "gm_dbg" $O/st_b$b.err | tail -30
done
