# k_gemvw phase stamps from a `make VARIANT=_a EXTRA=-DQTTS_STAMPS` build:
# the sub-talker (pass 5, layer 2, last frame; once as built and once with
# every stamped launch waiting for x before issuing its weights) and talker
# layer 10 (its O projection's merge prologue: 'w issued', 'merged').
#   bash tools/gpu_stamps.sh [tag]
TAG=${1:-st}
mkdir -p gpurun_out/$TAG
for XF in 0 1; do
QTTS_HIP_DBG_XFIRST=$XF QTTS_LIB=$GRAFT_REPO_ROOT/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/$TAG/b$XF.json 2> gpurun_out/$TAG/b$XF.err || exit 1
echo "== xfirst $XF"; grep gm_dbg gpurun_out/$TAG/b$XF.err | tail -15
done
QTTS_LIB=$GRAFT_REPO_ROOT/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so QTTS_HIP_GM_DBG=10 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/$TAG/t10.json 2> gpurun_out/$TAG/t10.err || exit 1
echo "== talker layer 10"; grep gm_dbg gpurun_out/$TAG/t10.err | tail -26
