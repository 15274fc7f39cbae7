# Sub-talker k_gemvw phase stamps (pass 5, layer 2, last frame) from a
# `make VARIANT=_a EXTRA=-DQTTS_STAMPS` build, once as built and once with
# every stamped launch waiting for x before issuing its weights.
#   bash tools/gpu_stamps.sh [tag]
TAG=${1:-st}
mkdir -p gpurun_out/$TAG
for XF in 0 1; do
QTTS_HIP_DBG_XFIRST=$XF QTTS_LIB=$GRAFT_REPO_ROOT/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/$TAG/b$XF.json 2> gpurun_out/$TAG/b$XF.err || exit 1
echo "== xfirst $XF"; grep gm_dbg gpurun_out/$TAG/b$XF.err | tail -15
done
