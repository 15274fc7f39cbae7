# Same-box A/B of two builds: lib_a (QTTS_LIB) vs the in-tree lib, alternating.
# usage: bash tools/gpu_ab.sh "<bench args>" [rounds]
set -o pipefail
ARGS=${1:-"--steps 3 --warmup 1"}
N=${2:-2}
L=$GRAFT_REPO_ROOT/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so
for i in $(seq $N); do
  for v in a b; do
    if [ $v = a ]; then export QTTS_LIB=$L; else unset QTTS_LIB; fi
    timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-profile > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', '$ARGS', d['value'], d['ms_per_step'], d.get('first_packet_ms'))"
  done
done
