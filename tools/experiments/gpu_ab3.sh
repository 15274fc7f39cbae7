# Same-box A/B/C: lib_a (QTTS_LIB), the in-tree lib, and the in-tree lib with
# an environment setting, alternating.
#   bash tools/gpu_ab3.sh "<bench args>" "<env for c>" [rounds]
set -o pipefail
ARGS=${1:-"--steps 3 --warmup 1"}
EC=$2
N=${3:-2}
L=$GRAFT_REPO_ROOT/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so
for i in $(seq $N); do
  for v in a b c; do
    ev=""
    if [ $v = a ]; then export QTTS_LIB=$L; else unset QTTS_LIB; fi
    [ $v = c ] && ev="$EC"
    env $ev timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-profile > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', '$ARGS', '$ev', d['value'], d['ms_per_step'], d.get('first_packet_ms'))"
  done
done
