# Same-box A/B of environment settings on the EOS-mode and fixed-mode batch-1 bench lines.
#   bash tools/gpu_eos_ab.sh <tag> "<env A>" "<env B>" ...   ("-" = none)
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    ev=""; [ "$e" != "-" ] && ev="$e"
    env $ev timeout -k 10 400 python3 bench.py --eos --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/eos_e${i}_r$r.json 2> $O/eos_e${i}_r$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/eos_e${i}_r$r.json'));print('eos [$e] r$r', d['value'], d['eos_mode']['fixed_same_length_audio_s_per_s'])"
  done
done
