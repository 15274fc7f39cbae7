# Same-box A/B of environment settings on one build: bench.py lines at the
# given batch sizes, each setting in turn, two rounds.
#   bash tools/gpu_env_ab.sh <tag> "<batch sizes>" "<env A>" "<env B>" ...
# (an env setting is e.g. "QTTS_HIP_BSELF_MIN=2", or "-" for none)
set -o pipefail
TAG=$1; shift
BATCHES=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for b in $BATCHES; do
  for r in 1 2; do
    i=0
    for e in "$@"; do
      i=$((i+1))
      ev=""; [ "$e" != "-" ] && ev="$e"
      env $ev timeout -k 10 400 python3 bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/b${b}_e${i}_r$r.json 2> $O/b${b}_e${i}_r$r.err || exit 1
      python3 -c "import json;d=json.load(open('$O/b${b}_e${i}_r$r.json'));print('batch $b [$e] r$r', d['value'], d['ms_per_step'])"
    done
  done
done
