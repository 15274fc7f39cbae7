# rocprofv3 kernel stats of the batch-1 bench under the given environment settings
#   bash tools/gpu_tl_prof.sh <tag> "<env A>" "<env B>" ...   ("-" = none)
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  ev=""; [ "$e" != "-" ] && ev="$e"
  rm -rf /tmp/tp$i
  env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tp$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  f=$(find /tmp/tp$i -name "*kernel_stats.csv" | head -1)
  cp $f $O/stats_$i.csv
  echo "== [$e] $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'])")"
  head -12 $O/stats_$i.csv | cut -d, -f1-4 | cut -c1-140
done
