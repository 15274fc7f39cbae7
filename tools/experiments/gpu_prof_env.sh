# rocprofv3 kernel traces of bench.py at one batch size under each environment
# setting, summarised per (kernel, grid).
#   bash tools/gpu_prof_env.sh <tag> <batch> "<env A>" "<env B>" ...   ("-" = none)
set -o pipefail
TAG=$1; shift
B=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  rm -rf /tmp/pe$i
  if [ "$e" != "-" ]; then export "$e"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/pe$i -o run -- python3 bench.py --batch $B --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_e$i.json 2> $O/bench_e$i.err || exit 1
  if [ "$e" != "-" ]; then unset "${e%%=*}"; fi
  f=$(find /tmp/pe$i -name "*kernel_trace.csv" | head -1)
  echo "== [$e]" > $O/by_grid_e$i.txt
  python3 tools/trace_by_grid.py $f 24 >> $O/by_grid_e$i.txt
  cat $O/by_grid_e$i.txt
done
