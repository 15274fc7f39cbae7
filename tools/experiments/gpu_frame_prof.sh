# rocprofv3 kernel trace of bench.py steps at the given batch sizes, summarised
# per (kernel, grid): the per-frame picture of the lock-step decode.
#   bash tools/gpu_frame_prof.sh <tag> "<batch sizes>"
set -o pipefail
TAG=${1:-fp}
BATCHES=${2:-"1 8"}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b in $BATCHES; do
  rm -rf /tmp/fp$b
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/fp$b -o run -- python3 bench.py --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_b$b.json 2> $O/bench_b$b.err || exit 1
  f=$(find /tmp/fp$b -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_by_grid.py $f 40 > $O/by_grid_b$b.txt
  head -30 $O/by_grid_b$b.txt
done
