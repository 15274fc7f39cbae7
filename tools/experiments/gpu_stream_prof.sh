# first-packet anatomy: the exact streaming codec push of 1 frame, kernel trace by (kernel, grid)
set -o pipefail
mkdir -p gpurun_out/sp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/sp -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_stream.py > $GRAFT_REPO_ROOT/gpurun_out/sp/prof_stream.log 2>&1 || exit 1
f=$(find /tmp/sp -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_by_grid.py $f 40 > $GRAFT_REPO_ROOT/gpurun_out/sp/by_grid.txt
cat $GRAFT_REPO_ROOT/gpurun_out/sp/prof_stream.log | tail -5
head -45 $GRAFT_REPO_ROOT/gpurun_out/sp/by_grid.txt
