# Launch-anatomy micro-benchmark (tools/mb_launch.hip) on the GPU box: plain and
# kernarg-preload builds, then the plain build under rocprofv3 --kernel-trace
# (per-dispatch begin/end beside the in-kernel stamps).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/mbl
mkdir -p $O
cd $GRAFT_REPO_ROOT/tools
timeout -k 10 120 ./mb_launch > $O/plain.txt 2>&1
timeout -k 10 120 ./mb_launch_pre > $O/preload.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d /tmp/mbl -o run -- $GRAFT_REPO_ROOT/tools/mb_launch > $O/prof_stdout.txt 2>&1
find /tmp/mbl -name "*.csv" -exec cp {} $O/ \;
ls $O
