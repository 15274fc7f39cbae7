# device time per launch of the decode GEMV dispatcher on the 1.7B shapes (x + norm, no partials), batch 1 and 8
set -o pipefail
mkdir -p gpurun_out/gs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d /tmp/gs -o run -- python3 $GRAFT_REPO_ROOT/tools/mb_gemvm.py --batch 1,8 --n 100 > $GRAFT_REPO_ROOT/gpurun_out/gs/mb.log 2>&1 || exit 1
f=$(find /tmp/gs -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_by_grid.py $f 30 > $GRAFT_REPO_ROOT/gpurun_out/gs/by_grid.txt
cat $GRAFT_REPO_ROOT/gpurun_out/gs/by_grid.txt
