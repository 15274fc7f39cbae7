# same-box A/B (lib_a vs in-tree) at batch 8 and 16, plus a batch-8 kernel trace of the in-tree build
set -o pipefail
mkdir -p gpurun_out/ab2
bash tools/gpu_ab.sh "--batch 8 --steps 3 --warmup 1" 2 > gpurun_out/ab2/ab_b8.txt 2>&1 || exit 1
cat gpurun_out/ab2/ab_b8.txt
bash tools/gpu_ab.sh "--batch 16 --steps 2 --warmup 1" 1 > gpurun_out/ab2/ab_b16.txt 2>&1 || exit 1
cat gpurun_out/ab2/ab_b16.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/pb8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > /dev/null 2>&1 || exit 1
f=$(find /tmp/pb8 -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_by_grid.py $f 14 > $GRAFT_REPO_ROOT/gpurun_out/ab2/b8_by_grid.txt
cat $GRAFT_REPO_ROOT/gpurun_out/ab2/b8_by_grid.txt
