set -o pipefail
mkdir -p gpurun_out/r02t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02t/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02t/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02t/gpu_tests.log
bash tools/gpu_ab.sh "--batch 8 --steps 3 --warmup 1" 2 > gpurun_out/r02t/ab_b8.txt 2>&1 || exit 1
cat gpurun_out/r02t/ab_b8.txt
bash tools/gpu_ab.sh "--batch 4 --steps 2 --warmup 1" 1 > gpurun_out/r02t/ab_b4.txt 2>&1 || exit 1
cat gpurun_out/r02t/ab_b4.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/pb8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > /dev/null 2>&1 || exit 1
f=$(find /tmp/pb8 -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_by_grid.py $f 40 > $GRAFT_REPO_ROOT/gpurun_out/r02t/b8_by_grid.txt
head -30 $GRAFT_REPO_ROOT/gpurun_out/r02t/b8_by_grid.txt
