# Sampler micro-benchmark, kernel + model GPU tests, same-box A/B lib_a (no
# kernarg preload) vs lib, and a rocprofv3 kernel-stats pass of the bench.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/chk3
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1
cat $O/mb_sample.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_ab.sh "--steps 3 --warmup 1" 2 > $O/ab_preload.txt 2>&1 || { cat $O/ab_preload.txt; exit 1; }
cat $O/ab_preload.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_bench.json 2> $O/prof_bench.err
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $O
head -16 $O/kernel_stats.csv | cut -c1-160
