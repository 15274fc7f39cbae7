# Launch-anatomy micro-benchmark (tools/mb_launch.hip) on the GPU box: plain and
# kernarg-preload builds, then the plain build under rocprofv3 --kernel-trace
# (per-dispatch begin/end beside the in-kernel stamps); the sampler phases and
# tests; the long-context / C2 / C4 reference goldens.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/mbl
mkdir -p $O
cd $GRAFT_REPO_ROOT/tools
timeout -k 10 120 ./mb_launch > $O/plain.txt 2>&1
timeout -k 10 120 ./mb_launch_pre > $O/preload.txt 2>&1
timeout -k 10 60 ./mb_sample > $O/mb_sample.txt 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sampler or expf" -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/sampler_tests.log 2>&1 || { tail -30 $O/sampler_tests.log; exit 1; }
tail -2 $O/sampler_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d /tmp/mbl -o run -- $GRAFT_REPO_ROOT/tools/mb_launch > $O/prof_stdout.txt 2>&1
find /tmp/mbl -name "*.csv" -exec cp {} $O/ \;
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/long_tests.log 2>&1 || { tail -30 $O/long_tests.log; exit 1; }
tail -3 $O/long_tests.log
# same-box A/B: lib_a (no kernarg preload) vs lib (preloaded k_gemvw arguments)
bash tools/gpu_ab.sh "--steps 3 --warmup 1" 2 > $O/ab_preload.txt 2>&1 || { cat $O/ab_preload.txt; exit 1; }
cat $O/ab_preload.txt
