# Round-4 check on the GPU box: sampler micro-benchmark and kernel tests, the
# long-context / C2 / C4 reference goldens, then a same-box A/B of lib_a vs lib.
#   bash tools/gpu_check.sh [ab-args]
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/chk
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1
cat $O/mb_sample.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sampler or expf" -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/sampler_tests.log 2>&1 || { tail -30 $O/sampler_tests.log; exit 1; }
tail -1 $O/sampler_tests.log
timeout -k 10 1200 python -u -m pytest tests/test_gpu_long.py -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/long_tests.log 2>&1 || { tail -30 $O/long_tests.log; exit 1; }
tail -1 $O/long_tests.log
bash tools/gpu_ab.sh "${1:---steps 3 --warmup 1}" 2 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
