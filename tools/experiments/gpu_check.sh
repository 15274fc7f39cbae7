# Round-4 check on the GPU box: micro-benchmarks (sampler phases, next-launch
# L2 prefetch), sampler kernel tests, the long-context / C2 / C4 reference
# goldens, then same-box A/Bs: QTTS_HIP_L2PF=0 vs on, lib_a (no kernarg
# preload) vs lib.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/chk
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1
cat $O/mb_sample.txt
timeout -k 10 120 ./tools/mb_l2pf > $O/mb_l2pf.txt 2>&1
cat $O/mb_l2pf.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sampler or expf" -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/sampler_tests.log 2>&1 || { tail -30 $O/sampler_tests.log; exit 1; }
tail -1 $O/sampler_tests.log
timeout -k 10 1200 python -u -m pytest tests/test_gpu_long.py -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/long_tests.log 2>&1 || { tail -30 $O/long_tests.log; exit 1; }
tail -1 $O/long_tests.log
bash tools/gpu_env_ab.sh chk/pf "1" "-" "QTTS_HIP_L2PF=0" > $O/ab_pf.txt 2>&1 || { cat $O/ab_pf.txt; exit 1; }
cat $O/ab_pf.txt
bash tools/gpu_ab.sh "--steps 3 --warmup 1" 1 > $O/ab_preload.txt 2>&1 || { cat $O/ab_preload.txt; exit 1; }
cat $O/ab_preload.txt
