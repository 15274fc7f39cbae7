# Which edges of the sub-talker chain the next-launch prefetch pays on
# (QTTS_HIP_L2PF masks), batch GEMV tests, and lib_a (no preload) vs lib at batch 8.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/chk4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mb_sample_h4 > $O/mb_sample_h4.txt 2>&1 && tail -3 $O/mb_sample_h4.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sampler" -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/sampler_tests.log 2>&1 || { tail -30 $O/sampler_tests.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_env_ab.sh chk4/pf "1" "-" "QTTS_HIP_L2PF=3" "QTTS_HIP_L2PF=7" "QTTS_HIP_L2PF=11" "QTTS_HIP_L2PF=0" > $O/ab_pf.txt 2>&1 || { cat $O/ab_pf.txt; exit 1; }
cat $O/ab_pf.txt
bash tools/gpu_ab.sh "--batch 8 --steps 3 --warmup 1" 2 > $O/ab_preload_b8.txt 2>&1 || { cat $O/ab_preload_b8.txt; exit 1; }
cat $O/ab_preload_b8.txt
