# Sampler micro-benchmark, the whole GPU suite, then same-box A/Bs: the talker
# next-launch prefetch options (QTTS_HIP_L2PF_TK) and lib_a (no kernarg preload) vs lib.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/chk2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1
timeout -k 10 120 ./tools/mb_l2pf > $O/mb_l2pf.txt 2>&1 && cat $O/mb_l2pf.txt
cat $O/mb_sample.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_env_ab.sh chk2/pftk "1" "-" "QTTS_HIP_L2PF_TK=1" "QTTS_HIP_L2PF_TK=2" "QTTS_HIP_L2PF_TK=3" > $O/ab_pftk.txt 2>&1 || { cat $O/ab_pftk.txt; exit 1; }
cat $O/ab_pftk.txt
bash tools/gpu_ab.sh "--steps 3 --warmup 1" 2 > $O/ab_preload.txt 2>&1 || { cat $O/ab_preload.txt; exit 1; }
cat $O/ab_preload.txt
