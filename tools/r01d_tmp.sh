set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r01ac; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_CONV_SPLIT=0" > $O/sweep_out.txt 2>&1
cp gpurun_out/envsweep/tmp.json $O/last_bench.json
echo done
