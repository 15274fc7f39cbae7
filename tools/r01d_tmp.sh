set -eo pipefail
O=gpurun_out/r01au; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 1000 bash tools/env_sweep.sh "X=1" "X=2" > $O/sweep_out.txt 2>&1
echo done
