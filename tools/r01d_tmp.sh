set -eo pipefail
O=gpurun_out/r01ah; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -k "matvec or e2e or full" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_GEMV_WIDE=0" "X=2" > $O/sweep_out.txt 2>&1
echo done
