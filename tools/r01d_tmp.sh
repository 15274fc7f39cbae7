set -eo pipefail
O=gpurun_out/r01x; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -k "matvec or e2e or full" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
for w in 1; do echo "== WIDE=$w"; MB_TALKER=1 QTTS_HIP_GEMV_WIDE=$w MB_AUTO=1 timeout -k 10 100 ./tools/mb_gemv; done > $O/mb_gemv_wide.txt 2>&1
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_GEMV_WIDE=0" > $O/sweep_out.txt 2>&1
echo done
