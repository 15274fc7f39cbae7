set -eo pipefail
O=gpurun_out/r01d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_ATT_PRO=0" "QTTS_HIP_ATT_PRO_WG=64" "QTTS_HIP_ATT_PRO_WG=128" "QTTS_HIP_ATT_PRO=0 QTTS_HIP_FUSE=1" "QTTS_HIP_ATT_PRO=0 QTTS_HIP_PTAB=0" > $O/sweep_out.txt 2>&1
echo done
