set -eo pipefail
O=gpurun_out/r01ai; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
echo done
