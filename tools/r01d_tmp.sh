set -eo pipefail
O=gpurun_out/r01av; mkdir -p $O; rm -f $O/configs.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
for c in "--batch 8" "--batch 16" "--batch 1"; do
  for e in X=1 QTTS_HIP_ATTN_O=0; do
  echo "== $c $e" >> $O/configs.txt
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 $c > $O/tmp.json 2>> $O/err.txt
  python3 -c "
import json; d = json.load(open('$O/tmp.json')); fp = d.get('frame_profile', {})
print(d['value'], d['ms_per_step'], fp.get('kernel_ms_per_frame'), fp.get('n_kernels'))" >> $O/configs.txt
  done
done
echo done
