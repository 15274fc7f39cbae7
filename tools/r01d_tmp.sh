set -eo pipefail
O=gpurun_out/r01t; mkdir -p $O; rm -f $O/configs.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -k "decode_matvec or batch or matvec" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
for b in 8 16 2; do MB_BATCH=$b timeout -k 10 100 ./tools/mb_gemv; done > $O/mb_gemvm.txt 2>&1
for c in "--batch 8" "--batch 16"; do
  echo "== $c" >> $O/configs.txt
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 $c > $O/tmp.json 2>> $O/err.txt
  python3 -c "
import json; d = json.load(open('$O/tmp.json')); fp = d.get('frame_profile', {})
print(d['value'], d['ms_per_step'], fp.get('kernel_ms_per_frame'), fp.get('n_kernels'))
for k, v in list(fp.get('kernels', {}).items())[:8]: print('   ', k, v)" >> $O/configs.txt
done
echo done
