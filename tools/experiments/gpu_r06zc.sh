#!/bin/bash
# Round 6: above 8 rows the 1.7B talker's down projection on 4 split-K
# columns (k_gemvb; QTTS_HIP_BKZ_WIDE default) instead of 2 (which overflow
# k_gemvb's LDS and fall back to k_gemvm): batch-16 parity both ways, then
# batch-16 / batch-12 lines in alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zc
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -k "batch16 or batch8_lock" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do
  for v in 0 1; do
    QTTS_HIP_BKZ_WIDE=$v timeout -k 10 400 python bench.py --batch 16 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/b16_$v.$i.json 2> $O/b16_$v.$i.err
  done
done
for v in 0 1; do
  QTTS_HIP_BKZ_WIDE=$v timeout -k 10 400 python bench.py --batch 12 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/b12_$v.json 2> $O/b12_$v.err
done
for f in $O/b*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['detail'].get('talker_ms'), d['detail'].get('codec_ms'))"; done
