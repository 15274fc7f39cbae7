#!/bin/bash
# Round-5 pass p: the whole-row batch GEMV (k_gemvwb) -- kernel numerics, the
# batch parity tests and the C4 reference goldens, then batch-8 A/B against
# k_gemvb (QTTS_HIP_GEMVWB=0) in alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05p
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_long.py tests/test_gpu_full.py -k "batch or matvec" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "FAIL|passed|failed" $O/tests.log | tail -5
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for gw in 0 1; do
    QTTS_HIP_GEMVWB=$gw timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_gw${gw}_$r.json 2> $O/b8_gw${gw}_$r.err
    echo "b8 round $r gemvwb $gw $(val $O/b8_gw${gw}_$r.json)"
  done
done
for gw in 0 1; do
  QTTS_HIP_GEMVWB=$gw timeout -k 10 300 python bench.py --batch 4 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b4_gw${gw}.json 2> $O/b4_gw${gw}.err
  echo "b4 gemvwb $gw $(val $O/b4_gw${gw}.json)"
done
echo done
