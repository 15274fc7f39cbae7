#!/bin/bash
# Round 6: the batch GEMV's tiles per workgroup capped (QTTS_HIP_GB_TPW=2 / 1:
# more, smaller workgroups for the talker's gate|up and q|k|v) against the
# default (up to 3), batch 8 and 16 in alternating processes; batch-8 parity
# on TPW=1 first.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zg
mkdir -p $O
cd $R
QTTS_HIP_GB_TPW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -k "bench_workload_batch8 and not BKZ and not GEMVB" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # name batch env...
  local n=$1 b=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/$n.json 2> $O/$n.err
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['detail'].get('talker_ms'), d['detail'].get('codec_ms'))"
}
for i in 1 2; do
  run b8_base.$i 8 QTTS_X=0
  run b8_tpw2.$i 8 QTTS_HIP_GB_TPW=2
  run b8_tpw1.$i 8 QTTS_HIP_GB_TPW=1
done
for i in 1 2; do
  run b16_base.$i 16 QTTS_X=0
  run b16_tpw2.$i 16 QTTS_HIP_GB_TPW=2
  run b16_tpw1.$i 16 QTTS_HIP_GB_TPW=1
done
