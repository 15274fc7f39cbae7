#!/bin/bash
# Round 6: batch 8 with the 1.7B talker's down projection on 4 split-K
# columns too (QTTS_HIP_BKZ_WIDE=2) and with every batch split on up to 4
# (BKZ_MAX=4), against the default 2, in alternating processes; batch-8
# parity on WIDE=2 first.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ze
mkdir -p $O
cd $R
QTTS_HIP_BKZ_WIDE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -k "bench_workload_batch8" -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/$n.json 2> $O/$n.err
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['detail'].get('talker_ms'), d['detail'].get('codec_ms'))"
}
for i in 1 2 3; do
  run base.$i QTTS_X=0
  run wide2.$i QTTS_HIP_BKZ_WIDE=2
  run bkz4.$i QTTS_HIP_BKZ_MAX=4
done
