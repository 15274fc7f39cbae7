#!/bin/bash
# Round 6: the persistent talker-layer engine (QTTS_HIP_TENGINE=1): parity
# against the reference goldens, then an alternating A/B of the bench line.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tengine.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/base_$i.json 2> $O/base_$i.err
  QTTS_HIP_TENGINE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/te_$i.json 2> $O/te_$i.err
done
for f in $O/base_*.json $O/te_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'])"; done
