#!/bin/bash
# Round-5 pass ak: prefill O / down split over K, self-reducing (QTTS_HIP_PREFILL_SPLIT=0:
# none) -- the reference goldens (bench workload, C2, C4, EOS), then the
# first packet A/B in alternating processes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ak
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_full.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['first_packet_ms'], d['detail']['prefill_ms'], d['detail']['first_packet_cold_ms'])"; }
for r in 1 2 3; do
  line="b1 round $r"
  for pg in 0 1; do
    QTTS_HIP_PREFILL_SPLIT=$pg timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $O/b1_pg${pg}_$r.json 2> $O/b1_pg${pg}_$r.err
    line="$line | prefill_split $pg (value, first packet, prefill, cold) $(val $O/b1_pg${pg}_$r.json)"
  done
  echo "$line"
done
