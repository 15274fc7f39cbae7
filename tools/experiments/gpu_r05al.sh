#!/bin/bash
# Round-5 pass al: prefill split kz 2 vs 4 (QTTS_HIP_PREFILL_SPLIT=2|4) at 1.7B and 0.6B;
# goldens at kz 4 -- the reference goldens (bench workload, C2, C4, EOS), then the
# first packet A/B in alternating processes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05al
mkdir -p $O
cd $R
QTTS_HIP_PREFILL_SPLIT=4 timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_full.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['first_packet_ms'], d['detail']['prefill_ms'], d['detail']['first_packet_cold_ms'])"; }
for r in 1 2 3; do
  line="b1 round $r"
  for pg in 2 4; do
    QTTS_HIP_PREFILL_SPLIT=$pg timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $O/b1_pg${pg}_$r.json 2> $O/b1_pg${pg}_$r.err
    line="$line | prefill_split $pg (value, first packet, prefill, cold) $(val $O/b1_pg${pg}_$r.json)"
  done
  echo "$line"
done
for r in 1 2; do
  line="0.6b greedy round $r"
  for pg in 2 4; do
    QTTS_HIP_PREFILL_SPLIT=$pg timeout -k 10 300 python bench.py --preset 0.6b --greedy --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $O/c2_pg${pg}_$r.json 2> $O/c2_pg${pg}_$r.err
    line="$line | prefill_split $pg (value, first packet, prefill, cold) $(val $O/c2_pg${pg}_$r.json)"
  done
  echo "$line"
done
