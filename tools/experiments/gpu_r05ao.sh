#!/bin/bash
# Round-5 pass ao: batch-1 bench with the prefill GEMM's split-K scratch (256 MB,
# default) vs none (QTTS_HIP_MGEMM_KZ=0), alternating processes on one box
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ao
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); dt=d.get('detail',{}); print(d['value'], d['first_packet_ms'], dt.get('step_talker_ms'), dt.get('step_prefill_ms'))"; }
for r in 1 2 3; do
  line="b1 round $r"
  for kz in 8 0; do
    QTTS_HIP_MGEMM_KZ=$kz timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $O/b1_kz${kz}_$r.json 2> $O/b1_kz${kz}_$r.err
    line="$line | kz $kz (value, first packet, talker, prefill) $(val $O/b1_kz${kz}_$r.json)"
  done
  echo "$line"
done
