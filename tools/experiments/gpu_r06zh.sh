#!/bin/bash
# Round 6: batch 16 with the sub-talker's split-K O / down on 2 columns
# (BKZ_MAX=2) while the talker's wide down keeps 4 (BKZ_WIDE=2) -- r06zd's
# BKZ_MAX=2 also sent the talker's down back to k_gemvm -- against the
# default (4 columns everywhere), alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zh
mkdir -p $O
cd $R
run() {  # name batch env...
  local n=$1 b=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/$n.json 2> $O/$n.err
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['detail'].get('talker_ms'), d['detail'].get('codec_ms'))"
}
for i in 1 2 3; do
  run b16_base.$i 16 QTTS_X=0
  run b16_st2.$i 16 QTTS_HIP_BKZ_MAX=2 QTTS_HIP_BKZ_WIDE=2
done
