#!/bin/bash
# Round 6: batch-16 dispatch switches on the tree with 4-column down
# projections (r06zc): the batch GEMV's workgroup size (GB_W=8), split-K
# column cap (BKZ_MAX=2), self-reduction threshold (BSELF_MIN=16: consumers
# add the partials), codec lanes (16), in alternating processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zd
mkdir -p $O
cd $R
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python bench.py --batch 16 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/$n.json 2> $O/$n.err
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['detail'].get('talker_ms'), d['detail'].get('codec_ms'))"
}
for i in 1 2; do
  run base.$i QTTS_X=0
  run gbw8.$i QTTS_HIP_GB_W=8
  run bkz2.$i QTTS_HIP_BKZ_MAX=2
  run lanes16.$i QTTS_HIP_CODEC_LANES=16
done
