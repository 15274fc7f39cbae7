#!/bin/bash
# Round-5 pass an: voice-clone batch 1 with the prefill GEMM split over K
# (default) vs not (QTTS_HIP_MGEMM_KZ=1), in alternating order, with the
# timed step's phases (detail.step_*)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05an
mkdir -p $O
cd $R
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); dt=d.get('detail',{}); print(d['value'], d['ms_per_step'], dt)"; }
i=0
for kz in 8 1 1 8 8 1; do
  i=$((i+1))
  QTTS_HIP_MGEMM_KZ=$kz timeout -k 10 300 python bench.py --voice-clone --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc1_${i}_kz${kz}.json 2> $O/vc1_${i}_kz${kz}.err
  echo "vc1 run $i kz $kz $(val $O/vc1_${i}_kz${kz}.json)"
done
