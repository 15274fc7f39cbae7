#!/bin/bash
# Round-5 pass aq: the prefill GEMM's split-K target grid 2048 vs 1024
# workgroups (QTTS_HIP_MGEMM_WG): voice-clone / full-model goldens at 2048,
# then voice clone batch 1 and batch 8 in alternating processes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aq
mkdir -p $O
cd $R
QTTS_HIP_MGEMM_WG=2048 timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_enc.py tests/test_gpu_model.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); dt=d.get('detail',{}); print(d['value'], dt.get('prefill_ms'), dt.get('step_prefill_ms'), dt.get('first_packet_ms'))"; }
for r in 1 2; do
  for wg in 1024 2048; do
    QTTS_HIP_MGEMM_WG=$wg timeout -k 10 300 python bench.py --voice-clone --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc1_wg${wg}_$r.json 2> $O/vc1_wg${wg}_$r.err
    echo "vc1 round $r wg $wg (value, prefill, step prefill, first packet) $(val $O/vc1_wg${wg}_$r.json)"
  done
done
for wg in 1024 2048; do
  QTTS_HIP_MGEMM_WG=$wg timeout -k 10 600 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_wg${wg}.json 2> $O/b8_wg${wg}.err
  echo "b8 wg $wg (value, prefill) $(python -c "import json; d=json.loads(open('$O/b8_wg${wg}.json').read().strip().splitlines()[-1]); print(d['value'], d['detail']['prefill_ms'])")"
done
