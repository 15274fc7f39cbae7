#!/bin/bash
# Round 6: k_pgemm with 128 x 256 tiles on 8 waves (default now) vs the
# 128 x 128 form (QTTS_HIP_PGEMM_BN=128): prefill parity tests, then
# alternating voice-clone batch-1 / batch-8 lines (prefill_ms, first packet).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06q
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_long.py -k "c5_bench_shape or prefill_gemm or 600_row or voice_clone" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log | cut -c1-120; tail -1 $O/tests.log
for i in 1 2; do
  for bn in 256 128; do
    QTTS_HIP_PGEMM_BN=$bn timeout -k 10 300 python bench.py --voice-clone --vc-codes --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/vc1_$bn.$i.json 2> $O/vc1_$bn.$i.err
    QTTS_HIP_PGEMM_BN=$bn timeout -k 10 400 python bench.py --voice-clone --vc-codes --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/vc8_$bn.$i.json 2> $O/vc8_$bn.$i.err
  done
done
for f in $O/vc*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); dd=d['detail']; print('$f'.split('/')[-1], d['value'], d.get('first_packet_ms'), dd.get('prefill_ms'), dd.get('step_prefill_ms'))"; done
