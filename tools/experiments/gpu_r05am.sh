#!/bin/bash
# Round-5 pass am: k_mgemm (the prefill GEMM over > 16 rows) split over K on
# grid.z with an in-order reduce + epilogue launch (QTTS_HIP_MGEMM_KZ=1: no
# split) -- the whole GPU suite, then voice-clone batch 1 / batch 8 and the
# batch-8 P128 bench in alternating processes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05am
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); dt=d.get('detail',{}); print(d['value'], {k: dt.get(k) for k in ('prefill_ms','first_packet_ms','talker_ms','codec_ms') if k in dt})"; }
for r in 1 2; do
  for kz in 1 8; do
    QTTS_HIP_MGEMM_KZ=$kz timeout -k 10 300 python bench.py --voice-clone --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc1_kz${kz}_$r.json 2> $O/vc1_kz${kz}_$r.err
    echo "vc1 round $r kz $kz $(val $O/vc1_kz${kz}_$r.json)"
    QTTS_HIP_MGEMM_KZ=$kz timeout -k 10 600 python bench.py --voice-clone --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc8_kz${kz}_$r.json 2> $O/vc8_kz${kz}_$r.err
    echo "vc8 round $r kz $kz $(val $O/vc8_kz${kz}_$r.json)"
    QTTS_HIP_MGEMM_KZ=$kz timeout -k 10 600 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_kz${kz}_$r.json 2> $O/b8_kz${kz}_$r.err
    echo "b8 round $r kz $kz $(val $O/b8_kz${kz}_$r.json)"
  done
done
