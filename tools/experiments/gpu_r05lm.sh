#!/bin/bash
# Round-5 passes l + m in one call: a batch's codec passes side by side
# (QTTS_HIP_CODEC_LANES) and one utterance's codec overlapped with the decode
# loop (QTTS_HIP_CODEC_OVERLAP) -- parity, then alternating A/Bs.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05lm
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_model.py tests/test_voice_clone.py -k "batch or overlap or stream_c3" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -30
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for ln in 1 4 8; do
    QTTS_HIP_CODEC_LANES=$ln timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_l${ln}_$r.json 2> $O/b8_l${ln}_$r.err
    echo "b8 round $r lanes $ln $(val $O/b8_l${ln}_$r.json)"
  done
  for ov in 0 16; do
    QTTS_HIP_CODEC_OVERLAP=$ov timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b1_ov${ov}_$r.json 2> $O/b1_ov${ov}_$r.err
    echo "b1 round $r overlap $ov $(val $O/b1_ov${ov}_$r.json)"
  done
done
for ln in 1 8; do
  QTTS_HIP_CODEC_LANES=$ln timeout -k 10 300 python bench.py --batch 16 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b16_l${ln}.json 2> $O/b16_l${ln}.err
  echo "b16 lanes $ln $(val $O/b16_l${ln}.json)"
done
echo done
