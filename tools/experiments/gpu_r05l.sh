#!/bin/bash
# Round-5 pass l: a batch's codec passes side by side (qtts_dev_codec_multi,
# QTTS_HIP_CODEC_LANES) -- parity (lanes bit-identical, batch / EOS / voice-clone
# batch tests), then batch-8 / 16 A/B over the lane count.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_model.py tests/test_voice_clone.py -k "batch" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -20
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for ln in 1 4 8; do
    QTTS_HIP_CODEC_LANES=$ln timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_l${ln}_$r.json 2> $O/b8_l${ln}_$r.err
    echo "b8 round $r lanes $ln $(val $O/b8_l${ln}_$r.json)"
  done
done
for ln in 1 4 8; do
  QTTS_HIP_CODEC_LANES=$ln timeout -k 10 300 python bench.py --batch 16 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b16_l${ln}.json 2> $O/b16_l${ln}.err
  echo "b16 lanes $ln $(val $O/b16_l${ln}.json)"
done
echo done
