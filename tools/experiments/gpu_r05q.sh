#!/bin/bash
# Round-5 pass q: where the EOS batch of 3 leaves the reference's codes, with
# and without the whole-row batch GEMV
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05q
mkdir -p $O
cd $R
for gw in 1 0; do
  echo "QTTS_HIP_GEMVWB=$gw"
  QTTS_HIP_GEMVWB=$gw timeout -k 10 300 python tools/eos_diverge.py > $O/gw$gw.txt 2> $O/gw$gw.err || { tail -20 $O/gw$gw.err; exit 1; }
  cat $O/gw$gw.txt
done
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for gw in 0 1; do
    QTTS_HIP_GEMVWB=$gw timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_gw${gw}_$r.json 2> $O/b8_gw${gw}_$r.err
    echo "b8 round $r gemvwb $gw $(val $O/b8_gw${gw}_$r.json)"
  done
done
