#!/bin/bash
# Round-5 pass h: batch-8 switch sweep on the current build (alternating, two
# rounds): talker attention split size (QTTS_HIP_ATTN_LPK 8 / 16: 32- / 16-key
# splits instead of 64), split-K columns up to 4 (QTTS_HIP_BKZ_MAX=4),
# self-reducing split-K from 2 rows (QTTS_HIP_BSELF_MIN=2), 512-thread batch
# GEMV workgroups (QTTS_HIP_GB_W=8).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
mkdir -p $O
cd $R
val() { python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
b8() { timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $1 2> $1.err; val $1; }
for i in 1 2; do
  a=$(b8 $O/base_$i.json)
  b=$(QTTS_HIP_ATTN_LPK=8 b8 $O/lpk8_$i.json)
  c=$(QTTS_HIP_ATTN_LPK=16 b8 $O/lpk16_$i.json)
  d=$(QTTS_HIP_BKZ_MAX=4 b8 $O/kz4_$i.json)
  e=$(QTTS_HIP_BSELF_MIN=2 b8 $O/self2_$i.json)
  f=$(QTTS_HIP_GB_W=8 b8 $O/w8_$i.json)
  echo "b8 round $i base $a lpk8 $b lpk16 $c kz4 $d self2 $e w8 $f"
done
echo done
