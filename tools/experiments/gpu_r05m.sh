#!/bin/bash
# Round-5 pass m: one utterance's codec decode overlapped with the decode loop
# (QTTS_HIP_CODEC_OVERLAP=<frames per push>) -- parity, then a batch-1 A/B.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -k "overlap or stream_c3 or default_12" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -20
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['codec_ms'], d['detail']['talker_ms'])"; }
for r in 1 2; do
  for ov in 0 8 16 32; do
    QTTS_HIP_CODEC_OVERLAP=$ov timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b1_ov${ov}_$r.json 2> $O/b1_ov${ov}_$r.err
    echo "b1 round $r overlap $ov (value, codec ms, talker ms of the breakdown call) $(val $O/b1_ov${ov}_$r.json)"
  done
done
echo done
