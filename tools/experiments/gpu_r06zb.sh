#!/bin/bash
# Round 6: the batch-1 talker attention's dead splits pull the O projection's
# weight slices into L2 while the live splits run (QTTS_HIP_ATTN_PF, default
# on) against no prefetch (=0): the attention + full-workload parity tests,
# in-graph spans both ways (stamp build), then batch-1 lines in alternating
# processes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zb
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_full.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
QTTS_HIP_ATTN_PF=0 timeout -k 10 300 python tools/graph_spans.py $O/spans_off.json > $O/spans_off.out 2>&1
timeout -k 10 300 python tools/graph_spans.py $O/spans_on.json > $O/spans_on.out 2>&1
python3 - <<PY
import json
for t in ("off", "on"):
    d = json.load(open("$O/spans_%s.json" % t))
    print(t, {k: (v["span_us"], v["period_us"]) for k, v in d.items() if k != "_note" and "talker layer" in v["group"]})
PY
for i in 1 2 3; do
  for v in 0 1; do
    QTTS_HIP_ATTN_PF=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/b1_$v.$i.json 2> $O/b1_$v.$i.err
  done
done
for f in $O/b1*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['detail'].get('talker_ms'))"; done
