#!/bin/bash
# Round-5 final: the whole GPU suite on the final tree, then the C5 line
# (voice clone from 5 s reference audio, encoders inside the step, batch 8)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ap
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python bench.py --voice-clone --batch 8 --steps 3 --warmup 1 > $O/bench_vc8.json 2> $O/bench_vc8.err
python -c "import json; d=json.loads(open('$O/bench_vc8.json').read().strip().splitlines()[-1]); print('vc8', d['value'], d.get('detail'))"
