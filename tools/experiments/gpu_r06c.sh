#!/bin/bash
# Round-6 pass c: the whole GPU suite on the round-6 tree (queue, divergence
# verdicts, advisor fixes), then the batch-8 / batch-16 lines with their own
# rocprof / PMC passes (<tag>_b8_*, <tag>_b16_*).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|ERROR" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_round.sh r06c batch
tail -c 600 $O/bench_b8.json; tail -c 600 $O/bench_b16.json
