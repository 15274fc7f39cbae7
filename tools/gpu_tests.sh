#!/bin/bash
# The whole GPU test suite as the driver runs it at round end (one process,
# per-test timeout), log under gpurun_out/<tag>/gpu_tests.log.
set -o pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
tail -2 $O/gpu_tests.log
exit $rc
