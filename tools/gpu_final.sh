#!/bin/bash
# Round-6 lines of record on the final tree, in one call: the batch-1 kernels'
# in-graph spans (stamp build), then tools/gpu_round.sh's core pass (the whole
# GPU suite, rocprofv3 stats + FETCH / WRITE passes for the 1.7B and C2 lines,
# both bench lines).  Usage: bash tools/gpu_final.sh <tag>
set -eo pipefail
TAG=${1:-r06z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python tools/graph_spans.py $O/graph_spans.json > $O/graph_spans.out 2>&1 || { tail -20 $O/graph_spans.out; exit 1; }
cp $O/graph_spans.json $R/profiles/${TAG}_graph_spans.json
bash tools/gpu_round.sh $TAG core
cp $O/gpu_tests.log $R/profiles/${TAG}_gpu_tests.log
cp $O/bench.json $R/profiles/${TAG}_bench.json
tail -2 $O/gpu_tests.log
cat $O/bench.json | tail -1 | cut -c1-600
