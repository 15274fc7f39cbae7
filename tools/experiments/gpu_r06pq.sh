#!/bin/bash
# Round 6: passes p and q in one call (the pool had no free box twice).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/experiments/gpu_r06q.sh
bash tools/experiments/gpu_r06p.sh
