#!/bin/bash
# Round-5 pass n: lock-step groups side by side on one GPU (tools/mb_concurrent.py):
# G contexts x batch B from G host threads, G frame graphs on G streams.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
for cfg in "1 8" "2 4" "1 16" "2 8" "4 2" "4 4" "2 1"; do
  set -- $cfg
  timeout -k 10 400 python tools/mb_concurrent.py --groups $1 --batch $2 --steps 3 --warmup 1 > $O/g$1_b$2.txt 2> $O/g$1_b$2.err || { tail -20 $O/g$1_b$2.err; exit 1; }
  cat $O/g$1_b$2.txt
done
echo done
