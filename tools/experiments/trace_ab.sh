#!/bin/bash
# Graph-mode kernel trace of a short bench under each given environment
# (development tool): bash tools/trace_ab.sh <tag> "ENV=.." "ENV=.." ...
# -> gpurun_out/<tag>/trace_<i>.txt (tools/trace_frame.py summaries)
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  env $e true   # validate
  ( export $e; timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/kt$i -o run -- python3 $R/bench.py --steps 1 --warmup 1 --frames 48 --no-cpu-baseline --no-profile > $O/kt$i.log 2>&1 )
  python3 $R/tools/trace_frame.py $O/kt$i --skip 60 > $O/trace_$i.txt
  echo "$e" >> $O/trace_$i.txt
  rm -rf $O/kt$i
  i=$((i+1))
done
echo done
