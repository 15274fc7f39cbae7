#!/bin/bash
# Round-5 pass i: does replicating a launch's output per XCD shorten the next
# launch's x fetch?  (tools/mb_launch x32k / x64k variants, plain run)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/mb_launch --quiet --only x4k,x32k,x32k_rep8,x64k,x64k_rep8,gemv_gu > $O/mb_xrep.txt 2>&1
cat $O/mb_xrep.txt
timeout -k 10 120 ./tools/mb_launch --quiet --only x4k,x32k,x32k_rep8,x64k,x64k_rep8 > $O/mb_xrep2.txt 2>&1
cat $O/mb_xrep2.txt
echo done
