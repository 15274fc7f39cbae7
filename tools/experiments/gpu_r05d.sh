#!/bin/bash
# Round-5 pass d (mostly host work on the GPU box): the CPU baseline's
# wait-policy A/B and an unextrapolated 128-frame reference run, the C1 line,
# then tools/mb_launch under rocprofv3 --kernel-trace (last: it segfaulted
# there in round 4; its per-call trace names the HIP call if it does again).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
timeout -k 10 900 python tools/cpu_wait_ab.py > $O/cpu_wait_ab.txt 2> $O/cpu_wait_ab.err
cat $O/cpu_wait_ab.txt
timeout -k 10 600 python bench.py --c1 --cpu-1thread > $O/c1.json 2> $O/c1.err
cat $O/c1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/mb_launch --quiet > $O/mb_launch_plain.txt 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d /tmp/mbl -o run -- $R/tools/mb_launch > $O/mb_launch_prof.txt 2> $O/mb_launch_prof.err
find /tmp/mbl -name "*.csv" -exec cp {} $O/ \;
tail -5 $O/mb_launch_prof.txt
echo done
