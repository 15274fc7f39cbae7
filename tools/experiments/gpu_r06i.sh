#!/bin/bash
# Round-6 pass i: mb_launch's kernarg sweep under rocprofv3 largest-first
# (r06g / r06h: ascending, it faults in kb232, its 4th variant, with or
# without destroying graphs): size or count?
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d /tmp/mbk2 -o run -- $R/tools/mb_launch --kernarg-sweep --desc > $O/desc.txt 2> $O/desc.err
rc=$?
echo "desc rc=$rc"; cat $O/desc.txt
grep -E "variant|SIGSEGV|Aborted|hipGraphLaunch" $O/desc.err | tail -12
exit 0
