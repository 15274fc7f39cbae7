#!/bin/bash
# Round-6 pass h: mb_launch's fault under rocprofv3 (r06g: the kernarg sweep
# faulted in its 4th variant, kb232, as round 5's run did in its 4th, x4k_big):
# the same sweep keeping every graph exec alive (--keep-graphs), then the
# sweep largest-first with graphs destroyed per variant (last: a fault ends it).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
set +e
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d /tmp/mbk1 -o run -- $R/tools/mb_launch --kernarg-sweep --keep-graphs > $O/keep.txt 2> $O/keep.err
rc=$?
echo "keep-graphs rc=$rc"; cat $O/keep.txt
[ $rc -ne 0 ] && { grep -E "variant|SIGSEGV" $O/keep.err | tail -5; exit 0; }
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d /tmp/mbk2 -o run -- $R/tools/mb_launch --kernarg-sweep --desc > $O/desc.txt 2> $O/desc.err
rc=$?
echo "desc rc=$rc"; cat $O/desc.txt
grep -E "variant|SIGSEGV|Aborted" $O/desc.err | tail -8
exit 0
