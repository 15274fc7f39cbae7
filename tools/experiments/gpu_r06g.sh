#!/bin/bash
# Round-6 pass g: in-graph spans of the batch-1 kernels from in-kernel stamps
# (stamp build lib_s: tools/graph_spans.py), then tools/mb_launch's by-value
# kernarg sweep (128..1024 B, ascending) under rocprofv3 --kernel-trace: the
# first size that faults names the boundary.  Last, since a
# host fault ends the call.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 600 python tools/graph_spans.py $O/graph_spans.json > $O/graph_spans.out 2>&1 || { tail -20 $O/graph_spans.out; exit 1; }
grep -A3 "k_attn_o" $O/graph_spans.json
timeout -k 10 120 $R/tools/mb_launch --kernarg-sweep > $O/mb_kb_plain.txt 2> $O/mb_kb_plain.err
cat $O/mb_kb_plain.txt
cd /tmp && export TMPDIR=/tmp
set +e
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d /tmp/mbk -o run -- $R/tools/mb_launch --kernarg-sweep > $O/mb_kb_prof.txt 2> $O/mb_kb_prof.err
rc=$?
echo "rocprofv3 kernarg sweep rc=$rc"
cat $O/mb_kb_prof.txt
grep -E "variant|SIGSEGV|Aborted" $O/mb_kb_prof.err | tail -8
exit 0
