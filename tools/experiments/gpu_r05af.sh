#!/bin/bash
# Round-5 pass af: first-packet timeline (prefill launched eagerly: host-bound?)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05af
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/prof_first_packet.py > $O/plain.txt 2>&1; tail -3 $O/plain.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/fp -o run -- python3 tools/prof_first_packet.py > $O/prof.txt 2>&1
f=$(find $O/fp -name "*kernel_trace.csv"); python3 tools/fp_timeline.py $f
python3 tools/trace_by_grid.py $f 25 > $O/by_grid.txt; head -20 $O/by_grid.txt
