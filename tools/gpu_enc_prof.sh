#!/bin/bash
# rocprof kernel stats + a per-(kernel, grid) breakdown of the encoder chain.
# Usage (on the box): bash tools/gpu_enc_prof.sh <tag>
set -o pipefail
T=${1:-ep}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/prof_enc.py > $O/enc_times.json 2> $O/enc_times.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o enc -- python3 tools/prof_enc.py --reps 2 > $O/prof.log 2>&1
rc=$?
tr=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$tr" ] && python3 tools/trace_by_grid.py "$tr" 45 > $O/enc_by_grid.txt
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/enc_kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -delete
exit $rc
