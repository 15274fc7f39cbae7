#!/bin/bash
# GPU pass for the voice-clone encoders: timings, rocprof
# kernel stats, the full-size parity test and the C5 bench line from
# reference audio.  Usage (on the box): bash tools/gpu_enc.sh <tag>
set -o pipefail
T=${1:-e}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
echo "[gpu_enc] timings" && timeout -k 10 600 python3 -u tools/prof_enc.py > $O/enc_times.json 2> $O/enc_times.err &&
echo "[gpu_enc] rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o enc -- python3 tools/prof_enc.py > $O/prof.log 2>&1 &&
echo "[gpu_enc] full-size parity" && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_enc.py -x -v --timeout 800 --timeout-method thread -m slow > $O/slow.log 2>&1 &&
echo "[gpu_enc] C5 bench" && timeout -k 10 900 python3 -u bench.py --voice-clone --batch 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_vc8.json 2> $O/bench_vc8.err
rc=$?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/enc_kernel_stats.csv \; 2>/dev/null
find $O/prof -name "*.db" -delete 2>/dev/null; find $O/prof -name "*kernel_trace.csv" -delete 2>/dev/null
echo "[gpu_enc] rc=$rc"
exit $rc
