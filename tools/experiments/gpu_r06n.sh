#!/bin/bash
# Round 6: where the voice-clone prefill's time goes (batch 1 and 8, kernel
# trace by grid) and k_pgemm's matrix-core busy fraction (PMC pass).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/vc1 -o run -- python3 $R/bench.py --voice-clone --vc-codes --steps 1 --warmup 1 --frames 4 --no-cpu-baseline --no-profile > $O/vc1.json 2> $O/vc1.err
python3 $R/tools/trace_by_grid.py $(find $O/vc1 -name "*kernel_trace.csv") 45 > $O/vc1_by_grid.txt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/vc8 -o run -- python3 $R/bench.py --voice-clone --vc-codes --batch 8 --steps 1 --warmup 1 --frames 4 --no-cpu-baseline --no-profile > $O/vc8.json 2> $O/vc8.err
python3 $R/tools/trace_by_grid.py $(find $O/vc8 -name "*kernel_trace.csv") 45 > $O/vc8_by_grid.txt
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/pmc_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --no-profile --voice-clone --vc-codes --batch 8 --steps 1 --warmup 0 --frames 4 > $O/pmc_mfma.log 2>&1
python3 $R/tools/prof_summary.py $O
find $O -name '*.csv' -size +2M -delete
head -30 $O/vc1_by_grid.txt; head -30 $O/vc8_by_grid.txt
