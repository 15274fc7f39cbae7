#!/bin/bash
# Round-6 pass b: the work queue with tail compaction (the running slots moved
# to the first rows once nothing is left to admit) -- queue parity, the EOS
# regression, then EOS batch-8 lines: lock-step, queue of 32 with and without
# compaction, queue of 96.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_long.py -k "queue and not six or eos_stop" -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python bench.py --eos --batch 8 --queue 32 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_q32.json 2> $O/bench_q32.err
tail -c 1500 $O/bench_q32.json
timeout -k 10 600 python bench.py --eos --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_eos_b8.json 2> $O/bench_eos_b8.err
tail -c 800 $O/bench_eos_b8.json
QTTS_QUEUE_COMPACT=0 timeout -k 10 600 python bench.py --eos --batch 8 --queue 32 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_q32_nocompact.json 2> $O/bench_q32_nocompact.err
tail -c 900 $O/bench_q32_nocompact.json
timeout -k 10 900 python bench.py --eos --batch 8 --queue 96 --steps 1 --warmup 0 --no-cpu-baseline --no-profile > $O/bench_q96.json 2> $O/bench_q96.err
tail -c 900 $O/bench_q96.json
