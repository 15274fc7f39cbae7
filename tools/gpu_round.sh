#!/bin/bash
# One GPU-box pass: parity tests, rocprofv3 kernel stats of the bench command,
# separate FETCH_SIZE / WRITE_SIZE PMC passes, then the bench line itself --
# after the summaries are in the box's profiles/ so the line's
# roofline.rocprof_avg_us / traffic come from the same code.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [all|all+mb|mb|prof|dist]
set -eo pipefail
TAG=${1:-r01}
MODE=${2:-all}   # all | all+mb (micro-benchmarks first) | mb | prof (no tests) | dist (2-rank gloo rehearsal)
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$MODE" = dist ]; then
  QTTS_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-profile > $O/dist2.json 2> $O/dist2.err
  echo done; exit 0
fi
if [ "$MODE" = mb ] || [ "$MODE" = all+mb ]; then
  # micro-benchmarks built in-tree on the CPU side (tools/mb_*)
  timeout -k 10 120 tools/mb_l2 > $O/mb_l2.txt 2>&1
  timeout -k 10 120 tools/mb_barrier > $O/mb_barrier.txt 2>&1
  timeout -k 10 300 tools/mb_gemv > $O/mb_gemv.txt 2>&1
  [ "$MODE" = mb ] && { echo done; exit 0; }
  MODE=all
fi
if [ "$MODE" = all ]; then
  rc=0
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
  # 1 = some test failed (keep measuring); anything else (timeout, abort, crash) ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc"; exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_write.log 2>&1
python3 $R/tools/prof_summary.py $O
# the bench reads the newest profiles/*kernel_stats.csv / *pmc.json
cp $O/kernel_stats.csv $R/profiles/${TAG}_kernel_stats.csv
cp $O/pmc.json $R/profiles/${TAG}_pmc.json
echo $TAG > $R/profiles/LATEST
cd $R
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
