#!/bin/bash
# One GPU-box pass: parity tests, rocprofv3 kernel stats of the bench command,
# separate FETCH_SIZE / WRITE_SIZE PMC passes, an MFMA-busy PMC pass over the
# voice-clone batch bench (prefill GEMM, batch decode GEMV, codec convs), then
# the bench line itself -- after the summaries are in the box's profiles/ so
# the line's roofline.rocprof_avg_us / traffic come from the same code.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [all|core|prof|prof1|vc|extra|batch|dist]
#   prof1 = the profiles and the 1.7B / 0.6B bench lines only (no tests)
#   vc    = the C5 line, the encoders and the MFMA pass only
#   core  = tests + profiles + the 1.7B and 0.6B (C2) bench lines (fits one call)
#   extra = C5 voice clone batch 8, batch 8 / 16 lines, encoders, MFMA pass
set -eo pipefail
TAG=${1:-r02}
MODE=${2:-all}   # all | core | prof (no tests) | extra | batch | dist (2-rank gloo rehearsal)
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
# keep the merge-back under gpurun's 64 MiB (raw per-dispatch traces are only
# needed for the summaries) and show where a failing call stopped
trim() { rc=$?; find $O -name '*.csv' -size +4M -delete; for f in gpu_tests.log prof_bench.err bench.err; do
  [ -f $O/$f ] && { echo "== $f"; tail -n 15 $O/$f; }; done; exit $rc; }
trap trim EXIT
if [ "$MODE" = dist ]; then
  QTTS_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-profile > $O/dist2.json 2> $O/dist2.err
  echo done; exit 0
fi
if [ "$MODE" = batch ]; then
  # the batch-8 line of record (C4's per-GPU shape) with its own rocprof stats
  # and FETCH / WRITE passes (<tag>_b8_kernel_stats.csv / _b8_pmc.json, read
  # by bench.py --batch 8), then the batch-16 line
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/b8/prof -o run -- python3 $R/bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_b8.json 2> $O/prof_b8.err
  f=$(find $O/b8/prof -name "*kernel_trace.csv"); python3 $R/tools/trace_by_grid.py $f > $O/b8_by_grid.txt 2>&1 || true
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/b8/pmc_fetch -o run -- python3 $R/bench.py --batch 8 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch_b8.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/b8/pmc_write -o run -- python3 $R/bench.py --batch 8 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_write_b8.log 2>&1
  python3 $R/tools/prof_summary.py $O/b8
  cp $O/b8/kernel_stats.csv $R/profiles/${TAG}_b8_kernel_stats.csv
  cp $O/b8/pmc.json $R/profiles/${TAG}_b8_pmc.json
  cp $O/b8_by_grid.txt $R/profiles/${TAG}_b8_by_grid.txt
  # the batch-16 line's own passes (<tag>_b16_*, read by bench.py --batch 16)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/b16/prof -o run -- python3 $R/bench.py --batch 16 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_b16.json 2> $O/prof_b16.err
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/b16/pmc_fetch -o run -- python3 $R/bench.py --batch 16 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch_b16.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/b16/pmc_write -o run -- python3 $R/bench.py --batch 16 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_write_b16.log 2>&1
  python3 $R/tools/prof_summary.py $O/b16
  cp $O/b16/kernel_stats.csv $R/profiles/${TAG}_b16_kernel_stats.csv
  cp $O/b16/pmc.json $R/profiles/${TAG}_b16_pmc.json
  echo $TAG > $R/profiles/LATEST
  cd $R
  timeout -k 10 600 python bench.py --batch 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_b8.json 2> $O/bench_b8.err
  cp $O/bench_b8.json $R/profiles/${TAG}_bench_batch8.json
  timeout -k 10 600 python bench.py --batch 16 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_b16.json 2> $O/bench_b16.err
  cp $O/bench_b16.json $R/profiles/${TAG}_bench_batch16.json
  echo done; exit 0
fi
if [ "$MODE" = extra ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests_extra.log 2>&1 || { echo "tests failed"; exit 1; }
  tail -1 $O/gpu_tests_extra.log
  timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1 && tail -3 $O/mb_sample.txt
  for b in 8 16; do
    timeout -k 10 600 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err
  done
fi
if [ "$MODE" = all ] || [ "$MODE" = core ]; then
  rc=0
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
  # 1 = some test failed (keep measuring); anything else (timeout, abort, crash) ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc"; exit $rc; fi
fi
if [ "$MODE" != extra ] && [ "$MODE" != vc ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_write.log 2>&1
python3 $R/tools/prof_summary.py $O
# the bench reads the newest profiles/*kernel_stats.csv / *pmc.json
cp $O/kernel_stats.csv $R/profiles/${TAG}_kernel_stats.csv
cp $O/pmc.json $R/profiles/${TAG}_pmc.json
echo $TAG > $R/profiles/LATEST
# BASELINE configs[1] (C2): 0.6B, batch 1, greedy -- its own profile passes
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/c2/prof -o run -- python3 $R/bench.py --preset 0.6b --greedy --no-cpu-baseline > $O/prof_bench_06b.json 2> $O/prof_bench_06b.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/c2/pmc_fetch -o run -- python3 $R/bench.py --preset 0.6b --greedy --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch_06b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/c2/pmc_write -o run -- python3 $R/bench.py --preset 0.6b --greedy --no-cpu-baseline --steps 1 --warmup 0 --frames 8 > $O/pmc_write_06b.log 2>&1
python3 $R/tools/prof_summary.py $O/c2
cp $O/c2/kernel_stats.csv $R/profiles/${TAG}_06b_kernel_stats.csv
cp $O/c2/pmc.json $R/profiles/${TAG}_06b_pmc.json
cd $R
timeout -k 10 900 python bench.py --preset 0.6b --greedy --no-cpu-1thread > $O/bench_06b.json 2> $O/bench_06b.err
cp $O/bench_06b.json $R/profiles/${TAG}_bench_06b.json
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
fi
{ [ "$MODE" = core ] || [ "$MODE" = prof1 ]; } && { echo done; exit 0; }
# BASELINE C5 as stated: voice clone from 5 s reference audio (encoders inside the step), batch 8 --
# its own rocprof / PMC passes first (<tag>_vc8_*, read by the C5 line's roofline)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/vc8/prof -o run -- python3 $R/bench.py --voice-clone --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_vc8.json 2> $O/prof_vc8.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/vc8/pmc_fetch -o run -- python3 $R/bench.py --voice-clone --batch 8 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_fetch_vc8.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/vc8/pmc_write -o run -- python3 $R/bench.py --voice-clone --batch 8 --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_write_vc8.log 2>&1
python3 $R/tools/prof_summary.py $O/vc8
cp $O/vc8/kernel_stats.csv $R/profiles/${TAG}_vc8_kernel_stats.csv
cp $O/vc8/pmc.json $R/profiles/${TAG}_vc8_pmc.json
[ -f $R/profiles/LATEST ] || echo $TAG > $R/profiles/LATEST
cd $R
timeout -k 10 900 python bench.py --voice-clone --batch 8 --steps 3 --warmup 1 > $O/bench_vc8.json 2> $O/bench_vc8.err
cp $O/bench_vc8.json $R/profiles/${TAG}_bench_vc8.json
# the encoders alone: timings, rocprof stats and the per-(kernel, grid) breakdown
bash tools/gpu_enc_prof.sh $TAG/enc
cp $O/enc/enc_times.json $R/profiles/${TAG}_enc_times.json
cp $O/enc/enc_by_grid.txt $R/profiles/${TAG}_enc_by_grid.txt
cp $O/enc/enc_kernel_stats.csv $R/profiles/${TAG}_enc_kernel_stats.csv
# last (a counter the box refuses ends only this pass): matrix-core busy cycles
# of the voice-clone batch-8 bench (prefill GEMM, batch decode GEMV, codec convs)
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/pmc_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --no-profile --voice-clone --batch 8 --steps 1 --warmup 0 --frames 16 > $O/pmc_mfma.log 2>&1
python3 $R/tools/prof_summary.py $O
cp $O/mfma.json $R/profiles/${TAG}_mfma.json
echo done
