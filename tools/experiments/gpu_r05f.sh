#!/bin/bash
# Round-5 pass f: batch-path parity on the current build (every weight step
# before the staging for SPW <= 2) over every batch switch, then the A/B of
# the same for the partial-free talker shapes (lib_b, -DQTTS_GB_ALLW4).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_long.py -k "batch" -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "FAIL|passed|failed" $O/tests.log | tail -3
val() { python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
b() { timeout -k 10 300 python bench.py --batch $2 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $1 2> $1.err; val $1; }
for i in 1 2 3; do
  a=$(b $O/b8_cur_$i.json 8)
  c=$(QTTS_LIB=$R/qwen3-tts-c_amd/lib_b/libqwen_tts_amd.so b $O/b8_allw4_$i.json 8)
  echo "b8 pair $i current $a allw4 $c"
done
for i in 1 2; do
  a=$(b $O/b16_cur_$i.json 16)
  c=$(QTTS_LIB=$R/qwen3-tts-c_amd/lib_b/libqwen_tts_amd.so b $O/b16_allw4_$i.json 16)
  echo "b16 pair $i current $a allw4 $c"
done
# last (a host fault under the profiler ends the call here): the launch
# micro-benchmark's relevant variants under rocprofv3, few replays
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d /tmp/mbl -o run -- $R/tools/mb_launch --only x4k,x4k_resid,gemv_gu --reps 3 > $O/mb_launch_prof.txt 2> $O/mb_launch_prof.err
find /tmp/mbl -name "*.csv" -exec cp {} $O/ \;
cat $O/mb_launch_prof.txt
echo done
