#!/bin/bash
# Batch path: parity of the attention tail + parallel epilogue reductions
# against the reference's 8-slot goldens, then same-box A/Bs with alternating
# processes (lib_a = the previous commit's build), stamps, rocprof stats.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_long.py -k "(c4_batch8 and (env0 or env4)) or (c4_bench_workload and env0)" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tail_tests.log 2>&1 || { tail -30 $O/tail_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tail_tests.log | tail -5
b8() { timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $1 2> $1.err; python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
for i in 1 2 3; do
  a=$(QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so b8 $O/ab_prev_$i.json)
  b=$(b8 $O/ab_new_$i.json)
  echo "b8 pair $i prev-commit $a new $b"
done
for i in 1 2; do
  a=$(QTTS_HIP_ATTN_TAIL=0 b8 $O/ab_notail_$i.json)
  b=$(b8 $O/ab_tail_$i.json)
  echo "b8 pair $i tail-off $a tail-on $b"
done
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b8.json 2> $O/st_b8.err
grep gm_dbg $O/st_b8.err | tail -26
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_b8 -o run -- python3 $R/bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_b8.json 2> $O/prof_b8.err
f=$(find $O/prof_b8 -name "*kernel_trace.csv"); python3 $R/tools/trace_by_grid.py $f > $O/b8_by_grid.txt 2>&1 || true
find $O/prof_b8 -name "*kernel_trace.csv" -delete
head -24 $O/b8_by_grid.txt
echo done
