#!/bin/bash
# Batch sub-talker attention as the q|k|v GEMV's tail: parity against the
# reference's 8-slot goldens first, then a same-box A/B (tail / separate launch)
# with alternating processes, then the batch-8 rocprof stats + PMC passes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -k "c4_batch8 and (env0 or env4)" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tail_tests.log 2>&1 || { tail -30 $O/tail_tests.log; exit 1; }
tail -3 $O/tail_tests.log
for i in 1 2 3; do
  QTTS_HIP_ATTN_TAIL=0 timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/ab_off_$i.json 2> $O/ab_off_$i.err
  timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/ab_on_$i.json 2> $O/ab_on_$i.err
  python -c "import json; f=lambda p: json.loads(open(p).read().strip().splitlines()[-1])['value']; print('b8 pair $i tail off', f('$O/ab_off_$i.json'), 'on', f('$O/ab_on_$i.json'))"
done
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b8.json 2> $O/st_b8.err
grep gm_dbg $O/st_b8.err | tail -24
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_b8 -o run -- python3 $R/bench.py --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/prof_b8.json 2> $O/prof_b8.err
f=$(find $O/prof_b8 -name "*kernel_trace.csv"); python3 $R/tools/trace_by_grid.py $f > $O/b8_by_grid.txt 2>&1 || true
head -30 $O/b8_by_grid.txt
echo done
