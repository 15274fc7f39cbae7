#!/bin/bash
# Round-5 pass e: the next-launch prefetch as a translation (TLB) warm-up --
# one load per 4 KB page (QTTS_HIP_PF_PAGE=1) vs one per 64-B chunk, and with
# the talker's edges on (QTTS_HIP_L2PF_TK=15) -- alternating processes; the
# batch GEMV with every weight step of SPW <= 2 before the staging (lib_b);
# parity of the page mode on the bench workload.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
QTTS_HIP_PF_PAGE=1 QTTS_HIP_L2PF_TK=15 timeout -k 10 400 python -u -m pytest tests/test_gpu_long.py -k "full_bench_workload and env0" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -3
val() { python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
b1() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $1 2> $1.err; val $1; }
for i in 1 2 3 4; do
  a=$(b1 $O/b1_chunk_$i.json)
  b=$(QTTS_HIP_PF_PAGE=1 b1 $O/b1_page_$i.json)
  c=$(QTTS_HIP_PF_PAGE=1 QTTS_HIP_L2PF_TK=15 b1 $O/b1_pagetk_$i.json)
  echo "b1 triple $i chunk64 $a page4k $b page4k+talker $c"
done
b8() { timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $1 2> $1.err; val $1; }
for i in 1 2 3; do
  a=$(b8 $O/b8_half_$i.json)
  b=$(QTTS_LIB=$R/qwen3-tts-c_amd/lib_b/libqwen_tts_amd.so b8 $O/b8_allw_$i.json)
  echo "b8 pair $i half-steps-first $a all-steps-first $b"
done
echo done
