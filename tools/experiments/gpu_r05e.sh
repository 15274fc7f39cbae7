#!/bin/bash
# (the QTTS_HIP_PF_MODE / QTTS_HIP_PF_BATCH switches this pass compared were removed after it: profiles/r05e_ab_prefetch_modes.txt)
# Round-5 pass e: the next-launch prefetch as a translation (TLB) warm-up.
# Batch 1: mode 0 (one load per 64-B chunk of the next slice, current) vs 1 (one
# per 4 KB page of it) vs 2 (one per 2 MB of the WHOLE next matrix) + the
# talker's edges (QTTS_HIP_L2PF_TK=15), alternating processes.  Batch 8: the
# whole-matrix form on the batch chain (QTTS_HIP_PF_BATCH=1), and the batch
# GEMV with every weight step of SPW <= 2 before the staging (lib_b).  TLB
# counters of mode 2.  Parity of the new forms on the bench workloads first.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
QTTS_HIP_PF_MODE=2 QTTS_HIP_L2PF_TK=15 QTTS_HIP_PF_BATCH=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_long.py -k "(full_bench_workload and env0) or (c4_batch8 and env0)" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -3
val() { python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
b1() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $1 2> $1.err; val $1; }
for i in 1 2 3; do
  a=$(b1 $O/b1_m0_$i.json)
  b=$(QTTS_HIP_PF_MODE=1 b1 $O/b1_m1_$i.json)
  c=$(QTTS_HIP_PF_MODE=2 b1 $O/b1_m2_$i.json)
  d=$(QTTS_HIP_PF_MODE=2 QTTS_HIP_L2PF_TK=15 b1 $O/b1_m2tk_$i.json)
  echo "b1 round $i mode0 $a mode1 $b mode2 $c mode2+talker $d"
done
b8() { timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $1 2> $1.err; val $1; }
for i in 1 2 3; do
  a=$(b8 $O/b8_base_$i.json)
  b=$(QTTS_HIP_PF_BATCH=1 QTTS_HIP_PF_MODE=2 b8 $O/b8_pf_$i.json)
  c=$(QTTS_LIB=$R/qwen3-tts-c_amd/lib_b/libqwen_tts_amd.so b8 $O/b8_allw_$i.json)
  echo "b8 round $i base $a pf-batch $b all-steps-first(lib_b) $c"
done
cd /tmp && export TMPDIR=/tmp
QTTS_HIP_PF_MODE=2 QTTS_HIP_L2PF_TK=15 timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-trace -f csv -d $O/pmc_tlb_m2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_tlb_m2.log 2>&1
python3 $R/tools/pmc_by_kernel.py $O/pmc_tlb_m2 $O/tlb_m2.json
echo done
