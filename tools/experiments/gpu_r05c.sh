#!/bin/bash
# Round-5 pass c: parity (EOS golden, C4 goldens, bench workload, stream-bw
# entry) on the batch GEMV's parallel epilogue; same-box A/Bs against the
# round-4 build (lib_a); batch-8 stamps; the L2-prefetch mechanism in L2 hit /
# TLB counters with and without the prefetch.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_kernels.py -k "eos_stop or (c4_batch8 and env0) or (c4_bench_workload and env0) or (full_bench_workload and env0) or hbm_stream" -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -8
val() { python -c "import json; print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
for i in 1 2 3; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_r04_$i.json 2> $O/b8_r04_$i.err
  timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_new_$i.json 2> $O/b8_new_$i.err
  echo "b8 pair $i r04-build $(val $O/b8_r04_$i.json) new $(val $O/b8_new_$i.json)"
done
for i in 1 2; do
  QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so timeout -k 10 300 python bench.py --batch 16 --no-cpu-baseline --no-profile --steps 2 --warmup 1 > $O/b16_r04_$i.json 2> $O/b16_r04_$i.err
  timeout -k 10 300 python bench.py --batch 16 --no-cpu-baseline --no-profile --steps 2 --warmup 1 > $O/b16_new_$i.json 2> $O/b16_new_$i.err
  echo "b16 pair $i r04-build $(val $O/b16_r04_$i.json) new $(val $O/b16_new_$i.json)"
done
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b8.json 2> $O/st_b8.err
grep gm_dbg $O/st_b8.err | tail -28
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
if grep -q "TCC_HIT" $O/avail.txt && grep -q "TCC_MISS" $O/avail.txt; then
  for pf in 0 31; do
    QTTS_HIP_L2PF=$pf timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d $O/pmc_tcc_$pf -o run -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_tcc_$pf.log 2>&1
    python3 $R/tools/pmc_by_kernel.py $O/pmc_tcc_$pf $O/tcc_l2pf$pf.json
  done
fi
if grep -q "TCP_UTCL1_TRANSLATION_MISS" $O/avail.txt && grep -q "TCP_UTCL1_TRANSLATION_HIT" $O/avail.txt; then
  for pf in 0 31; do
    QTTS_HIP_L2PF=$pf timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-trace -f csv -d $O/pmc_tlb_$pf -o run -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 --frames 8 > $O/pmc_tlb_$pf.log 2>&1
    python3 $R/tools/pmc_by_kernel.py $O/pmc_tlb_$pf $O/tlb_l2pf$pf.json
  done
fi
echo done
