#!/bin/bash
# Round-5 pass s: the codec's plain linears on k_xlin (3-plane bf16 MFMA, 128-wide
# K stages) -- codec parity at full size, then codec time A/B (QTTS_HIP_XLIN=0:
# k_xgemm) and the batch-8 line, alternating processes; a rocprof breakdown
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_long.py tests/test_gpu_model.py -k "codec or stream or bench_workload or greedy_prefix" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
  for xl in 0 1; do
    QTTS_HIP_XLIN=$xl timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_xl${xl}_$r.txt 2>&1
    echo "codec round $r xlin $xl: $(grep decode $O/codec_xl${xl}_$r.txt | tr '\n' ' ')"
  done
done
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for xl in 0 1; do
    QTTS_HIP_XLIN=$xl timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_xl${xl}_$r.json 2> $O/b8_xl${xl}_$r.err
    echo "b8 round $r xlin $xl $(val $O/b8_xl${xl}_$r.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/codec -o run -- python3 tools/prof_codec.py > $O/prof.log 2>&1
python3 tools/prof_codec.py --summarize $O/codec > $O/codec_kernels.txt
head -25 $O/codec_kernels.txt
