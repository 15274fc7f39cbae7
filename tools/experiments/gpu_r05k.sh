#!/bin/bash
# Round-5 pass k: the first packet's codec push replayed as a cached HIP graph
# -- streaming parity (bit-identical later streams, stream == full decode),
# then first-packet A/B against eager launches (QTTS_HIP_CODEC_G1=0).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_voice_clone.py tests/test_gpu_full.py tests/test_gpu_enc.py -k "stream" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -12
fp() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['first_packet_ms'], d['detail']['first_packet_cold_ms'], d['value'])"; }
for i in 1 2 3; do
  QTTS_HIP_CODEC_G1=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 > $O/eager_$i.json 2> $O/eager_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 > $O/graph_$i.json 2> $O/graph_$i.err
  echo "round $i eager (first packet, cold, value) $(fp $O/eager_$i.json) | graph $(fp $O/graph_$i.json)"
done
echo done
