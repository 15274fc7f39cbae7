#!/bin/bash
# Round-6 pass d: the prefill on the tiled GEMM over pre-split activations
# (k_pgemm; QTTS_HIP_PGEMM=0: k_mgemm) -- prefill / voice-clone / C5 parity
# (the new bench-shape C5 fixture), then voice-clone batch-1 first packet and
# C5 batch-8 prefill A/B in alternating processes, a rocprof of the new kernel.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_voice_clone.py tests/test_gpu_long.py -k "c5 or prefill or voice_clone or hd128_600" -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for pg in 1 0; do
    QTTS_HIP_PGEMM=$pg timeout -k 10 300 python bench.py --voice-clone --vc-codes --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/vc1_pg${pg}_$r.json 2> $O/vc1_pg${pg}_$r.err
    QTTS_HIP_PGEMM=$pg timeout -k 10 300 python bench.py --voice-clone --vc-codes --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/vc8_pg${pg}_$r.json 2> $O/vc8_pg${pg}_$r.err
    python3 - $O $pg $r <<'PY'
import json, sys
o, pg, r = sys.argv[1:]
for k in ("vc1", "vc8"):
    d = json.loads(open(f"{o}/{k}_pg{pg}_{r}.json").read().strip().splitlines()[-1])
    print(k, "pgemm", pg, "round", r, d["value"], {x: d["detail"].get(x) for x in ("first_packet_ms", "prefill_ms", "step_prefill_ms", "talker_ms", "codec_ms")})
PY
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --voice-clone --vc-codes --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --frames 8 > $O/prof.json 2> $O/prof.err
f=$(find $O/prof -name "*kernel_stats.csv"); grep -E "pgemm|mgemm|split3|row_rms" $f | cut -c1-200
