#!/bin/bash
# Round-6 pass f: k_pgemm, loads two stages ahead pinned at the stage start (sched_barrier), RMS
# fused into the plane split -- prefill parity, per-shape kernel times, VC lines.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_long.py -k "c5_bench or prefill_gemm or hd128_600" -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 8; do
  timeout -k 10 300 python bench.py --voice-clone --vc-codes --batch $k --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/vc$k.json 2> $O/vc$k.err
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for k in ("vc1", "vc8"):
    d = json.loads(open(f"{o}/{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], {x: d["detail"].get(x) for x in ("first_packet_ms", "prefill_ms", "step_prefill_ms", "talker_ms", "codec_ms")})
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --voice-clone --vc-codes --batch 8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --frames 8 > $O/prof.json 2> $O/prof.err
python3 - $O <<'PY'
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/prof/*kernel_trace.csv")[0]
d = collections.defaultdict(list)
for x in csv.DictReader(open(f)):
    n = x["Kernel_Name"]
    if any(k in n for k in ("pgemm", "split3", "mgemm", "row_rms")):
        d[(n.split("(")[0][-22:], x["Grid_Size_X"], x["Grid_Size_Y"], x["Grid_Size_Z"])].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print(k, len(v), round(sum(v) / len(v), 1))
PY
