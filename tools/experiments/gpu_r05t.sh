#!/bin/bash
# Round-5 pass t: k_convb's two MFMA chains interleaved (QTTS_HIP_CONV_IL=0:
# one after the other; bit-identical) and k_xlin on two accumulators -- codec
# parity, bit-identity of the conv switch, codec time and batch-8 A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_long.py tests/test_gpu_model.py tests/test_gpu_kernels.py -k "codec or stream or bench_workload or greedy_prefix or conv" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "passed|failed" $O/tests.log | tail -2
cat > $O/bitid.py <<'PY'
import os, sys, numpy as np
sys.path[:0] = ["qwen3-tts-c_amd", "tests", "tools"]
import qtts
from synth_model import ensure_model
md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
m = qtts.QwenTTS(md)
codes = np.random.default_rng(7).integers(0, 2048, size=(128, 16)).astype(np.int32)
np.save(sys.argv[1], m.codec_decode(codes))
m.close()
PY
QTTS_HIP_CONV_IL=0 timeout -k 10 200 python $O/bitid.py $O/il0.npy > /dev/null 2>&1
QTTS_HIP_CONV_IL=1 timeout -k 10 200 python $O/bitid.py $O/il1.npy > /dev/null 2>&1
python -c "import numpy as np; a=np.load('$O/il0.npy'); b=np.load('$O/il1.npy'); print('conv IL bit-identical:', np.array_equal(a, b), a.shape)"
rm -f $O/il0.npy $O/il1.npy
for r in 1 2; do
  for il in 0 1; do
    QTTS_HIP_CONV_IL=$il timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_il${il}_$r.txt 2>&1
    echo "codec round $r conv_il $il: $(grep decode $O/codec_il${il}_$r.txt | tr '\n' ' ')"
  done
done
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for il in 0 1; do
    QTTS_HIP_CONV_IL=$il timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_il${il}_$r.json 2> $O/b8_il${il}_$r.err
    echo "b8 round $r conv_il $il $(val $O/b8_il${il}_$r.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/codec -o run -- python3 tools/prof_codec.py > $O/prof.log 2>&1
python3 tools/prof_codec.py --summarize $O/codec > $O/codec_kernels.txt
head -25 $O/codec_kernels.txt
