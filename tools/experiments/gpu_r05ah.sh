#!/bin/bash
# Round-5 pass ah: 64-wide conv tiles for <= 64 output columns (the streaming
# decode's first frames; QTTS_HIP_CONV_NARROW=0: 128 / 256-wide) -- stream
# bit-identity, streaming / codec tests, first packet A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ah
mkdir -p $O
cd $R
cat > $O/bitid.py <<'PY'
import os, sys, numpy as np
sys.path[:0] = ["qwen3-tts-c_amd", "tests", "tools"]
import qtts
from synth_model import ensure_model
md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
m = qtts.QwenTTS(md)
codes = np.random.default_rng(9).integers(0, 2048, size=(40, 16)).astype(np.int32)
s = m.codec_stream([codes[:1], codes[1:3], codes[3:11], codes[11:40]])
np.save(sys.argv[1], np.concatenate(list(s) + [m.codec_decode(codes)]))
m.close()
PY
for nw in 0 1; do QTTS_HIP_CONV_NARROW=$nw timeout -k 10 200 python $O/bitid.py $O/n$nw.npy > $O/bitid$nw.log 2>&1 || { tail -5 $O/bitid$nw.log; exit 1; }; done
python -c "import numpy as np; print('narrow bit-identical:', np.array_equal(np.load('$O/n0.npy'), np.load('$O/n1.npy')))"
rm -f $O/n0.npy $O/n1.npy
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_full.py tests/test_voice_clone.py tests/test_gpu_enc.py tests/test_gpu_kernels.py -k "stream or codec or conv" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['first_packet_ms'], d['detail']['first_packet_cold_ms'], d['detail']['codec_ms'])"; }
for r in 1 2 3; do
  line="b1 round $r"
  for nw in 0 1; do
    QTTS_HIP_CONV_NARROW=$nw timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b1_n${nw}_$r.json 2> $O/b1_n${nw}_$r.err
    line="$line | narrow $nw (value, first packet, cold, codec) $(val $O/b1_n${nw}_$r.json)"
  done
  echo "$line"
done
