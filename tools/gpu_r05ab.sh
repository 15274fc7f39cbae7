#!/bin/bash
# Round-5 pass ab: k_convb with two stage buffers (the next stage split and
# written while this one's MFMAs run): QTTS_HIP_CONV_DB 0 / 1 / 2 --
# bit-identity of the codec output, codec time and the batch-8 line
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ab
mkdir -p $O
cd $R
cat > $O/bitid.py <<'PY'
import os, sys, numpy as np
sys.path[:0] = ["qwen3-tts-c_amd", "tests", "tools"]
import qtts
from synth_model import ensure_model
md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
m = qtts.QwenTTS(md)
codes = np.random.default_rng(7).integers(0, 2048, size=(128, 16)).astype(np.int32)
a = m.codec_decode(codes)
s = m.codec_stream([codes[:1], codes[1:9], codes[9:41]])
np.save(sys.argv[1], np.concatenate([a] + list(s)))
m.close()
PY
for db in 0 1 2; do QTTS_HIP_CONV_DB=$db timeout -k 10 200 python $O/bitid.py $O/db$db.npy > $O/bitid$db.log 2>&1 || { tail -5 $O/bitid$db.log; exit 1; }; done
python -c "import numpy as np; a=np.load('$O/db0.npy'); print('db1 bit-identical:', np.array_equal(a, np.load('$O/db1.npy')), 'db2 bit-identical:', np.array_equal(a, np.load('$O/db2.npy')), a.shape)"
rm -f $O/db*.npy
for r in 1 2; do
  line="codec round $r"
  for db in 0 1 2; do
    QTTS_HIP_CONV_DB=$db timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_db${db}_$r.txt 2>&1
    line="$line | db$db $(grep 'decode [12]' $O/codec_db${db}_$r.txt | awk '{print $3}' | tr '\n' ' ')"
  done
  echo "$line"
done
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail']['codec_ms'])"; }
for r in 1 2; do
  line="b8 round $r"
  for db in 0 1 2; do
    QTTS_HIP_CONV_DB=$db timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/b8_db${db}_$r.json 2> $O/b8_db${db}_$r.err
    line="$line | db$db $(val $O/b8_db${db}_$r.json)"
  done
  echo "$line"
done
