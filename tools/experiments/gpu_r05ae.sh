#!/bin/bash
# Round-5 pass ae: k_mgemm (prefill over > 16 rows) with G K steps' loads in
# flight per round -- kernel / voice-clone parity, bit-identity against the
# old build (lib_a), and the voice-clone prefill / first packet and C5 A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ae
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_voice_clone.py tests/test_gpu_full.py tests/test_gpu_enc.py -k "matvec or voice or vc or c5 or prefill" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cat > $O/bitid.py <<'PY'
import os, sys, numpy as np
sys.path[:0] = ["qwen3-tts-c_amd", "tests", "tools"]
import qtts
from synth_model import ensure_model, prompt_ids
md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
m = qtts.QwenTTS(md)
m.set_params(max_tokens=4096, fixed=4, seed=42)
r = np.random.default_rng(5)
codes = r.integers(0, 2048, size=(63, 16)).astype(np.int32)
rids = [151644, 77091, 198] + r.integers(1000, 100000, size=20).tolist() + [151645, 198]
a = m.generate_voice_clone(prompt_ids("p128", 1290), rids, codes, (r.standard_normal(m.cfg.talker_hidden) * 0.05).astype(np.float32), "english")
np.save(sys.argv[1], np.concatenate([a.astype(np.float64), m.last_codes().ravel().astype(np.float64)]))
m.close()
PY
QTTS_LIB=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so timeout -k 10 200 python $O/bitid.py $O/old.npy > $O/bitid_old.log 2>&1
timeout -k 10 200 python $O/bitid.py $O/new.npy > $O/bitid_new.log 2>&1
python -c "import numpy as np; print('voice-clone output bit-identical old vs new:', np.array_equal(np.load('$O/old.npy'), np.load('$O/new.npy')))"
rm -f $O/old.npy $O/new.npy
val() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['detail'])"; }
for r in 1 2; do
  for v in old new; do
    lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so; [ $v = old ] && lib=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so
    QTTS_LIB=$lib timeout -k 10 300 python bench.py --voice-clone --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc1_${v}_$r.json 2> $O/vc1_${v}_$r.err
    echo "vc1 round $r $v $(val $O/vc1_${v}_$r.json)"
  done
done
for v in old new; do
  lib=$R/qwen3-tts-c_amd/lib/libqwen_tts_amd.so; [ $v = old ] && lib=$R/qwen3-tts-c_amd/lib_a/libqwen_tts_amd.so
  QTTS_LIB=$lib timeout -k 10 400 python bench.py --voice-clone --batch 8 --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/vc8_${v}.json 2> $O/vc8_${v}.err
  echo "vc8 $v $(val $O/vc8_${v}.json)"
done
