"""Voice-clone (C5) time split on the GPU: prefill / decode / codec per call,
batch 1 and 8, next to the plain prompt (tools/r01az_vc.sh)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tools")]
import qtts  # noqa: E402
from synth_model import ensure_model, prompt_ids  # noqa: E402

md = ensure_model("/tmp/qtts_test_models/1.7b", "1.7b")
m = qtts.QwenTTS(md)
m.set_params(max_tokens=128, fixed=128, seed=42)
only = os.environ.get("QTTS_VC_ONLY")   # "8": batch-8 clone only (under rocprofv3)
for nb in ((8,) if only else (1, 8)):
    prompts = [prompt_ids("p128", seed=1234 + i) for i in range(nb)]
    r = np.random.default_rng(7)
    vc = [([151644, 77091, 198] + r.integers(1000, 100000, size=20).tolist() + [151645, 198],
           r.integers(0, 2048, size=(63, 16)).astype(np.int32), (r.standard_normal(2048) * 0.05).astype(np.float32))
          for _ in range(nb)]
    for mode in (("clone",) if only else ("plain", "clone")):
        for it in range(1 if only else 3):
            t = time.perf_counter()
            if mode == "plain":
                rc, _ = m.generate_batch(prompts, ["aiden"] * nb, ["english"] * nb)
            else:
                rc, _ = m.generate_voice_clone_batch(prompts, [v[0] for v in vc], [v[1] for v in vc],
                                                     [v[2] for v in vc], ["english"] * nb)
            w = (time.perf_counter() - t) * 1e3
        c = m.c
        print(f"nb={nb} {mode:5s} rc={rc} wall {w:7.1f} ms  prefill {c.perf_prefill_ms:6.1f}  "
              f"talker {c.perf_talker_ms:6.1f}  codec {c.perf_codec_ms:6.1f}  total {c.perf_total_ms:7.1f}", flush=True)
m.close()
