#!/usr/bin/env python3
"""Where a lock-step EOS batch leaves the reference's codes (development
diagnostic): the 1.7B EOS model's three golden utterances (long_eos17.npz)
as one batch; per slot, the first (frame, group) whose code differs from
the reference's and the stop step.  Env switches apply (QTTS_HIP_GEMVWB ...)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
import qtts  # noqa: E402
from conftest import model_dir  # noqa: E402
from oracle_py import DEFAULT  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
g = np.load(os.path.join(G, "long_eos17.npz"))
man = json.load(open(os.path.join(G, "long_manifest.json")))["eos17"]
prompts = [g["prompt_ids"][b, :int(g["prompt_len"][b])].tolist() for b in range(g["prompt_ids"].shape[0])]
m = qtts.QwenTTS(model_dir("1.7b", eos_gain=man["eos_gain"]))
m.set_params(max_tokens=int(sys.argv[1]) if len(sys.argv) > 1 else 4096, fixed=0, seed=man["seed"], **DEFAULT)
rc, aud = m.generate_batch(prompts, man["speakers"], [man["language"]] * len(prompts))
codes = m.last_codes_batch()
for b in range(len(prompts)):
    n = int(g["stop_step"][b])
    ref = g["codes"][b, :n]
    got = codes[b]
    k = min(len(got), n)
    d = np.argwhere(got[:k] != ref[:k])
    first = tuple(int(v) for v in d[0]) if len(d) else None
    print(f"slot {b}: frames {len(got)} (reference stop {n}); first differing (frame, group) {first}", flush=True)
m.close()
