"""Per-step wall times of the 1.7B batch-1 bench workload in one process
(development tool): is the run-to-run spread of bench.py per process or per
step?  python tools/step_spread.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "qwen3-tts-c_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import qtts  # noqa: E402
from synth_model import ensure_model, prompt_ids  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
md = os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b")
ensure_model(md, "1.7b", seed=0)
m = qtts.QwenTTS(md)
m.set_params(max_tokens=128, fixed=128, seed=42)
p = prompt_ids("p128", seed=1234)
m.generate(p, "aiden", "english")
ts = []
for _ in range(steps):
    t = time.perf_counter()
    m.generate(p, "aiden", "english")
    ts.append((time.perf_counter() - t) * 1e3)
print("step ms:", " ".join(f"{x:.1f}" for x in ts), f"| audio-s/s {10.24 / (sum(ts) / len(ts) / 1e3):.2f}", flush=True)
m.close()
