#!/usr/bin/env python3
"""Stop steps of EOS-mode utterances on bench.py --eos's model (1.7B, EOS row
x 1.4), so the EOS golden (tests/golden/make_golden_long.py eos17) only asks
the reference for runs that stop inside a bounded number of frames.
  python tools/eos_stop_probe.py 1234 1235 1236"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "qwen3-tts-c_amd")]
SPK = ["aiden", "vivian", "serena"]


def main():
    import qtts
    from synth_model import ensure_model, prompt_ids
    root = os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models")
    md = ensure_model(os.path.join(root, "1.7b_eos_gain1.4"), "1.7b", seed=0, overrides={"eos_gain": 1.4})
    m = qtts.QwenTTS(md)
    for i, sd in enumerate(int(x) for x in sys.argv[1:]):
        m.set_params(max_tokens=1024, fixed=0, seed=42)
        m.generate(prompt_ids("p128", seed=sd), SPK[i % 3], "english")
        st = int(m.c.last_stop_step) if m.c.last_stop_reason == 1 else -1
        print(f"seed {sd} speaker {SPK[i % 3]}: stop step {st} frames {m.c.last_frames}", flush=True)
    m.close()


if __name__ == "__main__":
    main()
