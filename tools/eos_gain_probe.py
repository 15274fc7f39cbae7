#!/usr/bin/env python3
"""Where does EOS land on the synthetic 1.7B model for a given codec-head EOS
gain (tools/synth_model.py eos_gain)?  For bench.py --eos: pick a gain whose
utterances stop inside 128-256 frames under the default sampling.
  python tools/eos_gain_probe.py 1.5 1.8 2.0"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "qwen3-tts-c_amd")]


def main():
    import qtts
    from synth_model import ensure_model, prompt_ids
    root = os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models")
    for g in [float(x) for x in sys.argv[1:]]:
        md = ensure_model(os.path.join(root, f"1.7b_eos_gain{g}"), "1.7b", seed=0, overrides={"eos_gain": g})
        m = qtts.QwenTTS(md)
        stops = []
        for sd in range(1234, 1250):
            m.set_params(max_tokens=1024, fixed=0, seed=42)
            m.generate(prompt_ids("p128", seed=sd), "aiden", "english")
            stops.append(int(m.c.last_stop_step) if m.c.last_stop_reason == 1 else -1)
        m.close()
        print(f"eos_gain {g}: stop steps {stops}", flush=True)


if __name__ == "__main__":
    main()
