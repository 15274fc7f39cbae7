#!/usr/bin/env python3
"""Voice-clone encoder timing: the speaker encoder and the
12 Hz encoder on B synthetic 5 s references (BASELINE C5: batch 8), repeated
so that `rocprofv3 --kernel-trace --stats -- python3 tools/prof_enc.py`
attributes per-kernel time.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "qwen3-tts-c_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="1.7b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--secs", type=float, default=5.0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch  # noqa: F401  (loads the HIP runtime first, as qtts.lib() expects)
    import qtts
    from synth_model import ensure_model, ref_wave
    from bench import encoder_gflop
    md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), a.preset), a.preset)
    m = qtts.QwenTTS(md)
    wavs = [ref_wave(1241 + i, a.secs) for i in range(a.batch)]
    m.speaker_embed(wavs)
    m.encode_audio(wavs)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        m.speaker_embed(wavs)
    t1 = time.perf_counter()
    for _ in range(a.reps):
        m.encode_audio(wavs)
    t2 = time.perf_counter()
    m.close()
    gs, gc = encoder_gflop(md, [w.shape[0] for w in wavs])
    sp, co = (t1 - t0) / a.reps * 1e3, (t2 - t1) / a.reps * 1e3
    print(json.dumps(dict(preset=a.preset, batch=a.batch, secs=a.secs, speaker_ms=round(sp, 3), codes_ms=round(co, 3),
                          speaker_gflop=round(gs, 2), codes_gflop=round(gc, 2), speaker_tflops=round(gs / sp, 2),
                          codes_tflops=round(gc / co, 2))), flush=True)


if __name__ == "__main__":
    main()
