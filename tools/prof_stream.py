#!/usr/bin/env python3
"""First-packet anatomy (development tool): times the exact streaming codec
push of 1 frame (the first packet's codec share) and of 8-frame chunks on the
synthetic 1.7B codec, host wall per push; run under rocprofv3 --kernel-trace
to split kernel time from launch overhead.

  python3 tools/prof_stream.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import torch  # noqa: F401
    import ctypes as C
    import qtts
    from synth_model import ensure_model
    md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
    m = qtts.QwenTTS(md)
    L = qtts.lib()
    codes = np.random.default_rng(0).integers(0, 2048, size=(64, 16)).astype(np.int32)
    for rep in range(3):
        if L.qwen_tts_codec_stream_begin(m.ctx, 256) != 0:
            raise RuntimeError("begin")
        ts = []
        t = 0
        for k in [1, 1, 1, 8, 8, 8]:
            c = np.ascontiguousarray(codes[t:t + k])
            o = np.zeros(k * 1920, np.float32)
            t0 = time.perf_counter()
            n = L.qwen_tts_codec_stream_push(m.ctx, c.ctypes.data_as(C.POINTER(C.c_int)), k,
                                             o.ctypes.data_as(C.POINTER(C.c_float)))
            ts.append((k, (time.perf_counter() - t0) * 1e3))
            assert n == k * 1920
            t += k
        print("rep", rep, " ".join(f"{k}f:{ms:.2f}ms" for k, ms in ts), flush=True)
    m.close()


if __name__ == "__main__":
    main()
