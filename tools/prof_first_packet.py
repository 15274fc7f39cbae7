#!/usr/bin/env python3
"""First-packet anatomy on the bench workload (development tool): the 1.7B
P128 prompt decoded for ONE frame through qwen_tts_generate_stream (prompt
build + prefill + frame 0 + the exact streaming codec on it), 2 warm-ups and
5 measured requests; under rocprofv3 --kernel-trace, summarise with
tools/trace_by_grid.py (totals / 7 requests).

  python3 tools/prof_first_packet.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]


def main():
    import torch  # noqa: F401
    import qtts
    from synth_model import ensure_model, prompt_ids
    md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
    m = qtts.QwenTTS(md)
    m.set_params(max_tokens=1, fixed=1, seed=42)
    ids = prompt_ids("p128")
    for i in range(7):
        t = time.perf_counter()
        m.generate_stream(ids, "aiden", "english", chunk_frames=8)
        print(f"request {i}: first packet {m.c.perf_first_packet_ms:.2f} ms (prefill {m.c.perf_prefill_ms:.2f}, "
              f"first frame {m.c.perf_first_frame_ms:.2f}), wall {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
    m.close()


if __name__ == "__main__":
    main()
