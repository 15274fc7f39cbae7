#!/usr/bin/env python3
"""Codec-only workload for rocprofv3 (development tool): decode 128 random
frames of the synthetic 1.7B codec twice through the C-ABI.

  rocprofv3 --kernel-trace -f csv -d gpurun_out/codec -o run -- python3 tools/prof_codec.py
  python3 tools/prof_codec.py --summarize gpurun_out/codec   # per-GEMM table of the 2nd decode
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "qwen3-tts-c_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]


def run():
    import numpy as np
    import torch  # noqa: F401  (HIP runtime first, qtts.lib())
    import time
    import qtts
    from synth_model import ensure_model
    md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b")
    m = qtts.QwenTTS(md)
    codes = np.random.default_rng(0).integers(0, 2048, size=(128, 16)).astype(np.int32)
    for i in range(3):
        t = time.perf_counter()
        a = m.codec_decode(codes)
        print(f"decode {i}: {(time.perf_counter() - t) * 1e3:.1f} ms, {len(a)} samples", flush=True)
    m.close()


def summarize(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the codec decodes are separated by host gaps; take the last third of the dispatches
    n = len(rows)
    last = rows[2 * n // 3:]
    tot = 0.0
    agg = {}
    for r in last:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (r["Kernel_Name"][:40], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
               r.get("Grid_Size_Z", ""))
        e = agg.setdefault(key, [0, 0.0])
        e[0] += 1
        e[1] += dur
        tot += dur
    print(f"{len(last)} dispatches, {tot / 1e3:.2f} ms kernel time")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{t:9.1f} us  x{c:3d}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
