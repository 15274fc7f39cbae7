#!/usr/bin/env python3
"""Micro-benchmark of the decode GEMV dispatcher (qtts_hip_decode_matvec_bf16)
at batch 1..16 on the 1.7B decode shapes: mean us per call over a burst of
back-to-back launches (torch events on the current stream), and the weight
stream rate.  QTTS_LIB selects a build (A/B).  The eager launches cost ~6.5 us
of host time each, so points below that are launch-rate bound: run it under
`rocprofv3 --kernel-trace` (tools/trace_by_grid.py) for device durations."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "qwen3-tts-c_amd"))

SHAPES = {  # name: (rows, cols, norm)
    "talker_qkv": (4096, 2048, True), "talker_o": (2048, 2048, False), "talker_gate_up": (12288, 2048, True),
    "talker_down": (2048, 6144, False), "st_qkv": (4096, 1024, True), "st_gate_up": (6144, 1024, True),
    "st_down": (1024, 3072, False), "st_head": (2048, 1024, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--batch", default="1,2,4,8,16", help="comma-separated batch sizes")
    ap.add_argument("--n", type=int, default=200, help="timed launches per point")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    batches = [int(b) for b in args.batch.split(",")]
    import torch
    import qtts
    dev = torch.device("cuda:0")
    out = {}
    for name, (R, Cc, norm) in SHAPES.items():
        if only and name not in only:
            continue
        A = torch.randint(0, 1 << 15, (R, Cc), dtype=torch.int16, device=dev).view(torch.uint16) \
            if hasattr(torch, "uint16") else torch.randint(0, 1 << 15, (R, Cc), dtype=torch.int16, device=dev)
        # keep the bf16 values finite and small: exponent bits of 0x3Fxx
        A = (A.to(torch.int32) & 0x007F | 0x3F00).to(torch.int16)
        w = torch.ones(Cc, device=dev) if norm else None
        for B in batches:
            x = torch.randn(B, Cc, device=dev)
            y = torch.zeros(B, R, device=dev)
            for _ in range(5):
                qtts.Kernels.decode_matvec_bf16(y, A, x, w, 1e-6, R, Cc, B)
            torch.cuda.synchronize()
            n = args.n
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                qtts.Kernels.decode_matvec_bf16(y, A, x, w, 1e-6, R, Cc, B)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / n * 1e3
            out[f"{name}/b{B}"] = dict(us=round(us, 2), GBs=round(R * Cc * 2 / us / 1e3, 1))
            print(f"{name:16s} b{B:2d} {us:8.2f} us  {R * Cc * 2 / us / 1e3:8.1f} GB/s", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
