#!/usr/bin/env python3
"""Per-kernel cost of one decode frame in graph replay, from a rocprofv3
--kernel-trace CSV (development tool).

  python tools/trace_frame.py <dir with *kernel_trace.csv> [--skip N]

Frames are delimited by k_embed_sum (the last kernel of a frame graph).  For
every kernel instance the 'slot' is end_i - end_{i-1} (what it adds to the
frame's wall time), 'dur' is end - start and 'gap' is start_i - end_{i-1}
(negative when the dispatch overlaps the predecessor's tail).  Prints the
per-name means over the frames after the first N (warm-up) and the mean
frame time.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 8
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start-Timestamp"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End-Timestamp"
    key_n = "Kernel_Name" if "Kernel_Name" in rows[0] else "Kernel-Name"
    rows.sort(key=lambda r: int(r[key_s]))
    ks = [(r[key_n], int(r[key_s]), int(r[key_e])) for r in rows]
    frames, cur = [], []
    for k in ks:
        cur.append(k)
        if "k_embed_sum" in k[0]:
            frames.append(cur)
            cur = []
    frames = [fr for fr in frames[skip:] if len(fr) > 100]
    if not frames:
        print("no frames")
        return
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    ftimes = []
    for fr in frames:
        ftimes.append((fr[-1][2] - fr[0][1]) / 1e3)
        for i in range(1, len(fr)):
            n, s, e = fr[i]
            pe = fr[i - 1][2]
            a = agg[n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]]
            a[0] += 1
            a[1] += (e - pe) / 1e3
            a[2] += (e - s) / 1e3
            a[3] += (s - pe) / 1e3
    nf = len(frames)
    print(f"{nf} frames, {len(frames[0])} kernels each, mean frame {sum(ftimes) / nf:.1f} us")
    print(f"{'kernel':50s} {'per frame':>9s} {'slot us':>8s} {'dur us':>7s} {'gap us':>7s} {'us/frame':>9s}")
    for n, (c, sl, du, gp) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n[:50]:50s} {c / nf:9.1f} {sl / c:8.2f} {du / c:7.2f} {gp / c:7.2f} {sl / nf:9.1f}")


if __name__ == "__main__":
    main()
