#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of tools/prof_first_packet.py (development
tool): for the last request, the GPU timeline from its first kernel to its last
-- busy time (union of kernel intervals) vs span, split at the prefill / frame /
codec boundaries by kernel name.  Usage: fp_timeline.py <kernel_trace.csv>"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # requests are separated by host gaps > 2 ms
    reqs, cur = [], [ev[0]]
    for a, b in zip(ev, ev[1:]):
        if b[0] - a[1] > 2_000_000:
            reqs.append(cur)
            cur = []
        cur.append(b)
    reqs.append(cur)
    last = reqs[-1]
    t0 = last[0][0]

    def phase(name):
        if "k_conv" in name or "k_xg" in name or "k_xlin" in name or "k_rvq" in name or "k_snake" in name or "k_dwconv" in name or "k_ln_t" in name or "k_clamp" in name or "copy2d" in name or "k_rms_rows" in name or "k_rope_rows" in name or "k_attn(" in name:
            return "codec"
        return "decode"
    segs = {}
    busy_end = t0
    for s, e, n in last:
        p = phase(n)
        d = segs.setdefault(p, [0, 0, None, None, 0])
        d[0] += 1
        d[1] += e - s
        d[2] = s if d[2] is None else min(d[2], s)
        d[3] = e if d[3] is None else max(d[3], e)
    print(f"{len(reqs)} requests; last: {len(last)} kernels, span {(last[-1][1] - t0) / 1e3:.1f} us")
    for p, (n, dur, s, e, _) in segs.items():
        print(f"  {p:7s} {n:4d} kernels  sum {dur / 1e3:8.1f} us  window {(s - t0) / 1e3:8.1f} - {(e - t0) / 1e3:8.1f} us")
    # prefill = the decode-phase kernels before the first frame graph's k_embed_sum / sampler
    names = [n for _, _, n in last]
    gaps = sorted(((b[0] - a[1]), i) for i, (a, b) in enumerate(zip(last, last[1:])))[-8:]
    print("  largest gaps (us, after kernel):", ", ".join(f"{g / 1e3:.1f}@{names[i][:30]}" for g, i in reversed(gaps)))
    # first 400 kernels (prefill + start of frame 0): busy vs span
    k = min(len(last), 400)
    span = last[k - 1][1] - t0
    busy = sum(e - s for s, e, _ in last[:k])
    print(f"  first {k} kernels: span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
