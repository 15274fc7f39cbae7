#!/usr/bin/env python3
"""Summarise one streaming-codec push from a rocprofv3 kernel trace of
tools/prof_stream.py (development tool): a push starts at k_rvq_sum.
  python3 tools/stream_trace.py <trace dir> [push index from the end, default 5]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 5
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
groups = []   # a push starts at its RVQ gather kernel
for r in rows:
    if "k_rvq_sum" in r["Kernel_Name"] or not groups:
        groups.append([])
    groups[-1].append(r)
g = groups[-idx]
span = (int(g[-1]["End_Timestamp"]) - int(g[0]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in g) / 1e3
print(f"{len(g)} kernels, span {span:.1f} us, busy {busy:.1f} us")
agg = {}
for r in g:
    k = (r["Kernel_Name"][:34], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    e = agg.setdefault(k, [0, 0.0])
    e[0] += 1
    e[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{t:8.1f} us x{c:3d} avg {t / c:6.1f}  {k}")
