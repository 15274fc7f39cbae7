#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv by (kernel, grid): launches, total
and mean duration -- the per-layer view of a launch chain whose layers share
one kernel (the encoders' k_econv).  Usage: trace_by_grid.py <trace.csv> [top]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    agg = collections.defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "?")
            name = name.replace("(anonymous namespace)::", "")[:60]
            grid = tuple(int(r.get(f"Grid_Size_{a}", 0) or 0) // max(1, int(r.get(f"Workgroup_Size_{a}", 1) or 1))
                         for a in "XYZ")
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = agg[(name, grid)]
            a[0] += 1
            a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':60s} {'grid (workgroups)':>22s} {'n':>5s} {'total_us':>10s} {'mean_us':>9s} {'share':>6s}")
    for (name, grid), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{name:60s} {str(grid):>22s} {n:5d} {t:10.1f} {t / n:9.1f} {t / tot:6.1%}")


if __name__ == "__main__":
    main()
