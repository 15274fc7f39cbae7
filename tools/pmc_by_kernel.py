#!/usr/bin/env python3
"""Mean per dispatch of every counter in a rocprofv3 --pmc output directory,
by kernel: python tools/pmc_by_kernel.py <dir> [out.json]  (the raw
counter_collection.csv files are deleted afterwards: gpurun's 64 MiB)."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import counters  # noqa: E402


def main():
    d = sys.argv[1]
    files = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    out = {k.replace("(anonymous namespace)::", ""): {c.replace("_kb_avg", "_avg"): v for c, v in e.items()}
           for k, e in counters(files).items()}
    for f in files:
        os.remove(f)
    js = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js)
    else:
        print(js)


if __name__ == "__main__":
    main()
