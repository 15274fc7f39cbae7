#!/usr/bin/env python3
"""Condense rocprofv3 output directories into small committed summaries.

  python tools/prof_summary.py <out_dir>

Looks under <out_dir> for
  prof/**/run_kernel_stats.csv        (--kernel-trace --stats)  -> kernel_stats.csv (copied)
  pmc_fetch/**/*counter_collection.csv (--pmc FETCH_SIZE)        -> pmc.json
  pmc_write/**/*counter_collection.csv (--pmc WRITE_SIZE)
  pmc_mfma/**/*counter_collection.csv  (--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE)
and writes pmc.json: per kernel name {dispatches, FETCH_SIZE_kb_avg,
WRITE_SIZE_kb_avg, hbm_read_bytes_avg (FETCH_SIZE x 1024 x 2: the gfx950
half-count correction of MI355X_MICROARCH.md "HBM"), hbm_write_bytes_avg}.
and mfma.json: per matrix-core kernel {dispatches, the three counters per
dispatch, mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs
x 4 SIMDs)} -- GRBM_GUI_ACTIVE is summed over the 8 XCDs and
SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per 32x32x16 bf16 MFMA per SIMD
(MI355X_MICROARCH.md), so mfma_util is the fraction of the chip's matrix-core
issue cycles the kernel kept busy while it ran.
The raw traces are deleted afterwards (they do not fit gpurun's 64 MiB).
"""
import csv
import glob
import json
import os
import shutil
import sys


def find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def counters(files):
    agg = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or "?"
                cn = row.get("Counter_Name")
                v = float(row.get("Counter_Value", 0) or 0)
                key = (name, cn)
                a = agg.setdefault(key, [0, 0.0, set()])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                a[2].add(disp)
                a[1] += v
    out = {}
    for (name, cn), (_, tot, ds) in agg.items():
        e = out.setdefault(name, {})
        e["dispatches"] = len(ds)
        e[f"{cn}_kb_avg"] = tot / max(len(ds), 1)
    return out


def main():
    d = sys.argv[1]
    st = find(os.path.join(d, "prof"), "*kernel_stats.csv")
    if st:
        shutil.copy(st[0], os.path.join(d, "kernel_stats.csv"))
    res = {}
    for sub in ("pmc_fetch", "pmc_write"):
        for name, e in counters(find(os.path.join(d, sub), "*counter_collection.csv")).items():
            res.setdefault(name, {}).update(e)
    for name, e in res.items():
        if "FETCH_SIZE_kb_avg" in e:
            e["hbm_read_bytes_avg"] = e["FETCH_SIZE_kb_avg"] * 1024 * 2
        if "WRITE_SIZE_kb_avg" in e:
            e["hbm_write_bytes_avg"] = e["WRITE_SIZE_kb_avg"] * 1024
    if res:   # (a second call after the mfma pass leaves the first call's pmc.json)
        with open(os.path.join(d, "pmc.json"), "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
    mf = {}
    for name, e in counters(find(os.path.join(d, "pmc_mfma"), "*counter_collection.csv")).items():
        busy = e.get("SQ_VALU_MFMA_BUSY_CYCLES_kb_avg", 0.0)
        if busy <= 0:
            continue
        act = e.get("GRBM_GUI_ACTIVE_kb_avg", 0.0)
        mf[name] = {"dispatches": e["dispatches"], "SQ_VALU_MFMA_BUSY_CYCLES_avg": busy,
                    "SQ_BUSY_CYCLES_avg": e.get("SQ_BUSY_CYCLES_kb_avg"), "GRBM_GUI_ACTIVE_avg": act,
                    "mfma_util": busy / (act / 8 * 256 * 4) if act > 0 else None}
    if mf:
        with open(os.path.join(d, "mfma.json"), "w") as f:
            json.dump(mf, f, indent=1, sort_keys=True)
    for sub in ("prof", "pmc_fetch", "pmc_write", "pmc_mfma"):
        shutil.rmtree(os.path.join(d, sub), ignore_errors=True)
    print(f"summaries in {d}: kernel_stats.csv, pmc.json ({len(res)} kernels), mfma.json ({len(mf)} kernels)")


if __name__ == "__main__":
    main()
