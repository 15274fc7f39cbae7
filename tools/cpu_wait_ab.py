#!/usr/bin/env python3
"""Why is the reference's 16-thread talker slower per frame than its 1-thread
talker?  The reference's kernel_matvec_bf16 has no
OpenMP (K.c:139-148), so during the talker the worker threads only wait; with
the default (active) OMP_WAIT_POLICY they spin.  Alternating A/B of the
bench's CPU leg at 16 threads with OMP_WAIT_POLICY unset vs passive, plus the
1-thread row and one unextrapolated run of the full 128 frames.
  python tools/cpu_wait_ab.py [threads]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]


def main():
    import threading
    import time
    t0 = time.time()

    def beat():   # a line a minute: the GPU box's runner takes 3 silent minutes for a hang
        while True:
            time.sleep(60)
            print(f"[cpu_wait_ab] {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    import bench
    from synth_model import ensure_model, prompt_ids
    thr = int(sys.argv[1]) if len(sys.argv) > 1 else bench.cpu_threads_default()
    md = ensure_model(os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), "1.7b"), "1.7b", seed=0)
    ids = prompt_ids("p128", seed=1234)
    out = []
    for pol in [None, "passive", None, "passive"]:
        r = bench.cpu_baseline(md, ids, thr, frames=8, runs=2, wait_policy=pol)
        rec = {"threads": thr, "OMP_WAIT_POLICY": pol or "(unset: active)",
               "talker_ms_per_frame": [round(x["talker_ms"] / x["tokens"], 1) for x in r["runs"]] if r else None,
               "value": round(r["value"], 4) if r else None}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    r = bench.cpu_baseline(md, ids, 1, frames=2, warmup=0, runs=2, timeout=3000)
    print(json.dumps({"threads": 1, "talker_ms_per_frame": [round(x["talker_ms"] / x["tokens"], 1) for x in r["runs"]]
                      if r else None, "value": round(r["value"], 4) if r else None}), flush=True)
    # one run of the whole 128-frame workload, nothing extrapolated (passive wait)
    r = bench.cpu_baseline(md, ids, thr, frames=128, warmup=0, runs=2, timeout=3000, wait_policy="passive")
    if r:
        print(json.dumps({"threads": thr, "frames": 128, "OMP_WAIT_POLICY": "passive", "runs": r["runs"],
                          "value": round(r["value"], 4)}), flush=True)


if __name__ == "__main__":
    main()
