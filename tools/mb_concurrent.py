#!/usr/bin/env python3
"""Lock-step groups side by side on one GPU (development measurement).

G model contexts on the same device, each decoding its own lock-step batch of
B utterances (bench.py's synthetic 1.7B, P128 prompts, fixed 128 frames) from
its own host thread -- so G frame graphs run concurrently on G HIP streams
and one group's latency-bound launches can fill the other's idle CUs.
Prints the whole job's audio-s/s (G x B utterances per step, max wall over
the threads), comparable with `bench.py --batch G*B`.

  python tools/mb_concurrent.py --groups 2 --batch 4 --steps 3 --warmup 1
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402  (sets sys.path for qtts / synth_model)
import qtts  # noqa: E402
from synth_model import prompt_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--preset", default="1.7b")
    a = ap.parse_args()
    md = os.path.join(os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models"), a.preset)
    bench.ensure_model_shared(md, a.preset, 1, 0, None)
    seeds = bench.rank_prompt_seeds(0, a.groups * a.batch)
    models = []
    for g in range(a.groups):
        m = qtts.QwenTTS(md, device=0)
        m.set_params(max_tokens=a.frames, fixed=a.frames, seed=42 + g)
        models.append(m)
    prompts = [[prompt_ids("p128", seed=s) for s in seeds[g * a.batch:(g + 1) * a.batch]] for g in range(a.groups)]
    bar = threading.Barrier(a.groups)
    res = [None] * a.groups
    err = []

    def step(g):
        m = models[g]
        if a.batch == 1:
            x = m.generate(prompts[g][0], "aiden", "english")
            return len(x)
        rc, aud = m.generate_batch(prompts[g], ["aiden"] * a.batch, ["english"] * a.batch)
        if rc != 0:
            raise RuntimeError("batch generation failed")
        return sum(len(x) for x in aud)

    def run(g):
        try:
            for _ in range(a.warmup):
                step(g)
            bar.wait()
            t0 = time.perf_counter()
            n = sum(step(g) for _ in range(a.steps))
            res[g] = (n, time.perf_counter() - t0)
        except Exception as e:  # noqa: BLE001
            err.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=run, args=(g,)) for g in range(a.groups)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for m in models:
        m.close()
    if err:
        raise SystemExit("; ".join(err))
    wall = max(r[1] for r in res)
    audio = sum(r[0] for r in res) / 24000.0
    print(f"groups {a.groups} x batch {a.batch}: {audio / wall:.2f} audio-s/s "
          f"(walls {' '.join(f'{r[1]:.3f}' for r in res)} s for {a.steps} steps)", flush=True)


if __name__ == "__main__":
    main()
