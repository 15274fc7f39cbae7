#!/usr/bin/env python3
"""Long-context golden fixtures from the REFERENCE build (TEST INFRASTRUCTURE).

Runs in the build container only (needs oracle/_ref/libqtts_ref.so, i.e.
`make -C oracle ref` against the unmodified /root/reference/c sources).  The
committed .npz files are data: seeded inputs and the reference's outputs.

  python tests/golden/make_golden_long.py            # all fixtures below
  python tests/golden/make_golden_long.py --only hd128

Fixtures
  long_hd128.npz   the `hd128` synthetic model (the 0.6B / 1.7B talker's
                   attention shape NH 16 / KV 8 / HD 128 in 2 narrow layers):
                   * a 640-frame default-sampling decode (P128 prompt, seed 42):
                     talker positions run to ~650, i.e. through 1, 2-8 and > 8
                     64-key splits of the decode attention (T.c:119-248); codes
                     and the waveform (every 16th sample, plus the first and
                     last frame in full);
                   * a 600-row prefill (> 512 rows, T.c:254-472) of seeded
                     embeddings (prefill_inputs(): regenerated from the seed), then 4 decode steps at positions 600-603:
                     prefill hidden, per-step logits and hidden.
  long_17b.npz     the BASELINE workload itself on the synthetic 1.7B model:
                   P128 prompt, fixed 128 frames, default sampling, seed 42
                   (bench.py's utterance): codes and the full waveform.
  long_06b.npz     BASELINE configs[1] (C2) on the synthetic 0.6B model: P128
                   prompt, GREEDY, fixed 128 frames, seed 42: codes and the
                   full waveform.
  long_17b_b8.npz  BASELINE C4's per-GPU shape on the synthetic 1.7B model:
                   8 prompts (p128 seeds 1400+i, speakers cycling
                   aiden / vivian / serena), default sampling, fixed 32
                   frames, seed 42 -- each slot ONE reference run (the
                   reference has no batch path); the GPU test decodes the 8
                   as one lock-step batch.  Codes, every 16th sample, and
                   each slot's last frame.
  long_17b_b8bench.npz  C4's per-GPU bench workload itself: exactly the 8
                   utterances `bench.py --batch 8` rank 0 decodes (p128 seeds
                   1234-1241, speaker aiden, seed 42, default sampling, fixed
                   128 frames) -- each slot ONE reference run.  Codes, every
                   16th sample, each slot's last frame.
  long_eos17.npz   EOS mode (the reference's default: max_new_tokens 4096, stop
                   at EOS, Q.c:1282-1330) on `bench.py --eos`'s model (1.7B,
                   codec-head EOS row x 1.4): p128 seeds 1234 / 1235 / 1236
                   with aiden / vivian / serena, seed 42, default sampling --
                   each one reference run: the stop step (= frames emitted),
                   all codes, every 16th sample.
  long_hd128_max.npz  the reference's full decode capacity on the `hd128`
                   model: max_new_tokens 4096 frames, fixed (P128 prompt,
                   seed 42, default sampling) -- talker positions to ~4200,
                   i.e. > 128 splits of 32 keys in the decode attention and
                   its merge (the maximum-size edge case of T.c:119-248).
                   Codes, every 256th sample, first and last frame.
  long_hd128_steps4k.npz  the `hd128` model's stage functions near the
                   capacity: a 4000-row prefill of seeded embeddings, then 4
                   decode steps at positions 4000-4003 (> 125 splits of 32
                   keys): the prefill's last hidden row, per-step logits and
                   hidden.
  long_17b_1100.npz  the synthetic 1.7B past 1024 keys: P128 prompt, fixed
                   1100 frames (positions to ~1140: > 32 splits of 32 keys per
                   kv head -- the talker layer engine's second split round),
                   seed 42, default sampling; codes, every 256th sample,
                   first and last frame.
  long_manifest.json  SHA-256 of the model files the fixtures were made from.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

from oracle_py import RefLib, REF_SO, DEFAULT, GREEDY  # noqa: E402
from synth_model import ensure_model, prompt_ids  # noqa: E402

MODEL_ROOT = os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models")
LONG_FRAMES = 640       # hd128 decode length (positions ~ 650: 11 splits of 64 keys)
PREFILL_ROWS = 600      # hd128 stage prefill (> 512 rows)
PREFILL_STEPS = 4
PREFILL_SEED = 20261017
AUDIO_STRIDE = 16
BENCH_FRAMES = 128      # bench.py workload
B8_FRAMES = 32          # C4 lock-step batch fixture
B8_SEEDS = [1400 + i for i in range(8)]
B8_SPEAKERS = ["aiden", "vivian", "serena", "aiden", "vivian", "serena", "aiden", "vivian"]
B8B_SEEDS = [1234 + i for i in range(8)]     # bench.py rank_prompt_seeds(0, 8)
EOS_GAIN = 1.4                               # bench.py EOS_GAIN
EOS_SEEDS = [1234, 1235, 1236]
EOS_SPEAKERS = ["aiden", "vivian", "serena"]
EOS_CAP = 1024                               # the fixture asserts every run stopped well before this
# (the cap bounds a run that would not stop; every fixture run stops well
# before it, so each result equals the reference's 4096-token run)
EOS_Q_SEEDS = [1237, 1238, 1239]             # long_eos17q: three more EOS utterances for the slot-refill queue
EOS_Q_SPEAKERS = ["aiden", "vivian", "serena"]


def model_hashes(md):
    out = {}
    for rel in ("config.json", "model.safetensors", "speech_tokenizer/config.json",
                "speech_tokenizer/model.safetensors"):
        h = hashlib.sha256()
        with open(os.path.join(md, rel), "rb") as f:
            for blk in iter(lambda: f.read(1 << 24), b""):
                h.update(blk)
        out[rel] = h.hexdigest()
    return out


def prefill_inputs(H, seed=PREFILL_SEED):
    """The stage inputs (regenerated by the tests from the seed, not stored)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    emb = (rng.standard_normal((PREFILL_ROWS, H)) * 0.5).astype(np.float32)
    steps = (rng.standard_normal((PREFILL_STEPS, H)) * 0.5).astype(np.float32)
    return emb, steps


MAX_FRAMES = 4096       # the reference's max_new_tokens default: the decode capacity
MAX_STRIDE = 256


def hd128_max_fixture():
    md = ensure_model(os.path.join(MODEL_ROOT, "hd128"), "hd128")
    ref = RefLib(md)
    ids = np.array(prompt_ids("p128"), np.int32)
    ref.set_params(max_tokens=MAX_FRAMES, fixed=MAX_FRAMES, seed=42, **DEFAULT)
    t = time.time()
    audio = ref.generate(ids, "aiden", "english")
    print(f"hd128 decode {MAX_FRAMES} frames: {time.time() - t:.1f} s", file=sys.stderr)
    codes = ref.recorded_codes()
    assert codes.shape == (MAX_FRAMES, ref.cfg["cq"]), codes.shape
    g = {"prompt_ids": ids, "codes": codes, "audio_sub": audio[::MAX_STRIDE].copy(),
         "audio_first": audio[:1920].copy(), "audio_last": audio[-1920:].copy(),
         "audio_len": np.array(len(audio), np.int64)}
    return g, md


STEPS4K_ROWS = 4000     # hd128 stage prefill near the decode capacity, then decode steps
STEPS4K_SEED = 20261019


def hd128_steps4k_fixture():
    """A 4000-row prefill of seeded embeddings, then 4 decode steps at
    positions 4000-4003 (125+ splits of 32 keys): prefill hidden (last row),
    per-step logits and hidden -- the decode attention near the capacity,
    compared with a tolerance (no sampling, so no near-tie can flip it)."""
    md = ensure_model(os.path.join(MODEL_ROOT, "hd128"), "hd128")
    ref = RefLib(md)
    rng = np.random.Generator(np.random.PCG64(STEPS4K_SEED))
    emb = (rng.standard_normal((STEPS4K_ROWS, ref.cfg["H"])) * 0.5).astype(np.float32)
    steps = (rng.standard_normal((PREFILL_STEPS, ref.cfg["H"])) * 0.5).astype(np.float32)
    t = time.time()
    hid = ref.prefill(emb)
    lg, hd = [], []
    for i in range(PREFILL_STEPS):
        l, h = ref.step(steps[i])
        lg.append(l)
        hd.append(h)
    print(f"hd128 {STEPS4K_ROWS}-row prefill + {PREFILL_STEPS} steps: {time.time() - t:.1f} s", file=sys.stderr)
    g = {"prefill_hidden": np.asarray(hid).copy(), "step_logits": np.stack(lg), "step_hidden": np.stack(hd)}
    return g, md


def hd128_fixtures():
    md = ensure_model(os.path.join(MODEL_ROOT, "hd128"), "hd128")
    ref = RefLib(md)
    g = {}
    ids = np.array(prompt_ids("p128"), np.int32)
    g["prompt_ids"] = ids
    ref.set_params(max_tokens=4096, fixed=LONG_FRAMES, seed=42, **DEFAULT)
    t = time.time()
    audio = ref.generate(ids, "aiden", "english")
    print(f"hd128 decode {LONG_FRAMES} frames: {time.time() - t:.1f} s", file=sys.stderr)
    codes = ref.recorded_codes()
    assert codes.shape == (LONG_FRAMES, ref.cfg["cq"]), codes.shape
    g["decode_codes"] = codes
    g["decode_audio_sub"] = audio[::AUDIO_STRIDE].copy()
    g["decode_audio_first"] = audio[:1920].copy()
    g["decode_audio_last"] = audio[-1920:].copy()
    g["decode_audio_len"] = np.array(len(audio), np.int64)
    # stage functions: > 512-row prefill, then decode steps over 600+ keys
    emb, steps_e = prefill_inputs(ref.cfg["H"])
    g["prefill_hidden"] = ref.prefill(emb)
    lg, hd = [], []
    for i in range(PREFILL_STEPS):
        l, h = ref.step(steps_e[i])
        lg.append(l)
        hd.append(h)
    g["step_logits"], g["step_hidden"] = np.stack(lg), np.stack(hd)
    ref.close()
    return g, md


def bench_fixtures():
    md = ensure_model(os.path.join(MODEL_ROOT, "1.7b"), "1.7b")
    ref = RefLib(md)
    ids = np.array(prompt_ids("p128"), np.int32)
    ref.set_params(max_tokens=BENCH_FRAMES, fixed=BENCH_FRAMES, seed=42, **DEFAULT)
    t = time.time()
    audio = ref.generate(ids, "aiden", "english")
    print(f"1.7b bench workload: {time.time() - t:.1f} s", file=sys.stderr)
    codes = ref.recorded_codes()
    assert codes.shape == (BENCH_FRAMES, ref.cfg["cq"]), codes.shape
    ref.close()
    return {"prompt_ids": ids, "codes": codes, "audio": audio}, md


K1100_FRAMES = 1100     # 1.7B past 1024 keys: > 32 splits of 32 keys per kv head


def k1100_fixture():
    md = ensure_model(os.path.join(MODEL_ROOT, "1.7b"), "1.7b")
    ref = RefLib(md)
    ids = np.array(prompt_ids("p128"), np.int32)
    ref.set_params(max_tokens=K1100_FRAMES, fixed=K1100_FRAMES, seed=42, **DEFAULT)
    t = time.time()
    audio = ref.generate(ids, "aiden", "english")
    print(f"1.7b {K1100_FRAMES} frames: {time.time() - t:.1f} s", file=sys.stderr)
    codes = ref.recorded_codes()
    assert codes.shape == (K1100_FRAMES, ref.cfg["cq"]), codes.shape
    ref.close()
    return {"prompt_ids": ids, "codes": codes, "audio_sub": audio[::MAX_STRIDE].copy(),
            "audio_first": audio[:1920].copy(), "audio_last": audio[-1920:].copy(),
            "audio_len": np.array(len(audio), np.int64)}, md


def c2_fixtures():
    md = ensure_model(os.path.join(MODEL_ROOT, "0.6b"), "0.6b")
    ref = RefLib(md)
    ids = np.array(prompt_ids("p128"), np.int32)
    ref.set_params(max_tokens=BENCH_FRAMES, fixed=BENCH_FRAMES, seed=42, **GREEDY)
    t = time.time()
    audio = ref.generate(ids, "aiden", "english")
    print(f"0.6b greedy {BENCH_FRAMES} frames: {time.time() - t:.1f} s", file=sys.stderr)
    codes = ref.recorded_codes()
    assert codes.shape == (BENCH_FRAMES, ref.cfg["cq"]), codes.shape
    ref.close()
    return {"prompt_ids": ids, "codes": codes, "audio": audio}, md


def b8_fixtures():
    md = ensure_model(os.path.join(MODEL_ROOT, "1.7b"), "1.7b")
    ref = RefLib(md)
    g = {}
    codes, sub, last = [], [], []
    ids_all = [np.array(prompt_ids("p128", s), np.int32) for s in B8_SEEDS]
    for b, ids in enumerate(ids_all):
        ref.set_params(max_tokens=4096, fixed=B8_FRAMES, seed=42, **DEFAULT)
        t = time.time()
        audio = ref.generate(ids, B8_SPEAKERS[b], "english")
        print(f"1.7b slot {b}: {B8_FRAMES} frames {time.time() - t:.1f} s", file=sys.stderr)
        c = ref.recorded_codes()
        assert c.shape == (B8_FRAMES, ref.cfg["cq"]), c.shape
        assert len(audio) == B8_FRAMES * 1920, len(audio)
        codes.append(c)
        sub.append(audio[::AUDIO_STRIDE].copy())
        last.append(audio[-1920:].copy())
    ref.close()
    L = max(len(x) for x in ids_all)
    g["prompt_ids"] = np.stack([np.pad(x, (0, L - len(x)), constant_values=-1) for x in ids_all])
    g["prompt_len"] = np.array([len(x) for x in ids_all], np.int32)
    g["codes"] = np.stack(codes)
    g["audio_sub"] = np.stack(sub)
    g["audio_last"] = np.stack(last)
    return g, md


def b8bench_fixtures():
    md = ensure_model(os.path.join(MODEL_ROOT, "1.7b"), "1.7b")
    ref = RefLib(md)
    codes, sub, last = [], [], []
    ids_all = [np.array(prompt_ids("p128", s), np.int32) for s in B8B_SEEDS]
    for b, ids in enumerate(ids_all):
        ref.set_params(max_tokens=BENCH_FRAMES, fixed=BENCH_FRAMES, seed=42, **DEFAULT)
        t = time.time()
        audio = ref.generate(ids, "aiden", "english")
        print(f"1.7b bench slot {b}: {BENCH_FRAMES} frames {time.time() - t:.1f} s", file=sys.stderr, flush=True)
        c = ref.recorded_codes()
        assert c.shape == (BENCH_FRAMES, ref.cfg["cq"]), c.shape
        assert len(audio) == BENCH_FRAMES * 1920, len(audio)
        codes.append(c)
        sub.append(audio[::AUDIO_STRIDE].copy())
        last.append(audio[-1920:].copy())
    ref.close()
    L = max(len(x) for x in ids_all)
    return {"prompt_ids": np.stack([np.pad(x, (0, L - len(x)), constant_values=-1) for x in ids_all]),
            "prompt_len": np.array([len(x) for x in ids_all], np.int32),
            "codes": np.stack(codes), "audio_sub": np.stack(sub), "audio_last": np.stack(last)}, md


def eos_model():
    return ensure_model(os.path.join(MODEL_ROOT, f"1.7b_eos_gain{EOS_GAIN}"), "1.7b", overrides={"eos_gain": EOS_GAIN})


def eos_seed_speaker(b):
    """Utterance b of the EOS set: 0-2 long_eos17, 3-5 long_eos17q."""
    seeds, spks = EOS_SEEDS + EOS_Q_SEEDS, EOS_SPEAKERS + EOS_Q_SPEAKERS
    return seeds[b], spks[b]


def eos17_slot(b):
    """One EOS-mode reference run (utterance b): codes [stop][G], every 16th sample."""
    ref = RefLib(eos_model())
    seed, spk = eos_seed_speaker(b)
    ids = np.array(prompt_ids("p128", seed), np.int32)
    # max_tokens is EOS_CAP, not 4096, only to bound a run that would not
    # stop; every fixture run stops well before it (asserted), so the result
    # equals the 4096-token run's
    ref.set_params(max_tokens=EOS_CAP, fixed=0, seed=42, **DEFAULT)
    t = time.time()
    audio = ref.generate(ids, spk, "english")
    c = ref.recorded_codes()
    print(f"1.7b eos slot {b}: stopped after {c.shape[0]} frames, {time.time() - t:.1f} s", file=sys.stderr, flush=True)
    assert 0 < c.shape[0] < EOS_CAP - 1, c.shape
    assert len(audio) == c.shape[0] * 1920, (len(audio), c.shape)
    ref.close()
    return c, audio[::AUDIO_STRIDE].copy()


def eos17_fixtures(slot_dir=None, utts=(0, 1, 2)):
    """slot_dir: the per-slot results of `--eos-slot b --slot-dir D` runs (one
    process per slot: the reference's recording hooks are process-global, and
    its talker GEMV is single-threaded, so the three runs go in parallel).
    utts: (0, 1, 2) long_eos17, (3, 4, 5) long_eos17q."""
    md = eos_model()
    g = {}
    ids_all = [np.array(prompt_ids("p128", eos_seed_speaker(b)[0]), np.int32) for b in utts]
    stops, codes, sub = [], [], []
    for b in utts:
        if slot_dir:
            z = np.load(os.path.join(slot_dir, f"eos_slot{b}.npz"))
            c, sb = z["codes"], z["audio_sub"]
        else:
            c, sb = eos17_slot(b)
        stops.append(c.shape[0])
        codes.append(c)
        sub.append(sb)
    L = max(len(x) for x in ids_all)
    T = max(stops)
    g["prompt_ids"] = np.stack([np.pad(x, (0, L - len(x)), constant_values=-1) for x in ids_all])
    g["prompt_len"] = np.array([len(x) for x in ids_all], np.int32)
    g["stop_step"] = np.array(stops, np.int32)
    g["codes"] = np.stack([np.pad(c, ((0, T - len(c)), (0, 0)), constant_values=-1) for c in codes])
    S = max(len(x) for x in sub)
    g["audio_sub"] = np.stack([np.pad(x, (0, S - len(x))) for x in sub])
    return g, md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["hd128", "hd128max", "steps4k", "k1100", "1.7b", "0.6b", "b8", "b8bench", "eos17", "eos17q"])
    ap.add_argument("--eos-slot", type=int, default=None, help="run one EOS slot into --slot-dir and exit")
    ap.add_argument("--slot-dir", default=None, help="eos17: per-slot results of --eos-slot runs")
    a = ap.parse_args()
    if a.eos_slot is not None:
        c, sb = eos17_slot(a.eos_slot)
        np.savez(os.path.join(a.slot_dir, f"eos_slot{a.eos_slot}.npz"), codes=c, audio_sub=sb)
        return
    if not os.path.exists(REF_SO):
        sys.exit(f"{REF_SO} missing: run `make -C oracle ref` first")
    mpath = os.path.join(HERE, "long_manifest.json")
    man = json.load(open(mpath)) if os.path.exists(mpath) else {}
    man.update({"generator": "tests/golden/make_golden_long.py",
                "reference": "oracle/_ref/libqtts_ref.so built from /root/reference/c by oracle/Makefile "
                             "(scalar + OpenMP, no BLAS)"})
    man.setdefault("models", {})
    if a.only in (None, "hd128"):
        g, md = hd128_fixtures()
        np.savez_compressed(os.path.join(HERE, "long_hd128.npz"), **g)
        man["models"]["hd128"] = model_hashes(md)
        man["hd128"] = {"frames": LONG_FRAMES, "prompt": "p128", "seed": 42, "sampling": "default",
                        "audio_stride": AUDIO_STRIDE, "prefill_rows": PREFILL_ROWS, "prefill_steps": PREFILL_STEPS,
                        "prefill_seed": PREFILL_SEED}
    if a.only == "hd128max":   # (not in the default set: a 4096-frame reference run)
        g, md = hd128_max_fixture()
        np.savez_compressed(os.path.join(HERE, "long_hd128_max.npz"), **g)
        man["models"]["hd128"] = model_hashes(md)
        man["hd128max"] = {"frames": MAX_FRAMES, "prompt": "p128", "seed": 42, "sampling": "default",
                           "speaker": "aiden", "language": "english", "audio_stride": MAX_STRIDE}
    if a.only == "steps4k":
        g, md = hd128_steps4k_fixture()
        np.savez_compressed(os.path.join(HERE, "long_hd128_steps4k.npz"), **g)
        man["models"]["hd128"] = model_hashes(md)
        man["steps4k"] = {"prefill_rows": STEPS4K_ROWS, "prefill_seed": STEPS4K_SEED, "steps": PREFILL_STEPS}
    if a.only == "k1100":   # (not in the default set: a 1100-frame 1.7B reference run, ~30 min)
        g, md = k1100_fixture()
        np.savez_compressed(os.path.join(HERE, "long_17b_1100.npz"), **g)
        man["models"]["1.7b"] = model_hashes(md)
        man["k1100"] = {"frames": K1100_FRAMES, "prompt": "p128", "seed": 42, "sampling": "default",
                        "speaker": "aiden", "language": "english", "audio_stride": MAX_STRIDE}
    if a.only in (None, "1.7b"):
        g, md = bench_fixtures()
        np.savez_compressed(os.path.join(HERE, "long_17b.npz"), **g)
        man["models"]["1.7b"] = model_hashes(md)
        man["1.7b"] = {"frames": BENCH_FRAMES, "prompt": "p128", "seed": 42, "sampling": "default",
                       "speaker": "aiden", "language": "english"}
    if a.only in (None, "0.6b"):
        g, md = c2_fixtures()
        np.savez_compressed(os.path.join(HERE, "long_06b.npz"), **g)
        man["models"]["0.6b"] = model_hashes(md)
        man["0.6b"] = {"frames": BENCH_FRAMES, "prompt": "p128", "seed": 42, "sampling": "greedy",
                       "speaker": "aiden", "language": "english"}
    if a.only in (None, "b8"):
        g, md = b8_fixtures()
        np.savez_compressed(os.path.join(HERE, "long_17b_b8.npz"), **g)
        man["models"]["1.7b"] = model_hashes(md)
        man["b8"] = {"frames": B8_FRAMES, "prompt": "p128", "prompt_seeds": B8_SEEDS, "seed": 42,
                     "sampling": "default", "speakers": B8_SPEAKERS, "language": "english",
                     "audio_stride": AUDIO_STRIDE}
    if a.only in (None, "b8bench"):
        g, md = b8bench_fixtures()
        np.savez_compressed(os.path.join(HERE, "long_17b_b8bench.npz"), **g)
        man["models"]["1.7b"] = model_hashes(md)
        man["b8bench"] = {"frames": BENCH_FRAMES, "prompt": "p128", "prompt_seeds": B8B_SEEDS, "seed": 42,
                          "sampling": "default", "speakers": ["aiden"] * 8, "language": "english",
                          "audio_stride": AUDIO_STRIDE}
    if a.only in (None, "eos17"):
        g, md = eos17_fixtures(a.slot_dir)
        np.savez_compressed(os.path.join(HERE, "long_eos17.npz"), **g)
        man["models"][f"1.7b_eos_gain{EOS_GAIN}"] = model_hashes(md)
        man["eos17"] = {"eos_gain": EOS_GAIN, "prompt": "p128", "prompt_seeds": EOS_SEEDS, "seed": 42,
                        "sampling": "default", "speakers": EOS_SPEAKERS, "language": "english",
                        "max_tokens": EOS_CAP, "audio_stride": AUDIO_STRIDE}
    if a.only == "eos17q":   # (not in the default set: its three reference runs take ~1 h in parallel)
        g, md = eos17_fixtures(a.slot_dir, utts=(3, 4, 5))
        np.savez_compressed(os.path.join(HERE, "long_eos17q.npz"), **g)
        man["models"][f"1.7b_eos_gain{EOS_GAIN}"] = model_hashes(md)
        man["eos17q"] = {"eos_gain": EOS_GAIN, "prompt": "p128", "prompt_seeds": EOS_Q_SEEDS, "seed": 42,
                         "sampling": "default", "speakers": EOS_Q_SPEAKERS, "language": "english",
                         "max_tokens": EOS_CAP, "audio_stride": AUDIO_STRIDE,
                         "note": "max_tokens is a bound on a run that would not stop; every run stopped well "
                                 "before it, so the codes equal the reference's 4096-token run"}
    if "eos17" in man and "note" not in man["eos17"]:
        man["eos17"]["note"] = ("max_tokens is a bound on a run that would not stop; every run stopped well "
                                "before it, so the codes equal the reference's 4096-token run")
    with open(mpath, "w") as f:
        json.dump(man, f, indent=1)
    for fn in ("long_hd128.npz", "long_hd128_max.npz", "long_hd128_steps4k.npz", "long_17b_1100.npz", "long_17b.npz", "long_06b.npz", "long_17b_b8.npz", "long_17b_b8bench.npz",
               "long_eos17.npz", "long_eos17q.npz", "long_manifest.json"):
        p = os.path.join(HERE, fn)
        if os.path.exists(p):
            print(fn, os.path.getsize(p))


if __name__ == "__main__":
    main()
