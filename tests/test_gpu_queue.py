"""Work queue: utterances of EOS-variable length on a live
lock-step batch, each freed slot refilled with the next queued utterance
(`qwen_tts_generate_queue`, `qtts_dev_refill`).

The bar is the reference's own: every utterance's codes and stop step equal
its single run -- the reference decodes one utterance per call
(Q.c:1059-1443) and stops it at its own EOS (Q.c:1323-1330) or at
max_new_tokens -- whatever slot it lands in and whatever the other slots do.

* tiny EOS model (the stage goldens' model, codec-head EOS x3): 10 prompts on
  3 slots against the oracle's single runs (EOS stops and the max_new_tokens
  cap mixed), in order and in a caller-chosen admission order;
* tiny, fixed length: 7 prompts on 3 slots (every slot retired by the host
  count and refilled on the same frame);
* synthetic 1.7B, the reference's own runs: long_eos17 (EOS stops at
  157 / 395 / 218) on 2 slots, long_eos17 + long_eos17q (6 EOS utterances) on 3
  slots, and C4's 8-utterance golden (32 fixed frames) on 3 slots.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, manifest, model_dir
from parity import codes_equal
from oracle_py import DEFAULT, Oracle
from qtts_io import lookup_ids
from synth_model import prompt_ids

import qtts

pytestmark = pytest.mark.gpu


def _codes_equal(got, want, what, ctx=None):
    codes_equal(got, want, what, ctx)


def _audio_close(a, ref, what, mse_bar=1e-4, max_bar=1e-3):
    assert a is not None and a.shape == ref.shape, (what, None if a is None else a.shape, ref.shape)
    d = a.astype(np.float64) - ref
    mse, mx = float(np.mean(d * d)), float(np.abs(d).max())
    assert mse < mse_bar and mx < max_bar, (what, mse, mx)


def _tiny_prompts():
    return [prompt_ids("short"), prompt_ids("p128", 1300), prompt_ids("p128", 1301), prompt_ids("short")] + \
        [prompt_ids("p128", 1310 + i) for i in range(6)]


@pytest.fixture(scope="module")
def tiny_eos():
    md = model_dir("tiny", eos_gain=manifest()["eos_gain"])
    m = qtts.QwenTTS(md)
    o = Oracle(md)
    yield m, o
    m.close()
    o.close()


_ORC = {}


def _single(o, ids, max_tokens, fixed, seed):
    """the oracle's single run of one utterance (codes, stop reason 1 eos / 2
    max_tokens, waveform), cached"""
    key = (tuple(int(i) for i in ids), max_tokens, fixed, seed)
    if key not in _ORC:
        s, l = lookup_ids(o.cfg, "aiden", "english")
        want, stop = o.generate_codes(ids, s, l, max_tokens=max_tokens, fixed=fixed, seed=seed, **DEFAULT)
        _ORC[key] = (want, stop, o.codec_decode(want))
    return _ORC[key]


def _tiny_check(m, o, prompts, audio, max_tokens, fixed, seed):
    st = m.queue_stats()
    for i, ids in enumerate(prompts):
        want, stop, wav = _single(o, ids, max_tokens, fixed, seed)
        s, l = lookup_ids(o.cfg, "aiden", "english")
        ctx = dict(oracle=o, ids=ids, spk=s, lang=l,
                   params=dict(max_tokens=max_tokens, fixed=fixed, seed=seed, **DEFAULT))
        _codes_equal(m.queue_codes(i), want, f"utterance {i} (slot {st['slot'][i]})", ctx)
        assert st["stop_reason"][i] == stop, (i, st["stop_reason"][i], stop)   # 1 eos, 2 max_tokens
        _audio_close(audio[i], wav, f"utterance {i} audio")


def test_queue_tiny_eos_refill_matches_single_runs(tiny_eos):
    """10 EOS-mode utterances on 3 slots: each freed slot takes the next one
    inside the live batch; every utterance equals its single oracle run
    (codes bit-exact, stop reason, audio), EOS stops and the cap mixed."""
    m, o = tiny_eos
    prompts = _tiny_prompts()
    m.set_params(max_tokens=32, fixed=0, seed=7, **DEFAULT)
    rc, audio = m.generate_queue(prompts, ["aiden"] * 10, ["english"] * 10, slots=3)
    assert rc == 0
    st = m.queue_stats()
    assert st["slots"] == 3 and st["refills"] == 7, st
    assert st["used"] == sum(st["frames_per_utt"]), st
    # the set mixes EOS stops (5 to 17 frames) and the max_new_tokens cap (utterance 9)
    assert set(st["stop_reason"]) == {1, 2}, st
    # the tail ran compacted (fewer rows than slots x frames)
    assert st["rows_launched"] < 3 * st["frames"], st
    _tiny_check(m, o, prompts, audio, 32, 0, 7)


def test_queue_tiny_admission_order_and_plain_batch(tiny_eos):
    """A caller-chosen admission order (the cross-GPU counter's hook) gives
    every utterance the same codes; nq == slots is the plain lock-step batch."""
    m, o = tiny_eos
    prompts = _tiny_prompts()
    m.set_params(max_tokens=32, fixed=0, seed=7, **DEFAULT)
    order = iter([9, 2, 7, 0, 5, 1, 8, 3, 6, 4])
    rc, audio = m.generate_queue(prompts, ["aiden"] * 10, ["english"] * 10, slots=4,
                                 next_fn=lambda: next(order, -1))
    assert rc == 0
    assert m.queue_stats()["slot"][9] == 0 and m.queue_stats()["slot"][2] == 1
    _tiny_check(m, o, prompts, audio, 32, 0, 7)
    rc, qa = m.generate_queue(prompts[:4], ["aiden"] * 4, ["english"] * 4, slots=4)
    assert rc == 0 and m.queue_stats()["refills"] == 0
    rc, ba = m.generate_batch(prompts[:4], ["aiden"] * 4, ["english"] * 4)
    assert rc == 0
    for b in range(4):
        np.testing.assert_array_equal(qa[b], ba[b])


def test_queue_tiny_partial_take(tiny_eos):
    """next_fn handing this ctx only some utterances (another GPU takes the
    rest): the others come back as None and their codes as absent."""
    m, o = tiny_eos
    prompts = _tiny_prompts()[:6]
    m.set_params(max_tokens=32, fixed=0, seed=7, **DEFAULT)
    order = iter([1, 3, 5])
    rc, audio = m.generate_queue(prompts, ["aiden"] * 6, ["english"] * 6, slots=2, next_fn=lambda: next(order, -1))
    assert rc == 0
    for i in range(6):
        if i % 2 == 0:
            assert audio[i] is None and m.queue_codes(i) is None
        else:
            _codes_equal(m.queue_codes(i), _single(o, prompts[i], 32, 0, 7)[0], f"utterance {i}")


def test_queue_tiny_fixed_length(tiny_eos):
    """Fixed-length mode (no EOS stop; the EOS re-draw below the length,
    Q.c:1315-1321): every slot is retired by the host's frame count and
    refilled on the same frame."""
    m, o = tiny_eos
    prompts = _tiny_prompts()[:7]
    m.set_params(max_tokens=4096, fixed=8, seed=42, **DEFAULT)
    rc, audio = m.generate_queue(prompts, ["aiden"] * 7, ["english"] * 7, slots=3)
    assert rc == 0
    st = m.queue_stats()
    assert st["frames_per_utt"] == [8] * 7 and st["refills"] == 4, st
    _tiny_check(m, o, prompts, audio, 4096, 8, 42)


def _man():
    return json.load(open(os.path.join(GOLDEN, "long_manifest.json")))


def _prompts(g):
    return [g["prompt_ids"][b, :int(g["prompt_len"][b])] for b in range(g["prompt_ids"].shape[0])]


def _eos_check(m, audio, g, man, i, u, what):
    n = int(g["stop_step"][u])
    st = m.queue_stats()
    assert st["stop_reason"][i] == 1 and st["frames_per_utt"][i] == n, (what, i, st["stop_reason"][i],
                                                                         st["frames_per_utt"][i], n)
    _codes_equal(m.queue_codes(i), g["codes"][u, :n], f"{what}: utterance {i} (slot {st['slot'][i]})")
    a = audio[i]
    assert a is not None and len(a) == n * 1920, (what, i)
    _audio_close(a[::man["audio_stride"]], g["audio_sub"][u, :len(a[::man["audio_stride"]])],
                 f"{what}: utterance {i} every 16th sample")


@pytest.mark.parametrize("compact", ["1", "0"])
def test_queue_eos17_two_slots_vs_reference(gpu, monkeypatch, compact):
    """The reference's three full-size EOS utterances (stops 157 / 395 / 218)
    on 2 slots: the third starts in the slot the first frees at its step 157,
    inside the live batch; once it stops, nothing is left to admit, so the
    second utterance's state moves to slot 0 and its last frames run as a
    batch of one (QTTS_QUEUE_COMPACT=0: on its own slot in the batch of 2).
    Every utterance's stop step and codes equal its own reference run."""
    monkeypatch.setenv("QTTS_QUEUE_COMPACT", compact)
    g = np.load(os.path.join(GOLDEN, "long_eos17.npz"))
    man = _man()["eos17"]
    m = qtts.QwenTTS(model_dir("1.7b", eos_gain=man["eos_gain"]))
    try:
        m.set_params(max_tokens=4096, fixed=0, seed=man["seed"], **DEFAULT)
        prompts = _prompts(g)
        rc, audio = m.generate_queue(prompts, man["speakers"], [man["language"]] * 3, slots=2)
        assert rc == 0
        st = m.queue_stats()
        assert st["refills"] == 1 and st["slot"][2] == 0, st
        # (compacted: utterance 1 finishes on slot 0, its tail frames one row each)
        assert st["slot"][1] == (0 if compact == "1" else 1), st
        assert (st["rows_launched"] < 2 * st["frames"]) == (compact == "1"), st
        for i in range(3):
            _eos_check(m, audio, g, man, i, i, "eos17 on 2 slots")
    finally:
        m.close()


def test_queue_eos17_six_on_three_slots_vs_reference(gpu):
    """Six full-size EOS utterances (long_eos17 + long_eos17q, each one
    reference run) on 3 slots: three refills, each utterance's stop step and
    codes equal its own reference run; occupancy beats the lock-step batch's."""
    ga = np.load(os.path.join(GOLDEN, "long_eos17.npz"))
    gb = np.load(os.path.join(GOLDEN, "long_eos17q.npz"))
    man = _man()
    ma, mb = man["eos17"], man["eos17q"]
    m = qtts.QwenTTS(model_dir("1.7b", eos_gain=ma["eos_gain"]))
    try:
        m.set_params(max_tokens=4096, fixed=0, seed=ma["seed"], **DEFAULT)
        prompts = _prompts(ga) + _prompts(gb)
        spk = ma["speakers"] + mb["speakers"]
        rc, audio = m.generate_queue(prompts, spk, ["english"] * 6, slots=3)
        assert rc == 0
        st = m.queue_stats()
        assert st["refills"] == 3, st
        for i in range(6):
            g, u = (ga, i) if i < 3 else (gb, i - 3)
            _eos_check(m, audio, g, ma, i, u, "6 EOS utterances on 3 slots")
        stops = [int(x) for x in ga["stop_step"]] + [int(x) for x in gb["stop_step"]]
        lockstep = sum(stops) / (3.0 * (max(stops[:3]) + max(stops[3:])))   # two lock-step batches of 3
        assert st["occupancy"] > lockstep, (st, lockstep)
    finally:
        m.close()


@pytest.mark.slow
def test_queue_c4_fixed_32_on_three_slots_vs_reference(gpu):
    """C4's 8 reference utterances (32 fixed frames each) on 3 slots: each
    slot retired by the host count and refilled twice or thrice; every
    utterance's 32 x 16 codes bit-exact against its reference run."""
    g = np.load(os.path.join(GOLDEN, "long_17b_b8.npz"))
    man = _man()["b8"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=4096, fixed=man["frames"], seed=man["seed"], **DEFAULT)
        rc, audio = m.generate_queue(_prompts(g), man["speakers"], [man["language"]] * 8, slots=3)
        assert rc == 0
        assert m.queue_stats()["refills"] == 5
        for i in range(8):
            _codes_equal(m.queue_codes(i), g["codes"][i], f"C4 queue utterance {i}")
            _audio_close(audio[i][::man["audio_stride"]], g["audio_sub"][i], f"utterance {i} every 16th sample")
    finally:
        m.close()
