"""Full-size (synthetic 1.7B; 0.6B for BASELINE.json configs[1]) parity and
size-independent properties on the GPU.

At full size the oracle is slow on the CPU, so it checks a short greedy
prefix (3 frames: talker prefill over the P128 prompt, 3 decode steps, 3
sub-talker passes; greedy and default sampling) and a 4-frame codec decode; the 128-frame benchmark
workload is checked through properties: determinism, identical slots for
identical inputs in a lock-step batch, code ranges, waveform length and range.
"""
import numpy as np
import pytest

from conftest import model_dir
from oracle_py import GREEDY, DEFAULT, Oracle
from qtts_io import lookup_ids
from synth_model import prompt_ids

import qtts

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def full_dir():
    return model_dir("1.7b")


@pytest.fixture(scope="module")
def full_tts(gpu, full_dir):
    m = qtts.QwenTTS(full_dir)
    yield m
    m.close()


def test_full_greedy_prefix_and_codec_vs_oracle(full_tts, full_dir):
    ids = prompt_ids("p128")
    o = Oracle(full_dir)
    try:
        s, l = lookup_ids(o.cfg, "aiden", "english")
        for pp in (GREEDY, DEFAULT):   # greedy, then the default sampling (top-k 50 / 0.9 / 1.05)
            codes_o, _ = o.generate_codes(ids, s, l, max_tokens=4096, fixed=3, seed=42, **pp)
            full_tts.set_params(max_tokens=4096, fixed=3, seed=42, **pp)
            full_tts.generate(ids, "aiden", "english")
            np.testing.assert_array_equal(full_tts.last_codes(), codes_o)
        rng = np.random.default_rng(0)
        codes = rng.integers(0, 2048, size=(4, 16)).astype(np.int32)
        a = full_tts.codec_decode(codes)
        r = o.codec_decode(codes)
        assert a.shape == r.shape
        assert float(np.mean((a.astype(np.float64) - r) ** 2)) < 1e-4
        assert np.abs(a - r).max() < 1e-3
    finally:
        o.close()


def test_full_bench_workload_properties(full_tts):
    """The bench workload (P128, fixed 128 frames, default sampling)."""
    ids = prompt_ids("p128")
    full_tts.set_params(max_tokens=128, fixed=128, seed=42, **DEFAULT)
    a1 = full_tts.generate(ids, "aiden", "english")
    c1 = full_tts.last_codes()
    a2 = full_tts.generate(ids, "aiden", "english")
    c2 = full_tts.last_codes()
    assert c1.shape == (128, 16)
    np.testing.assert_array_equal(c1, c2)                     # deterministic
    np.testing.assert_array_equal(a1, a2)
    assert c1.min() >= 0 and c1[:, 0].max() < 2048 and c1[:, 1:].max() < 2048
    assert a1.shape == (128 * 1920,) and np.isfinite(a1).all() and np.abs(a1).max() <= 1.0


def test_full_batch_identical_slots(full_tts):
    ids = prompt_ids("p128", 1300)
    full_tts.set_params(max_tokens=32, fixed=32, seed=5, **DEFAULT)
    rc, audio = full_tts.generate_batch([ids, prompt_ids("p128", 1301), ids], ["aiden"] * 3, ["english"] * 3)
    assert rc == 0
    np.testing.assert_array_equal(audio[0], audio[2])
    assert not np.array_equal(audio[0], audio[1])
    assert all(len(x) == 32 * 1920 for x in audio)


def test_06b_greedy_prefix_vs_oracle(gpu):
    """BASELINE.json configs[1] (0.6B, batch 1, greedy, P128): a 3-frame
    prefix bit-exact against the oracle (no sub-talker input projection:
    H == H_s)."""
    md = model_dir("0.6b")
    ids = prompt_ids("p128")
    o = Oracle(md)
    m = qtts.QwenTTS(md)
    try:
        s, l = lookup_ids(o.cfg, "aiden", "english")
        codes_o, _ = o.generate_codes(ids, s, l, max_tokens=4096, fixed=3, seed=42, **GREEDY)
        m.set_params(max_tokens=4096, fixed=3, seed=42, **GREEDY)
        m.generate(ids, "aiden", "english")
        np.testing.assert_array_equal(m.last_codes(), codes_o)
    finally:
        m.close()
        o.close()
