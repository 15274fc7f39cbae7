"""The batch-1 talker layer as ONE persistent launch (QTTS_HIP_TENGINE=1|2|3,
k_tengine.hip) against the reference's own outputs.

The engine computes every value with the launch-per-op layer's arithmetic
(k_gemvw rows, its RMS statistic, k_attn_dec's attention and split merge), so
the bar is the same as the default path's: codes bit-exact against the
reference runs of tests/golden/long_17b.npz (the bench workload, 128 frames)
and long_eos17.npz (three EOS-mode utterances to their stop, positions past
the 32-key splits' 8-split preload), waveform MSE < 1e-4.  Positions cover
1..32 splits per kv head (one split per workgroup) and the hand-offs of all
28 layers every frame; a hand-off that times out fails generate (the error
word is read back with the codes).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, model_dir
from parity import codes_equal
from oracle_py import DEFAULT

import qtts

pytestmark = [pytest.mark.gpu]


def _man():
    return json.load(open(os.path.join(GOLDEN, "long_manifest.json")))


def _audio_close(a, ref, what):
    assert a is not None and a.shape == ref.shape, (what, None if a is None else a.shape, ref.shape)
    d = a.astype(np.float64) - ref
    mse, mx = float(np.mean(d * d)), float(np.abs(d).max())
    assert mse < 1e-4 and mx < 1e-3, (what, mse, mx)


def _engine_layers():
    return int(qtts.lib().qtts_hip_tengine_layers())


# 1: the register form (k_tlayer); 2 / 3: the LDS-DMA ring engine with 1 / 2
# weight slots left in flight after each issue (k_tlayer_ring<2> / <3>)
MODES = [m for m in os.environ.get("QTTS_TEST_TENGINE", "2,3").split(",") if m]


@pytest.mark.parametrize("mode", MODES)
def test_tengine_bench_workload_vs_reference(gpu, monkeypatch, mode):
    monkeypatch.setenv("QTTS_HIP_TENGINE", mode)
    g = np.load(os.path.join(GOLDEN, "long_17b.npz"))
    man = _man()["1.7b"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        n0 = _engine_layers()
        a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        # the decode frames ran on the engine (28 layers per captured / enqueued talker pass)
        assert _engine_layers() - n0 >= 28, "the talker layer engine was not selected"
        codes_equal(m.last_codes(), g["codes"], "engine: 1.7B bench workload")
        _audio_close(a, g["audio"], "engine: 1.7B bench workload waveform")
        # a second utterance on the same context: new tags (epoch), same codes
        a2 = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        codes_equal(m.last_codes(), g["codes"], "engine: repeat run")
        assert np.array_equal(a, a2)
    finally:
        m.close()


@pytest.mark.parametrize("mode", MODES)
def test_tengine_eos_batch_1_vs_reference(gpu, monkeypatch, mode):
    monkeypatch.setenv("QTTS_HIP_TENGINE", mode)
    g = np.load(os.path.join(GOLDEN, "long_eos17.npz"))
    man = _man()["eos17"]
    m = qtts.QwenTTS(model_dir("1.7b", eos_gain=man["eos_gain"]))
    n0 = _engine_layers()
    try:
        for b in range(g["prompt_ids"].shape[0]):
            ids = g["prompt_ids"][b, :int(g["prompt_len"][b])]
            n = int(g["stop_step"][b])
            m.set_params(max_tokens=4096, fixed=0, seed=man["seed"], **DEFAULT)
            a = m.generate(ids, man["speakers"][b], man["language"])
            assert m.c.last_stop_reason == 1 and m.c.last_stop_step == n, (b, m.c.last_stop_step, n)
            codes_equal(m.last_codes(), g["codes"][b, :n], f"engine: EOS utterance {b}")
            assert a is not None and len(a) == n * 1920
            sub = a[::man["audio_stride"]]
            _audio_close(sub, g["audio_sub"][b, :len(sub)], f"engine: EOS utterance {b} every 16th sample")
        assert _engine_layers() - n0 >= 28, "the talker layer engine was not selected"
    finally:
        m.close()


@pytest.mark.parametrize("mode", MODES)
def test_tengine_past_1024_keys_vs_reference(gpu, monkeypatch, mode):
    """Positions past 1024 (fixed 1100 frames): the engine's attention runs a
    second round of splits (split j32 + 32) in the workgroups of each kv head,
    with the cache rows loaded inside the loop; codes bit-exact against the
    reference's own run (long_17b_1100.npz)."""
    path = os.path.join(GOLDEN, "long_17b_1100.npz")
    if not os.path.exists(path):
        pytest.skip("long_17b_1100.npz not generated (make_golden_long.py --only k1100)")
    monkeypatch.setenv("QTTS_HIP_TENGINE", mode)
    g = np.load(path)
    man = _man()["k1100"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    n0 = _engine_layers()
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        assert _engine_layers() - n0 >= 28, "the talker layer engine was not selected"
        codes_equal(m.last_codes(), g["codes"], f"engine {mode}: 1.7B 1100-frame decode")
        sub = a[::man["audio_stride"]]
        _audio_close(sub, g["audio_sub"], f"engine {mode}: every 256th sample")
    finally:
        m.close()
