"""Reference audio at other sample rates (CPU only; host C, no GPU).

The Python reference resamples reference audio to 24 kHz with
librosa.resample (qwen_tts/inference/qwen3_tts_model.py:441-444).
qwen_tts_resample implements librosa's res_type="polyphase", which is
scipy.signal.resample_poly; it is pinned to scipy here.  librosa's default
res_type (soxr_hq) is a different filter and is not importable in this image:
parity with it is unpinned.
"""
import numpy as np
import pytest
from scipy.signal import resample_poly

import qtts


@pytest.mark.parametrize("sr_in", [16000, 22050, 44100, 48000, 8000, 24000, 32000])
def test_resample_matches_scipy_resample_poly(sr_in):
    rng = np.random.default_rng(sr_in)
    n = int(sr_in * 0.37) + 11
    x = (rng.standard_normal(n) * 0.3).astype(np.float32)
    x[n // 3: n // 3 + 50] += np.sin(np.arange(50) * 0.2).astype(np.float32)
    g = np.gcd(24000, sr_in)
    want = resample_poly(x.astype(np.float64), 24000 // g, sr_in // g)
    got = qtts.resample(x, sr_in, 24000)
    assert got is not None and got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-6)


def test_resample_edge_lengths():
    for n in (1, 2, 7):
        x = np.linspace(-0.5, 0.5, n).astype(np.float32)
        want = resample_poly(x.astype(np.float64), 3, 2)
        got = qtts.resample(x, 16000, 24000)
        np.testing.assert_allclose(got, want, atol=2e-6)
    assert qtts.resample(np.zeros(0, np.float32), 16000, 24000) is None
