"""Voice-clone encoder oracle (oracle/enc_oracle.py) against the golden
vectors of tests/golden/make_golden_enc.py (transformers' MimiModel and
ECAPA_TimeDelayNet, torch.stft + the slaney mel filterbank) -- CPU only.

Tolerances: both sides are float64, except the golden codebook distances
(float32 torch.cdist, as MimiEuclideanCodebook computes them): codes must be
equal except at near ties (best vs second-best squared distance within 1e-3).
"""
import numpy as np
import pytest

from conftest import golden, model_dir

import enc_oracle as E

G = golden("enc_tiny.npz")


@pytest.fixture(scope="module")
def enc_weights():
    return E.load_encoder_weights(model_dir("tiny_vc"))


def test_mel_filterbank_matches_transformers_slaney():
    np.testing.assert_allclose(E.mel_filterbank(), G["mel_fb"], rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_mel_spectrogram(i):
    w = G[f"wav{i}"]
    mel = E.mel_spectrogram(w)
    assert mel.shape == G[f"mel{i}"].shape == (128, E.mel_frames(w.shape[0]))
    np.testing.assert_allclose(mel, G[f"mel{i}"], atol=2e-5)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_speaker_embedding(enc_weights, i):
    W, scfg, _, _ = enc_weights
    x = E.speaker_embedding(W, scfg, G[f"wav{i}"])
    ref = G[f"xvec{i}"].astype(np.float64)
    assert x.shape == ref.shape == (scfg["enc_dim"],)
    np.testing.assert_allclose(x, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


def test_mimi_encode_batch_and_single(enc_weights):
    _, _, M, mcfg = enc_weights
    outs = E.encode_batch(M, mcfg, [G["wav0"], G["wav1"]])
    outs.append(E.mimi_encode(M, mcfg, G["wav2"], return_latent=False))
    tags = ["b0", "b1", "s0"]
    for (codes, margins), tag, w in zip(outs, tags, [G["wav0"], G["wav1"], G["wav2"]]):
        ref = G[f"codes_{tag}"]
        assert codes.shape == ref.shape == (-(-w.shape[0] // 1920), 16)
        excused, bad = E.compare_codes(codes, ref, margins, 1e-3)
        assert not bad, (tag, bad)
        assert excused <= max(1, codes.shape[0] // 10), (tag, excused)


def test_mimi_latent(enc_weights):
    _, _, M, mcfg = enc_weights
    n = max(G["wav0"].shape[0], G["wav1"].shape[0])
    for b, key in enumerate(["wav0", "wav1"]):
        w = np.zeros(n)
        w[:G[key].shape[0]] = G[key]
        _, _, lat = E.mimi_encode(M, mcfg, w, n_keep=G[key].shape[0], return_latent=True)
        ref = G[f"latent_b{b}"]
        np.testing.assert_allclose(lat, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


def test_mimi_frames_formula():
    for n in (1, 1919, 1920, 1921, 48000, 120000, 29630):
        assert E.mimi_frames(n) == -(-n // 1920)
