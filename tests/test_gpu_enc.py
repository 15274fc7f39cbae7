"""Voice-clone audio encoders on the GPU against the golden
vectors (tests/golden/make_golden_enc.py: transformers' MimiModel and
ECAPA_TimeDelayNet) and the float64 oracle (oracle/enc_oracle.py).

Tolerances (the device computes fp32-exact products with fp32 accumulation):
  mel          |d| <= 1e-4 (log domain)
  x-vector     |d| <= 2e-4 * max|x|
  latent       |d| <= 2e-4 * max|latent|
  codes        equal, except a frame's first differing codebook may be a near
               tie: oracle best vs second-best squared distance within
               1e-3 * (1 + best distance) (MimiModel itself decides these in
               float32 torch.cdist, modeling_mimi.py:985-990)
"""
import numpy as np
import pytest

from conftest import golden, model_dir

import enc_oracle as E

pytestmark = pytest.mark.gpu
G = golden("enc_tiny.npz")


@pytest.fixture(scope="module")
def tts_vc(gpu):
    import qtts
    m = qtts.QwenTTS(model_dir("tiny_vc"))
    assert m.encoders_available() == 3
    yield m
    m.close()


@pytest.fixture(scope="module")
def enc_w():
    return E.load_encoder_weights(model_dir("tiny_vc"))


def _check_codes(codes, ref, margins, best):
    tol = 1e-3 * (1.0 + best)
    excused, bad = 0, []
    for f in range(codes.shape[0]):
        d = np.nonzero(codes[f] != ref[f])[0]
        if d.size == 0:
            continue
        q = int(d[0])
        if margins[f, q] <= tol[f, q]:
            excused += 1
        else:
            bad.append((f, q, float(margins[f, q])))
    assert not bad, bad
    assert excused <= max(1, codes.shape[0] // 10), excused


def test_speaker_embedding_vs_golden(tts_vc):
    wavs = [G[f"wav{i}"] for i in range(3)]
    xv, mels = tts_vc.speaker_embed(wavs, mel=True)
    for i in range(3):
        np.testing.assert_allclose(mels[i], G[f"mel{i}"], atol=1e-4)
        ref = G[f"xvec{i}"]
        np.testing.assert_allclose(xv[i], ref, atol=2e-4 * np.abs(ref).max())


def test_speaker_embedding_batch_equals_single(tts_vc):
    """Each utterance of a ragged batch runs at its own length: equal to its
    single run up to the split-K order of the padded length (1e-5 relative)."""
    wavs = [G[f"wav{i}"] for i in range(3)]
    xb = tts_vc.speaker_embed(wavs)
    for i in range(3):
        np.testing.assert_allclose(tts_vc.speaker_embed([wavs[i]])[0], xb[i], rtol=1e-5,
                                   atol=1e-5 * np.abs(xb[i]).max())
    np.testing.assert_array_equal(tts_vc.speaker_embed([wavs[0]])[0], xb[0])   # the longest: same padding
    api = tts_vc.speaker_embedding_api(wavs[1])
    np.testing.assert_array_equal(api, xb[1])


def test_speaker_embedding_vs_oracle_long(tts_vc, enc_w):
    W, scfg, _, _ = enc_w
    rng = np.random.default_rng(7)
    w = (0.2 * rng.standard_normal(24000 * 5 + 123)).astype(np.float32)   # 5 s, ragged
    ref = E.speaker_embedding(W, scfg, w)
    got = tts_vc.speaker_embed([w])[0]
    np.testing.assert_allclose(got, ref, atol=2e-4 * np.abs(ref).max())


def test_speaker_embedding_rejects_short(tts_vc):
    assert tts_vc.speaker_embedding_api(np.zeros(300, np.float32)) is None


def test_encode_audio_vs_golden(tts_vc, enc_w):
    _, _, M, mcfg = enc_w
    w0, w1 = G["wav0"], G["wav1"]
    codes, lats = tts_vc.encode_audio([w0, w1], latent=True)
    n = max(w0.shape[0], w1.shape[0])
    for b, w in enumerate([w0, w1]):
        ref_lat = G[f"latent_b{b}"]
        np.testing.assert_allclose(lats[b], ref_lat, atol=2e-4 * np.abs(ref_lat).max())
        wp = np.zeros(n)
        wp[:w.shape[0]] = w
        oc, om = E.mimi_encode(M, mcfg, wp, n_keep=w.shape[0])
        best = _best_dist(M, mcfg, wp, w.shape[0])
        _check_codes(codes[b], G[f"codes_b{b}"], om, best)
        _check_codes(codes[b], oc, om, best)
    c2 = tts_vc.encode_audio([G["wav2"]])[0]
    oc, om = E.mimi_encode(M, mcfg, G["wav2"])
    _check_codes(c2, G["codes_s0"], om, _best_dist(M, mcfg, G["wav2"], G["wav2"].shape[0]))


def _best_dist(M, mcfg, wav, n_keep):
    """oracle best squared distance per (frame, codebook) (tolerance scale)."""
    _, _, lat = E.mimi_encode(M, mcfg, wav, n_keep=n_keep, return_latent=True)
    out = []
    for pre, n_q in (("quantizer.semantic_residual_vector_quantizer.", 1),
                     ("quantizer.acoustic_residual_vector_quantizer.", 15)):
        r = E.conv1d(lat, M[pre + "input_proj.weight"]).T
        for qi in range(n_q):
            e = E.codebook(M, f"{pre}layers.{qi}.")
            d = (r * r).sum(1)[:, None] - 2.0 * r @ e.T + (e * e).sum(1)[None, :]
            idx = d.argmin(1)
            out.append(d[np.arange(d.shape[0]), idx])
            r = r - e[idx]
    return np.stack(out).T


@pytest.mark.parametrize("n", [1, 1919, 1920, 1921, 3840 + 7])
def test_encode_audio_edge_lengths(tts_vc, enc_w, n):
    _, _, M, mcfg = enc_w
    rng = np.random.default_rng(n)
    w = (0.3 * rng.standard_normal(n)).astype(np.float32)
    c = tts_vc.encode_audio_api(w)
    assert c is not None and c.shape == (-(-n // 1920), 16)
    assert ((c >= 0) & (c < 2048)).all()
    oc, om = E.mimi_encode(M, mcfg, w)
    _check_codes(c, oc, om, _best_dist(M, mcfg, w, n))


def test_encode_batch_padding_semantics(tts_vc):
    """A batch is zero-padded to its longest member (the tokenizer's batch
    encode): each member equals its own encode on the same padded waveform."""
    w0, w1 = G["wav0"], G["wav1"]
    cb = tts_vc.encode_audio([w0, w1])
    wp = np.zeros(w0.shape[0], np.float32)
    wp[:w1.shape[0]] = w1
    c1 = tts_vc.encode_audio([wp])[0][:cb[1].shape[0]]
    np.testing.assert_array_equal(cb[1], c1)
    np.testing.assert_array_equal(cb[0], tts_vc.encode_audio([w0])[0])


def test_voice_clone_from_audio_equals_codes_path(tts_vc):
    """qwen_tts_generate_voice_clone_audio == encode + x-vector + the codes
    voice clone (ICL and x-vector-only modes)."""
    from oracle_py import GREEDY
    from synth_model import prompt_ids
    tts_vc.set_params(max_tokens=4096, fixed=6, seed=42, **GREEDY)
    ids = prompt_ids("short")
    ref_ids = [151644, 77091, 198, 2354, 2244, 151645, 198]
    w = G["wav0"]
    a = tts_vc.generate_voice_clone_audio(ids, w, ref_ids=ref_ids, language="english")
    codes = tts_vc.encode_audio([w])[0]
    xv = tts_vc.speaker_embed([w])[0]
    b = tts_vc.generate_voice_clone(ids, ref_ids=ref_ids, ref_codes=codes, spk_embed=xv, language="english")
    assert a is not None and b is not None
    np.testing.assert_array_equal(a, b)
    ax = tts_vc.generate_voice_clone_audio(ids, w, language="english", x_vector_only=True)
    bx = tts_vc.generate_voice_clone(ids, spk_embed=xv, language="english")
    np.testing.assert_array_equal(ax, bx)


def test_voice_clone_audio_stream_equals_codes_stream(tts_vc):
    """qwen_tts_generate_voice_clone_audio_stream == encode + the codes stream."""
    from oracle_py import GREEDY
    from synth_model import prompt_ids
    tts_vc.set_params(max_tokens=4096, fixed=6, seed=42, **GREEDY)
    ids = prompt_ids("short")
    ref_ids = [151644, 77091, 198, 2354, 2244, 151645, 198]
    w = G["wav1"]
    chunks = []
    a = tts_vc.generate_voice_clone_audio_stream(ids, w, ref_ids=ref_ids, language="english", chunk_frames=2,
                                                 on_chunk=chunks.append)
    codes = tts_vc.encode_audio([w])[0]
    xv = tts_vc.speaker_embed([w])[0]
    b = tts_vc.generate_voice_clone_stream(ids, ref_ids=ref_ids, ref_codes=codes, spk_embed=xv, language="english",
                                           chunk_frames=2)
    assert a is not None and chunks
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(np.concatenate(chunks), a)
    assert tts_vc.c.perf_first_packet_ms > 0


def test_voice_clone_audio_batch_equals_singles(tts_vc):
    from oracle_py import GREEDY
    from synth_model import prompt_ids
    tts_vc.set_params(max_tokens=4096, fixed=5, seed=42, **GREEDY)
    ids = [prompt_ids("short"), prompt_ids("p128", seed=1235)]
    ref_ids = [[151644, 77091, 198, 2354, 151645, 198], [151644, 77091, 198, 4041, 2244, 151645, 198]]
    wavs = [G["wav0"], G["wav1"]]
    rc, outs = tts_vc.generate_voice_clone_audio_batch(ids, wavs, ref_id_lists=ref_ids, languages=["english"] * 2)
    assert rc == 0
    codes = tts_vc.encode_audio(wavs)          # the same padded batch encode
    xv = tts_vc.speaker_embed(wavs)
    rc2, ref = tts_vc.generate_voice_clone_batch(ids, ref_ids, codes, spk_embeds=list(xv), languages=["english"] * 2)
    assert rc2 == 0
    for a, b in zip(outs, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.slow
def test_full_size_encoders_vs_oracle(gpu):
    """1.7B model dir (reference-default encoder sizes: ECAPA 512/1536,
    Mimi hidden 512, 8 layers, window 250): a 5.2 s reference."""
    import qtts
    md = model_dir("1.7b")
    W, scfg, M, mcfg = E.load_encoder_weights(md)
    rng = np.random.default_rng(3)
    t = np.arange(int(24000 * 5.2)) / 24000.0
    w = (0.3 * np.sin(2 * np.pi * 220 * t) + 0.05 * rng.standard_normal(t.shape[0])).astype(np.float32)
    m = qtts.QwenTTS(md)
    try:
        assert m.encoders_available() == 3
        xv = m.speaker_embed([w])[0]
        codes, lats = m.encode_audio([w], latent=True)
    finally:
        m.close()
    ref = E.speaker_embedding(W, scfg, w)
    np.testing.assert_allclose(xv, ref, atol=2e-4 * np.abs(ref).max())
    oc, om, ol = E.mimi_encode(M, mcfg, w, return_latent=True)
    np.testing.assert_allclose(lats[0], ol, atol=2e-4 * np.abs(ol).max())
    _check_codes(codes[0], oc, om, _best_dist(M, mcfg, w, w.shape[0]))
