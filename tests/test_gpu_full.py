"""Full-size (synthetic 1.7B; 0.6B for BASELINE.json configs[1]) parity and
size-independent properties on the GPU.

Against the oracle (oracle/qtts_oracle.c, pinned to the reference c/ build):
  * a 3-frame greedy / default-sampling prefix and a 12-frame default-sampling
    decode (the per-occurrence repetition penalty bites, KV grows past the
    prompt), codes bit-exact;
  * codec decode at T = 4 and T = 128 (the 72-frame window and every real
    vocoder width; waveform MSE < 1e-4, max |d| < 1e-3);
  * BASELINE C3: the streamed chunks of a 1.7B utterance equal its
    non-streamed waveform, and the first packet (frame 0 through the exact
    streaming codec) equals the oracle's decode of that frame;
  * BASELINE C4 per-GPU shape: 8 utterances in lock step (split-K O / down
    projections), every slot bit-exact against its own oracle run;
  * BASELINE C5: 8 voice-clone slots (ICL prompts of 20-34 reference frames +
    x-vectors: the prefill GEMM over > 64 rows), every slot against the
    oracle's ICL layout (parity of that layout itself is unpinned, see
    tests/test_voice_clone.py).
The 128-frame benchmark workload is also checked through properties:
determinism, identical slots for identical inputs in a lock-step batch, code
ranges, waveform length and range.
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


def _audio_close(a, ref, mse_bar=1e-4, max_bar=1e-3):
    assert a is not None and a.shape == ref.shape, (None if a is None else a.shape, ref.shape)
    d = a.astype(np.float64) - ref
    assert float(np.mean(d * d)) < mse_bar, float(np.mean(d * d))
    assert np.abs(d).max() < max_bar, np.abs(d).max()


@pytest.fixture(scope="module")
def full_oracle(full_dir):
    o = Oracle(full_dir)
    yield o
    o.close()


def test_full_default_12_frames_vs_oracle(full_tts, full_oracle):
    """12 frames under the default sampling: repeated group-0 ids are
    penalised once per occurrence (K.c:395-405), KV grows 12 rows past the
    prompt; codes bit-exact."""
    ids = prompt_ids("p128", 1277)
    s, l = lookup_ids(full_oracle.cfg, "aiden", "english")
    codes_o, _ = full_oracle.generate_codes(ids, s, l, max_tokens=4096, fixed=12, seed=42, **DEFAULT)
    full_tts.set_params(max_tokens=4096, fixed=12, seed=42, **DEFAULT)
    a = full_tts.generate(ids, "aiden", "english")
    np.testing.assert_array_equal(full_tts.last_codes(), codes_o)
    _audio_close(a, full_oracle.codec_decode(codes_o))


def test_full_codec_128_vs_oracle(full_tts, full_oracle):
    """The bench's 128-frame codec decode at real widths (1536-channel
    vocoder, hidden 1024, the 72-frame attention window crossed)."""
    codes = np.random.default_rng(128).integers(0, 2048, size=(128, 16)).astype(np.int32)
    _audio_close(full_tts.codec_decode(codes), full_oracle.codec_decode(codes))


def test_full_stream_c3(full_tts, full_oracle):
    """BASELINE C3 (1.7B, batch 1, streaming): chunks concatenate to the
    non-streamed utterance; the first packet is frame 0 alone through the
    exact streaming codec = the oracle's decode of frame 0."""
    ids = prompt_ids("p128", 1278)
    full_tts.set_params(max_tokens=4096, fixed=16, seed=42, **DEFAULT)
    chunks = []
    a = full_tts.generate_stream(ids, "aiden", "english", chunk_frames=8, on_chunk=chunks.append)
    codes = full_tts.last_codes()
    assert a is not None and len(chunks) >= 2 and len(chunks[0]) == 1920
    np.testing.assert_array_equal(np.concatenate(chunks), a)
    b = full_tts.generate(ids, "aiden", "english")
    np.testing.assert_array_equal(full_tts.last_codes(), codes)
    _audio_close(a, b)
    _audio_close(chunks[0], full_oracle.codec_decode(codes[:1]))
    s, l = lookup_ids(full_oracle.cfg, "aiden", "english")
    codes_o, _ = full_oracle.generate_codes(ids, s, l, max_tokens=4096, fixed=16, seed=42, **DEFAULT)
    np.testing.assert_array_equal(codes, codes_o)


def test_full_batch8_vs_oracle_c4(full_tts, full_oracle):
    """BASELINE C4's per-GPU shape: 8 utterances in lock step (the batch GEMV
    on the matrix cores, O / down projections split over K); every slot's
    3 frames bit-exact against its own single oracle run."""
    prompts = [prompt_ids("p128", 1400 + i) for i in range(8)]
    spk = ["aiden", "vivian", "serena", "aiden", "vivian", "serena", "aiden", "vivian"]
    full_tts.set_params(max_tokens=4096, fixed=3, seed=42, **DEFAULT)
    rc, audio = full_tts.generate_batch(prompts, spk, ["english"] * 8)
    assert rc == 0
    for b in range(8):
        s, l = lookup_ids(full_oracle.cfg, spk[b], "english")
        codes_o, _ = full_oracle.generate_codes(prompts[b], s, l, max_tokens=4096, fixed=3, seed=42, **DEFAULT)
        _audio_close(audio[b], full_oracle.codec_decode(codes_o))


def test_full_batch12_self_reducing_split_k(full_tts, full_oracle):
    """12 utterances in lock step (above 8 rows the O / down split-K producer
    reduces its own partials): 3 distinct prompts x 4; the distinct slots
    against their oracle runs, the repeats bit-equal to them."""
    prompts = [prompt_ids("p128", 1450 + i % 3) for i in range(12)]
    spk = ["aiden", "vivian", "serena"] * 4
    full_tts.set_params(max_tokens=4096, fixed=3, seed=42, **DEFAULT)
    rc, audio = full_tts.generate_batch(prompts, spk, ["english"] * 12)
    assert rc == 0
    for b in range(3):
        s, l = lookup_ids(full_oracle.cfg, spk[b], "english")
        codes_o, _ = full_oracle.generate_codes(prompts[b], s, l, max_tokens=4096, fixed=3, seed=42, **DEFAULT)
        _audio_close(audio[b], full_oracle.codec_decode(codes_o))
    for b in range(3, 12):
        np.testing.assert_array_equal(audio[b], audio[b % 3])


def test_full_batch_codec_lanes_bit_identical(full_tts, full_oracle, monkeypatch):
    """A batch's codec passes side by side (qtts_dev_codec_multi, lane k
    decodes slots k, k + lanes, ...): 1, 3 and 8 lanes give the same audio bit
    for bit, each slot the lone decode of its own codes (qwen_tts_codec_decode)
    and the oracle's decode (slots of different lengths side by side:
    test_batch_eos_slots_stop_independently)."""
    prompts = [prompt_ids("p128", 1500 + i) for i in range(8)]
    full_tts.set_params(max_tokens=4096, fixed=24, seed=42, **DEFAULT)
    runs = {}
    for lanes in ("1", "3", "8"):
        monkeypatch.setenv("QTTS_HIP_CODEC_LANES", lanes)
        rc, audio = full_tts.generate_batch(prompts, ["aiden"] * 8, ["english"] * 8)
        assert rc == 0 and all(len(a) == 24 * 1920 for a in audio)
        runs[lanes] = audio
    for b in range(8):
        np.testing.assert_array_equal(runs["3"][b], runs["1"][b])
        np.testing.assert_array_equal(runs["8"][b], runs["1"][b])
    codes = full_tts.last_codes_batch(8)
    for b in (0, 5):
        np.testing.assert_array_equal(full_tts.codec_decode(codes[b]), runs["8"][b])
    _audio_close(runs["8"][7], full_oracle.codec_decode(codes[7]))


def test_full_voice_clone_b8_vs_oracle_c5(full_tts, full_oracle):
    """BASELINE C5 (1.7B voice clone, batch 8): ICL prompts of 20-34
    reference frames + x-vectors (> 64 prefill rows: the matrix-core
    prefill GEMM); every slot's 3 generated frames and audio against the
    oracle's ICL prompt (orc_build_icl_prompt)."""
    cfg = full_oracle.cfg
    _, lang = lookup_ids(cfg, "aiden", "english")
    prompts, rids, refs, spks = [], [], [], []
    for i in range(8):
        r = np.random.default_rng(500 + i)
        prompts.append(prompt_ids("p128", 1500 + i))
        rids.append([151644, 77091, 198] + r.integers(1000, 100000, size=12).tolist() + [151645, 198])
        refs.append(r.integers(0, 2048, size=(20 + 2 * i, cfg["G"])).astype(np.int32))
        spks.append((r.standard_normal(cfg["H"]) * 0.05).astype(np.float32))
    full_tts.set_params(max_tokens=4096, fixed=3, seed=42, **DEFAULT)
    rc, audio = full_tts.generate_voice_clone_batch(prompts, rids, refs, spks, ["english"] * 8)
    assert rc == 0
    for b in range(8):
        pre, tr = full_oracle.build_icl_prompt(prompts[b], rids[b], refs[b], spks[b], lang, 0)
        want, _ = full_oracle.generate_from_prompt(pre, tr, max_tokens=4096, fixed=3, seed=42, **DEFAULT)
        full = full_oracle.codec_decode(np.concatenate([refs[b], want]))
        T = refs[b].shape[0]
        cut = int(T / (T + len(want)) * full.shape[0])
        _audio_close(audio[b], full[cut:])


def test_c5_bench_shape_vs_oracle_fixture(full_tts, monkeypatch):
    """BASELINE C5 at the bench's own shape: exactly the
    8 voice-clone utterances `bench.py --voice-clone --vc-codes --batch 8`
    rank 0 decodes -- 63 reference frames + a 20-id reference text + an
    x-vector per slot (73 prefill rows each, 584 in the batch's prefill
    GEMM) -- 32 generated frames per slot, against the oracle's ICL layout
    (tests/golden/vc_c5_b8.npz, tests/golden/make_golden_vc.py; the reference
    c/ has no voice clone, so this pin is the oracle's restatement): every
    slot's 32 x 16 codes bit-exact, its audio within the bar.  Also on the
    round-5 prefill GEMM (QTTS_HIP_PGEMM=0, a fresh context) and on k_pgemm's
    128 x 128 tile form (QTTS_HIP_PGEMM_BN=128, read per launch)."""
    import os
    from conftest import GOLDEN
    from parity import codes_equal
    from make_golden_vc import bench_inputs
    g = np.load(os.path.join(GOLDEN, "vc_c5_b8.npz"))
    inp = bench_inputs(full_tts.cfg.num_code_groups, full_tts.cfg.talker_hidden)
    T = int(g["frames"])
    for env in ("1", "bn128", "0"):
        m = full_tts
        if env == "bn128":   # the 128 x 128 tile form of k_pgemm (the default takes 128 x 256 at 584 rows)
            monkeypatch.setenv("QTTS_HIP_PGEMM_BN", "128")
        if env == "0":
            monkeypatch.delenv("QTTS_HIP_PGEMM_BN", raising=False)
            monkeypatch.setenv("QTTS_HIP_PGEMM", "0")
            m = qtts.QwenTTS(model_dir("1.7b"))
        try:
            m.set_params(max_tokens=4096, fixed=T, seed=42, **DEFAULT)
            rc, audio = m.generate_voice_clone_batch([x[0] for x in inp], [x[1] for x in inp], [x[2] for x in inp],
                                                     [x[3] for x in inp], ["english"] * 8)
            assert rc == 0
            codes = m.last_codes_batch(8)
            for b in range(8):
                codes_equal(codes[b], g["codes"][b], f"C5 bench-shape slot {b} (PGEMM={env})")
                assert len(audio[b]) == int(g["audio_len"][b]), (b, len(audio[b]))
                _audio_close(audio[b][::int(g["audio_stride"])], g["audio_sub"][b])
                _audio_close(audio[b][-1920:], g["audio_last"][b])
        finally:
            if m is not full_tts:
                m.close()


def test_prefill_gemm_matches_round5_gemm(gpu, monkeypatch):
    """The prefill's tiled GEMM over pre-split activations (k_pgemm) against
    the round-5 GEMM (k_mgemm, QTTS_HIP_PGEMM=0) on the 1.7B talker: 24 / 97 /
    300 seeded prompt rows (the 16 < rows <= 64 chunk path, the one-tile and
    the multi-tile-plus-split-K shapes) -- prefill hidden allclose, the same
    products summed in another order."""
    outs = {}
    for env in ("1", "bn128", "bn256", "0"):   # "1": the tile width by row count
        monkeypatch.setenv("QTTS_HIP_PGEMM", "0" if env == "0" else "1")
        monkeypatch.setenv("QTTS_HIP_PGEMM_BN", env[2:] if env.startswith("bn") else "auto")
        m = qtts.QwenTTS(model_dir("1.7b"))
        try:
            outs[env] = [m.prefill((np.random.default_rng(n).standard_normal((n, m.cfg.talker_hidden)) * 0.5)
                                   .astype(np.float32)) for n in (24, 97, 300)]
        finally:
            m.close()
    for a, b, b2, c in zip(outs["1"], outs["bn128"], outs["bn256"], outs["0"]):
        np.testing.assert_allclose(a, c, atol=1e-4, rtol=1e-4)
        np.testing.assert_allclose(b2, c, atol=1e-4, rtol=1e-4)
        # (the tile widths split K into different column counts where the tiles
        # alone would not fill the chip: the same products, grouped otherwise)
        np.testing.assert_allclose(a, b, atol=1e-4, rtol=1e-4)
