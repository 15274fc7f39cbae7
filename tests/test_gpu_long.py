"""Long-context parity on the GPU against the REFERENCE's own outputs.

Fixtures (tests/golden/make_golden_long.py, from the reference c/ build):

* `long_hd128.npz` -- the `hd128` synthetic model (the talker's real attention
  shape NH 16 / KV 8 / HD 128, 2 narrow layers): a 640-frame default-sampling
  decode, talker positions 38 .. 678.  At batch 1 `k_attn_dec` takes 32-key
  splits whose merge runs in the O projection's prologue (up to 22 splits
  here); the batch-3 test runs the 64-key splits the kernel merges itself,
  through the 1-split, 2-8-split and > 8-split merges.  QTTS_HIP_ATTN_DEFER=0
  (batch 1 merging its own 64-key splits) runs all 640 frames, so batch 1
  also reaches > 8 splits of 64 keys.  The codes must be bit-exact all the
  way.  A 600-row prefill (> 512 rows) and 4 decode steps over 600+ keys.
* `long_hd128_max.npz` -- the same model over the reference's whole decode
  capacity (4096 frames, positions to ~4200: > 128 key splits).
* `long_17b_1100.npz` -- the synthetic 1.7B past 1024 keys (fixed 1100 frames).
* `long_17b.npz` -- the benchmark workload itself (bench.py): synthetic 1.7B,
  P128 prompt, fixed 128 frames, default sampling, seed 42.
* `long_06b.npz` -- BASELINE configs[1] (C2): synthetic 0.6B (H = H_s = 1024,
  no sub-talker input projection), P128, GREEDY, fixed 128 frames.
* `long_17b_b8.npz` -- BASELINE C4's per-GPU shape: 8 prompts, default
  sampling, 32 frames, each slot one reference run; decoded here as ONE
  lock-step batch on the batch GEMV (`k_gemvb`, RMS scale applied after the
  dot product, split-K O / down), codes compared slot by slot.
* `long_17b_b8bench.npz` -- C4's bench workload itself: the 8 utterances of
  `bench.py --batch 8` (p128 seeds 1234-1241, aiden), the whole 128 frames.
* `long_eos17.npz` -- EOS mode on bench.py --eos's model: three utterances,
  each one reference run to its EOS stop; the stop steps and codes.

Bars: codes bit-exact (the first divergent frame / group is reported if not,
with tests/divergence.py's verdict -- fp near-tie or bug -- where the oracle
can replay the utterance to it: the C2 greedy run and frames <= 48);
waveform MSE < 1e-4 and max |d| < 1e-3 (north star); hidden / logits
allclose(1e-4, 1e-4) as the tiny stage goldens.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, model_dir
from parity import codes_equal, codes_equal_upto_classified
from make_golden_long import prefill_inputs
from oracle_py import DEFAULT, GREEDY, Oracle
from qtts_io import lookup_ids

import qtts

pytestmark = [pytest.mark.gpu]


def _man():
    return json.load(open(os.path.join(GOLDEN, "long_manifest.json")))


def _codes_equal(got, want, what, ctx=None):
    codes_equal(got, want, what, ctx)


def _audio_close(a, ref, what, mse_bar=1e-4, max_bar=1e-3):
    assert a is not None and a.shape == ref.shape, (what, None if a is None else a.shape, ref.shape)
    d = a.astype(np.float64) - ref
    mse, mx = float(np.mean(d * d)), float(np.abs(d).max())
    assert mse < mse_bar and mx < max_bar, (what, mse, mx)


@pytest.fixture(scope="module")
def hd128(gpu):
    md = model_dir("hd128")
    m = qtts.QwenTTS(md)
    yield m, md, np.load(os.path.join(GOLDEN, "long_hd128.npz")), _man()["hd128"]
    m.close()


def test_hd128_640_frames_vs_reference(hd128):
    """640 frames: every split-merge path of the talker's decode attention,
    codes bit-exact against the reference, waveform against its samples."""
    m, md, g, man = hd128
    m.set_params(max_tokens=4096, fixed=man["frames"], seed=man["seed"], **DEFAULT)
    a = m.generate(g["prompt_ids"], "aiden", "english")
    _codes_equal(m.last_codes(), g["decode_codes"], "hd128 640-frame decode")
    assert a.shape[0] == int(g["decode_audio_len"])
    _audio_close(a[::man["audio_stride"]], g["decode_audio_sub"], "every 16th sample")
    _audio_close(a[:1920], g["decode_audio_first"], "first frame")
    _audio_close(a[-1920:], g["decode_audio_last"], "last frame")
    # the whole waveform against the oracle port's decode of the same codes
    o = Oracle(md)
    try:
        _audio_close(a, o.codec_decode(g["decode_codes"]), "full waveform vs oracle")
    finally:
        o.close()


def test_hd128_max_capacity_vs_reference(hd128):
    """The reference's whole decode capacity (max_new_tokens 4096, fixed): talker
    positions to ~4200, i.e. > 128 key splits per kv head in the decode
    attention and the O prologue's merge of them (the maximum-size edge case),
    codes bit-exact against the reference's own 4096-frame run
    (long_hd128_max.npz) up to a recorded fp near-tie, the waveform against
    its samples before it."""
    path = os.path.join(GOLDEN, "long_hd128_max.npz")
    if not os.path.exists(path):
        pytest.skip("long_hd128_max.npz not generated (make_golden_long.py --only hd128max)")
    m, md, _, _ = hd128
    g = np.load(path)
    man = _man()["hd128max"]
    m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
    a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
    # 65,536 draws: bit-exact up to the first divergence, which must be the
    # recorded, classified fp near-tie (profiles/r06_classify_hd128max.txt)
    f = codes_equal_upto_classified(m.last_codes(), g["codes"], "hd128 4096-frame decode",
                                    man.get("near_ties"))
    assert a.shape[0] == int(g["audio_len"])
    n = len(a) if f is None else f * 1920   # (the codec is causal: samples before frame f see only equal codes)
    st = man["audio_stride"]
    _audio_close(a[:n:st], g["audio_sub"][:(n + st - 1) // st], "every 256th sample (before any divergence)")
    _audio_close(a[:1920], g["audio_first"], "first frame")
    if f is None:
        _audio_close(a[-1920:], g["audio_last"], "last frame")


def test_17b_past_1024_keys_vs_reference(gpu):
    """The synthetic 1.7B past 1024 keys (fixed 1100 frames, P128): > 32 splits
    of 32 keys per kv head in the talker's decode attention and its merge in
    the O prologue; codes bit-exact against the reference's own run
    (long_17b_1100.npz)."""
    path = os.path.join(GOLDEN, "long_17b_1100.npz")
    if not os.path.exists(path):
        pytest.skip("long_17b_1100.npz not generated (make_golden_long.py --only k1100)")
    g = np.load(path)
    man = _man()["k1100"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        _codes_equal(m.last_codes(), g["codes"], "1.7B 1100-frame decode")
        assert a.shape[0] == int(g["audio_len"])
        _audio_close(a[::man["audio_stride"]], g["audio_sub"], "every 256th sample")
        _audio_close(a[-1920:], g["audio_last"], "last frame")
    finally:
        m.close()


def test_hd128_640_frames_lock_step_batch(hd128):
    """The same utterance as slot 0 and 2 of a lock-step batch of 3 (batch
    attention rows through the same split merges): bit-equal to the reference."""
    m, md, g, man = hd128
    other = g["prompt_ids"].copy()
    other[5] += 17
    m.set_params(max_tokens=4096, fixed=man["frames"], seed=man["seed"], **DEFAULT)
    rc, audio = m.generate_batch([g["prompt_ids"], other, g["prompt_ids"]], ["aiden", "vivian", "aiden"],
                                 ["english"] * 3)
    assert rc == 0
    np.testing.assert_array_equal(audio[0], audio[2])
    _audio_close(audio[0][::man["audio_stride"]], g["decode_audio_sub"], "batch slot 0, every 16th sample")
    _audio_close(audio[0][-1920:], g["decode_audio_last"], "batch slot 0, last frame")


def test_hd128_600_row_prefill_and_steps_vs_reference(hd128):
    """A 600-row prefill (the matrix-core prefill GEMM, prefill attention over
    600 rows), then decode steps at positions 600-603 (10 key splits)."""
    m, md, g, man = hd128
    emb, steps = prefill_inputs(m.cfg.talker_hidden, man["prefill_seed"])
    h = m.prefill(emb)
    np.testing.assert_allclose(h, g["prefill_hidden"], atol=1e-4, rtol=1e-4)
    for i in range(man["prefill_steps"]):
        lg, hid = m.step(steps[i])
        np.testing.assert_allclose(lg, g["step_logits"][i], atol=1e-4, rtol=1e-4)
        np.testing.assert_allclose(hid, g["step_hidden"][i], atol=1e-4, rtol=1e-4)


def test_hd128_4000_row_prefill_and_steps_vs_reference(hd128):
    """Near the decode capacity: a 4000-row prefill of seeded embeddings, then
    decode steps at positions 4000-4003 -- 125+ splits of 32 keys per kv head
    and their merge in the O prologue -- hidden and logits within the stage
    bar against the reference's (long_hd128_steps4k.npz; no sampling, so no
    near-tie can turn a rounding difference into a different id)."""
    path = os.path.join(GOLDEN, "long_hd128_steps4k.npz")
    if not os.path.exists(path):
        pytest.skip("long_hd128_steps4k.npz not generated (make_golden_long.py --only steps4k)")
    m, md, _, _ = hd128
    g = np.load(path)
    man = _man()["steps4k"]
    rng = np.random.Generator(np.random.PCG64(man["prefill_seed"]))
    emb = (rng.standard_normal((man["prefill_rows"], m.cfg.talker_hidden)) * 0.5).astype(np.float32)
    steps = (rng.standard_normal((man["steps"], m.cfg.talker_hidden)) * 0.5).astype(np.float32)
    h = m.prefill(emb)
    np.testing.assert_allclose(h, g["prefill_hidden"], atol=1e-4, rtol=1e-4)
    for i in range(man["steps"]):
        lg, hid = m.step(steps[i])
        np.testing.assert_allclose(lg, g["step_logits"][i], atol=1e-4, rtol=1e-4)
        np.testing.assert_allclose(hid, g["step_hidden"][i], atol=1e-4, rtol=1e-4)


@pytest.mark.slow
@pytest.mark.parametrize("env", [{}, {"QTTS_HIP_L2PF": "0"}, {"QTTS_HIP_L2PF_TK": "3"}, {"QTTS_HIP_L2PF": "5"}])
def test_full_bench_workload_vs_reference(gpu, monkeypatch, env):
    """BASELINE's workload as bench.py runs it (1.7B, P128, fixed 128 frames,
    default sampling, seed 42): codes bit-exact, waveform MSE < 1e-4 -- also
    without the next-launch L2 prefetch, with part of its edges, and with the
    talker's prefetch edges on (these loads never change a value)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = np.load(os.path.join(GOLDEN, "long_17b.npz"))
    man = _man()["1.7b"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        _codes_equal(m.last_codes(), g["codes"], "1.7B bench workload")
        _audio_close(a, g["audio"], "1.7B bench workload waveform")
    finally:
        m.close()


def test_c2_06b_greedy_128_frames_vs_reference(gpu):
    """BASELINE configs[1] (0.6B, batch 1, greedy, P128), the whole 128-frame
    utterance: codes bit-exact against the reference, waveform MSE < 1e-4."""
    g = np.load(os.path.join(GOLDEN, "long_06b.npz"))
    man = _man()["0.6b"]
    m = qtts.QwenTTS(model_dir("0.6b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **GREEDY)
        a = m.generate(g["prompt_ids"], man["speaker"], man["language"])
        codes = m.last_codes()
        if not np.array_equal(codes, g["codes"]):   # (the verdict needs the oracle on the 0.6B model)
            o = Oracle(model_dir("0.6b"))
            s, l = lookup_ids(o.cfg, man["speaker"], man["language"])
            ctx = dict(oracle=o, ids=g["prompt_ids"], spk=s, lang=l, max_frame=man["frames"],
                       params=dict(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **GREEDY))
            _codes_equal(codes, g["codes"], "0.6B greedy 128 frames", ctx)
        _audio_close(a, g["audio"], "0.6B greedy waveform")
    finally:
        m.close()


def _b8_prompts(g):
    return [g["prompt_ids"][b, :int(g["prompt_len"][b])] for b in range(g["prompt_ids"].shape[0])]


@pytest.mark.slow
@pytest.mark.parametrize("env", [{}, {"QTTS_HIP_GEMVB": "0"}, {"QTTS_HIP_BSELF_MIN": "2"}, {"QTTS_HIP_TAB0B": "0"}])
def test_c4_batch8_lock_step_vs_reference(gpu, monkeypatch, env):
    """C4's per-GPU shape: the 8 reference utterances (32 frames, default
    sampling) decoded as ONE lock-step batch -- the batch GEMV with its RMS
    scale after the dot product, split-K O / down -- every slot's codes
    bit-exact against its own reference run, audio against the reference's
    samples.  Also on the staged-plane batch GEMV (GEMVB=0), with the
    split-K producers reducing their own partials from 2 rows, and with layer
    0's q|k|v by GEMV instead of the load-time table (TAB0B=0)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = np.load(os.path.join(GOLDEN, "long_17b_b8.npz"))
    man = _man()["b8"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=4096, fixed=man["frames"], seed=man["seed"], **DEFAULT)
        rc, audio = m.generate_batch(_b8_prompts(g), man["speakers"], [man["language"]] * 8)
        assert rc == 0
        codes = m.last_codes_batch()
        for b in range(8):
            _codes_equal(codes[b], g["codes"][b], f"batch-8 slot {b} {env}")
            _audio_close(audio[b][::man["audio_stride"]], g["audio_sub"][b], f"slot {b} every 16th sample")
            _audio_close(audio[b][-1920:], g["audio_last"][b], f"slot {b} last frame")
    finally:
        m.close()


@pytest.mark.parametrize("env,frames", [({"QTTS_HIP_ATTN_DEFER": "0"}, 640), ({"QTTS_HIP_ATTN_LPK": "4"}, 300),
                                        ({"QTTS_HIP_ATTN_LPK": "16"}, 300)])
def test_hd128_attention_switch_paths_vs_reference(gpu, monkeypatch, env, frames):
    """The talker attention's A/B switches at HD 128: the merge in the last
    split instead of the O projection's prologue (64-key splits, all 640
    frames: positions to 678, so batch 1 runs the 1-, 2-8- and > 8-split
    merges), and the other split sizes of the deferred merge (64- / 16-key
    splits, 300 frames) -- codes bit-exact against the reference's.  The
    split size is latched at model creation (the scratch is sized by it)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = np.load(os.path.join(GOLDEN, "long_hd128.npz"))
    man = _man()["hd128"]
    m = qtts.QwenTTS(model_dir("hd128"))
    try:
        m.set_params(max_tokens=4096, fixed=frames, seed=man["seed"], **DEFAULT)
        m.generate(g["prompt_ids"], "aiden", "english")
        _codes_equal(m.last_codes(), g["decode_codes"][:frames], f"hd128 {frames} frames {env}")
    finally:
        m.close()


@pytest.mark.slow
@pytest.mark.parametrize("env", [{}, {"QTTS_HIP_GEMVB": "0"}, {"QTTS_HIP_BKZ_WIDE": "2"}])
def test_c4_bench_workload_batch8_vs_reference(gpu, monkeypatch, env):
    """C4's per-GPU bench workload itself (`bench.py --batch 8`, rank 0): p128
    seeds 1234-1241, speaker aiden, seed 42, default sampling, the whole 128
    frames -- decoded as ONE lock-step batch, every slot's 128 x 16 codes
    bit-exact against its own reference run (long_17b_b8bench.npz), audio
    against the reference's samples.  Also on the staged-plane batch GEMV,
    and with the talker's down projection on 4 split-K columns (BKZ_WIDE=2)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = np.load(os.path.join(GOLDEN, "long_17b_b8bench.npz"))
    man = _man()["b8bench"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        rc, audio = m.generate_batch(_b8_prompts(g), man["speakers"], [man["language"]] * 8)
        assert rc == 0
        codes = m.last_codes_batch()
        for b in range(8):
            _codes_equal(codes[b], g["codes"][b], f"bench batch-8 slot {b} {env}")
            _audio_close(audio[b][::man["audio_stride"]], g["audio_sub"][b], f"slot {b} every 16th sample")
            _audio_close(audio[b][-1920:], g["audio_last"][b], f"slot {b} last frame")
    finally:
        m.close()


@pytest.mark.slow
@pytest.mark.parametrize("env", [{}, {"QTTS_HIP_BKZ_WIDE": "0"}])
def test_c4_bench_workload_batch16_vs_reference(gpu, monkeypatch, env):
    """`bench.py --batch 16`'s shape: the bench workload's 8 utterances twice
    in ONE lock-step batch of 16 -- above 8 rows the split-K producers reduce
    their own partials, and the 1.7B talker's down projection runs on 4
    split-K columns (bsplit_kz; BKZ_WIDE=0: 2 columns on k_gemvm) -- slots b
    and b + 8 bit-exact against reference run b (long_17b_b8bench.npz)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = np.load(os.path.join(GOLDEN, "long_17b_b8bench.npz"))
    man = _man()["b8bench"]
    m = qtts.QwenTTS(model_dir("1.7b"))
    try:
        m.set_params(max_tokens=man["frames"], fixed=man["frames"], seed=man["seed"], **DEFAULT)
        rc, audio = m.generate_batch(_b8_prompts(g) * 2, man["speakers"] * 2, [man["language"]] * 16)
        assert rc == 0
        codes = m.last_codes_batch()
        for s in range(16):
            b = s % 8
            _codes_equal(codes[s], g["codes"][b], f"bench batch-16 slot {s} {env}")
            _audio_close(audio[s][-1920:], g["audio_last"][b], f"slot {s} last frame")
    finally:
        m.close()


def _eos_slot_check(codes, audio, g, man, b, what):
    n = int(g["stop_step"][b])
    _codes_equal(codes, g["codes"][b, :n], f"{what}: slot {b} codes up to the reference's stop")
    assert audio is not None and len(audio) == n * 1920, (what, b, None if audio is None else len(audio), n)
    _audio_close(audio[::man["audio_stride"]], g["audio_sub"][b, :len(audio[::man["audio_stride"]])],
                 f"{what}: slot {b} every 16th sample")


def test_eos_stop_17b_batch_1_and_3(gpu):
    """EOS mode (the reference's default: max_new_tokens 4096, stop at EOS,
    Q.c:1282-1330) on the synthetic 1.7B whose codec-head EOS row is scaled
    x1.4 (bench.py --eos), against the reference's own EOS runs
    (long_eos17.npz): each of the three utterances alone stops at the
    reference's step with its codes bit-exact, and the same three as ONE
    lock-step batch -- where the rows that stop first keep riding along while
    the others decode -- give every slot the same stop step and codes.
    Regression: a stopped row's table id (the talker's EOS id, >= the
    sub-talker vocabulary) indexed past the last pass's q|k|v / input table."""
    g = np.load(os.path.join(GOLDEN, "long_eos17.npz"))
    man = _man()["eos17"]
    m = qtts.QwenTTS(model_dir("1.7b", eos_gain=man["eos_gain"]))
    try:
        prompts = _b8_prompts(g)
        stops = [int(x) for x in g["stop_step"]]
        assert len(set(stops)) > 1, stops   # the batch run must have a row stopping before the others
        for b, ids in enumerate(prompts):
            m.set_params(max_tokens=4096, fixed=0, seed=man["seed"], **DEFAULT)
            a = m.generate(ids, man["speakers"][b], man["language"])
            assert m.c.last_stop_reason == 1, "no EOS stop"
            assert m.c.last_stop_step == stops[b], (b, m.c.last_stop_step, stops[b])
            _eos_slot_check(m.last_codes(), a, g, man, b, "batch 1")
        m.set_params(max_tokens=4096, fixed=0, seed=man["seed"], **DEFAULT)
        rc, aud = m.generate_batch(prompts, man["speakers"], [man["language"]] * len(prompts))
        assert rc == 0
        codes = m.last_codes_batch()
        for b in range(len(prompts)):
            _eos_slot_check(codes[b], aud[b], g, man, b, "lock-step batch of 3")
    finally:
        m.close()
