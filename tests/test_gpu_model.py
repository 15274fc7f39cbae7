"""The HIP hot path (talker + sub-talker decode, on-device sampling, codec)
through the drop-in C-ABI (include/qwen_tts.h) against the reference's golden
outputs (tests/golden/, produced by the reference c/ build) and the oracle.

Bars (BASELINE.json north_star): codebook ids bit-exact; waveform MSE < 1e-4
(asserted, plus a tighter max-abs regression bar of 1e-4 since the fp32 path
differs from the reference only in summation order).  Hidden states / logits:
allclose(atol=1e-4, rtol=1e-4).
"""
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import golden, manifest, model_dir
from oracle_py import GREEDY, DEFAULT, Oracle
from qtts_io import lookup_ids
from synth_model import prompt_ids
from test_oracle_golden import RUNS

import qtts

pytestmark = pytest.mark.gpu
S = golden("stages_tiny.npz")
E = golden("e2e_tiny.npz")


def audio_close(a, ref):
    assert a is not None and a.shape == ref.shape, (None if a is None else a.shape, ref.shape)
    mse = float(np.mean((a.astype(np.float64) - ref) ** 2)) if len(ref) else 0.0
    assert mse < 1e-4, mse
    if len(ref):
        assert np.abs(a - ref).max() < 1e-4, np.abs(a - ref).max()


def test_stage_prefill_and_step(tts_tiny):
    h = tts_tiny.prefill(S["prefill_embeds"])
    np.testing.assert_allclose(h, S["prefill_hidden"], atol=1e-4, rtol=1e-4)
    lg, hid = tts_tiny.step(S["step_embed"])
    np.testing.assert_allclose(lg, S["step_logits"], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(hid, S["step_hidden"], atol=1e-4, rtol=1e-4)


def test_stage_subtalker(tts_tiny):
    m = tts_tiny
    m.set_params(**{"st_top_k": 1, "st_temperature": 1.0, "st_top_p": 1.0})
    np.testing.assert_array_equal(m.subtalker(S["step_hidden"], 5), S["st_greedy_codes"])
    m.set_params(seed=42, st_top_k=50, st_temperature=0.9, st_top_p=1.0)
    np.testing.assert_array_equal(m.subtalker(S["step_hidden"], 5), S["st_sampled_codes"])


def test_stage_codec(tts_tiny):
    a = tts_tiny.codec_decode(S["codec_codes"])
    audio_close(a, S["codec_audio"])


def test_codec_edge_lengths(tts_tiny, oracle):
    """T = 1 (first packet), T crossing the 72-frame attention window, and
    codes out of range (zero contribution, Cd.c:150-160)."""
    rng = np.random.default_rng(3)
    for T in (1, 2, 73, 150):
        codes = rng.integers(0, 2048, size=(T, 16)).astype(np.int32)
        codes[0, 3] = -1
        codes[-1, 5] = 4096
        audio_close(tts_tiny.codec_decode(codes), oracle.codec_decode(codes))


@pytest.mark.parametrize("P", [17, 64, 65, 200])
def test_long_prefill_vs_oracle(tts_tiny, oracle, P):
    """ICL-length prefill (100-250 prompt rows, T.c:254-472):
    rows past 16 go to the 64-row MFMA GEMM (k_mgemm) in chunks, attention
    runs causal over the whole prompt; the next decode step then reads all P
    cached keys.  Hidden and logits against the oracle at the stage bar."""
    rng = np.random.default_rng(100 + P)
    H = S["prefill_embeds"].shape[1]
    e = (rng.standard_normal((P, H)) * 0.5).astype(np.float32)
    np.testing.assert_allclose(tts_tiny.prefill(e), oracle.prefill(e), atol=1e-4, rtol=1e-4)
    x = (rng.standard_normal(H) * 0.5).astype(np.float32)
    lg, hid = tts_tiny.step(x)
    lgo, hido = oracle.step(x)
    np.testing.assert_allclose(lg, lgo, atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(hid, hido, atol=1e-4, rtol=1e-4)


def _gen(m, name):
    fx, pp, fixed, mx, seed = RUNS[name]
    m.set_params(max_tokens=mx, fixed=fixed, seed=seed, **pp)
    return m.generate(prompt_ids("short"), "aiden", "english")


@pytest.mark.parametrize("name", sorted(RUNS))
def test_e2e_codes_bit_exact_and_audio(name, request):
    fx = RUNS[name][0]
    m = qtts.QwenTTS(request.getfixturevalue(fx))
    try:
        a = _gen(m, name)
        codes = m.last_codes()
        np.testing.assert_array_equal(codes, E[f"{name}_codes"])
        audio_close(a, E[f"{name}_audio"])
        assert m.c.perf_codec_tokens == len(E[f"{name}_codes"])
        # determinism: a second run on the same ctx gives the same codes
        _gen(m, name)
        np.testing.assert_array_equal(m.last_codes(), codes)
    finally:
        m.close()


def test_eos_stop_reported_like_reference(gpu):
    m = qtts.QwenTTS(model_dir("tiny", eos_gain=manifest()["eos_gain"]))
    try:
        _gen(m, "eosg")
        want = int(re.search(r"step (\d+)", manifest()["cli_eos"]["stop_line"]).group(1))
        assert m.c.last_stop_reason == 1 and m.c.last_stop_step == want
    finally:
        m.close()


@pytest.mark.parametrize("env", [{}, {"QTTS_HIP_BSPLIT": "0"}, {"QTTS_HIP_GEMVB": "0"}, {"QTTS_HIP_BSELF_MIN": "2"},
                                 {"QTTS_HIP_BKZ_MAX": "4"}, {"QTTS_HIP_TAB0B": "0"}])
def test_batch_slots_match_single_runs(tiny_dir, oracle, monkeypatch, env):
    """Lock-step batch (B GEMV columns, one weight read per frame): every
    slot's audio equals the oracle's for its own prompt / speaker -- with the
    O / down projections split over K (partials added by the next residual
    reader) and without, on the staged-plane batch GEMV (k_gemvm) instead of
    the per-wave-slice one (k_gemvb), with every split-K producer reducing its
    own partials, with up to 4 split-K columns, and with layer 0's q|k|v by
    GEMV instead of the load-time table (passes >= 1)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = qtts.QwenTTS(tiny_dir)
    try:
        prompts = [prompt_ids("short"), prompt_ids("p128", 1240), prompt_ids("p128", 1241)]
        spk = ["aiden", "vivian", "serena"]
        lang = ["english", "japanese", "chinese"]
        for pp, fixed, mx in ((GREEDY, 12, 4096), (DEFAULT, 12, 4096)):
            m.set_params(max_tokens=mx, fixed=fixed, seed=42, **pp)
            rc, audio = m.generate_batch(prompts, spk, lang)
            assert rc == 0
            for b in range(3):
                s, l = lookup_ids(oracle.cfg, spk[b], lang[b])
                codes, _ = oracle.generate_codes(prompts[b], s, l, max_tokens=mx, fixed=fixed, seed=42, **pp)
                audio_close(audio[b], oracle.codec_decode(codes))
    finally:
        m.close()


def test_batch12_self_reducing_split_k(tiny_dir, oracle):
    """Above 8 slots the O / down split-K producer adds its own partials to
    the residual (the last workgroup column of a row block, k_gemvm ticket);
    12 slots, each equal to its own oracle run, twice on one ctx (the tickets
    are reset by their last arriver)."""
    m = qtts.QwenTTS(tiny_dir)
    try:
        prompts = [prompt_ids("p128", 1250 + i) for i in range(12)]
        spk = ["aiden", "vivian", "serena"] * 4
        lang = ["english", "japanese", "chinese", "english"] * 3
        m.set_params(max_tokens=4096, fixed=8, seed=42, **DEFAULT)
        rc, audio = m.generate_batch(prompts, spk, lang)
        assert rc == 0
        for b in range(12):
            s, l = lookup_ids(oracle.cfg, spk[b], lang[b])
            codes, _ = oracle.generate_codes(prompts[b], s, l, max_tokens=4096, fixed=8, seed=42, **DEFAULT)
            audio_close(audio[b], oracle.codec_decode(codes))
        rc, again = m.generate_batch(prompts, spk, lang)
        assert rc == 0
        for b in range(12):
            np.testing.assert_array_equal(again[b], audio[b])
    finally:
        m.close()


def test_batch_eos_slots_stop_independently(tiny_eos_dir):
    """Slots stop at their own EOS; finished slots keep their frame count (and
    their codec passes, of different lengths, run side by side)."""
    o = Oracle(tiny_eos_dir)
    m = qtts.QwenTTS(tiny_eos_dir)
    try:
        prompts = [prompt_ids("short"), prompt_ids("p128", 1300), prompt_ids("p128", 1301), prompt_ids("short")]
        m.set_params(max_tokens=32, fixed=0, seed=7, **DEFAULT)
        rc, audio = m.generate_batch(prompts, ["aiden"] * 4, ["english"] * 4)
        assert rc == 0
        s, l = lookup_ids(o.cfg, "aiden", "english")
        for b in range(4):
            codes, _ = o.generate_codes(prompts[b], s, l, max_tokens=32, fixed=0, seed=7, **DEFAULT)
            audio_close(audio[b], o.codec_decode(codes))
    finally:
        m.close()
        o.close()


def test_cli_eos_regression_like_reference(tiny_eos_dir):
    """test/test_eos_regression.py's check on our CLI: greedy flags, the same
    `Stop: eos at step N` line and WAV as the reference CLI (+-1 LSB)."""
    man = manifest()["cli_eos"]
    ids = ",".join(str(i) for i in prompt_ids("short"))
    with tempfile.TemporaryDirectory() as d:
        wav = os.path.join(d, "o.wav")
        r = subprocess.run([qtts.CLI_PATH, "-d", tiny_eos_dir, "-t", ids, "-o", wav] + man["args"],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert man["stop_line"] in r.stderr
        g = re.search(r"Generated (\d+) codec tokens in [\d.]+ ms \([\d.]+ ms/token\)", r.stderr)
        assert g and int(g.group(1)) == man["generated"]
        assert re.search(r"Total: [\d.]+ ms \([\d.]+ s audio, [\d.]+x realtime\)", r.stderr)
        pcm = np.frombuffer(open(wav, "rb").read()[44:], np.int16)
    ref = golden("wav.npz")["cli_eos_pcm"]
    assert pcm.shape == ref.shape
    assert np.abs(pcm.astype(np.int32) - ref).max() <= 1


def test_cli_codec_verbose_lines_like_reference(tiny_eos_dir):
    """The codec's stderr lines: at -v the reference CLI's own
    `Codec decode: N timesteps, 16 quantizers` / `Codec decode complete: S
    samples (X seconds)` (tests/golden/manifest.json, c/qwen_tts_codec.c:598,
    740-742); at -v -v also `Codec stages (ms): rvq=.. preconv=.. transformer=..
    upsample=.. vocoder=..` (:743-746), timed on the device by HIP events."""
    man = manifest()["cli_eos"]
    ids = ",".join(str(i) for i in prompt_ids("short"))
    stages = re.compile(r"Codec stages \(ms\): rvq=[\d.]+ preconv=[\d.]+ transformer=[\d.]+ upsample=[\d.]+ "
                        r"vocoder=[\d.]+")
    with tempfile.TemporaryDirectory() as d:
        for extra, want_stages in ((["-v"], False), (["-v", "-v"], True)):
            args = [a for a in man["args"] if a != "-v"] + extra
            r = subprocess.run([qtts.CLI_PATH, "-d", tiny_eos_dir, "-t", ids, "-o", os.path.join(d, "o.wav")] + args,
                               capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, r.stderr
            lines = r.stderr.splitlines()
            for want in man["codec_lines"]:
                assert want in lines, (want, r.stderr)
            assert bool(stages.search(r.stderr)) == want_stages, r.stderr


def test_cli_persistent_benchmark_lines(tiny_dir):
    ids = ",".join(str(i) for i in prompt_ids("short"))
    with tempfile.TemporaryDirectory() as d:   # the writer goes through <path>.tmp like the reference's
        r = subprocess.run([qtts.CLI_PATH, "-d", tiny_dir, "-t", ids, "-o", os.path.join(d, "o.wav"),
                            "--fixed-codec-tokens", "8", "--benchmark-runs", "2", "--benchmark-warmup", "1"],
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    runs = re.findall(r"\[persistent\] run (\d+)/(\d+): elapsed=[\d.]+ ms, audio=[\d.]+s, talker=[\d.]+ ms, "
                      r"codec=[\d.]+ ms, total=[\d.]+ ms, tokens=(\d+)", r.stderr + r.stdout)
    assert len(runs) == 2 and all(t == "8" for _, _, t in runs)


def test_progress_callback_and_params(tts_tiny):
    import ctypes as C
    steps = []
    cb = qtts.PROGRESS_CB(lambda s, t, u: steps.append((s, t)))
    qtts.lib().qwen_tts_set_progress_callback(tts_tiny.ctx, cb, None)
    try:
        tts_tiny.set_params(max_tokens=4096, fixed=6, seed=1, **GREEDY)
        a = tts_tiny.generate(prompt_ids("short"), "aiden", "english")
        assert a is not None and len(a) == 6 * 1920
        assert [s for s, _ in steps] == list(range(1, 7)) or len(steps) == 6
    finally:
        qtts.lib().qwen_tts_set_progress_callback(tts_tiny.ctx, C.cast(None, qtts.PROGRESS_CB), None)


def test_unknown_speaker_warns_and_continues(tts_tiny):
    tts_tiny.set_params(max_tokens=4096, fixed=3, seed=1, **GREEDY)
    a = tts_tiny.generate(prompt_ids("short"), "nobody", "klingon")
    assert a is not None and len(a) == 3 * 1920


# ---------------------------------------------------------------- streaming
@pytest.mark.parametrize("T,chunks", [(50, [1, 3, 7, 16, 23]), (150, [1, 40, 16, 5, 88])])
def test_codec_stream_equals_full_decode(tts_tiny, oracle, T, chunks):
    """Incremental decode with carried state (conv histories, transposed-conv
    tails, window-72 K/V) reproduces the full decode; T=150 crosses the
    attention window."""
    rng = np.random.default_rng(T)
    codes = rng.integers(0, 2048, size=(T, 16)).astype(np.int32)
    full = tts_tiny.codec_decode(codes)
    parts, t = [], 0
    for c in chunks:
        parts.append(codes[t:t + c])
        t += c
    assert t == T
    outs = tts_tiny.codec_stream(parts)
    for p, o in zip(parts, outs):
        assert len(o) == len(p) * 1920
    s = np.concatenate(outs)
    assert s.shape == full.shape
    assert np.abs(s - full).max() < 1e-5, np.abs(s - full).max()
    audio_close(s, oracle.codec_decode(codes))


def test_generate_stream_equals_generate(tiny_dir):
    m = qtts.QwenTTS(tiny_dir)
    try:
        m.set_params(max_tokens=4096, fixed=16, seed=42, **GREEDY)
        full = m.generate(prompt_ids("short"), "aiden", "english")
        chunks = []
        s = m.generate_stream(prompt_ids("short"), "aiden", "english", chunk_frames=4, on_chunk=chunks.append)
        assert [len(c) for c in chunks] == [1920, 4 * 1920, 4 * 1920, 4 * 1920, 3 * 1920]
        np.testing.assert_array_equal(np.concatenate(chunks), s)
        assert s.shape == full.shape and np.abs(s - full).max() < 1e-5
        np.testing.assert_array_equal(m.last_codes(), E["greedy_codes"])
        assert 0 < m.c.perf_first_packet_ms < m.c.perf_total_ms
        # later streams on the same context (reused stream state): identical audio
        for _ in range(2):
            chunks2 = []
            s2 = m.generate_stream(prompt_ids("short"), "aiden", "english", chunk_frames=4, on_chunk=chunks2.append)
            np.testing.assert_array_equal(s2, s)
            np.testing.assert_array_equal(chunks2[0], chunks[0])
    finally:
        m.close()


def test_generate_stream_eos(tiny_eos_dir):
    """Streaming in EOS mode stops with the reference's stop step and yields
    the same audio as the non-streaming call."""
    m = qtts.QwenTTS(tiny_eos_dir)
    try:
        _gen(m, "eosg")
        full = m.generate(prompt_ids("short"), "aiden", "english")
        s = m.generate_stream(prompt_ids("short"), "aiden", "english", chunk_frames=5)
        np.testing.assert_array_equal(m.last_codes(), E["eosg_codes"])
        assert s.shape == full.shape and np.abs(s - full).max() < 1e-5
    finally:
        m.close()


def test_cli_stream_flag(tiny_dir):
    ids = ",".join(str(i) for i in prompt_ids("short"))
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([qtts.CLI_PATH, "-d", tiny_dir, "-t", ids, "-o", os.path.join(d, "o.wav"), "-v",
                            "--fixed-codec-tokens", "8", "--stream", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert re.search(r"First packet: [\d.]+ ms", r.stderr)


@pytest.mark.parametrize("env", [{"QTTS_HIP_PTAB": "0"}, {"QTTS_HIP_ATTN_O": "0"}, {"QTTS_HIP_NO_GRAPH": "1"},
                                 {"QTTS_HIP_L2PF": "0"}, {"QTTS_HIP_SAMPLE_W": "0"}, {"QTTS_HIP_ARENA": "1"}])
def test_e2e_debug_switch_paths(tiny_dir, monkeypatch, env):
    """The debug switches' paths stay bit-exact: the per-pass input projection
    instead of the projected tables, sub-talker attention and O projection as
    two kernels, eager launches instead of the frame graphs, no next-launch
    L2 prefetch, the 256-thread sampler, small buffers carved from 32 MB blocks
    (the default path is covered by
    test_e2e_codes_bit_exact_and_audio)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    m = qtts.QwenTTS(tiny_dir)
    try:
        for name in ("greedy", "sampled"):
            a = _gen(m, name)
            np.testing.assert_array_equal(m.last_codes(), E[f"{name}_codes"])
            audio_close(a, E[f"{name}_audio"])
    finally:
        m.close()


@pytest.mark.parametrize("heads", [(8, 2), (4, 4)])
def test_subtalker_head_layouts_vs_oracle(gpu, heads):
    """Sub-talker head layouts the fused attention + O kernel does not take
    (NH != 2 KV): the layer-0 q|k|v table must not be read there (its skipped
    GEMV is what writes the residual), so the generic attention path runs
    with the GEMV.  Codes bit-exact and audio against the oracle."""
    nh, kv = heads
    md = model_dir("tiny", NHs=nh, KVs=kv)
    ids = prompt_ids("short")
    o = Oracle(md)
    m = qtts.QwenTTS(md)
    try:
        s, l = lookup_ids(o.cfg, "aiden", "english")
        for pp in (GREEDY, DEFAULT):
            want, _ = o.generate_codes(ids, s, l, max_tokens=4096, fixed=6, seed=42, **pp)
            m.set_params(max_tokens=4096, fixed=6, seed=42, **pp)
            a = m.generate(ids, "aiden", "english")
            np.testing.assert_array_equal(m.last_codes(), want)
            audio_close(a, o.codec_decode(want))
    finally:
        m.close()
        o.close()
