"""Voice clone (the ICL prompt and its long prefill).

The c/ reference has no voice-clone path; the layout follows the Python
reference (modeling_qwen3_tts.py:1967-2019 generate_icl_prompt, :2104-2232
prompt assembly; qwen3_tts_model.py:612-630 decode-with-reference and cut).
The oracle restates it (oracle/qtts_oracle.c orc_build_icl_prompt).  PARITY
UNPINNED against the Python reference itself (not importable here, SURVEY.md
§8c): the pin is the oracle's own identity with the c/-pinned plain prompt
(x-vector-only without a vector == the custom-voice layout).  The audio
encoders (ECAPA speaker encoder, 12 Hz tokenizer encoder, §8f N3) are out of
scope: tests feed synthetic reference codes and x-vectors.

Bars: codes bit-exact (greedy and default sampling), audio as test_gpu_model.
"""
import numpy as np
import pytest

from oracle_py import DEFAULT, GREEDY
from qtts_io import lookup_ids
from synth_model import prompt_ids

REF_IDS = [151644, 77091, 198] + list(range(3000, 3012)) + [151645, 198]   # 12 content ids


def _inputs(o, T, seed=0, spk=False):
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, min(o.cfg["V"], o.cfg["Vs"]), size=(T, o.cfg["G"])).astype(np.int32)
    sv = (rng.standard_normal(o.cfg["H"]) * 0.05).astype(np.float32) if spk else None
    return codes, sv


# ------------------------------------------------------------------ CPU: the oracle's layout
def test_xvector_only_without_vector_is_plain_prompt(oracle):
    _, lang = lookup_ids(oracle.cfg, "aiden", "english")
    ids = prompt_ids("short")
    for l in (-1, lang):
        a = oracle.build_prompt(ids, -1, l)
        b = oracle.build_icl_prompt(ids, lang=l)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("T,ns", [(5, 0), (20, 0), (20, 1), (3, 1)])
def test_icl_layout_lengths(oracle, T, ns):
    _, lang = lookup_ids(oracle.cfg, "aiden", "english")
    ids = prompt_ids("short")
    codes, sv = _inputs(oracle, T, spk=True)
    pre, tr = oracle.build_icl_prompt(ids, REF_IDS, codes, sv, lang, ns)
    head = 3 + (4 + 1 + 2) - 1                       # role + tag/lang/spk/pad rows
    Lt, Lc = (len(REF_IDS) - 5) + (len(ids) - 8) + 1, T + 1
    if ns:
        assert pre.shape[0] == head + Lt + Lc and tr.shape[0] == 1
    else:
        assert pre.shape[0] == head + Lc
        assert tr.shape[0] == (Lt - Lc if Lt > Lc else 1)
    pad = oracle.embed_text(151671)
    if ns or Lt <= Lc:
        np.testing.assert_array_equal(tr[0], pad)
    else:   # the text that did not fit under the reference frames, then tts_eos
        np.testing.assert_array_equal(tr[-1], oracle.embed_text(151673))
        nr = len(REF_IDS) - 5
        first = REF_IDS[3 + Lc] if Lc < nr else ids[3 + Lc - nr]
        np.testing.assert_array_equal(tr[0], oracle.embed_text(first))


# ------------------------------------------------------------------ GPU: HIP path vs oracle
CASES = {
    # name: (ref frames, spk vector, non_streaming, params)
    "icl_text_shorter": (20, False, 0, GREEDY),
    "icl_text_longer": (4, False, 0, GREEDY),
    "icl_nonstream_spk": (12, True, 1, GREEDY),
    "icl_spk_sampled": (12, True, 0, DEFAULT),
    "icl_long_prefill": (150, True, 0, GREEDY),     # ~160 prefill rows: the 64-row MFMA GEMM
    "xvec_only": (0, True, 0, GREEDY),
    "xvec_only_nonstream": (0, True, 1, GREEDY),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_voice_clone_vs_oracle(tts_tiny, oracle, name):
    from test_gpu_model import audio_close
    T, spk, ns, pp = CASES[name]
    _, lang = lookup_ids(oracle.cfg, "aiden", "english")
    ids = prompt_ids("short")
    codes, sv = _inputs(oracle, max(T, 1), seed=T, spk=spk)
    rc = codes if T > 0 else None
    fixed = 4
    m = tts_tiny
    m.set_params(max_tokens=4096, fixed=fixed, seed=42, **pp)
    a = m.generate_voice_clone(ids, REF_IDS if T else None, rc, sv, "english", ns)
    got = m.last_codes()
    pre, tr = oracle.build_icl_prompt(ids, REF_IDS if T else None, rc, sv, lang, ns)
    want, _ = oracle.generate_from_prompt(pre, tr, max_tokens=4096, fixed=fixed, seed=42, **pp)
    np.testing.assert_array_equal(got, want)
    full = oracle.codec_decode(np.concatenate([codes, want]) if T else want)
    tot = T + len(want)
    cut = int(T / tot * full.shape[0])
    audio_close(a, full[cut:])


@pytest.mark.gpu
def test_voice_clone_needs_codes_or_vector(tts_tiny):
    assert tts_tiny.generate_voice_clone(prompt_ids("short")) is None


@pytest.mark.gpu
def test_voice_clone_batch_slots_vs_oracle(tts_tiny, oracle):
    """Lock-step voice-clone batch (BASELINE C5): slots with different
    reference lengths, one x-vector-only slot and different prompts; every
    slot's audio equals the oracle's for its own prompt, reference and cut."""
    from test_gpu_model import audio_close
    prompts = [prompt_ids("short"), prompt_ids("p128", 1240), prompt_ids("p128", 1241)]
    refs = [_inputs(oracle, 9, seed=1, spk=True), _inputs(oracle, 30, seed=2), _inputs(oracle, 1, seed=3, spk=True)]
    codes = [refs[0][0], refs[1][0], None]
    spk = [refs[0][1], None, refs[2][1]]
    rids = [REF_IDS, REF_IDS[:3] + [4000, 4001] + REF_IDS[-2:], None]
    _, lang = lookup_ids(oracle.cfg, "aiden", "english")
    for pp in (GREEDY, DEFAULT):
        tts_tiny.set_params(max_tokens=4096, fixed=6, seed=42, **pp)
        rc, audio = tts_tiny.generate_voice_clone_batch(prompts, rids, codes, spk, ["english"] * 3)
        assert rc == 0
        for b in range(3):
            pre, tr = oracle.build_icl_prompt(prompts[b], rids[b], codes[b], spk[b], lang, 0)
            want, _ = oracle.generate_from_prompt(pre, tr, max_tokens=4096, fixed=6, seed=42, **pp)
            T = 0 if codes[b] is None else codes[b].shape[0]
            full = oracle.codec_decode(np.concatenate([codes[b], want]) if T else want)
            audio_close(audio[b], full[int(T / (T + len(want)) * full.shape[0]):])


@pytest.mark.gpu
@pytest.mark.parametrize("ns", [0, 1])
def test_cli_voice_clone_flags(tiny_dir, tts_tiny, oracle, ns):
    """qwen-tts --ref-codes / --ref-text / --xvector [--non-streaming] writes
    the same wav as the API call on the same inputs (text files in, as a
    caller of the audio encoders would write them)."""
    import os
    import subprocess
    import tempfile

    import qtts
    codes, sv = _inputs(oracle, 10, seed=5, spk=True)
    ids = prompt_ids("short")
    with tempfile.TemporaryDirectory() as d:
        cf, xf = os.path.join(d, "ref_codes.txt"), os.path.join(d, "xvec.txt")
        np.savetxt(cf, codes, fmt="%d")
        np.savetxt(xf, sv[None], fmt="%.9g")
        cmd = [qtts.CLI_PATH, "-d", tiny_dir, "-t", ",".join(map(str, ids)), "-l", "english", "-o",
               os.path.join(d, "cli.wav"), "--fixed-codec-tokens", "5", "--seed", "42", "--ref-codes", cf,
               "--ref-text", ",".join(map(str, REF_IDS)), "--xvector", xf] + (["--non-streaming"] if ns else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        tts_tiny.set_params(max_tokens=4096, fixed=5, seed=42)
        a = tts_tiny.generate_voice_clone(ids, REF_IDS, codes, sv, "english", ns)
        api = os.path.join(d, "api.wav")
        assert qtts.lib().qwen_tts_write_wav(api.encode(), a.ctypes.data_as(qtts._fp), len(a), 24000) == 0
        assert open(os.path.join(d, "cli.wav"), "rb").read() == open(api, "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [0, 7, 63])
def test_voice_clone_stream(tts_tiny, oracle, T):
    """Streaming voice clone: same codes as the oracle, chunks concatenate to
    the reference ++ generated decode from the exact frame boundary T * 1920
    (the reference frames are pushed through the streaming codec first).
    Runs on the session ctx after test_gpu_model's direct codec_stream_* use
    and the batch tests above (which re-allocate the decode state)."""
    from test_gpu_model import audio_close
    codes, sv = _inputs(oracle, max(T, 1), seed=11 + T, spk=True)
    rc = codes if T else None
    ids = prompt_ids("short")
    _, lang = lookup_ids(oracle.cfg, "aiden", "english")
    tts_tiny.set_params(max_tokens=4096, fixed=6, seed=42, **DEFAULT)
    chunks = []
    a = tts_tiny.generate_voice_clone_stream(ids, REF_IDS if T else None, rc, sv, "english", 0, chunk_frames=2,
                                             on_chunk=chunks.append)
    assert a is not None and chunks, "no audio / no chunks"
    assert len(chunks[0]) == 1920 and np.array_equal(np.concatenate(chunks), a)
    pre, tr = oracle.build_icl_prompt(ids, REF_IDS if T else None, rc, sv, lang, 0)
    want, _ = oracle.generate_from_prompt(pre, tr, max_tokens=4096, fixed=6, seed=42, **DEFAULT)
    np.testing.assert_array_equal(tts_tiny.last_codes(), want)
    full = oracle.codec_decode(np.concatenate([codes, want]) if T else want)
    audio_close(a, full[T * 1920:])
    # the non-streamed call cuts where the Python reference does,
    # int(T / tot * samples) (qwen3_tts_model.py:612-630), which is one sample
    # before the frame boundary for some (T, tot): the streamed chunks start at
    # T * 1920 because tot is unknown while streaming
    b = tts_tiny.generate_voice_clone(ids, REF_IDS if T else None, rc, sv, "english", 0)
    tot = T + len(want)
    off = T * 1920 - int(T / tot * (tot * 1920))   # the C host's (double) ref / tot * samples
    assert off in (0, 1) and len(b) == len(a) + off
    audio_close(b[off:], a)


@pytest.mark.gpu
def test_stream_after_state_realloc_same_ctx(tts_tiny, tiny_dir, oracle):
    """Regression (round-1 use-after-free): a codec stream is started, then a
    batch call re-allocates the decode state (and with it the codec GEMMs'
    split-K workspace), then a streaming voice clone reuses the stream's
    buffers on the same ctx.  Its chunks must be there and bit-equal to the
    same call on a fresh ctx."""
    import qtts
    codes, sv = _inputs(oracle, 7, seed=21, spk=True)
    ids = prompt_ids("short")
    tts_tiny.codec_stream([codes[:3], codes[3:]])                       # stream begun directly
    tts_tiny.set_params(max_tokens=4096, fixed=4, seed=42, **DEFAULT)
    rc, _ = tts_tiny.generate_voice_clone_batch([ids, ids], [REF_IDS, REF_IDS], [codes, codes], [sv, sv],
                                                ["english"] * 2)      # nb = 2: state re-allocated
    assert rc == 0

    def run(m):
        m.set_params(max_tokens=4096, fixed=6, seed=42, **DEFAULT)
        ch = []
        a = m.generate_voice_clone_stream(ids, REF_IDS, codes, sv, "english", 0, chunk_frames=2,
                                          on_chunk=ch.append)
        return a, ch, m.last_codes()

    a, ch, c = run(tts_tiny)
    assert a is not None and ch and np.array_equal(np.concatenate(ch), a)
    fresh = qtts.QwenTTS(tiny_dir)
    try:
        a2, ch2, c2 = run(fresh)
    finally:
        fresh.close()
    np.testing.assert_array_equal(c, c2)
    np.testing.assert_array_equal(a, a2)
