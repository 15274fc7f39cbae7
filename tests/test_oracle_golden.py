"""The CPU oracle (oracle/qtts_oracle.c) against the reference's own outputs
(tests/golden/*.npz, made by tests/golden/make_golden.py from the reference
c/ sources compiled unmodified).  This pins the oracle: every later GPU
parity claim is a claim against it.

The oracle restates the reference's scalar arithmetic in the same order
(-ffp-contract=off), so everything here is bit-exact.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import golden, manifest
from oracle_py import Oracle, GREEDY, DEFAULT, fptr
from synth_model import prompt_ids

K = golden("kernels.npz")


def _lib():
    from oracle_py import _lib_oracle
    return _lib_oracle()


def model_hashes(md):
    return {rel: hashlib.sha256(open(os.path.join(md, rel), "rb").read()).hexdigest()
            for rel in ("config.json", "model.safetensors", "speech_tokenizer/config.json",
                        "speech_tokenizer/model.safetensors")}


def test_model_generator_reproduces_golden_models(tiny_dir, tiny_eq_dir, tiny_eos_dir):
    man = manifest()["models"]
    assert model_hashes(tiny_dir) == man["tiny"]
    assert model_hashes(tiny_eq_dir) == man["tiny_eq"]
    assert model_hashes(tiny_eos_dir) == man["tiny_eos"]


@pytest.mark.parametrize("i", [0, 1, 2])
def test_matvec_bf16(i):
    A, x, y = K[f"matvec{i}_A"], K[f"matvec{i}_x"], K[f"matvec{i}_y"]
    out = np.zeros_like(y)
    _lib().orc_matvec_bf16(fptr(out), A.ctypes.data, fptr(x), A.shape[0], A.shape[1])
    np.testing.assert_array_equal(out, y)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_rms_norm(i):
    x, w, y = K[f"rms{i}_x"], K[f"rms{i}_w"], K[f"rms{i}_y"]
    out = np.zeros_like(y)
    _lib().orc_rmsnorm(fptr(out), fptr(x), fptr(w), len(x), 1e-6)
    np.testing.assert_array_equal(out, y)


def test_softmax():
    x = K["softmax_x"].copy()
    _lib().orc_softmax(fptr(x), len(x))
    np.testing.assert_array_equal(x, K["softmax_y"])


@pytest.mark.parametrize("i", range(5))
def test_causal_conv1d(i):
    ci, co, k, L, d, g = (int(v) for v in K[f"conv{i}_cfg"])
    out = np.zeros((co, L), np.float32)
    _lib().orc_conv1d(fptr(out), fptr(K[f"conv{i}_x"]), fptr(K[f"conv{i}_w"]), K[f"conv{i}_b"].ctypes.data,
                      ci, co, k, L, d, g)
    np.testing.assert_array_equal(out, K[f"conv{i}_y"])


@pytest.mark.parametrize("i", range(5))
def test_transposed_conv1d(i):
    ci, co, k, s, L = (int(v) for v in K[f"tconv{i}_cfg"])
    out = np.zeros((co, L * s), np.float32)
    _lib().orc_tconv1d(fptr(out), fptr(K[f"tconv{i}_x"]), fptr(K[f"tconv{i}_w"]), K[f"tconv{i}_b"].ctypes.data,
                       ci, co, k, s, L)
    np.testing.assert_array_equal(out, K[f"tconv{i}_y"])


def test_snake_beta():
    x = K["snake_x"]
    out = np.zeros_like(x)
    _lib().orc_snake(fptr(out), fptr(x), fptr(K["snake_a"]), fptr(K["snake_ib"]), x.shape[0], x.shape[1])
    np.testing.assert_array_equal(out, K["snake_y"])


@pytest.mark.parametrize("V", [2048, 3072])
def test_sampler_draws_and_rng(V):
    lib = _lib()
    lg, meta, fm, rs = K[f"samp{V}_logits"], K[f"samp{V}_meta"], K[f"samp{V}_fmeta"], K[f"samp{V}_rng"]
    for i in range(len(lg)):
        st = np.array([rs[i, 0]], np.uint32).view(np.float32).copy()
        r = lib.orc_sample(fptr(lg[i].copy()), V, int(meta[i, 0]), float(fm[i, 0]), float(fm[i, 1]), fptr(st))
        assert r == meta[i, 1], (i, r, meta[i])
        assert st.view(np.uint32)[0] == rs[i, 1], i


S = golden("stages_tiny.npz")


def test_stage_prefill_step(oracle):
    h = oracle.prefill(S["prefill_embeds"])
    np.testing.assert_array_equal(h, S["prefill_hidden"])
    lg, hid = oracle.step(S["step_embed"])
    np.testing.assert_array_equal(lg, S["step_logits"])
    np.testing.assert_array_equal(hid, S["step_hidden"])


def test_stage_subtalker(oracle):
    hid = S["step_hidden"]
    np.testing.assert_array_equal(oracle.subtalker(hid, 5, top_k=1, top_p=1.0, temp=1.0), S["st_greedy_codes"])
    np.testing.assert_array_equal(oracle.subtalker(hid, 5, top_k=50, top_p=1.0, temp=0.9, seed=42),
                                  S["st_sampled_codes"])


def test_stage_codec(oracle):
    a = oracle.codec_decode(S["codec_codes"])
    np.testing.assert_array_equal(a, S["codec_audio"])


E = golden("e2e_tiny.npz")
RUNS = {  # name -> (model fixture, sampling, fixed, max_tokens, seed)
    "greedy": ("tiny_dir", GREEDY, 16, 4096, 42),
    "sampled": ("tiny_dir", DEFAULT, 16, 4096, 42),
    "eos": ("tiny_dir", DEFAULT, 0, 32, 42),
    "eosg": ("tiny_eos_dir", GREEDY, 0, 32, 7),
    "eoss": ("tiny_eos_dir", DEFAULT, 0, 32, 7),
    "resample": ("tiny_eos_dir", DEFAULT, 24, 4096, 7),
    "eq_greedy": ("tiny_eq_dir", GREEDY, 16, 4096, 42),
}


@pytest.mark.parametrize("name", sorted(RUNS))
def test_e2e_codes_and_audio(name, request):
    fx, pp, fixed, mx, seed = RUNS[name]
    md = request.getfixturevalue(fx)
    o = Oracle(md)
    from qtts_io import lookup_ids
    spk, lang = lookup_ids(o.cfg, "aiden", "english")
    codes, stop = o.generate_codes(prompt_ids("short"), spk, lang, max_tokens=mx, fixed=fixed, seed=seed, **pp)
    np.testing.assert_array_equal(codes, E[f"{name}_codes"])
    audio = o.codec_decode(codes)
    np.testing.assert_array_equal(audio, E[f"{name}_audio"])
    o.close()


def test_e2e_fixture_covers_stops():
    st = manifest()["stop_tokens"]
    assert st["eosg"] < 32 and st["eoss"] < 32, "EOS-stop runs must stop on EOS"
    assert st["eos"] == 32, "max_tokens stop"
    assert manifest()["resample_eos_draws"] >= 1, "fixed-mode EOS re-sample must be exercised"
