#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE build.

TEST INFRASTRUCTURE.  Runs in the build container only (needs
oracle/_ref/libqtts_ref.so, i.e. `make -C oracle ref` against the unmodified
/root/reference/c sources).  The committed .npz files are data: seeded inputs
and the reference's outputs for them; nothing of the reference travels.

  python tests/golden/make_golden.py          # rewrites tests/golden/*.npz + manifest.json

Fixtures
  kernels.npz       per-kernel I/O of the reference kernel layer
                    (c/qwen_tts_kernels.h): matvec_bf16, rms_norm, softmax,
                    causal_conv1d (dense d=1/3/9, depthwise, k=1), transposed
                    conv1d (the vocoder's stride/kernel pairs), snake_beta,
                    sample_top_k (logits, params, RNG state in/out, id out).
  stages_tiny.npz   stage functions (c/qwen_tts.h:483-502) on the `tiny`
                    synthetic model: prefill hidden, one decode step's logits
                    and hidden, sub-talker codes (greedy + sampled), codec
                    waveform for random codes.
  e2e_tiny.npz      qwen_tts_generate on the short prompt (test/tokens_great_power.txt,
                    SURVEY.md 4): greedy / seed-42 sampled fixed-length runs,
                    an EOS-mode run (codes + stop step) and their waveforms;
                    the same greedy run on `tiny_eq` (no sub-talker input
                    projection).
                    An EOS-heavy variant of `tiny` (EOS logit row x EOS_GAIN)
                    adds EOS-stopped runs and a fixed-length run whose EOS draws
                    are re-sampled.
  wav.npz           bytes of qwen_tts_write_wav for a short signal; PCM of the
                    reference CLI's WAV for the greedy EOS run (flags of
                    test/test_eos_regression.py) whose stderr Stop line is in
                    manifest.json.
  manifest.json     SHA-256 of the synthetic model files the fixtures were
                    made from (tests check the generator still reproduces them).
"""
import ctypes as C
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

from oracle_py import RefLib, REF_SO, GREEDY, DEFAULT, fptr, iptr  # noqa: E402
from qtts_io import f32_to_bf16  # noqa: E402
from synth_model import ensure_model, prompt_ids  # noqa: E402

E2E_FRAMES = 16
EOS_MAX = 32
EOS_GAIN = 3.0


def model_hashes(md):
    out = {}
    for rel in ("config.json", "model.safetensors", "speech_tokenizer/config.json",
                "speech_tokenizer/model.safetensors"):
        with open(os.path.join(md, rel), "rb") as f:
            out[rel] = hashlib.sha256(f.read()).hexdigest()
    return out


def kernel_fixtures(lib, rng):
    g = {}
    # matvec_bf16 (K.c:95): rows x cols bf16 weights, fp32 x
    for i, (R, Cc) in enumerate([(96, 128), (64, 1024), (40, 3072)]):
        A = f32_to_bf16(rng.standard_normal((R, Cc)).astype(np.float32) * 0.05)
        x = rng.standard_normal(Cc).astype(np.float32)
        y = np.zeros(R, np.float32)
        lib.kernel_matvec_bf16(fptr(y), A.ctypes.data, fptr(x), R, Cc)
        g[f"matvec{i}_A"], g[f"matvec{i}_x"], g[f"matvec{i}_y"] = A, x, y
    # rms_norm (K.c:27)
    for i, n in enumerate([128, 1024, 2048]):
        x = rng.standard_normal(n).astype(np.float32) * 3
        w = (1 + 0.1 * rng.standard_normal(n)).astype(np.float32)
        y = np.zeros(n, np.float32)
        lib.kernel_rms_norm(fptr(y), fptr(x), fptr(w), n, C.c_float(1e-6))
        g[f"rms{i}_x"], g[f"rms{i}_w"], g[f"rms{i}_y"] = x, w, y
    # softmax (K.c:371)
    x = (rng.standard_normal(257) * 4).astype(np.float32)
    g["softmax_x"] = x.copy()
    lib.kernel_softmax(fptr(x), 257)
    g["softmax_y"] = x
    # causal conv1d (K.c:659): (ci, co, k, L, dilation, groups)
    convs = [(16, 24, 7, 40, 1, 1), (12, 12, 7, 33, 3, 1), (8, 8, 7, 50, 9, 1),
             (16, 16, 7, 37, 1, 16), (24, 16, 1, 29, 1, 1)]
    for i, (ci, co, k, L, d, gr) in enumerate(convs):
        x = rng.standard_normal((ci, L)).astype(np.float32)
        w = (rng.standard_normal((co, ci // gr, k)) / np.sqrt(ci // gr * k)).astype(np.float32)
        b = (0.1 * rng.standard_normal(co)).astype(np.float32)
        y = np.zeros((co, L), np.float32)
        lib.kernel_causal_conv1d(fptr(y), fptr(x), fptr(w), b.ctypes.data, ci, co, k, L, d, gr)
        g[f"conv{i}_cfg"] = np.array([ci, co, k, L, d, gr], np.int32)
        g[f"conv{i}_x"], g[f"conv{i}_w"], g[f"conv{i}_b"], g[f"conv{i}_y"] = x, w, b, y
    # transposed conv1d (K.c:873): (ci, co, k, stride, L) - the vocoder's k/s pairs
    tconvs = [(16, 16, 2, 2, 9), (24, 12, 16, 8, 5), (12, 8, 10, 5, 7), (8, 8, 8, 4, 6), (8, 4, 6, 3, 11)]
    for i, (ci, co, k, s, L) in enumerate(tconvs):
        x = rng.standard_normal((ci, L)).astype(np.float32)
        w = (rng.standard_normal((ci, co, k)) / np.sqrt(ci)).astype(np.float32)
        b = (0.1 * rng.standard_normal(co)).astype(np.float32)
        y = np.zeros(co * (L * s + k), np.float32)    # flat [co, out_length]
        ol = C.c_int(0)
        lib.kernel_transposed_conv1d(fptr(y), fptr(x), fptr(w), b.ctypes.data, ci, co, k, s, L, C.byref(ol))
        g[f"tconv{i}_cfg"] = np.array([ci, co, k, s, L], np.int32)
        g[f"tconv{i}_x"], g[f"tconv{i}_w"], g[f"tconv{i}_b"] = x, w, b
        g[f"tconv{i}_y"] = y[: co * ol.value].reshape(co, ol.value).copy()
    # snake_beta (K.c:251) on pre-processed alpha' / inv_beta'
    Cc, L = 12, 77
    x = (rng.standard_normal((Cc, L)) * 2).astype(np.float32)
    a = np.exp(0.3 * rng.standard_normal(Cc)).astype(np.float32)
    ib = (1.0 / (np.exp(0.3 * rng.standard_normal(Cc)) + 1e-9)).astype(np.float32)
    y = np.zeros((Cc, L), np.float32)
    lib.kernel_snake_beta(fptr(y), fptr(x), fptr(a), fptr(ib), Cc, L)
    g["snake_x"], g["snake_a"], g["snake_ib"], g["snake_y"] = x, a, ib, y
    # sampler (K.c:407): talker (3072) and sub-talker (2048) vocab sizes
    for V, n in ((2048, 24), (3072, 12)):
        lg = np.zeros((n, V), np.float32)
        meta = np.zeros((n, 2), np.int32)           # top_k, result
        fm = np.zeros((n, 2), np.float32)           # top_p, temperature
        rs = np.zeros((n, 2), np.uint32)            # rng in / out (float bits)
        for i in range(n):
            l = (rng.standard_normal(V) * 3).astype(np.float32)
            if i % 5 == 0:
                l[rng.integers(0, V, 24)] = l.max()   # ties at the top
            if i % 7 == 3:
                l[rng.integers(0, V, 64)] = -np.inf    # suppressed entries
            k = [1, 50, 7, 300, 0, 50][i % 6]
            tp = [1.0, 0.8, 1.0, 0.95, 1.0, 0.5][i % 6]
            temp = [1.0, 0.9, 0.7, 1.3, 0.9, 0.9][i % 6]
            st = np.array([np.float32(17 + 31 * i)], np.float32)
            rin = st.view(np.uint32)[0]
            r = lib.kernel_sample_top_k(fptr(l), V, k, C.c_float(tp), C.c_float(temp), fptr(st))
            lg[i], meta[i], fm[i] = l, (k, r), (tp, temp)
            rs[i] = (rin, st.view(np.uint32)[0])
        g[f"samp{V}_logits"], g[f"samp{V}_meta"], g[f"samp{V}_fmeta"], g[f"samp{V}_rng"] = lg, meta, fm, rs
    return g


def stage_fixtures(md, rng):
    ref = RefLib(md)
    c = ref.cfg
    g = {}
    P = 9
    emb = (rng.standard_normal((P, c["H"])) * 0.5).astype(np.float32)
    g["prefill_embeds"] = emb
    g["prefill_hidden"] = ref.prefill(emb)
    e1 = (rng.standard_normal(c["H"]) * 0.5).astype(np.float32)
    lg, hid = ref.step(e1)
    g["step_embed"], g["step_logits"], g["step_hidden"] = e1, lg, hid
    # sub-talker greedy / sampled on the decode hidden, first code 5
    ref.set_params(**GREEDY)
    g["st_greedy_codes"] = ref.subtalker(hid, 5)
    ref.set_params(seed=42, **DEFAULT)
    g["st_sampled_codes"] = ref.subtalker(hid, 5)
    codes = rng.integers(0, c["ccb"], size=(24, c["cq"])).astype(np.int32)
    codes[3, 2] = c["ccb"] + 7       # out of range -> zero contribution (Cd.c:150-160)
    g["codec_codes"] = codes
    g["codec_audio"] = ref.codec_decode(codes)
    ref.close()
    return g


def e2e_fixtures(md, md_eq, md_eos):
    g = {}
    ids = np.array(prompt_ids("short"), np.int32)
    g["prompt_ids"] = ids
    ref = RefLib(md)
    runs = [("greedy", GREEDY, E2E_FRAMES, 4096), ("sampled", DEFAULT, E2E_FRAMES, 4096), ("eos", DEFAULT, 0, EOS_MAX)]
    for name, pp, fixed, mx in runs:
        ref.set_params(max_tokens=mx, fixed=fixed, seed=42, **pp)
        audio = ref.generate(ids, "aiden", "english")
        g[f"{name}_codes"] = ref.recorded_codes()
        g[f"{name}_audio"] = audio if audio is not None else np.zeros(0, np.float32)
        g[f"{name}_tokens"] = np.array(ref.perf()["tokens"], np.int32)
        hid, cod = ref.recorded_subtalker()
        g[f"{name}_st_hidden0"] = hid[:2].copy()
    ref.close()
    # EOS-heavy model (codec_head EOS row x EOS_GAIN): EOS stops under greedy
    # and sampling; in fixed mode the EOS draws are re-sampled (Q.c:1315-1321)
    ref = RefLib(md_eos)
    runs = [("eosg", GREEDY, 0, EOS_MAX), ("eoss", DEFAULT, 0, EOS_MAX), ("resample", DEFAULT, 24, 4096)]
    for name, pp, fixed, mx in runs:
        ref.set_params(max_tokens=mx, fixed=fixed, seed=7, **pp)
        audio = ref.generate(ids, "aiden", "english")
        g[f"{name}_codes"] = ref.recorded_codes()
        g[f"{name}_audio"] = audio if audio is not None else np.zeros(0, np.float32)
        g[f"{name}_tokens"] = np.array(ref.perf()["tokens"], np.int32)
        if name == "resample":
            eos = ref.cfg["eos"]
            g["resample_eos_draws"] = np.array(sum(1 for r in ref.recorded_samples()
                                                   if r["vocab"] == ref.cfg["V"] and r["result"] == eos), np.int32)
    ref.close()
    ref = RefLib(md_eq)
    ref.set_params(max_tokens=4096, fixed=E2E_FRAMES, seed=42, **GREEDY)
    a = ref.generate(ids, "aiden", "english")
    g["eq_greedy_codes"] = ref.recorded_codes()
    g["eq_greedy_audio"] = a
    ref.close()
    return g


def wav_fixture(lib):
    t = np.arange(480, dtype=np.float32)
    x = (np.sin(t * 0.05) * 1.2).astype(np.float32)   # includes clipping
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.wav")
        lib.qwen_tts_write_wav(p.encode(), fptr(x), len(x), 24000)
        data = np.frombuffer(open(p, "rb").read(), np.uint8).copy()
    return {"wav_in": x, "wav_bytes": data}


def cli_fixture(md_eos):
    """The reference CLI (c/main.c) on the EOS model with the greedy flags of
    test/test_eos_regression.py: its stderr Stop/Generated lines and WAV."""
    import re
    import subprocess
    cli = os.path.join(os.path.dirname(REF_SO), "qwen-tts")
    ids = ",".join(str(i) for i in prompt_ids("short"))
    with tempfile.TemporaryDirectory() as d:
        wav = os.path.join(d, "o.wav")
        args = ["-s", "aiden", "-l", "english", "--top-k", "1", "--temperature", "1.0", "--repetition-penalty", "1.0",
                "--subtalker-top-k", "1", "--subtalker-temperature", "1.0", "--max-tokens", "32", "-v"]
        r = subprocess.run([cli, "-d", md_eos, "-t", ids, "-o", wav] + args, capture_output=True, text=True,
                           check=True)
        pcm = np.frombuffer(open(wav, "rb").read()[44:], np.int16).copy()
    stop = re.search(r"Stop: (eos|max_tokens) at step (\d+)", r.stderr)
    gen = re.search(r"Generated (\d+) codec tokens", r.stderr)
    # the codec's -v lines (c/qwen_tts_codec.c:598-599, 740-742)
    codec = [ln for ln in r.stderr.splitlines() if ln.startswith("Codec decode:") and "timesteps" in ln
             or ln.startswith("Codec decode complete:")]
    meta = {"args": args, "stop_line": stop.group(0), "generated": int(gen.group(1)), "codec_lines": codec}
    return {"cli_eos_pcm": pcm}, meta


def main():
    if not os.path.exists(REF_SO):
        sys.exit(f"{REF_SO} missing: run `make -C oracle ref` first")
    lib = C.CDLL(REF_SO)
    fp, ip, vp = C.POINTER(C.c_float), C.POINTER(C.c_int), C.c_void_p
    lib.kernel_sample_top_k.restype = C.c_int
    lib.kernel_sample_top_k.argtypes = [fp, C.c_int, C.c_int, C.c_float, C.c_float, fp]
    lib.kernel_matvec_bf16.argtypes = [fp, vp, fp, C.c_int, C.c_int]
    lib.kernel_rms_norm.argtypes = [fp, fp, fp, C.c_int, C.c_float]
    lib.kernel_softmax.argtypes = [fp, C.c_int]
    lib.kernel_causal_conv1d.argtypes = [fp, fp, fp, vp] + [C.c_int] * 6
    lib.kernel_transposed_conv1d.argtypes = [fp, fp, fp, vp] + [C.c_int] * 5 + [ip]
    lib.kernel_snake_beta.argtypes = [fp, fp, fp, fp, C.c_int, C.c_int]
    lib.qwen_tts_write_wav.argtypes = [C.c_char_p, C.POINTER(C.c_float), C.c_int, C.c_int]
    rng = np.random.Generator(np.random.PCG64(20261015))
    md = ensure_model("/tmp/qtts_golden_tiny", "tiny")
    md_eq = ensure_model("/tmp/qtts_golden_tiny_eq", "tiny_eq")
    md_eos = ensure_model("/tmp/qtts_golden_tiny_eos", "tiny", overrides={"eos_gain": EOS_GAIN})
    np.savez_compressed(os.path.join(HERE, "kernels.npz"), **kernel_fixtures(lib, rng))
    np.savez_compressed(os.path.join(HERE, "stages_tiny.npz"), **stage_fixtures(md, rng))
    e = e2e_fixtures(md, md_eq, md_eos)
    np.savez_compressed(os.path.join(HERE, "e2e_tiny.npz"), **e)
    w = wav_fixture(lib)
    cli, cli_meta = cli_fixture(md_eos)
    w.update(cli)
    np.savez_compressed(os.path.join(HERE, "wav.npz"), **w)
    man = {"generator": "tests/golden/make_golden.py",
           "reference": "oracle/_ref/libqtts_ref.so built from /root/reference/c by oracle/Makefile "
                        "(scalar + OpenMP, no BLAS)",
           "models": {"tiny": model_hashes(md), "tiny_eq": model_hashes(md_eq),
                      "tiny_eos": model_hashes(md_eos)}, "eos_gain": EOS_GAIN,
           "e2e_frames": E2E_FRAMES, "eos_max_tokens": EOS_MAX,
           "stop_tokens": {k: int(e[k + "_tokens"]) for k in ("greedy", "sampled", "eos", "eosg", "eoss", "resample")},
           "resample_eos_draws": int(e["resample_eos_draws"]),
           "cli_eos": cli_meta}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1)
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
