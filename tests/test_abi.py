"""The drop-in boundary on a CPU box: the C-ABI library loads, exports every
function include/*.h declares, has the ctx layout the ctypes mirror assumes,
its host-only code (WAV writer, CLI) matches the reference, and every compute
entry fails loudly - never silently on the CPU - when no HIP device exists."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT, golden, has_gpu

import qtts


def header_symbols(path):
    """Function (and extern variable) names declared at file scope."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"#ifdef __cplusplus.*?#endif", "", src, flags=re.S)
    src = re.sub(r"^\s*#[^\n]*", "", src, flags=re.M)
    out, depth, stmt = [], 0, ""
    for ch in src:
        if ch == "{":
            depth += 1
            if depth == 1:
                stmt = ""
            continue
        if ch == "}":
            depth -= 1
            continue
        if depth:
            continue
        if ch == ";":
            s = " ".join(stmt.split())
            stmt = ""
            if not s or s.startswith("typedef") or s.startswith("static"):
                continue
            m = re.match(r"^extern\s+[\w\s\*]+?\b(\w+)$", s)
            if m:
                out.append(m.group(1))
                continue
            m = re.search(r"\b(\w+)\s*\(", s)
            if m:
                out.append(m.group(1))
            continue
        stmt += ch
    return out


HEADERS = [os.path.join(ROOT, "include", h) for h in ("qwen_tts.h", "qtts_hip.h")]


def test_library_exports_every_declared_symbol():
    lib = qtts.lib()
    declared = [s for h in HEADERS for s in header_symbols(h)]
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # the Python mirror lists the same set
    assert sorted(set(declared)) == sorted(set(qtts.EXPORTS))


def test_ctx_layout_matches_ctypes_mirror():
    assert qtts.lib().qwen_tts_abi_sizeof_ctx() == C.sizeof(qtts.Ctx)


def test_reference_api_names_kept():
    """Every function of the reference's public header c/qwen_tts.h:448-502
    exists under the same name (the drop-in contract)."""
    ref_api = ["qwen_tts_load", "qwen_tts_free", "qwen_tts_set_progress_callback", "qwen_tts_generate",
               "qwen_tts_write_wav", "qwen_tts_talker_prefill", "qwen_tts_talker_forward",
               "qwen_tts_subtalker_generate", "qwen_tts_codec_decode"]
    declared = header_symbols(HEADERS[0])
    assert all(n in declared for n in ref_api)
    fields = {f for f, _ in qtts.Ctx._fields_}
    # ctx fields the reference CLI pokes / reads (c/main.c:214-223, 268-270, 306-312)
    for f in ("temperature", "subtalker_temperature", "top_k", "subtalker_top_k", "top_p", "subtalker_top_p",
              "repetition_penalty", "max_new_tokens", "fixed_codec_tokens", "sample_seed", "perf_total_ms",
              "perf_talker_ms", "perf_codec_ms", "perf_codec_tokens"):
        assert f in fields, f


def test_write_wav_bytes_match_reference():
    g = golden("wav.npz")
    x = g["wav_in"]
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "o.wav")
        rc = qtts.lib().qwen_tts_write_wav(p.encode(), x.ctypes.data_as(C.POINTER(C.c_float)), len(x), 24000)
        assert rc == 0
        got = np.frombuffer(open(p, "rb").read(), np.uint8)
    np.testing.assert_array_equal(got, g["wav_bytes"])


def test_write_wav_bad_path_returns_error():
    x = np.zeros(4, np.float32)
    rc = qtts.lib().qwen_tts_write_wav(b"/nonexistent-dir/x.wav", x.ctypes.data_as(C.POINTER(C.c_float)), 4, 24000)
    assert rc == -1


def test_cli_usage_lists_reference_flags():
    r = subprocess.run([qtts.CLI_PATH], capture_output=True, text=True)
    assert r.returncode != 0
    txt = r.stdout + r.stderr
    for flag in ("-d", "-t", "-f", "-s", "-l", "-o", "-v", "--temperature", "--top-k", "--top-p",
                 "--repetition-penalty", "--max-tokens", "--fixed-codec-tokens", "--seed",
                 "--subtalker-temperature", "--subtalker-top-k", "--subtalker-top-p", "--benchmark-runs",
                 "--benchmark-warmup"):
        assert flag in txt, flag


@pytest.mark.skipif(has_gpu(), reason="checks the no-device failure mode")
def test_no_device_fails_loudly(tiny_dir):
    """No CPU fallback: without a HIP device the product path refuses to run."""
    lib = qtts.lib()
    assert lib.qtts_hip_device_count() == 0
    r = subprocess.run([qtts.CLI_PATH, "-d", tiny_dir, "-t", "151644,77091,198,1,2,3,151645,198,151644,77091,198",
                        "-o", os.devnull], capture_output=True, text=True)
    assert r.returncode != 0 and "no HIP device" in r.stderr
    assert not lib.qwen_tts_load(tiny_dir.encode())
    with pytest.raises(RuntimeError):
        qtts.QwenTTS(tiny_dir)


def test_product_never_links_the_oracle():
    """The product library and CLI must not depend on oracle/ (test-only)."""
    for p in (qtts.LIB_PATH, qtts.CLI_PATH):
        r = subprocess.run(["ldd", p], capture_output=True, text=True)
        assert "oracle" not in r.stdout and "qtts_ref" not in r.stdout
        data = open(p, "rb").read()
        assert b"orc_talker_step" not in data and b"liboracle" not in data
