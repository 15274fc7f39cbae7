"""Shared fixtures.  `-m "not gpu"` runs on any CPU box; `-m gpu` needs an
MI355X and drives the HIP path through the C-ABI (qwen3-tts-c_amd/qtts.py).

The oracle (oracle/_port/liboracle.so) and, where it was built, the reference
build (oracle/_ref/libqtts_ref.so) are the checkers; the golden fixtures in
tests/golden/ were produced by the reference build (tests/golden/make_golden.py).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "qwen3-tts-c_amd")
GOLDEN = os.path.join(HERE, "golden")
for p in (HERE, os.path.join(ROOT, "tools"), PKG, ROOT, os.path.join(ROOT, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)

MODEL_ROOT = os.environ.get("QTTS_TEST_MODELS", "/tmp/qtts_test_models")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: full-size (1.7B) property tests")


def _ensure_built():
    """Build the oracle port and the product library if the tree has no
    prebuilt copies (the GPU box receives the prebuilt .so files)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_port", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "port"], check=True)
    if not os.path.exists(os.path.join(PKG, "lib", "libqwen_tts_amd.so")):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)


_ensure_built()


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def model_dir(preset, **overrides):
    from synth_model import ensure_model
    tag = preset + "".join(f"_{k}{v}" for k, v in sorted(overrides.items()))
    return ensure_model(os.path.join(MODEL_ROOT, tag), preset, seed=0, overrides=overrides or None)


@pytest.fixture(scope="session")
def tiny_dir():
    return model_dir("tiny")


@pytest.fixture(scope="session")
def tiny_eq_dir():
    return model_dir("tiny_eq")


@pytest.fixture(scope="session")
def tiny_eos_dir():
    return model_dir("tiny", eos_gain=manifest()["eos_gain"])


@pytest.fixture(scope="session")
def oracle(tiny_dir):
    from oracle_py import Oracle
    o = Oracle(tiny_dir)
    yield o
    o.close()


def has_gpu():
    try:
        import qtts
        return qtts.lib().qtts_hip_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """The HIP device must be there for -m gpu tests: fail, do not skip."""
    import torch
    import qtts
    n = qtts.lib().qtts_hip_device_count()
    assert n > 0 and torch.cuda.is_available(), "no HIP device visible to the gpu tests"
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def tts_tiny(gpu, tiny_dir):
    import qtts
    m = qtts.QwenTTS(tiny_dir)
    yield m
    m.close()
