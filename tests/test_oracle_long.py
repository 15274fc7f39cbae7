"""The oracle port against the long-context reference fixtures (CPU only).

tests/golden/long_hd128.npz comes from the reference c/ build
(tests/golden/make_golden_long.py) on the `hd128` synthetic model: the
talker's real attention shape (NH 16 / KV 8 / HD 128) decoding 640 frames
(positions up to ~680) and a 600-row prefill followed by 4 decode steps.  The
oracle must reproduce it bit-exactly before it checks the GPU at those
lengths (tests/test_gpu_long.py).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, model_dir
from make_golden_long import model_hashes, prefill_inputs
from oracle_py import DEFAULT, Oracle
from qtts_io import lookup_ids


@pytest.fixture(scope="module")
def hd128():
    md = model_dir("hd128")
    man = json.load(open(os.path.join(GOLDEN, "long_manifest.json")))
    assert model_hashes(md) == man["models"]["hd128"], "synthetic hd128 model no longer reproduces"
    o = Oracle(md)
    yield o, np.load(os.path.join(GOLDEN, "long_hd128.npz")), man["hd128"]
    o.close()


def test_oracle_long_decode_bit_exact(hd128):
    o, g, m = hd128
    s, l = lookup_ids(o.cfg, "aiden", "english")
    codes, _ = o.generate_codes(g["prompt_ids"], s, l, max_tokens=4096, fixed=m["frames"], seed=m["seed"],
                                **DEFAULT)
    np.testing.assert_array_equal(codes, g["decode_codes"])
    a = o.codec_decode(codes)
    assert a.shape[0] == int(g["decode_audio_len"])
    np.testing.assert_array_equal(a[::m["audio_stride"]], g["decode_audio_sub"])
    np.testing.assert_array_equal(a[-1920:], g["decode_audio_last"])


def test_oracle_long_prefill_and_steps_bit_exact(hd128):
    o, g, m = hd128
    emb, steps = prefill_inputs(o.cfg["H"], m["prefill_seed"])
    np.testing.assert_array_equal(o.prefill(emb), g["prefill_hidden"])
    for i in range(m["prefill_steps"]):
        lg, hid = o.step(steps[i])
        np.testing.assert_array_equal(lg, g["step_logits"][i])
        np.testing.assert_array_equal(hid, g["step_hidden"][i])


def test_long_fixtures_describe_the_bench_workloads():
    """The round-5 reference fixtures hold what bench.py runs (no compute):
    long_17b_b8bench = rank 0's 8 utterances of `bench.py --batch 8`
    (rank_prompt_seeds), long_eos17 = the P128 prompts of bench.py --eos's
    model with each slot's codes up to the reference's EOS stop (and
    long_eos17q three more of them)."""
    import bench
    from synth_model import prompt_ids
    man = json.load(open(os.path.join(GOLDEN, "long_manifest.json")))
    g = np.load(os.path.join(GOLDEN, "long_17b_b8bench.npz"))
    m = man["b8bench"]
    assert m["prompt_seeds"] == bench.rank_prompt_seeds(0, 8) and m["frames"] == 128 and m["speakers"] == ["aiden"] * 8
    for b, sd in enumerate(m["prompt_seeds"]):
        n = int(g["prompt_len"][b])
        np.testing.assert_array_equal(g["prompt_ids"][b, :n], prompt_ids("p128", sd))
    assert g["codes"].shape == (8, 128, 16) and g["codes"].min() >= 0 and g["codes"].max() < 3072
    e = np.load(os.path.join(GOLDEN, "long_eos17.npz"))
    m = man["eos17"]
    assert m["eos_gain"] == bench.EOS_GAIN and m["max_tokens"] > max(int(x) for x in e["stop_step"])
    for b, sd in enumerate(m["prompt_seeds"]):
        n, T = int(e["prompt_len"][b]), int(e["stop_step"][b])
        np.testing.assert_array_equal(e["prompt_ids"][b, :n], prompt_ids("p128", sd))
        assert (e["codes"][b, :T] >= 0).all() and (e["codes"][b, T:] == -1).all()
    assert len(set(int(x) for x in e["stop_step"])) == len(m["prompt_seeds"])   # the batch test needs rows stopping apart
    # long_eos17q: three more utterances of the same model for the work-queue test
    q = np.load(os.path.join(GOLDEN, "long_eos17q.npz"))
    m = man["eos17q"]
    assert m["eos_gain"] == bench.EOS_GAIN and m["max_tokens"] > max(int(x) for x in q["stop_step"])
    for b, sd in enumerate(m["prompt_seeds"]):
        n, T = int(q["prompt_len"][b]), int(q["stop_step"][b])
        np.testing.assert_array_equal(q["prompt_ids"][b, :n], prompt_ids("p128", sd))
        assert (q["codes"][b, :T] >= 0).all() and (q["codes"][b, T:] == -1).all()


def test_long_capacity_fixtures_extend_the_shorter_runs():
    """The long-capacity reference fixtures (no compute): long_hd128_max (4096
    frames, fixed) starts with the 640-frame run of long_hd128, and
    long_17b_1100 (1100 frames, fixed) with the bench workload of long_17b --
    the same prompt, seed and sampling, so the reference drew the same codes
    for the shared frames (fixed mode only re-draws an EOS, never a code)."""
    man = json.load(open(os.path.join(GOLDEN, "long_manifest.json")))
    p = os.path.join(GOLDEN, "long_hd128_max.npz")
    if os.path.exists(p):
        a, b = np.load(p), np.load(os.path.join(GOLDEN, "long_hd128.npz"))
        assert a["codes"].shape == (man["hd128max"]["frames"], 16)
        np.testing.assert_array_equal(a["codes"][:man["hd128"]["frames"]], b["decode_codes"])
        np.testing.assert_array_equal(a["audio_first"], b["decode_audio_first"])
        np.testing.assert_array_equal(a["prompt_ids"], b["prompt_ids"])
    p = os.path.join(GOLDEN, "long_17b_1100.npz")
    if os.path.exists(p):
        a, b = np.load(p), np.load(os.path.join(GOLDEN, "long_17b.npz"))
        assert a["codes"].shape == (man["k1100"]["frames"], 16)
        np.testing.assert_array_equal(a["codes"][:man["1.7b"]["frames"]], b["codes"])
        np.testing.assert_array_equal(a["audio_first"], b["audio"][:1920])
