"""Live cross-check of the CPU restatement against the reference build on
fresh seeded inputs (beyond the committed goldens).  Skipped where
oracle/_ref/libqtts_ref.so was not built (it is built from /root/reference by
`make -C oracle ref`; the .so travels with the tree)."""
import os

import numpy as np
import pytest

from oracle_py import REF_SO, Oracle, RefLib, DEFAULT, GREEDY, fptr
from qtts_io import lookup_ids
from synth_model import prompt_ids

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference build not present")


def test_sampler_random_draws(oracle):
    import ctypes as C
    lib = C.CDLL(REF_SO)
    lib.kernel_sample_top_k.restype = C.c_int
    lib.kernel_sample_top_k.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_float, C.c_float,
                                        C.POINTER(C.c_float)]
    rng = np.random.default_rng(99)
    for i in range(150):
        V = [2048, 3072, 1000][i % 3]
        lg = (rng.standard_normal(V) * rng.uniform(0.5, 6)).astype(np.float32)
        if i % 4 == 0:
            lg[rng.integers(0, V, 40)] = lg.max()
        k, tp, t = int(rng.integers(0, 400)), float(rng.choice([1.0, 0.9, 0.6])), float(rng.uniform(0.5, 1.5))
        s1 = np.array([np.float32(rng.integers(1, 10**6))], np.float32)
        s2 = s1.copy()
        a = lib.kernel_sample_top_k(fptr(lg.copy()), V, k, tp, t, fptr(s1))
        b = oracle.lib.orc_sample(fptr(lg.copy()), V, k, tp, t, fptr(s2))
        assert a == b and s1.view(np.uint32)[0] == s2.view(np.uint32)[0], i


@pytest.mark.parametrize("seed,pp,fixed", [(3, DEFAULT, 8), (11, GREEDY, 6), (5, dict(DEFAULT, top_p=0.8), 6)])
def test_e2e_p128_codes_and_audio(tiny_dir, seed, pp, fixed):
    ids = prompt_ids("p128", seed=1234 + seed)
    ref = RefLib(tiny_dir)
    ref.set_params(max_tokens=4096, fixed=fixed, seed=seed, **pp)
    audio_r = ref.generate(ids, "serena", "chinese")
    codes_r = ref.recorded_codes()
    ref.close()
    o = Oracle(tiny_dir)
    spk, lang = lookup_ids(o.cfg, "serena", "chinese")
    codes_o, _ = o.generate_codes(ids, spk, lang, max_tokens=4096, fixed=fixed, seed=seed, **pp)
    audio_o = o.codec_decode(codes_o)
    o.close()
    np.testing.assert_array_equal(codes_o, codes_r)
    np.testing.assert_array_equal(audio_o, audio_r)
