"""The divergence classifier's draw analysis (tests/divergence.py) against the
oracle's sampler (K.c:407-484 restated, pinned to the reference): the same
drawn id, and a logit perturbation just above the reported flip distance,
built adversarially, changes the draw while one just below never does."""
import ctypes as C

import numpy as np

from divergence import _u, flip_distance
from oracle_py import _lib_oracle, fptr


def _orc_draw(lib, lg, k, T, bits):
    st = np.array([bits], np.uint32).view(np.float32).copy()
    return lib.orc_sample(fptr(np.ascontiguousarray(lg, np.float32)), lg.shape[0], k, C.c_float(1.0), C.c_float(T),
                          fptr(st))


def test_uniform_matches_oracle():
    lib = _lib_oracle()
    for bits in (1109917696, 0x3F800000, 12345, 0xFFFFFFFF, 7):
        st = np.array([bits], np.uint32).view(np.float32).copy()
        assert np.float32(lib.orc_rand_uniform(fptr(st))) == _u(bits)


def test_flip_distance_matches_draw_and_bounds_flips():
    lib = _lib_oracle()
    rs = np.random.default_rng(5)
    flipped_above = 0
    for t in range(400):
        n, k, T = 512, int(rs.choice([1, 5, 50])), float(rs.choice([0.9, 1.0]))
        lg = (rs.standard_normal(n) * rs.choice([0.5, 3.0])).astype(np.float32)
        bits = int(rs.integers(1, 2**31))
        fd = flip_distance(lg, k, 1.0, T, bits)
        assert fd["result"] == _orc_draw(lib, lg, k, T, bits), t
        eps = fd["eps_flip"]
        if not np.isfinite(eps) or eps < 1e-4:
            continue
        cand, j = fd["candidates"], fd["rank"]
        # below the distance: random and adversarial perturbations keep the id
        for s in (0.5, 0.9):
            for d in (rs.uniform(-1, 1, n) * eps * s,):
                assert _orc_draw(lib, (lg + d).astype(np.float32), k, T, bits) == fd["result"], (t, s)
            if fd["eps_down"] == eps and j > 0:
                d = np.full(n, -eps * s)
                d[cand[:j]] = eps * s
                assert _orc_draw(lib, (lg + d).astype(np.float32), k, T, bits) == fd["result"], (t, s)
        # just above it, the adversarial perturbation of the binding boundary flips it
        s = 1.02
        if fd["eps_down"] == eps and j > 0:
            d = np.full(n, -eps * s)
            d[cand[:j]] = eps * s
        elif fd["eps_up"] == eps:
            d = np.full(n, eps * s)
            d[cand[:j + 1]] = -eps * s
        else:
            continue
        flipped_above += _orc_draw(lib, (lg + d).astype(np.float32), k, T, bits) != fd["result"]
    assert flipped_above > 20


def test_trace_and_classify_tiny_draws(tiny_dir):
    """The oracle's draw trace hands back the sampler inputs of draw (f, g):
    re-drawing from them gives the generation's own code there, and the
    classifier's verdict on that (agreeing) draw is finite and consistent."""
    from divergence import classify
    from oracle_py import DEFAULT, Oracle
    from qtts_io import lookup_ids
    from synth_model import prompt_ids
    o = Oracle(tiny_dir)
    try:
        ids = prompt_ids("p128", 1300)
        s, l = lookup_ids(o.cfg, "aiden", "english")
        par = dict(max_tokens=8, fixed=8, seed=42, **DEFAULT)
        codes, _ = o.generate_codes(ids, s, l, **par)
        lib = _lib_oracle()
        for f, g in ((0, 0), (3, 0), (2, 1), (5, 7), (7, 15)):
            tr = o.trace_draw(ids, s, l, f, g, **par)
            assert tr is not None and tr["result"] == codes[f, g], (f, g)
            k, T = (50, 0.9)
            assert _orc_draw(lib, tr["logits"], k, T, tr["rng_bits"]) == codes[f, g]
            c = classify(o, ids, s, l, f, g, par, got=int(codes[f, g]))
            assert c["reference"] == codes[f, g] and c["eps_gemv"] > 1e-6 and c["eps_flip"] >= 0, c
    finally:
        o.close()
