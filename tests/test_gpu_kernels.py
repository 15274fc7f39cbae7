"""HIP kernels through the kernel-level C-ABI (include/qtts_hip.h) against
the reference's golden I/O and the CPU oracle.

Bars: integer outputs (sampled ids, RNG state) bit-exact; fp32 GEMV within
|err| <= 2e-6 * sum|a_i x_i| + 1e-6 (accumulation order differs: 8-lane
partials + KSPLIT slots vs the reference's sequential loop); codec convs on
the fp32 MFMA path within 2e-5 abs + 1e-4 rel.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import golden
from oracle_py import fptr
from qtts_io import f32_to_bf16

import qtts

pytestmark = pytest.mark.gpu
K = golden("kernels.npz")


def T(a, dev, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.view(dtype)
    return t.to(dev)


def bf16_f64(A):
    return (A.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def gemv_bound(A, x):
    return 2e-6 * (np.abs(bf16_f64(A)) @ np.abs(x.astype(np.float64).T)).T + 1e-6


def run_matvec(dev, A, x, B):
    import torch
    R, Cc = A.shape
    out = torch.zeros(B * R, device=dev)
    qtts.Kernels.matvec_bf16(out, T(A, dev, torch.int16), T(x, dev), R, Cc, B)
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(B, R)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_matvec_golden(gpu, i):
    A, x, y = K[f"matvec{i}_A"], K[f"matvec{i}_x"], K[f"matvec{i}_y"]
    got = run_matvec(gpu, A, x[None], 1)[0]
    assert np.all(np.abs(got - y) <= gemv_bound(A, x[None])[0])


# decode shapes of the 1.7B talker / sub-talker + ragged ones
SHAPES = [(4096, 2048, 1), (2048, 2048, 1), (12288, 2048, 1), (2048, 6144, 1), (3072, 2048, 1), (4096, 1024, 1),
          (1024, 2048, 1), (6144, 1024, 1), (1024, 3072, 1), (2048, 1024, 1), (100, 64, 1), (37, 8192, 1),
          (2048, 2048, 2), (4096, 1024, 4), (1000, 192, 3), (3072, 2048, 8), (257, 1024, 16),
          # matrix-core path (batch 2..64: prefill / text projection rows)
          (12288, 2048, 10), (2048, 6144, 33), (4096, 2048, 64), (2048, 2048, 17), (96, 64, 5)]


@pytest.mark.parametrize("R,Cc,B", SHAPES)
def test_matvec_shapes(gpu, R, Cc, B):
    rng = np.random.default_rng(R * 7 + Cc + B)
    A = f32_to_bf16((rng.standard_normal((R, Cc)) / np.sqrt(Cc)).astype(np.float32))
    x = rng.standard_normal((B, Cc)).astype(np.float32)
    got = run_matvec(gpu, A, x, B)
    ref = x.astype(np.float64) @ bf16_f64(A).T
    assert np.all(np.abs(got - ref) <= gemv_bound(A, x)), np.abs(got - ref).max()


@pytest.mark.parametrize("R,Cc,B", [(4096, 2048, 1), (2048, 1024, 1), (512, 128, 1), (1024, 2048, 4),
                                     (4096, 2048, 40)])
def test_rmsnorm_matvec(gpu, R, Cc, B):
    import torch
    rng = np.random.default_rng(5 + B)
    A = f32_to_bf16((rng.standard_normal((R, Cc)) / np.sqrt(Cc)).astype(np.float32))
    x = (rng.standard_normal((B, Cc)) * 3).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(Cc)).astype(np.float32)
    out = torch.zeros(B * R, device=gpu)
    qtts.Kernels.rmsnorm_matvec_bf16(out, T(A, gpu, torch.int16), T(x, gpu), T(w, gpu), 1e-6, R, Cc, B)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(B, R)
    xn = x / np.sqrt((x.astype(np.float64) ** 2).mean(1, keepdims=True) + 1e-6) * w
    ref = xn @ bf16_f64(A).T
    assert np.all(np.abs(got - ref) <= gemv_bound(A, xn) + 1e-5 * np.abs(ref)), np.abs(got - ref).max()


# lock-step batch decode shapes (k_gemvm: matrix cores, x staged whole or in
# column chunks for the down projections at B >= 8) + the tiny model's
DECODE_SHAPES = [(4096, 2048, 8, True), (12288, 2048, 8, True), (2048, 6144, 8, False), (2048, 6144, 16, False),
                 (1024, 3072, 16, False), (4096, 1024, 2, True), (6144, 1024, 4, True), (2048, 1024, 16, True),
                 (3072, 2048, 3, True), (1024, 2048, 5, False), (256, 128, 3, True), (128, 64, 2, True),
                 (2048, 64, 7, False)]


@pytest.mark.parametrize("R,Cc,B,norm", DECODE_SHAPES)
def test_decode_matvec_batch(gpu, R, Cc, B, norm):
    """The decode-loop dispatcher at batch 2..16 (one weight read serves
    every utterance) against float64, with and without the RMSNorm prologue."""
    import torch
    rng = np.random.default_rng(R + Cc * 3 + B)
    A = f32_to_bf16((rng.standard_normal((R, Cc)) / np.sqrt(Cc)).astype(np.float32))
    x = (rng.standard_normal((B, Cc)) * 2).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(Cc)).astype(np.float32)
    out = torch.zeros(B * R, device=gpu)
    qtts.Kernels.decode_matvec_bf16(out, T(A, gpu, torch.int16), T(x, gpu), T(w, gpu) if norm else None, 1e-6,
                                    R, Cc, B)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(B, R)
    xn = x.astype(np.float64)
    if norm:
        xn = (x / np.sqrt((x.astype(np.float64) ** 2).mean(1, keepdims=True) + 1e-6) * w)
    ref = xn @ bf16_f64(A).T
    assert np.all(np.abs(got - ref) <= gemv_bound(A, xn) + 1e-5 * np.abs(ref)), np.abs(got - ref).max()


# the sub-talker chain's batch-1 GEMV (k_gemvw: Infinity-Cache-resident weights)
# at the 1.7B / 0.6B sub-talker shapes, every epilogue, + shapes it leaves to k_gemv1
RESIDENT = [(4096, 1024, 0, True), (6144, 1024, 4, True), (1024, 3072, 3, False), (2048, 1024, 0, True),
            (1024, 2048, 3, False), (3072, 1024, 0, True), (2048, 2048, 0, True), (4096, 2048, 0, False),
            (1024, 1024, 3, True), (6144, 2048, 4, True), (96, 64, 0, True), (200, 1024, 3, False)]


@pytest.mark.parametrize("R,Cc,epi,norm", RESIDENT)
def test_resident_matvec(gpu, R, Cc, epi, norm):
    import torch
    rng = np.random.default_rng(R + 5 * Cc + epi)
    A = f32_to_bf16((rng.standard_normal((R, Cc)) / np.sqrt(Cc)).astype(np.float32))
    x = (rng.standard_normal((1, Cc)) * 2).astype(np.float32)
    w = (1 + 0.1 * rng.standard_normal(Cc)).astype(np.float32)
    nout = R // 2 if epi == 4 else R
    y0 = rng.standard_normal(nout).astype(np.float32) if epi == 3 else np.zeros(nout, np.float32)
    out = T(y0.copy(), gpu)
    qtts.Kernels.resident_matvec_bf16(out, T(A, gpu, torch.int16), T(x, gpu), T(w, gpu) if norm else None, 1e-6,
                                      R, Cc, epi)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    xn = x.astype(np.float64)
    if norm:
        xn = x / np.sqrt((x.astype(np.float64) ** 2).mean(1, keepdims=True) + 1e-6) * w
    acc = (xn @ bf16_f64(A).T)[0]
    bound = gemv_bound(A, xn)[0] + 1e-5 * np.abs(acc)
    if epi == 0:
        ref = acc
    elif epi == 3:
        ref = y0 + acc
    else:   # SwiGLU over gate|up quads: rows 8q..8q+3 gate, 8q+4..8q+7 up
        q = acc.reshape(-1, 2, 4)
        g, u = q[:, 0, :].reshape(-1), q[:, 1, :].reshape(-1)
        ref = g / (1 + np.exp(-g)) * u
        bound = (bound.reshape(-1, 2, 4)[:, 0, :].reshape(-1) + bound.reshape(-1, 2, 4)[:, 1, :].reshape(-1)) * \
            (np.abs(u) + np.abs(g) + 1)
    assert np.all(np.abs(got - ref) <= bound), np.abs(got - ref).max()


def sample_gpu(dev, lg, V, k, tp, temp, rng_bits):
    import torch
    B = lg.shape[0]
    out = torch.zeros(B, dtype=torch.int32, device=dev)
    rs = T(np.asarray(rng_bits, np.uint32).view(np.int32), dev)
    qtts.Kernels.sample_top_k(out, T(lg, dev), V, k, tp, temp, rs, B)
    torch.cuda.synchronize()
    return out.cpu().numpy(), rs.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("V", [2048, 3072])
def test_sampler_golden_bit_exact(gpu, V):
    lg, meta, fm, rs = K[f"samp{V}_logits"], K[f"samp{V}_meta"], K[f"samp{V}_fmeta"], K[f"samp{V}_rng"]
    for i in range(len(lg)):
        r, st = sample_gpu(gpu, lg[i:i + 1], V, int(meta[i, 0]), float(fm[i, 0]), float(fm[i, 1]), [rs[i, 0]])
        assert r[0] == meta[i, 1], (i, r[0], meta[i])
        assert st[0] == rs[i, 1], i


@pytest.mark.parametrize("sw", ["1", "0"])
def test_sampler_random_vs_oracle(gpu, oracle, monkeypatch, sw):
    """Many draws, ties, -inf, top_p cut, k=0/1/large, batched rows with their
    own RNG states: ids and RNG state bit-exact.  On the 1024-thread fast path
    (k_sample_w) and the 256-thread one (QTTS_HIP_SAMPLE_W=0)."""
    monkeypatch.setenv("QTTS_HIP_SAMPLE_W", sw)
    rng = np.random.default_rng(123)
    for it in range(40):
        V = [2048, 3072, 1500, 64][it % 4]
        B = [1, 3, 8][it % 3]
        lg = (rng.standard_normal((B, V)) * rng.uniform(0.3, 8)).astype(np.float32)
        if it % 3 == 0:
            lg[:, rng.integers(0, V, 30)] = lg.max()
        if it % 5 == 1:
            lg[:, rng.integers(0, V, V // 3)] = -1e9
        k = int([1, 50, 0, 7, 300, 2048][it % 6])
        tp = float([1.0, 0.9, 0.5, 0.99][it % 4])
        temp = float(rng.uniform(0.4, 1.6))
        st0 = (rng.integers(1, 10**6, B)).astype(np.float32)
        r, st = sample_gpu(gpu, lg, V, k, tp, temp, st0.view(np.uint32))
        for b in range(B):
            s = np.array([st0[b]], np.float32)
            e = oracle.lib.orc_sample(fptr(lg[b].copy()), V, k, tp, temp, fptr(s))
            assert r[b] == e, (it, b, r[b], e)
            assert st[b] == s.view(np.uint32)[0], (it, b)


@pytest.mark.parametrize("sw", ["1", "0"])
def test_sampler_candidate_bins_vs_oracle(gpu, oracle, monkeypatch, sw):
    """The k <= 64 distance-binned path (qtts_sample_dev.h sample_dist /
    sample_dist_nt) and its radix fallback: boundary bins dense with ties
    (more than 64 candidates), every logit equal, +0 / -0 mixtures,
    ineligible -FLT_MAX entries, values spanning zero, k at the 64 cap and
    one past it, narrow and wide logit scales; ids and RNG state bit-exact.
    On the 1024-thread fast path and the 256-thread one (QTTS_HIP_SAMPLE_W=0)."""
    monkeypatch.setenv("QTTS_HIP_SAMPLE_W", sw)
    rng = np.random.default_rng(7)
    fmax = np.finfo(np.float32).max
    cases = []
    for it in range(48):
        V = [2048, 3072, 4096, 1500, 100][it % 5]
        lg = (rng.standard_normal(V) * [0.01, 0.3, 3.0, 40.0][it % 4]).astype(np.float32)
        kind = it % 8
        if kind == 1:    # ties straddling the k-th key (fallback: > 64 candidates)
            srt = np.sort(lg)[::-1]
            lg[rng.integers(0, V, 80)] = srt[45]
        elif kind == 2:  # every logit equal
            lg[:] = np.float32(rng.standard_normal())
        elif kind == 3:  # +0 / -0 and values around zero
            lg[rng.integers(0, V, V // 2)] = 0.0
            lg[rng.integers(0, V, V // 4)] = -0.0
        elif kind == 4:  # ineligible entries (v <= -FLT_MAX after / T)
            lg[rng.integers(0, V, V - 20)] = -fmax
        elif kind == 5:  # a sharp head and a long tail
            lg[rng.integers(0, V, 5)] += 30.0
        elif kind == 6:  # many copies of the maximum
            lg[rng.integers(0, V, 70)] = lg.max()
        k = int([50, 64, 65, 1, 63, 2, 50, 50][(it // 8 + it) % 8])
        temp = float([0.9, 1.0, 0.5, 1.7][it % 4])
        cases.append((lg, V, k, temp))
    for it, (lg, V, k, temp) in enumerate(cases):
        st0 = np.array([float(rng.integers(1, 10**6))], np.float32)
        r, st = sample_gpu(gpu, lg[None, :], V, k, 1.0, temp, st0.view(np.uint32))
        s = st0.copy()
        e = oracle.lib.orc_sample(fptr(lg.copy()), V, k, 1.0, temp, fptr(s))
        assert r[0] == e, (it, r[0], e)
        assert st[0] == s.view(np.uint32)[0], it


@pytest.mark.parametrize("i", range(5))
def test_causal_conv1d_golden(gpu, i):
    import torch
    ci, co, k, L, d, g = (int(v) for v in K[f"conv{i}_cfg"])
    out = torch.zeros(co * L, device=gpu)
    qtts.Kernels.causal_conv1d(out, T(K[f"conv{i}_x"], gpu), T(K[f"conv{i}_w"], gpu), T(K[f"conv{i}_b"], gpu),
                               ci, co, k, L, d, g)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy().reshape(co, L), K[f"conv{i}_y"], atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("ci,co,k,L,d", [(96, 96, 7, 8192, 9), (64, 192, 3, 4096, 1), (32, 128, 1, 6144, 1),
                                         (768, 768, 7, 1024, 3)])
def test_causal_conv1d_vocoder_shapes(gpu, ci, co, k, L, d):
    """Vocoder-sized convs (the tap-staged k_conv path: channels in stages of
    16, dilation up to 9) against a float64 restatement of kernel_causal_conv1d
    (K.c:659-871): zero left pad (k-1)*d, bias, stride 1."""
    import torch
    rng = np.random.default_rng(ci + co + k + d)
    x = rng.standard_normal((ci, L)).astype(np.float32)
    w = (rng.standard_normal((co, ci, k)) / np.sqrt(ci * k)).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    out = torch.zeros(co * L, device=gpu)
    qtts.Kernels.causal_conv1d(out, T(x, gpu), T(w, gpu), T(b, gpu), ci, co, k, L, d, 1)
    torch.cuda.synchronize()
    pad = (k - 1) * d
    xp = np.concatenate([np.zeros((ci, pad)), x.astype(np.float64)], axis=1)
    ref = np.tile(b.astype(np.float64)[:, None], (1, L))
    for tap in range(k):
        ref += w[:, :, tap].astype(np.float64) @ xp[:, tap * d: tap * d + L]
    np.testing.assert_allclose(out.cpu().numpy().reshape(co, L), ref, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("i", range(5))
def test_transposed_conv1d_golden(gpu, i):
    import torch
    ci, co, k, s, L = (int(v) for v in K[f"tconv{i}_cfg"])
    out = torch.zeros(co * L * s, device=gpu)
    qtts.Kernels.transposed_conv1d(out, T(K[f"tconv{i}_x"], gpu), T(K[f"tconv{i}_w"], gpu),
                                   T(K[f"tconv{i}_b"], gpu), ci, co, k, s, L)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy().reshape(co, L * s), K[f"tconv{i}_y"], atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("ci,co,k,s,L", [(1536, 768, 16, 8, 512), (192, 96, 6, 3, 8192), (768, 384, 10, 5, 1024),
                                         (1024, 1024, 2, 2, 2048), (384, 192, 8, 4, 2048)])
def test_transposed_conv1d_vocoder_shapes(gpu, ci, co, k, s, L):
    """Vocoder-sized transposed convs (all phases in one k_conv launch, each a
    causal conv of k/s taps) against a float64 restatement of
    kernel_transposed_conv1d (K.c:873-940) trimmed to L*s outputs."""
    import torch
    rng = np.random.default_rng(ci + k + L)
    x = rng.standard_normal((ci, L)).astype(np.float32)
    w = (rng.standard_normal((ci, co, k)) / np.sqrt(ci * k / s)).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    out = torch.zeros(co * L * s, device=gpu)
    qtts.Kernels.transposed_conv1d(out, T(x, gpu), T(w, gpu), T(b, gpu), ci, co, k, s, L)
    torch.cuda.synchronize()
    full = np.zeros((co, (L - 1) * s + k))
    xd = x.astype(np.float64)
    for j in range(k):
        full[:, j: j + (L - 1) * s + 1: s] += w[:, :, j].astype(np.float64).T @ xd
    ref = full[:, :L * s] + b.astype(np.float64)[:, None]
    np.testing.assert_allclose(out.cpu().numpy().reshape(co, L * s), ref, atol=2e-5, rtol=1e-4)


def test_snake_golden(gpu):
    import torch
    x = K["snake_x"]
    out = torch.zeros(x.size, device=gpu)
    qtts.Kernels.snake_beta(out, T(x, gpu), T(K["snake_a"], gpu), T(K["snake_ib"], gpu), x.shape[0], x.shape[1])
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy().reshape(x.shape), K["snake_y"], atol=2e-6, rtol=2e-6)


def test_expf_glibc_matches_libm(gpu):
    """The sampler's expf replica is bit-identical to glibc expf (the
    reference's softmax/top-p arithmetic, K.c:371-378, 480-520)."""
    import torch
    libm = C.CDLL("libm.so.6")
    libm.expf.restype = C.c_float
    libm.expf.argtypes = [C.c_float]
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-104, 89, 150000), rng.uniform(-1, 1, 30000), np.linspace(-87.4, 88.7, 20000),
                        [0.0, -0.0, 88.72283, -103.97, 1e-30, -1e-30]]).astype(np.float32)
    out = torch.zeros(len(x), device=gpu)
    qtts.Kernels.expf_glibc(out, T(x, gpu), len(x))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = np.array([libm.expf(float(v)) for v in x], np.float32)
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
    assert len(bad) == 0, (len(bad), x[bad[:5]], got[bad[:5]], ref[bad[:5]])


def test_hbm_stream_bandwidth_entry(gpu):
    """qtts_hip_hbm_bw (the bench line's measured stream bandwidth): both
    figures positive and below the 8 TB/s nominal peak; sizes it refuses."""
    lib = qtts.lib()
    lib.qtts_hip_hbm_bw.restype = C.c_int
    lib.qtts_hip_hbm_bw.argtypes = [C.c_size_t, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    rd, cp = C.c_double(0), C.c_double(0)
    assert lib.qtts_hip_hbm_bw(1 << 30, 3, C.byref(rd), C.byref(cp)) == 0
    assert 500.0 < rd.value < 8000.0 and 500.0 < cp.value < 8000.0, (rd.value, cp.value)
    assert lib.qtts_hip_hbm_bw(1024, 3, C.byref(rd), C.byref(cp)) == -1
    assert lib.qtts_hip_hbm_bw(512 << 20, 0, C.byref(rd), C.byref(cp)) == -1
