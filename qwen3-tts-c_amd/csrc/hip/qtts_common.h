// qtts_common.h - shared device helpers for the gfx950 kernels (HIP C++).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define QTTS_CHECK(x)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorName(e_), __FILE__, \
                    __LINE__, #x);                                                       \
            return -1;                                                                   \
        }                                                                                \
    } while (0)

typedef uint16_t bf16_t;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));  // 16 B = 8 packed bf16

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
// 8 packed bf16 (one 16-B load) -> 8 floats
__device__ __forceinline__ void unpack8(const v4u &w, float (&f)[8]) {
    f[0] = __uint_as_float(w.x << 16); f[1] = __uint_as_float(w.x & 0xFFFF0000u);
    f[2] = __uint_as_float(w.y << 16); f[3] = __uint_as_float(w.y & 0xFFFF0000u);
    f[4] = __uint_as_float(w.z << 16); f[5] = __uint_as_float(w.z & 0xFFFF0000u);
    f[6] = __uint_as_float(w.w << 16); f[7] = __uint_as_float(w.w & 0xFFFF0000u);
}

// wave64 reductions
// Wave-wide reductions on the VALU cross-lane paths: DPP inside rows of 16
// lanes, v_permlane16/32_swap across rows (gfx950).  __shfl_xor compiles to
// ds_bpermute_b32, an LDS round trip per step (~0.3 us for a dependent
// 6-step sum, profiles/r02r_batch_gemvm_decomp.txt).  A butterfly: lane ^ 1,
// lane ^ 2 (quad_perm), then the other quad of the 8 (row_half_mirror) and
// the other 8 of the row (row_mirror) -- every lane of the partner group
// already holds the same bits, so the mirror partners are as good as xor 4 /
// xor 8 -- then row pairs and halves (each swap's two results are the lane's
// value and its partner's).  Every lane returns the same bits.
template <int CTRL>
__device__ __forceinline__ float dpp_get(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swap16_other(float v, float &mine) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    mine = __uint_as_float(r[0]);
    return __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap32_other(float v, float &mine) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    mine = __uint_as_float(r[0]);
    return __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_get<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_get<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_get<0x141>(v);   // row_half_mirror
    v += dpp_get<0x140>(v);   // row_mirror
    float a, b = swap16_other(v, a);
    v = a + b;
    b = swap32_other(v, a);
    return a + b;
}
// Sums / maxima over aligned groups of N lanes (N a power of two <= 64; every
// lane of a group gets the group's value) on the same DPP / permlane steps as
// wave_sum -- the __shfl_xor butterflies they replace were one ds_bpermute
// (an LDS round trip) per step.
template <int N>
__device__ __forceinline__ float group_sum(float v) {
    if constexpr (N >= 2) v += dpp_get<0xB1>(v);
    if constexpr (N >= 4) v += dpp_get<0x4E>(v);
    if constexpr (N >= 8) v += dpp_get<0x141>(v);
    if constexpr (N >= 16) v += dpp_get<0x140>(v);
    if constexpr (N >= 32) { float a, b = swap16_other(v, a); v = a + b; }
    if constexpr (N >= 64) { float a, b = swap32_other(v, a); v = a + b; }
    return v;
}
template <int N>
__device__ __forceinline__ float group_max(float v) {
    if constexpr (N >= 2) v = fmaxf(v, dpp_get<0xB1>(v));
    if constexpr (N >= 4) v = fmaxf(v, dpp_get<0x4E>(v));
    if constexpr (N >= 8) v = fmaxf(v, dpp_get<0x141>(v));
    if constexpr (N >= 16) v = fmaxf(v, dpp_get<0x140>(v));
    if constexpr (N >= 32) { float a, b = swap16_other(v, a); v = fmaxf(a, b); }
    if constexpr (N >= 64) { float a, b = swap32_other(v, a); v = fmaxf(a, b); }
    return v;
}
// value of lane ^ 16: v_permlane16_swap(v, v) swaps the odd rows of its first
// result with the even rows of its second, so an even row finds its partner
// in the second result and an odd row in the first (swap16_other returns the
// second, which only a symmetric use -- a + b -- may take as "the other")
__device__ __forceinline__ float xor16_get(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(((threadIdx.x >> 4) & 1) ? r[0] : r[1]);
}

// Inclusive wave prefix sum of ints on DPP: row_shr 1, 2, 4, 8 inside rows of
// 16 (zeros shifted in), then row_bcast:15 / row_bcast:31 carry the row
// totals (the 6-step __shfl_up scan is six LDS round trips).
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_get<0xB1>(v));
    v = fmaxf(v, dpp_get<0x4E>(v));
    v = fmaxf(v, dpp_get<0x141>(v));
    v = fmaxf(v, dpp_get<0x140>(v));
    float a, b = swap16_other(v, a);
    v = fmaxf(a, b);
    b = swap32_other(v, a);
    return fmaxf(a, b);
}
// 256-thread block reduction (4 waves); red must hold >= 4 floats; all threads get the result
__device__ __forceinline__ float block_sum256(float v, float *red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}
__device__ __forceinline__ float block_max256(float v, float *red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// IEEE single-precision helpers (correctly rounded, as the host C does)
__device__ __forceinline__ float div_rn(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ float sqrt_rn(float a) { return __fsqrt_rn(a); }

// RMSNorm scale exactly as written in the reference (K.c:27-39):
// inv = 1/sqrtf(ss/dim + eps)
__device__ __forceinline__ float rms_inv(float ss, int dim, float eps) {
    return div_rn(1.0f, sqrt_rn(div_rn(ss, (float)dim) + eps));
}

// expf with glibc 2.35's exact result (sysdeps/ieee754/flt-32/e_expf.c algorithm:
// 32-entry 2^(i/32) table + cubic in double, FMA ifunc variant).  Verified
// bit-identical to the host libm expf over every float in [-87, 88]
// (tests/test_expf.py re-checks it on the box).  Used where the reference's
// discrete output depends on the exact bits (the sampler's softmax).
__constant__ uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
template <class Tab>
__device__ __forceinline__ float expf_glibc_core(float x, Tab tab) {
#pragma clang fp contract(off)
    if (x > 0x1.62e42ep6f) return __builtin_inff();
    if (x < -0x1.9fe368p6f) return 0.0f;
    const double kInvLn2N = 0x1.71547652b82fep+0 * 32.0;
    const double kShift = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32;
    const double C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32;
    const double C2 = 0x1.62e42ff0c52d6p-1 / 32;
    double xd = (double)x;
    double z = kInvLn2N * xd;
    double kd = z + kShift;
    uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= kShift;
    double r = __fma_rn(kInvLn2N, xd, -kd);
    uint64_t t = tab((int)(ki % 32));
    t += ki << (52 - 5);
    double s = __longlong_as_double((long long)t);
    double zz = __fma_rn(C0, r, C1);
    double r2 = r * r;
    double y = __fma_rn(C2, r, 1.0);
    y = __fma_rn(zz, r2, y);
    y = y * s;
    return (float)y;
}
__device__ __forceinline__ float expf_glibc(float x) {
    return expf_glibc_core(x, [](int i) { return kExp2fTab[i]; });
}
// The same with the table held by the wave (lane l: kExp2fTab[l & 31], loaded
// with the kernel's first loads) and read across lanes: the global table read
// is a dependent memory round trip per call.  Every lane of the wave must be
// active.
__device__ __forceinline__ float expf_glibc_wave(float x, uint64_t tab_lane) {
    return expf_glibc_core(x, [&](int i) {
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)tab_lane, i, 64);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(tab_lane >> 32), i, 64);
        return ((uint64_t)hi << 32) | lo;
    });
}

// Write-through ("sc1") 4-byte store / load at agent scope: the hand-off form
// of cdna_hip_programming.md Guideline 16 R1 for data another workgroup of the
// SAME launch consumes (no release fence; every storing wave drains vmcnt
// before the ticket; the consumer reads with these loads, no acquire).
__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
    return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

