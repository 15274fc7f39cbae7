// k_codec.hip - 12 Hz codec decoder / vocoder on gfx950 (c/qwen_tts_codec.c).
//
// Every dense contraction of the codec -- causal conv1d (K.c:659-871),
// transposed conv1d (K.c:873-972), the 1x1 RVQ/ConvNeXt projections and the
// sliding-window transformer's linears (Cd.c:267-522) -- runs through ONE
// implicit-GEMM kernel on the fp32-input MFMA v_mfma_f32_32x32x2_f32 (exact
// fp32 products, f32 accumulate; the codec weights are f32 like the
// reference's).  The operand loaders do the im2col / transposed-conv gather
// and apply SnakeBeta (K.c:251-311) to the input channels on the fly; the
// epilogues fuse bias, GELU(tanh), SiLU*up, LayerScale+residual, gamma,
// transposed stores and the ResUnit residual (Cd.c:549-575).
//
// Tile 64x64 per 256-thread workgroup (2x2 waves of 32x32), K step 16 staged
// through LDS with +1 padding (conflict-free column reads).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "qtts_codec.h"
#include "qtts_common.h"
#include "qtts_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = 64, BN = 64, BK = 32;

// sin^2(r): the sign of sin drops out, so one Cody-Waite step by pi
// (pi = PI_HI + PI_LO; both products exact inside the fmas, k exact below
// 2^24) and the odd Taylor series through y^13 on [-pi/2, pi/2] (truncation
// < 1e-9) give sinf(r)^2 to 2.2e-7 absolute (checked over |r| <= 8192) in
// ~15 instructions instead of the general sinf's ~90 plus its inlined
// large-argument path.
__device__ __forceinline__ float sin2(float r) {
    const float k = rintf(r * 0.318309886183790672f);
    float y = fmaf(-k, 3.14159274101257324f, r);
    y = fmaf(-k, -8.74227765734758577e-08f, y);
    const float y2 = y * y;
    float p = 1.6059043836821613e-10f;                 // 1/13!
    p = fmaf(p, y2, -2.5052108385441720e-08f);         // -1/11!
    p = fmaf(p, y2, 2.7557319223985893e-06f);          // 1/9!
    p = fmaf(p, y2, -1.9841269841269841e-04f);         // -1/7!
    p = fmaf(p, y2, 8.3333333333333333e-03f);          // 1/5!
    p = fmaf(p, y2, -1.6666666666666667e-01f);         // -1/3!
    const float sn = fmaf(y * y2, p, y);
    return sn * sn;
}

__device__ __forceinline__ float snake1(float x, float a, float ib) { return x + ib * sin2(x * a); }

__device__ __forceinline__ float loadB(const XGemm &g, int k, int n) {
    if (k >= g.K || n >= g.N) return 0.f;
    if (g.bmode == XB_WT) return g.B[(size_t)n * g.ldb + k];
    int ic, t;
    if (g.bmode == XB_CONV) {
        ic = k / g.Kw;
        const int tap = k - ic * g.Kw;
        t = n + tap * g.dil - g.pad;
    } else {  // XB_TCONV: k = ic*ntap + j, input position q - j
        const int ntap = g.Kw / g.stride;
        ic = k / ntap;
        t = n - (k - ic * ntap);
    }
    if (t < g.tmin || t >= g.L) return 0.f;
    const float x = g.B[(size_t)ic * g.ldb + t];
    return g.sa ? snake1(x, g.sa[ic], g.sb[ic]) : x;
}

__device__ __forceinline__ float loadA(const XGemm &g, int m, int k) {
    if (m >= g.M || k >= g.K) return 0.f;
    if (g.amode == XA_ROWS) return g.A[(size_t)m * g.lda + k];
    if (g.amode == XA_TRANS) return g.A[(size_t)k * g.lda + m];
    const int ntap = g.Kw / g.stride;  // tconv weight [ci][co][Kw], k = ic*ntap + j
    const int ic = k / ntap, j = k - ic * ntap;
    return g.A[((size_t)ic * g.co + m) * g.Kw + g.phase + j * g.stride];
}

__device__ __forceinline__ float gelu_tanh(float v) {
    return 0.5f * v * (1.0f + tanhf(0.7978845608028654f * (v + 0.044715f * v * v * v)));
}

__device__ __forceinline__ void xg_epi(const XGemm &g, int m, int n, float v) {
    switch (g.emode) {
        case XE_STORE: g.C[(size_t)m * g.ldc + n] = v; break;
        case XE_BIAS_N: g.C[(size_t)m * g.ldc + n] = v + g.bias[n]; break;
        case XE_BIAS_N_GELU: g.C[(size_t)m * g.ldc + n] = gelu_tanh(v + g.bias[n]); break;
        case XE_SILU_MUL: {
            const float gt = g.aux[(size_t)m * g.ldaux + n];
            g.C[(size_t)m * g.ldc + n] = (gt / (1.0f + expf(-gt))) * v;
            break;
        }
        case XE_SCALE_RESID_N: g.C[(size_t)m * g.ldc + n] += v * g.vec[n]; break;
        case XE_BIAS_T: g.C[(size_t)n * g.ldc + m] = v + g.bias[n]; break;
        case XE_BIAS_GAMMA_RES_T:
            g.C[(size_t)n * g.ldc + m] = (v + g.bias[n]) * g.vec[n] + g.res[(size_t)n * g.ldres + m];
            break;
        case XE_BIAS_M: {
            float y = v + (g.bias ? g.bias[m] : 0.f);
            if (g.stride > 1 || g.phase > 0) g.C[(size_t)m * g.ldc + (size_t)n * g.stride + g.phase] = y;
            else g.C[(size_t)m * g.ldc + n] = y;
            break;
        }
        case XE_BIAS_M_RES: g.C[(size_t)m * g.ldc + n] = v + g.bias[m] + g.res[(size_t)m * g.ldres + n]; break;
        case XE_BIAS_M_SNAKE: g.C[(size_t)m * g.ldc + n] = snake1(v + g.bias[m], g.ea[m], g.eb[m]); break;
    }
}

// 64x64 output tile per workgroup (2x2 waves of 32x32 on v_mfma_f32_32x32x2f32),
// K in steps of BK = 32 staged through LDS; the next step's operands are
// loaded into registers while the MFMAs consume the current one.  With
// gridDim.z > 1 (split-K for small output tiles) each z covers one K range and
// writes raw partials to g.part[z][M][N]; k_xg_reduce sums them in z order and
// applies the epilogue.
__global__ __launch_bounds__(256) void k_xgemm(XGemm g) {
    __shared__ float As[BM][BK + 1];
    __shared__ float Bs[BN][BK + 1];
    constexpr int NA = (BM * BK) / 256, NB_ = (BN * BK) / 256;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    const int nz = gridDim.z, z = blockIdx.z;
    const int ksteps = (g.K + BK - 1) / BK;
    const int s0 = (int)((long)ksteps * z / nz), s1 = (int)((long)ksteps * (z + 1) / nz);
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const bool a_k_fast = g.amode == XA_ROWS;   // consecutive threads along k
    const bool b_k_fast = g.bmode == XB_WT;
    float ra[NA], rb[NB_];
    auto load = [&](int k0) {
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            const int e = tid + 256 * j;
            int mi, ki;
            if (a_k_fast) { mi = e / BK; ki = e % BK; }
            else { ki = e / BM; mi = e % BM; }
            ra[j] = loadA(g, m0 + mi, k0 + ki);
        }
#pragma unroll
        for (int j = 0; j < NB_; ++j) {
            const int e = tid + 256 * j;
            int ni, ki;
            if (b_k_fast) { ni = e / BK; ki = e % BK; }
            else { ki = e / BN; ni = e % BN; }
            rb[j] = loadB(g, k0 + ki, n0 + ni);
        }
    };
    if (s0 < s1) load(s0 * BK);
    for (int s2 = s0; s2 < s1; ++s2) {
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            const int e = tid + 256 * j;
            int mi, ki;
            if (a_k_fast) { mi = e / BK; ki = e % BK; }
            else { ki = e / BM; mi = e % BM; }
            As[mi][ki] = ra[j];
        }
#pragma unroll
        for (int j = 0; j < NB_; ++j) {
            const int e = tid + 256 * j;
            int ni, ki;
            if (b_k_fast) { ni = e / BK; ki = e % BK; }
            else { ki = e / BN; ni = e % BN; }
            Bs[ni][ki] = rb[j];
        }
        __syncthreads();
        if (s2 + 1 < s1) load((s2 + 1) * BK);
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float a = As[wm + (lane & 31)][kk + (lane >> 5)];
            const float b = Bs[wn + (lane & 31)][kk + (lane >> 5)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + (lane & 31);
        if (m >= g.M || n >= g.N) continue;
        if (nz > 1) g.part[((size_t)z * g.M + m) * g.N + n] = acc[r];
        else xg_epi(g, m, n, acc[r]);
    }
}

// Causal conv, stride 1 (Cd.c conv stacks, K.c:659-871), as Kw accumulated
// per-tap GEMMs: out[co][t] = b[co] + sum_tap sum_ci Wt[tap][co][ci] * x'[ci][t + tap*dil - pad],
// x' = SnakeBeta(x) when g.sa is set (K.c:251-311).  64 (co) x 128 (t) tile
// per workgroup, 4 waves of 32 x 64 (two v_mfma_f32_32x32x2f32 blocks: exact
// fp32 products).  Per stage of 16 input channels the B window
// x'[16][t0 - pad, t0 + 128) is staged ONCE in LDS -- SnakeBeta applied once
// per element -- and every tap reads it shifted by tap*dil; the stage's
// Kw x 64 x 16 weights come from the re-laid [Kw][co][ci] copy as float4.
// The next stage's loads are in registers while the MFMAs consume this one.
constexpr int CV_BM = 64, CV_BN = 128, CV_BC = 16, CV_HALO = 64;   // halo >= (Kw-1)*dil (host-checked)

// blockIdx.z = phase * kz + split: the transposed-conv output phase
// (tconv_run: weights g.wt + phase*KW*M*ci, outputs at column
// n*stride + phase) and, when g.kz > 1, the input-channel split whose raw
// partial tile goes to g.part[z][M][N] (k_conv_reduce applies the epilogue).
template <int KW>
__global__ __launch_bounds__(256) void k_conv(XGemm g) {
    const int nzk = g.kz > 1 ? g.kz : 1, ph = blockIdx.z / nzk, kzi = blockIdx.z - ph * nzk;
    if (ph) {
        g.wt += (size_t)ph * KW * g.M * (g.K / KW);
        g.phase += ph;
    }
    constexpr int NBW = CV_BN + CV_HALO;                     // staged window columns
    constexpr int NA4 = KW * CV_BM * CV_BC / 4 / 256;       // float4 weight loads per thread (ceil below)
    constexpr int NA4C = (KW * CV_BM * CV_BC / 4 + 255) / 256;
    constexpr int NB = (CV_BC * NBW + 255) / 256;            // window loads per thread
    __shared__ __attribute__((aligned(16))) float As[KW][CV_BM][CV_BC + 1];
    __shared__ float Bs[CV_BC][NBW + 1];
    (void)NA4;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * CV_BM, n0 = blockIdx.x * CV_BN;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 64;
    const int ci = g.K / KW, dil = g.dil, t0 = n0 - g.pad;
    const int cpz = ci / nzk, cbeg = kzi * cpz, cend = cbeg + cpz;   // this split's input channels
    const int win = CV_BN + (KW - 1) * dil;                  // columns actually needed
    floatx16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; }
    float4 ra[NA4C];
    float rb[NB];
    auto load = [&](int c0) {
#pragma unroll
        for (int j = 0; j < NA4C; ++j) {
            const int e = tid + 256 * j;                     // float4 index in [KW][BM][BC/4]
            const int c4 = e % (CV_BC / 4), m = (e / (CV_BC / 4)) % CV_BM, tap = e / (CV_BC / 4 * CV_BM);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (tap < KW && m0 + m < g.M)
                v = *reinterpret_cast<const float4 *>(g.wt + ((size_t)tap * g.M + m0 + m) * ci + c0 + 4 * c4);
            ra[j] = v;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int e = tid + 256 * j, c = e / NBW, x = e - c * NBW, t = t0 + x;
            float v = 0.f;
            if (c < CV_BC && x < win && t >= g.tmin && t < g.L) {
                v = g.B[(size_t)(c0 + c) * g.ldb + t];
                if (g.sa) v = snake1(v, g.sa[c0 + c], g.sb[c0 + c]);
            }
            rb[j] = v;
        }
    };
    load(cbeg);
    for (int c0 = cbeg; c0 < cend; c0 += CV_BC) {
#pragma unroll
        for (int j = 0; j < NA4C; ++j) {
            const int e = tid + 256 * j;
            const int c4 = e % (CV_BC / 4), m = (e / (CV_BC / 4)) % CV_BM, tap = e / (CV_BC / 4 * CV_BM);
            if (tap < KW) {
                As[tap][m][4 * c4 + 0] = ra[j].x; As[tap][m][4 * c4 + 1] = ra[j].y;
                As[tap][m][4 * c4 + 2] = ra[j].z; As[tap][m][4 * c4 + 3] = ra[j].w;
            }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int e = tid + 256 * j, c = e / NBW, x = e - c * NBW;
            if (c < CV_BC) Bs[c][x] = rb[j];
        }
        __syncthreads();
        if (c0 + CV_BC < cend) load(c0 + CV_BC);
#pragma unroll
        for (int tap = 0; tap < KW; ++tap) {
            const int sh = tap * dil;
#pragma unroll
            for (int kk = 0; kk < CV_BC; kk += 2) {
                const int kr = kk + (lane >> 5);
                const float a = As[tap][wm + (lane & 31)][kr];
                const float b0 = Bs[kr][wn + (lane & 31) + sh];
                const float b1 = Bs[kr][wn + 32 + (lane & 31) + sh];
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float *pz = nzk > 1 ? g.part + (size_t)blockIdx.z * g.M * g.N : nullptr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + (lane & 31);
        if (m >= g.M) continue;
        if (pz) {
            if (n < g.N) pz[(size_t)m * g.N + n] = acc0[r];
            if (n + 32 < g.N) pz[(size_t)m * g.N + n + 32] = acc1[r];
            continue;
        }
        if (n < g.N) xg_epi(g, m, n, acc0[r]);
        if (n + 32 < g.N) xg_epi(g, m, n + 32, acc1[r]);
    }
}

// k_conv on the bf16 matrix cores: same
// tiles, grid, splits and epilogues, fp32-equivalent products.  The weights
// and the staged input are split exactly into three bf16 planes, w = w1 + w2
// + w3 and x = x1 + x2 + x3, and the six products with i + j <= 4 are
// accumulated (the three dropped ones are below 2^-24 of |w x|):
//   v_mfma_f32_32x32x16_bf16 is 16x the fp32-input MFMA's rate, so six of
//   them cost 3/8 of the eight v_mfma_f32_32x32x2_f32 a 16-channel stage
//   took.
// LDS rows are 16 channels (32 B) with the two 16-B halves swapped on odd
// 8-row groups: conflict-free ds_read_b128 fragments.  The weight planes
// follow the fp32 relayout in the same allocation (wt_planes).
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int CB_SNAKE_MAX = 1536;   // input channels per split k_convb takes with SnakeBeta (larger: k_conv)

__device__ __forceinline__ int cb_swz(int row, int half) { return row * 16 + 8 * (half ^ ((row >> 3) & 1)); }

__device__ __forceinline__ uint32_t cb_pk(float lo, float hi) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    const bf2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float cb_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float cb_hi(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

// 8 floats -> three bf16 planes (16 B each)
__device__ __forceinline__ void cb_split8(const float (&v)[8], uint4 &p1, uint4 &p2, uint4 &p3) {
    uint32_t a[4], b[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = cb_pk(v[2 * i], v[2 * i + 1]);
        const float e0 = v[2 * i] - cb_lo(a[i]), e1 = v[2 * i + 1] - cb_hi(a[i]);
        b[i] = cb_pk(e0, e1);
        c[i] = cb_pk(e0 - cb_lo(b[i]), e1 - cb_hi(b[i]));
    }
    p1 = make_uint4(a[0], a[1], a[2], a[3]);
    p2 = make_uint4(b[0], b[1], b[2], b[3]);
    p3 = make_uint4(c[0], c[1], c[2], c[3]);
}

// WN waves along t (2 or 4): a 64 x 64*WN tile per workgroup of 128*WN
// threads; the staged weights serve WN waves per 32-row half.
// (a 128-VGPR bound lets two 8-wave k_convb<7,4> workgroups share a CU now
// that its LDS fits twice: batch-8 codec 53.1-53.4 -> 51.9-52.0 ms, batch 1
// 7.87 -> 7.65 ms, one spilled VGPR; profiles/r06p_ab_convb.txt)
#ifndef QTTS_CONVB_MINB
#define QTTS_CONVB_MINB 4
#endif
template <int KW, int WN>
__global__ __launch_bounds__(128 * WN, QTTS_CONVB_MINB) void k_convb(XGemm g) {
    constexpr int NT = 128 * WN, BNT = 64 * WN;
    const int nzk = g.kz > 1 ? g.kz : 1, ph = blockIdx.z / nzk, kzi = blockIdx.z - ph * nzk;
    const int nph = gridDim.z / nzk, ci = g.K / KW;
    const size_t ps = (size_t)nph * g.M * g.K;   // plane stride (elements)
    const unsigned short *wb = reinterpret_cast<const unsigned short *>(g.wt + ps) + (size_t)ph * KW * g.M * ci;
    g.phase += ph;
    constexpr int NBW = BNT + CV_HALO;
    constexpr int NA = 3 * KW * CV_BM * 2;                   // 16-B weight items per stage
    constexpr int NAT = (NA + NT - 1) / NT;
    constexpr int NBT = (2 * NBW + NT - 1) / NT;             // (half, column) input items per thread
    __shared__ __attribute__((aligned(16))) unsigned short As[3 * KW * CV_BM * 16];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[3 * NBW * 16];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * CV_BM, n0 = blockIdx.x * BNT;
    const int wm = (wave / WN) * 32, wn = (wave % WN) * 64;
    const int dil = g.dil, t0 = n0 - g.pad;
    const int cpz = ci / nzk, cbeg = kzi * cpz, cend = cbeg + cpz;
    const int win = BNT + (KW - 1) * dil;
    floatx16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; }
    uint4 ra[NAT];
    float rb[NBT][8];
    auto load = [&](int c0) {
#pragma unroll
        for (int j = 0; j < NAT; ++j) {
            const int e = tid + NT * j;
            const int p = e / (KW * CV_BM * 2), rem = e - p * (KW * CV_BM * 2);
            const int tap = rem / (CV_BM * 2), m = (rem >> 1) % CV_BM, h = rem & 1;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (e < NA && m0 + m < g.M)
                v = *reinterpret_cast<const uint4 *>(wb + p * ps + ((size_t)tap * g.M + m0 + m) * ci + c0 + 8 * h);
            ra[j] = v;
        }
#pragma unroll
        for (int j = 0; j < NBT; ++j) {
            const int e = tid + NT * j, h = e / NBW, x = e - h * NBW, t = t0 + x;
            const bool ok = h < 2 && x < win && t >= g.tmin && t < g.L;
#pragma unroll
            for (int q = 0; q < 8; ++q) rb[j][q] = ok ? g.B[(size_t)(c0 + 8 * h + q) * g.ldb + t] : 0.f;
        }
    };
    load(cbeg);
    // SnakeBeta of the input channels is applied when a stage is written to
    // LDS (its loads have landed by then).  Its parameters come through the
    // scalar cache: an item's 8 channels are wave-uniform (NBW is a multiple
    // of 64), so no LDS copy of them (12 KB at 1536 channels) is needed.
    static_assert(NBW % 64 == 0, "k_convb: staged window columns must be whole waves");
    const bool snake = g.sa != nullptr;
    const int r = lane & 31, hh = lane >> 5;
    for (int c0 = cbeg; c0 < cend; c0 += CV_BC) {
#pragma unroll
        for (int j = 0; j < NAT; ++j) {
            const int e = tid + NT * j;
            if (e < NA) {
                const int pt = e / (CV_BM * 2), m = (e >> 1) % CV_BM, h = e & 1;   // pt = plane * KW + tap
                *reinterpret_cast<uint4 *>(&As[pt * CV_BM * 16 + cb_swz(m, h)]) = ra[j];
            }
        }
#pragma unroll
        for (int j = 0; j < NBT; ++j) {
            const int e = tid + NT * j, h = e / NBW, x = e - h * NBW;
            if (h < 2) {
                if (snake) {
                    const int cu = __builtin_amdgcn_readfirstlane(c0 + 8 * h);
#pragma unroll
                    for (int q = 0; q < 8; ++q) rb[j][q] = snake1(rb[j][q], g.sa[cu + q], g.sb[cu + q]);
                }
                uint4 p1, p2, p3;
                cb_split8(rb[j], p1, p2, p3);
                const int o = cb_swz(x, h);
                *reinterpret_cast<uint4 *>(&Bs[o]) = p1;
                *reinterpret_cast<uint4 *>(&Bs[NBW * 16 + o]) = p2;
                *reinterpret_cast<uint4 *>(&Bs[2 * NBW * 16 + o]) = p3;
            }
        }
        __syncthreads();
        if (c0 + CV_BC < cend) load(c0 + CV_BC);
#pragma unroll
        for (int tap = 0; tap < KW; ++tap) {
            const int sh = tap * dil, oa = cb_swz(wm + r, hh);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8 *>(&As[(0 * KW + tap) * CV_BM * 16 + oa]);
            const bf16x8 a2 = *reinterpret_cast<const bf16x8 *>(&As[(1 * KW + tap) * CV_BM * 16 + oa]);
            const bf16x8 a3 = *reinterpret_cast<const bf16x8 *>(&As[(2 * KW + tap) * CV_BM * 16 + oa]);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int ob = cb_swz(wn + 32 * nb + r + sh, hh);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(&Bs[ob]);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(&Bs[NBW * 16 + ob]);
                const bf16x8 b3 = *reinterpret_cast<const bf16x8 *>(&Bs[2 * NBW * 16 + ob]);
                floatx16 &acc = nb ? acc1 : acc0;
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b3, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, b1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float *pz = nzk > 1 ? g.part + (size_t)blockIdx.z * g.M * g.N : nullptr;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + (lane & 31);
        if (m >= g.M) continue;
        if (pz) {
            if (n < g.N) pz[(size_t)m * g.N + n] = acc0[i];
            if (n + 32 < g.N) pz[(size_t)m * g.N + n + 32] = acc1[i];
            continue;
        }
        if (n < g.N) xg_epi(g, m, n, acc0[i]);
        if (n + 32 < g.N) xg_epi(g, m, n + 32, acc1[i]);
    }
}

// The codec's plain linears (XA_ROWS x XB_WT: the transformer's projections,
// Cd.c:267-461, and the ConvNeXt pointwise convs, Cd.c:493-507, at T / 2T / 4T
// rows): C = A W^T, fp32 A [M][K] and W [N][K], on the bf16 matrix cores with
// k_convb's exact split (both operands as three bf16 planes, the six products
// with i + j <= 4; fp32-equivalent).  k_xgemm ran them at 21-34 us per
// 128-row projection (profiles/r05o_codec_kernels.txt): one float per thread
// per load, 32-wide K steps, each step's loads one stage ahead.  Here a
// workgroup (4 waves of 32 x 32 on a 64 x 64 tile) takes XL_KS = 128 columns
// of K per stage as 16 float4 loads per thread (the next stage's issued before
// this one's MFMAs), both tiles fp32 in LDS, and each wave splits its
// fragments in registers: 8 blocks of 16 K x 6 v_mfma_f32_32x32x16_bf16 per
// stage, alternate blocks on two accumulators.  Split-K over blockIdx.z (K / XL_KS stages dealt evenly) with the
// raw partials in g.part for k_xg_reduce, as k_xgemm.
constexpr int XL_KS = 128, XL_LD = XL_KS + 4;

__device__ __forceinline__ void xl_split2(float x0, float x1, uint32_t &a, uint32_t &b, uint32_t &c) {
    a = cb_pk(x0, x1);
    const float e0 = x0 - cb_lo(a), e1 = x1 - cb_hi(a);
    b = cb_pk(e0, e1);
    c = cb_pk(e0 - cb_lo(b), e1 - cb_hi(b));
}
__device__ __forceinline__ void xl_split8(const float4 &u, const float4 &v, bf16x8 &h1, bf16x8 &h2, bf16x8 &h3) {
    uint4 p1, p2, p3;
    xl_split2(u.x, u.y, p1.x, p2.x, p3.x);
    xl_split2(u.z, u.w, p1.y, p2.y, p3.y);
    xl_split2(v.x, v.y, p1.z, p2.z, p3.z);
    xl_split2(v.z, v.w, p1.w, p2.w, p3.w);
    h1 = __builtin_bit_cast(bf16x8, p1);
    h2 = __builtin_bit_cast(bf16x8, p2);
    h3 = __builtin_bit_cast(bf16x8, p3);
}

__global__ __launch_bounds__(256, 1) void k_xlin(XGemm g) {
    __shared__ __attribute__((aligned(16))) float As[64 * XL_LD];
    __shared__ __attribute__((aligned(16))) float Bs[64 * XL_LD];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    const int nz = gridDim.z, z = blockIdx.z;
    const int nst = g.K / XL_KS;
    const int s0 = (int)((long)nst * z / nz), s1 = (int)((long)nst * (z + 1) / nz);
    // stage loads: element e = tid + 256 j of the 64 x 32 float4 tile: row e / 32, float4 column e % 32
    // the stage's 16 float4 per thread as named registers (an indexed array
    // here stayed in scratch: the compiler kept it addressable across the
    // stage loop)
    float4 ra0, ra1, ra2, ra3, ra4, ra5, ra6, ra7, rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7;
    // (rows past M read row M - 1 and are zeroed when staged)
    const int lr = tid >> 5, lc = 4 * (tid & 31);
    auto arow = [&](int j) { const int m = m0 + lr + 8 * j; return g.A + (size_t)(m < g.M ? m : g.M - 1) * g.lda + lc; };
    const float *pa0 = arow(0), *pa1 = arow(1), *pa2 = arow(2), *pa3 = arow(3), *pa4 = arow(4), *pa5 = arow(5),
                *pa6 = arow(6), *pa7 = arow(7);
    const float *pb0 = g.B + (size_t)(n0 + lr) * g.ldb + lc;
    const size_t sb = (size_t)8 * g.ldb;
#define XL_L1(j, k0)                                                                                       \
    ra##j = *reinterpret_cast<const float4 *>(pa##j + (k0));                                               \
    rb##j = *reinterpret_cast<const float4 *>(pb0 + j * sb + (k0));
#define XL_LOAD(k0) XL_L1(0, k0) XL_L1(1, k0) XL_L1(2, k0) XL_L1(3, k0) XL_L1(4, k0) XL_L1(5, k0) XL_L1(6, k0) XL_L1(7, k0)
#define XL_S1(j)                                                                                           \
    *reinterpret_cast<float4 *>(As + (lr + 8 * j) * XL_LD + lc) = m0 + lr + 8 * j < g.M ? ra##j : make_float4(0.f, 0.f, 0.f, 0.f); \
    *reinterpret_cast<float4 *>(Bs + (lr + 8 * j) * XL_LD + lc) = rb##j;
    floatx16 acc, acc2;
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc[i] = 0.f; acc2[i] = 0.f; }
    if (s0 < s1) { XL_LOAD(s0 * XL_KS) }
    const int ra_row = wm + (lane & 31), rb_row = wn + (lane & 31), kh = 8 * (lane >> 5);
    for (int s = s0; s < s1; ++s) {
        XL_S1(0) XL_S1(1) XL_S1(2) XL_S1(3) XL_S1(4) XL_S1(5) XL_S1(6) XL_S1(7)
        __syncthreads();
        if (s + 1 < s1) { XL_LOAD((s + 1) * XL_KS) }
        // two 16-K blocks per step on two accumulators, their chains
        // interleaved (no MFMA waits on the one just issued)
#pragma unroll
        for (int kb = 0; kb < XL_KS; kb += 32) {
            const float *pa = As + ra_row * XL_LD + kb + kh, *pb = Bs + rb_row * XL_LD + kb + kh;
            bf16x8 a1, a2, a3, b1, b2, b3, c1, c2, c3, d1, d2, d3;
            xl_split8(*reinterpret_cast<const float4 *>(pa), *reinterpret_cast<const float4 *>(pa + 4), a1, a2, a3);
            xl_split8(*reinterpret_cast<const float4 *>(pb), *reinterpret_cast<const float4 *>(pb + 4), b1, b2, b3);
            xl_split8(*reinterpret_cast<const float4 *>(pa + 16), *reinterpret_cast<const float4 *>(pa + 20), c1, c2, c3);
            xl_split8(*reinterpret_cast<const float4 *>(pb + 16), *reinterpret_cast<const float4 *>(pb + 20), d1, d2, d3);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b3, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, d3, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c2, d2, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, b1, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c3, d1, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, d2, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c2, d1, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, d1, acc2, 0, 0, 0);
        }
        __syncthreads();
    }
    acc += acc2;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn + (lane & 31);
        if (m >= g.M) continue;
        if (nz > 1) g.part[((size_t)z * g.M + m) * g.N + n] = acc[i];
        else xg_epi(g, m, n, acc[i]);
    }
#undef XL_LOAD
#undef XL_L1
#undef XL_S1
}

// w (fp32, n elements) -> three exact bf16 planes at planes[p * n + i]
__global__ void k_wt_split(const float *w, size_t n, unsigned short *planes) {
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i >= n) return;
    const float v0 = w[i], v1 = i + 1 < n ? w[i + 1] : 0.f;
    const uint32_t a = cb_pk(v0, v1);
    const float e0 = v0 - cb_lo(a), e1 = v1 - cb_hi(a);
    const uint32_t b = cb_pk(e0, e1);
    const uint32_t c = cb_pk(e0 - cb_lo(b), e1 - cb_hi(b));
    const uint32_t pl[3] = {a, b, c};
    for (int p = 0; p < 3; ++p) {
        planes[p * n + i] = (unsigned short)(pl[p] & 0xFFFFu);
        if (i + 1 < n) planes[p * n + i + 1] = (unsigned short)(pl[p] >> 16);
    }
}

// sum of k_conv's channel-split partials (in split order) + the epilogue, per
// (phase, m, n)
__global__ void k_conv_reduce(XGemm g, int nph) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x, mn = (size_t)g.M * g.N;
    if (idx >= mn * nph) return;
    const int ph = (int)(idx / mn);
    const size_t e = idx - (size_t)ph * mn;
    const float *p = g.part + (size_t)ph * g.kz * mn + e;
    float v = p[0];
    for (int z = 1; z < g.kz; ++z) v += p[(size_t)z * mn];
    g.phase += ph;
    xg_epi(g, (int)(e / g.N), (int)(e % g.N), v);
}

// Weight-streaming GEMV for the codec's linears at M <= 4 rows (the first-
// packet / small-chunk streaming decode: transformer, ConvNeXt pointwise
// convs at T = 1..4 frames).  C[m][n] = sum_k A(m, k) * W[n][k] with fp32
// weights W (ldb), A rows (XA_ROWS) or columns (XA_TRANS).  256 threads = 32
// slots x 8 lanes; a lane loads 16 B (4 floats) per 32-column block; a row's
// blocks are dealt to KS slots; A is staged in LDS; epilogue xg_epi.
constexpr int XV_U = 8;   // loads in flight per lane
typedef float floatx4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_xgemv(XGemm g, int ks) {
    extern __shared__ __attribute__((aligned(16))) float xsm[];
    const int tid = threadIdx.x, slot = tid >> 3, sub = tid & 7;
    const int RPW = 32 / ks, rloc = slot % RPW, kss = slot / RPW;
    const int n0 = blockIdx.x * RPW, n = n0 + rloc, nc = n < g.N ? n : g.N - 1;
    const int K = g.K, M = g.M;
    float *xs = xsm;                 // [M][K]
    float *red = xs + 4 * K;         // [32][4]
    const floatx4v *wr = reinterpret_cast<const floatx4v *>(g.B + (size_t)nc * g.ldb) + sub;
    const int nblk = K / 32 / ks;
    floatx4v wv[XV_U];
    auto load = [&](int j0) {
#pragma unroll
        for (int u = 0; u < XV_U; ++u) {
            int j = j0 + u;
            j = j < nblk ? j : nblk - 1;
            wv[u] = __builtin_nontemporal_load(wr + 8 * (kss + j * ks));
        }
    };
    load(0);
    for (int i = tid; i < M * K; i += 256) {
        const int m = i / K, k = i - m * K;
        xs[i] = g.amode == XA_TRANS ? g.A[(size_t)k * g.lda + m] : g.A[(size_t)m * g.lda + k];
    }
    __syncthreads();
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < nblk; j0 += XV_U) {
        floatx4v cur[XV_U];
#pragma unroll
        for (int u = 0; u < XV_U; ++u) cur[u] = wv[u];
        if (j0 + XV_U < nblk) load(j0 + XV_U);
#pragma unroll
        for (int u = 0; u < XV_U; ++u) {
            if (j0 + u < nblk) {
                const int c = 32 * (kss + (j0 + u) * ks) + 4 * sub;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    if (m < M) {
                        const float4 x = *reinterpret_cast<const float4 *>(xs + m * K + c);
                        acc[m] = fmaf(cur[u][0], x.x, acc[m]); acc[m] = fmaf(cur[u][1], x.y, acc[m]);
                        acc[m] = fmaf(cur[u][2], x.z, acc[m]); acc[m] = fmaf(cur[u][3], x.w, acc[m]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float v = acc[m];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        acc[m] = v;
    }
    if (sub == 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) red[(kss * RPW + rloc) * 4 + m] = acc[m];
    }
    __syncthreads();
    if (tid < RPW * M) {
        const int rl = tid / M, m = tid - rl * M, nn = n0 + rl;
        if (nn < g.N) {
            float v = red[rl * 4 + m];
            for (int k2 = 1; k2 < ks; ++k2) v += red[(k2 * RPW + rl) * 4 + m];
            xg_epi(g, m, nn, v);
        }
    }
}

// w [co][ci][Kw] -> wt [Kw][co][ci]
__global__ void k_wt_relayout(const float *w, int co, int ci, int Kw, float *wt) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, n = (size_t)co * ci * Kw;
    if (i >= n) return;
    const int tap = (int)(i % Kw), c = (int)((i / Kw) % ci), o = (int)(i / ((size_t)Kw * ci));
    wt[((size_t)tap * co + o) * ci + c] = w[i];
}

// transposed conv w [ci][co][Kw] (Kw = ntap*s) -> per phase causal-conv weights
// wt [s][ntap][co][ci]: phase ph, conv tap j' (input t - (ntap-1-j')) uses w[..][ph + (ntap-1-j')*s]
__global__ void k_wt_tconv(const float *w, int ci, int co, int Kw, int s, float *wt) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, n = (size_t)co * ci * Kw;
    if (i >= n) return;
    const int nt = Kw / s;
    const int c = (int)(i % ci), o = (int)((i / ci) % co), tap = (int)((i / ((size_t)ci * co)) % nt),
              ph = (int)(i / ((size_t)ci * co * nt));
    wt[i] = w[((size_t)c * co + o) * Kw + ph + (nt - 1 - tap) * s];
}

__global__ void k_xg_reduce(XGemm g, int nz) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)g.M * g.N) return;
    float v = 0.f;
    for (int z = 0; z < nz; ++z) v += g.part[(size_t)z * g.M * g.N + idx];
    xg_epi(g, (int)(idx / g.N), (int)(idx % g.N), v);
}

// RVQ gather-sums (Cd.c:166-227), bit-identical order: sem = 0 + e0[c0];
// ac = 0 + e1[c1] + ... + e15[c15]; out-of-range codes -> 0
__global__ void k_rvq_sum(const int *codes, int T, int Q, int CB, int vq, const float *cb, float *ss, float *as) {
#pragma clang fp contract(off)
    const int t = blockIdx.x, k = threadIdx.x;
    if (k >= vq) return;
    float s = 0.f, a = 0.f;
    for (int q = 0; q < Q; ++q) {
        int c = codes[(size_t)t * Q + q];
        if (c < 0 || c >= CB) c = 0;
        const float e = cb[((size_t)q * CB + c) * vq + k];
        if (q == 0) s += e;
        else a += e;
    }
    ss[(size_t)k * T + t] = s;
    as[(size_t)k * T + t] = a;
}
// output projections (1x1, no bias) summed (Cd.c:178-255): one wave per
// output (o, t), lanes stride over k, shuffle-tree sums (s1 + s2 as the reference)
__global__ void k_rvq_proj(const float *ps, const float *pa, const float *ss, const float *as, int vq, int half, int T,
                           int ldo, float *out) {
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (idx >= half * T) return;
    const int o = idx / T, t = idx - o * T;
    float s1 = 0.f, s2 = 0.f;
    for (int k = lane; k < vq; k += 64) {
        s1 = fmaf(ps[(size_t)o * vq + k], ss[(size_t)k * T + t], s1);
        s2 = fmaf(pa[(size_t)o * vq + k], as[(size_t)k * T + t], s2);
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) out[(size_t)o * ldo + t] = s1 + s2;
}
// depthwise causal conv k=7 (ConvNeXt dwconv), reference order b + sum_k
// (ldx / ldy: row strides; tmin < 0 reads the streaming history in the margin)
__global__ void k_dwconv(const float *x, int ldx, int tmin, const float *w, const float *b, int C, int L, int K,
                         float *y, int ldy) {
#pragma clang fp contract(off)
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)C * L) return;
    const int c = (int)(idx / L), t = (int)(idx - (size_t)c * L);
    float acc = b ? b[c] : 0.f;
    for (int k = 0; k < K; ++k) {
        const int ti = t - (K - 1) + k;
        if (ti >= tmin) acc += w[(size_t)c * K + k] * x[(size_t)c * ldx + ti];
    }
    y[(size_t)c * ldy + t] = acc;
}
// strided 2-D copy (streaming history in / out)
__global__ void k_copy2d(float *dst, int ldd, const float *src, int lds, int rows, int cols) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)rows * cols) return;
    const int r = (int)(idx / cols), c = (int)(idx - (size_t)r * cols);
    dst[(size_t)r * ldd + c] = src[(size_t)r * lds + c];
}
// LayerNorm over channels of a channel-major [C][L] tensor, written time-major [L][C] (Cd.c:480-488)
__global__ __launch_bounds__(256) void k_ln_t(const float *x, int ldx, int C, const float *w, const float *b,
                                              float eps, float *y) {
    __shared__ float red[8];
    const int t = blockIdx.x;
    float s = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) s += x[(size_t)c * ldx + t];
    const float mean = block_sum256(s, red) / (float)C;
    float v = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) { const float d = x[(size_t)c * ldx + t] - mean; v += d * d; }
    const float var = block_sum256(v, red + 4) / (float)C;
    const float inv = div_rn(1.0f, sqrt_rn(var + eps));
    for (int c = threadIdx.x; c < C; c += 256) {
        float o = (x[(size_t)c * ldx + t] - mean) * inv;
        o *= w[c];
        y[(size_t)t * C + c] = o + b[c];
    }
}
// RMSNorm rows [T][D] -> out rows (K.c:27-39)
__global__ __launch_bounds__(256) void k_rms_rows(const float *x, int D, const float *w, float eps, float *y) {
    __shared__ float red[4];
    const int t = blockIdx.x;
    const float *xr = x + (size_t)t * D;
    float s = 0.f;
    for (int c = threadIdx.x; c < D; c += 256) s += xr[c] * xr[c];
    const float inv = rms_inv(block_sum256(s, red), D, eps);
    for (int c = threadIdx.x; c < D; c += 256) y[(size_t)t * D + c] = xr[c] * inv * w[c];
}
// rotate-half RoPE in place on rows [T][nh*hd] (K.c:564-587)
__global__ void k_rope_rows(float *x, int ld, int nh, int hd, const float *cs, const float *sn) {
    const int t = blockIdx.x;
    const int half = hd / 2;
    for (int i = threadIdx.x; i < nh * half; i += blockDim.x) {
        const int h = i / half, e = i - h * half;
        float *q = x + (size_t)t * ld + h * hd;
        const float a = q[e], bb = q[e + half];
        q[e] = a * cs[(size_t)t * hd + e] - bb * sn[(size_t)t * hd + e];
        q[e + half] = bb * cs[(size_t)t * hd + e + half] + a * sn[(size_t)t * hd + e + half];
    }
}
__global__ void k_snake(const float *x, const float *a, const float *ib, int C, int L, float *y) {
#pragma clang fp contract(off)
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)C * L) return;
    const int c = (int)(idx / L);
    const float s = sinf(x[idx] * a[c]);
    y[idx] = x[idx] + ib[c] * s * s;
}
__global__ void k_clamp(float *x, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        float v = x[i];
        if (v < -1.0f) v = -1.0f;
        if (v > 1.0f) v = 1.0f;
        x[i] = v;
    }
}
__global__ void k_expf_glibc(const float *x, float *y, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = expf_glibc(x[i]);
}
__global__ void k_iota(int *p, int n, int zero) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = zero ? 0 : i;
}

}  // namespace

// k_conv covers the conv when its re-laid weights are given, the channels
// come in whole stages, the window halo fits and the output fills the chip
// (small first-packet decodes keep the split-K GEMM).
static int conv_splits(const XGemm &g);
static bool conv_ok(const XGemm &g) {
    constexpr int min_tiles = 96;
    if (!g.wt || g.bmode != XB_CONV || g.amode != XA_ROWS ||
        !(g.Kw == 1 || g.Kw == 2 || g.Kw == 3 || g.Kw == 7) || (g.K / g.Kw) % CV_BC ||
        (g.Kw - 1) * g.dil > CV_HALO || ((uintptr_t)g.wt & 15))
        return false;
    const int tiles = ((g.N + CV_BN - 1) / CV_BN) * ((g.M + CV_BM - 1) / CV_BM) * (g.stride > 1 ? g.stride : 1);
    return tiles >= min_tiles || (g.part && conv_splits(g) > 1);
}

// input-channel splits for a grid that would not fill the chip: up to 1024
// workgroups, >= 2 channel stages each
static int conv_splits(const XGemm &g) {
    if (!g.part) return 1;
    const int nph = g.stride > 1 ? g.stride : 1;
    const int tiles = ((g.N + CV_BN - 1) / CV_BN) * ((g.M + CV_BM - 1) / CV_BM) * nph;
    const int ci = g.K / g.Kw;
    int nz = 1;
    while (tiles * nz * 2 <= 1024 && (ci / CV_BC) % (nz * 2) == 0 && ci / CV_BC / (nz * 2) >= 2 &&
           (size_t)nz * 2 * nph * g.M * g.N <= g.part_elems)
        nz *= 2;
    return nz;
}

static int conv_launch(const XGemm &gin, int nph, hipStream_t st) {
    XGemm g = gin;
    g.kz = conv_splits(g);
    const dim3 cg((g.N + CV_BN - 1) / CV_BN, (g.M + CV_BM - 1) / CV_BM, nph * g.kz);
    // bf16 3-plane MFMA path, except a SnakeBeta prologue over more input
    // channels than its staging covers (then the fp32 MFMA k_conv)
    const bool bf = !g.sa || g.K / g.Kw / (g.kz > 1 ? g.kz : 1) <= CB_SNAKE_MAX;
    if (bf) {
        // 256-column tiles where the grid still holds >= 2 workgroups per CU
        // (the two column blocks' MFMA chains interleaved measured the same:
        // codec 7.9 ms per 128 frames either way, profiles/r05st_ab_codec.txt)
        const int tiles4 = ((g.N + 255) / 256) * cg.y * cg.z;
        if (tiles4 >= 512) {
            const dim3 c4((g.N + 255) / 256, cg.y, cg.z);
            switch (g.Kw) {
                case 7: hipLaunchKernelGGL((k_convb<7, 4>), c4, dim3(512), 0, st, g); break;
                case 3: hipLaunchKernelGGL((k_convb<3, 4>), c4, dim3(512), 0, st, g); break;
                case 2: hipLaunchKernelGGL((k_convb<2, 4>), c4, dim3(512), 0, st, g); break;
                default: hipLaunchKernelGGL((k_convb<1, 4>), c4, dim3(512), 0, st, g); break;
            }
        } else {
            switch (g.Kw) {
                case 7: hipLaunchKernelGGL((k_convb<7, 2>), cg, dim3(256), 0, st, g); break;
                case 3: hipLaunchKernelGGL((k_convb<3, 2>), cg, dim3(256), 0, st, g); break;
                case 2: hipLaunchKernelGGL((k_convb<2, 2>), cg, dim3(256), 0, st, g); break;
                default: hipLaunchKernelGGL((k_convb<1, 2>), cg, dim3(256), 0, st, g); break;
            }
        }
    } else {
        switch (g.Kw) {
            case 7: hipLaunchKernelGGL(k_conv<7>, cg, dim3(256), 0, st, g); break;
            case 3: hipLaunchKernelGGL(k_conv<3>, cg, dim3(256), 0, st, g); break;
            case 2: hipLaunchKernelGGL(k_conv<2>, cg, dim3(256), 0, st, g); break;
            default: hipLaunchKernelGGL(k_conv<1>, cg, dim3(256), 0, st, g); break;
        }
    }
    if (g.kz > 1) {
        const size_t n = (size_t)nph * g.M * g.N;
        hipLaunchKernelGGL(k_conv_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, nph);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// k_xgemv covers a linear at <= 4 rows
static bool xgemv_ok(const XGemm &g) {
    return g.M <= 4 && g.bmode == XB_WT && (g.amode == XA_ROWS || g.amode == XA_TRANS) && g.K % 256 == 0 &&
           g.ldb % 4 == 0 && ((uintptr_t)g.B & 15) == 0 && (size_t)4 * g.K * 4 + 512 <= 64 * 1024;
}

// k_xlin covers plain fp32 linears above k_xgemv's 4 rows with 16-B rows
static bool xlin_ok(const XGemm &g) {
    return g.amode == XA_ROWS && g.bmode == XB_WT && g.M > 4 && g.N % 64 == 0 && g.K % XL_KS == 0 &&
           g.lda % 4 == 0 && g.ldb % 4 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0;
}

int qtts_xgemm(const XGemm &g, hipStream_t st) {
    if (g.M <= 0 || g.N <= 0 || g.K <= 0) return 0;
    static const bool xl_on = [] { const char *e = getenv("QTTS_HIP_XLIN"); return !(e && !atoi(e)); }();
    if (xl_on && xlin_ok(g)) {
        dim3 grid(g.N / 64, (g.M + 63) / 64, 1);
        // split-K where the tiles would not fill the chip: >= 1 stage each,
        // partials within the workspace
        const int tiles = grid.x * grid.y, nst = g.K / XL_KS;
        int nz = 1;
        if (g.part && tiles < 256) {
            nz = (256 + tiles - 1) / tiles;
            if (nz > nst) nz = nst;
            while (nz > 1 && (size_t)nz * g.M * g.N > g.part_elems) --nz;
        }
        grid.z = nz;
        hipLaunchKernelGGL(k_xlin, grid, dim3(256), 0, st, g);
        if (nz > 1) {
            const size_t n = (size_t)g.M * g.N;
            hipLaunchKernelGGL(k_xg_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, nz);
        }
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (xgemv_ok(g)) {
        int ks = 1;   // KSPLIT: grid >= 512 workgroups, >= 1 block per lane
        while (ks < 32 && (g.N + 32 / ks - 1) / (32 / ks) < 512 && g.K / 32 / (2 * ks) >= 1) ks *= 2;
        const int rpw = 32 / ks;
        hipLaunchKernelGGL(k_xgemv, dim3((g.N + rpw - 1) / rpw), dim3(256), (size_t)(4 * g.K + 128) * 4, st, g, ks);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (conv_ok(g)) return conv_launch(g, g.stride > 1 ? g.stride : 1, st);
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, 1);
    // split-K when the output has too few tiles to fill the chip (first-packet
    // sized decodes): z ranges of >= 8 K-steps, partials in g.part
    const int tiles = grid.x * grid.y, ksteps = (g.K + BK - 1) / BK;
    int nz = 1;
    if (g.part && tiles < 192 && ksteps >= 16) {
        nz = (256 + tiles - 1) / tiles;
        if (nz > ksteps / 8) nz = ksteps / 8;
        if (nz > 32) nz = 32;
        while (nz > 1 && (size_t)nz * g.M * g.N > g.part_elems) --nz;
    }
    grid.z = nz;
    hipLaunchKernelGGL(k_xgemm, grid, dim3(256), 0, st, g);
    if (nz > 1) {
        const size_t n = (size_t)g.M * g.N;
        hipLaunchKernelGGL(k_xg_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, nz);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ===================================================================== model
static float *cw(CodecModel *m, const std::string &n) {
    auto it = m->w.find(n);
    return it == m->w.end() ? nullptr : it->second;
}

// a relayout of cnt floats is followed in its allocation (cnt * 10 bytes) by
// its three bf16 planes (k_convb)
static void wt_planes(float *t, size_t cnt, hipStream_t st) {
    hipLaunchKernelGGL(k_wt_split, dim3((unsigned)((cnt / 2 + 256) / 256)), dim3(256), 0, st, t, cnt,
                       reinterpret_cast<unsigned short *>(t + cnt));
}

// conv weight `n` ([co][ci][Kw]) re-laid as [Kw][co][ci] for k_conv, made on first use
static const float *cwt(CodecModel *m, const std::string &n, int co, int ci, int Kw) {
    auto it = m->wt.find(n);
    if (it != m->wt.end()) return it->second;
    const float *w = cw(m, n);
    float *t = nullptr;
    const size_t cnt = (size_t)co * ci * Kw;
    if (!w || hipMalloc(&t, cnt * 10) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(k_wt_relayout, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, m->st, w, co, ci, Kw, t);
    wt_planes(t, cnt, m->st);
    m->wt[n] = t;
    m->wbytes += cnt * 10;
    return t;
}

void codec_init(CodecModel *m, const qtts_dims_t *d, hipStream_t st) {
    m->d = *d;
    m->st = st;
}

void codec_free_state(CodecModel *m) {
    for (void *p : m->scratch) hipFree(p);
    m->scratch.clear();
    m->scratch_bytes = 0;
    m->buf_elems = 0;
    m->t_cap = 0;
    m->rope_cap = 0;
    m->bufA = m->bufB = m->bufC = m->bufD = nullptr;
    m->tq = m->tx = m->txn = m->tatt = m->tg = m->tu = nullptr;
    m->rope_cos = m->rope_sin = nullptr;
    m->codes_tmp = nullptr;
    // the split-K workspace lives in `scratch` too: a stream that outlives this
    // state (codec_stream_begin's reuse path) must re-create it, never reuse it
    m->xg_part = nullptr;
    m->xg_part_elems = 0;
}

void codec_destroy(CodecModel *m) {
    for (hipEvent_t &e : m->tev)
        if (e) { hipEventDestroy(e); e = nullptr; }
    codec_stream_free(m);
    codec_free_state(m);
    for (auto &kv : m->w) hipFree(kv.second);
    m->w.clear();
    for (auto &kv : m->wt) hipFree(kv.second);
    m->wt.clear();
    if (m->cb) hipFree(m->cb);
    m->cb = nullptr;
}

size_t codec_weight_bytes(const CodecModel *m) { return m->wbytes; }

static float f32_of(const void *h, int dtype, size_t i) {
    if (dtype == 0) return ((const float *)h)[i];
    uint16_t v = ((const uint16_t *)h)[i];
    if (dtype == 1) {
        uint32_t u = (uint32_t)v << 16;
        float f;
        memcpy(&f, &u, 4);
        return f;
    }
    _Float16 x;
    memcpy(&x, &v, 2);
    return (float)x;
}

static int build_codebook(CodecModel *m, int q) {
    const qtts_dims_t &d = m->d;
    std::string u, e;
    if (q == 0) {
        u = "decoder.quantizer.rvq_first.vq.layers.0._codebook.cluster_usage";
        e = "decoder.quantizer.rvq_first.vq.layers.0._codebook.embedding_sum";
    } else {
        u = "decoder.quantizer.rvq_rest.vq.layers." + std::to_string(q - 1) + "._codebook.cluster_usage";
        e = "decoder.quantizer.rvq_rest.vq.layers." + std::to_string(q - 1) + "._codebook.embedding_sum";
    }
    if (!m->host_keep.count(u) || !m->host_keep.count(e)) return 0;  // wait for both
    const int CB = d.ccb, vq = d.ccbdim / 2;
    std::vector<float> &us = m->host_keep[u], &es = m->host_keep[e];
    if ((int)us.size() != CB || (int)es.size() != CB * vq) {
        fprintf(stderr, "qtts codec: codebook %d has unexpected shape\n", q);
        return -1;
    }
    std::vector<float> cb((size_t)CB * vq);
    for (int c = 0; c < CB; ++c) {  // Q.c:584-592
        float usage = us[c];
        if (usage < 1e-5f) usage = 1e-5f;
        const float inv = 1.0f / usage;
        for (int k = 0; k < vq; ++k) cb[(size_t)c * vq + k] = es[(size_t)c * vq + k] * inv;
    }
    if (!m->cb) {
        size_t bytes = (size_t)d.cq * CB * vq * 4;
        if (hipMalloc(&m->cb, bytes) != hipSuccess) return -1;
        m->wbytes += bytes;
    }
    if (hipMemcpy(m->cb + (size_t)q * CB * vq, cb.data(), cb.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return -1;
    m->host_keep.erase(u);
    m->host_keep.erase(e);
    m->w["__cb" + std::to_string(q)] = nullptr;  // marker
    return 0;
}

int codec_put_tensor(CodecModel *m, const std::string &name, const void *host, int dtype, const int64_t *shape,
                     int ndim, size_t n) {
    std::vector<float> f(n);
    for (size_t i = 0; i < n; ++i) f[i] = f32_of(host, dtype, i);
    const bool is_usage = name.find("._codebook.cluster_usage") != std::string::npos;
    const bool is_esum = name.find("._codebook.embedding_sum") != std::string::npos;
    if (is_usage || is_esum) {
        m->host_keep[name] = std::move(f);
        const std::string pre1 = "decoder.quantizer.rvq_first.vq.layers.0.";
        const std::string pre2 = "decoder.quantizer.rvq_rest.vq.layers.";
        int q = -1;
        if (name.compare(0, pre1.size(), pre1) == 0) q = 0;
        else if (name.compare(0, pre2.size(), pre2) == 0) q = 1 + atoi(name.c_str() + pre2.size());
        if (q < 0 || q >= m->d.cq) return 0;
        return build_codebook(m, q);
    }
    // SnakeBeta parameters pre-exponentiated with libm (Q.c:596-602)
    const size_t L = name.size();
    if (L > 6 && (name.compare(L - 6, 6, ".alpha") == 0)) {
        for (auto &v : f) v = expf(v);
    } else if (L > 5 && name.compare(L - 5, 5, ".beta") == 0) {
        for (auto &v : f) v = 1.0f / (expf(v) + 1e-9f);
    }
    float *p = nullptr;
    if (hipMalloc(&p, n * 4) != hipSuccess) return -1;
    m->wbytes += n * 4;
    if (hipMemcpy(p, f.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (m->w.count(name) && m->w[name]) hipFree(m->w[name]);
    m->w[name] = p;
    m->shape[name] = std::vector<int64_t>(shape, shape + ndim);
    return 0;
}

int codec_finalize(CodecModel *m) {
    const qtts_dims_t &d = m->d;
    std::vector<std::string> need = {"decoder.quantizer.rvq_first.output_proj.weight",
                                     "decoder.quantizer.rvq_rest.output_proj.weight", "decoder.pre_conv.conv.weight",
                                     "decoder.pre_transformer.input_proj.weight",
                                     "decoder.pre_transformer.output_proj.weight", "decoder.decoder.0.conv.weight",
                                     "decoder.decoder.6.conv.weight"};
    for (int q = 0; q < d.cq; ++q) need.push_back("__cb" + std::to_string(q));
    for (int l = 0; l < d.clayers; ++l)
        for (const char *s : {"input_layernorm.weight", "post_attention_layernorm.weight", "self_attn.q_proj.weight",
                              "self_attn.k_proj.weight", "self_attn.v_proj.weight", "self_attn.o_proj.weight",
                              "mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight"})
            need.push_back("decoder.pre_transformer.layers." + std::to_string(l) + "." + s);
    for (int s = 0; s < 2; ++s)
        for (const char *t : {"0.conv.weight", "0.conv.bias", "1.dwconv.conv.weight", "1.norm.weight", "1.norm.bias",
                              "1.pwconv1.weight", "1.pwconv1.bias", "1.pwconv2.weight", "1.pwconv2.bias", "1.gamma"})
            need.push_back("decoder.upsample." + std::to_string(s) + "." + t);
    for (int b = 0; b < 4; ++b) {
        const std::string p = "decoder.decoder." + std::to_string(b + 1) + ".block.";
        for (const char *t : {"0.alpha", "0.beta", "1.conv.weight", "1.conv.bias"}) need.push_back(p + t);
        for (int r = 0; r < 3; ++r)
            for (const char *t : {"act1.alpha", "act1.beta", "conv1.conv.weight", "conv1.conv.bias", "act2.alpha",
                                  "act2.beta", "conv2.conv.weight", "conv2.conv.bias"})
                need.push_back(p + std::to_string(r + 2) + "." + t);
    }
    for (auto &n : need)
        if (!m->w.count(n)) {
            fprintf(stderr, "Error: codec decoder is not fully loaded (missing %s)\n", n.c_str());
            return -1;
        }
    if (d.clat / 2 != d.ccbdim) {
        fprintf(stderr, "Error: codec requires codebook_dim == latent_dim/2 (got %d, %d)\n", d.ccbdim, d.clat);
        return -1;
    }
    return 0;
}

static void *scratch_alloc(CodecModel *m, size_t bytes) {
    void *p = nullptr;
    const hipError_t prior = hipPeekAtLastError();
    const hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        fprintf(stderr, "qtts codec: hipMalloc(%zu) failed: %s (last error before it: %s)\n", bytes,
                hipGetErrorName(e), hipGetErrorName(prior));
        return nullptr;
    }
    m->scratch.push_back(p);
    m->scratch_bytes += bytes;
    return p;
}

// largest channel-major intermediate over the decoder at `cap` frames (elements)
static size_t codec_buf_elems(const qtts_dims_t &d, int cap) {
    size_t L = (size_t)cap * d.ratios[0] * d.ratios[1];
    size_t mx = (size_t)d.clat * L * 4;  // ConvNeXt pw1 [L][4C]
    if ((size_t)d.cdec * L > mx) mx = (size_t)d.cdec * L;
    int C = d.cdec;
    for (int b = 0; b < 4; ++b) {
        L *= d.rates[b];
        C /= 2;
        if ((size_t)C * L > mx) mx = (size_t)C * L;
    }
    const size_t lat_t = (size_t)d.clat * cap;
    return lat_t > mx ? lat_t : mx;
}

// device bytes of one decode state for T frames (ensure_codec_state's allocations)
size_t codec_state_bytes(const CodecModel *m, int T) {
    const qtts_dims_t &d = m->d;
    const size_t cap = T < 64 ? 64 : T;
    const size_t hid = d.chid, kvd = (size_t)d.ckv * (d.chid / d.cheads);
    return 4 * codec_buf_elems(d, (int)cap) * 4 + cap * (4 * hid + 2 * kvd + 2 * (size_t)d.cinter + 2) * 4 +
           ((size_t)8 << 20) * 4 + 2 * cap * (hid / d.cheads) * 4;
}

static int ensure_codec_state(CodecModel *m, int T) {
    const qtts_dims_t &d = m->d;
    if (T <= m->t_cap) return 0;
    codec_free_state(m);
    const int cap = T < 64 ? 64 : T;
    const size_t mx = codec_buf_elems(d, cap);
    m->buf_elems = mx;
    m->bufA = (float *)scratch_alloc(m, mx * 4);
    m->bufB = (float *)scratch_alloc(m, mx * 4);
    m->bufC = (float *)scratch_alloc(m, mx * 4);
    m->bufD = (float *)scratch_alloc(m, mx * 4);
    const int hid = d.chid, kvd = d.ckv * (d.chid / d.cheads);
    m->tx = (float *)scratch_alloc(m, (size_t)cap * hid * 4);
    m->txn = (float *)scratch_alloc(m, (size_t)cap * hid * 4);
    m->tq = (float *)scratch_alloc(m, (size_t)cap * (hid + 2 * kvd) * 4);
    m->tatt = (float *)scratch_alloc(m, (size_t)cap * hid * 4);
    m->tg = (float *)scratch_alloc(m, (size_t)cap * d.cinter * 4);
    m->tu = (float *)scratch_alloc(m, (size_t)cap * d.cinter * 4);
    m->codes_tmp = (int *)scratch_alloc(m, (size_t)cap * 2 * 4);  // [0..cap) positions, [cap..2cap) zeros
    m->xg_part_elems = (size_t)8 << 20;
    m->xg_part = (float *)scratch_alloc(m, m->xg_part_elems * 4);
    if (!m->xg_part) return -1;
    if (!m->bufA || !m->bufB || !m->bufC || !m->bufD || !m->tx || !m->txn || !m->tq || !m->tatt || !m->tg || !m->tu ||
        !m->codes_tmp)
        return -1;
    hipLaunchKernelGGL(k_iota, dim3((cap + 255) / 256), dim3(256), 0, m->st, m->codes_tmp, cap, 0);
    hipLaunchKernelGGL(k_iota, dim3((cap + 255) / 256), dim3(256), 0, m->st, m->codes_tmp + cap, cap, 1);
    // RoPE table (theta fixed at 1e4 in the reference, Cd.c:309; head_dim = hidden/heads, Cd.c:275)
    const int hd = d.chid / d.cheads, half = hd / 2;
    std::vector<float> c((size_t)cap * hd), s((size_t)cap * hd);
    for (int p = 0; p < cap; ++p)
        for (int i = 0; i < half; ++i) {
            float freq = 1.0f / powf(10000.0f, (float)(2 * i) / (float)hd);
            float ang = (float)p * freq;
            c[(size_t)p * hd + i] = c[(size_t)p * hd + i + half] = cosf(ang);
            s[(size_t)p * hd + i] = s[(size_t)p * hd + i + half] = sinf(ang);
        }
    m->rope_cos = (float *)scratch_alloc(m, c.size() * 4);
    m->rope_sin = (float *)scratch_alloc(m, s.size() * 4);
    if (!m->rope_cos || !m->rope_sin) return -1;
    if (hipMemcpy(m->rope_cos, c.data(), c.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (hipMemcpy(m->rope_sin, s.data(), s.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    m->t_cap = cap;
    return 0;
}

#define KCK(x) do { if ((x) != 0) return -1; } while (0)

// codec GEMMs get the split-K workspace
static int xgm(CodecModel *m, XGemm g, hipStream_t st) {
    g.part = m->xg_part;   // nullptr (kernel-level entries' stateless model): no split
    g.part_elems = m->xg_part_elems;
    return qtts_xgemm(g, st);
}

static XGemm lin(const float *A, int M, int K, const float *W, int N, float *C, int emode) {
    XGemm g;
    g.M = M; g.N = N; g.K = K; g.amode = XA_ROWS; g.A = A; g.lda = K; g.bmode = XB_WT; g.B = W; g.ldb = K;
    g.C = C; g.ldc = N; g.emode = emode;
    return g;
}

// causal conv as implicit GEMM: out[co][L] = W[co][ci*K] . im2col(snake?(x))
static int conv(CodecModel *m, const float *x, int ci, int L, const std::string &wn, const std::string &bn, int co,
                int K, int dil, float *out, int emode, const float *sa, const float *sb, const float *res,
                const float *ea = nullptr, const float *eb = nullptr) {
    XGemm g;
    g.M = co; g.N = L; g.K = ci * K;
    g.amode = XA_ROWS; g.A = cw(m, wn); g.lda = ci * K; g.wt = cwt(m, wn, co, ci, K);
    g.bmode = XB_CONV; g.B = x; g.ldb = L; g.Kw = K; g.dil = dil; g.pad = (K - 1) * dil; g.L = L;
    g.sa = sa; g.sb = sb;
    g.C = out; g.ldc = L; g.emode = emode; g.bias = bn.empty() ? nullptr : cw(m, bn); g.res = res; g.ldres = L;
    g.ea = ea; g.eb = eb;
    if (!g.A) return -1;
    return xgm(m, g, m->st);
}

// transposed conv (stride s, kernel Kw = s * ntap) as s phase GEMMs
// transposed-conv weights re-laid per phase for k_conv (k_wt_tconv), made on first use
static const float *ctwt(CodecModel *m, const float *w, int ci, int co, int Kw, int s, hipStream_t st) {
    const std::string key = "tconv#" + std::to_string((uintptr_t)w);
    auto it = m->wt.find(key);
    if (it != m->wt.end()) return it->second;
    float *t = nullptr;
    const size_t cnt = (size_t)co * ci * Kw;
    if (!w || hipMalloc(&t, cnt * 10) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(k_wt_tconv, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, w, ci, co, Kw, s, t);
    wt_planes(t, cnt, st);
    m->wt[key] = t;
    m->wbytes += cnt * 10;
    return t;
}

// a transposed conv (kernel Kw = ntap*s, stride s) as s causal convs of ntap
// taps over the same input, one per output phase, in one k_conv launch
// (grid z = phase) when k_conv covers it; else one implicit GEMM per phase
static int tconv_run(CodecModel *m, const XGemm &g, hipStream_t st) {
    const int s = g.stride, nt = g.Kw / s, ci = g.K / nt;
    XGemm c = g;
    c.amode = XA_ROWS; c.A = nullptr; c.bmode = XB_CONV; c.Kw = nt; c.dil = 1; c.pad = nt - 1; c.phase = 0;
    c.wt = (const float *)16;  // shape-only probe before the relayout is made
    c.part = m->xg_part;
    c.part_elems = m->xg_part_elems;
    if (conv_ok(c)) {
        c.wt = ctwt(m, g.A, ci, g.co, g.Kw, s, st);
        if (c.wt) return xgm(m, c, st);
    }
    for (int ph = 0; ph < s; ++ph) {
        XGemm p = g;
        p.phase = ph;
        KCK(xgm(m, p, st));
    }
    return 0;
}

static int tconv(CodecModel *m, const float *x, int ci, int L, const float *w, const float *bias, int co, int Kw,
                 int s, float *out, const float *sa, const float *sb, hipStream_t st) {
    XGemm g;
    g.M = co; g.N = L; g.K = ci * (Kw / s);
    g.amode = XA_TCONV_W; g.A = w; g.co = co; g.Kw = Kw; g.stride = s;
    g.bmode = XB_TCONV; g.B = x; g.ldb = L; g.L = L; g.sa = sa; g.sb = sb;
    g.C = out; g.ldc = L * s; g.emode = XE_BIAS_M; g.bias = bias;
    return tconv_run(m, g, st);
}

static int codec_transformer(CodecModel *m, const float *pc /*[lat][T]*/, int T, float *out /*[lat][T]*/) {
    const qtts_dims_t &d = m->d;
    const int lat = d.clat, hid = d.chid, nh = d.cheads, nkv = d.ckv, hd = hid / nh, kvd = nkv * hd, I = d.cinter;
    hipStream_t st = m->st;
    const std::string P = "decoder.pre_transformer.";
    XGemm g;
    g.M = T; g.N = hid; g.K = lat; g.amode = XA_TRANS; g.A = pc; g.lda = T; g.bmode = XB_WT;
    g.B = cw(m, P + "input_proj.weight"); g.ldb = lat; g.C = m->tx; g.ldc = hid;
    g.bias = cw(m, P + "input_proj.bias");
    g.emode = g.bias ? XE_BIAS_N : XE_STORE;
    KCK(xgm(m, g, st));
    float *q = m->tq, *k = m->tq + (size_t)T * hid, *v = k + (size_t)T * kvd;
    for (int l = 0; l < d.clayers; ++l) {
        const std::string p = P + "layers." + std::to_string(l) + ".";
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, m->tx, hid, cw(m, p + "input_layernorm.weight"),
                           d.ceps, m->txn);
        KCK(xgm(m, lin(m->txn, T, hid, cw(m, p + "self_attn.q_proj.weight"), hid, q, XE_STORE), st));
        KCK(xgm(m, lin(m->txn, T, hid, cw(m, p + "self_attn.k_proj.weight"), kvd, k, XE_STORE), st));
        KCK(xgm(m, lin(m->txn, T, hid, cw(m, p + "self_attn.v_proj.weight"), kvd, v, XE_STORE), st));
        hipLaunchKernelGGL(k_rope_rows, dim3(T), dim3(256), 0, st, q, hid, nh, hd, m->rope_cos, m->rope_sin);
        hipLaunchKernelGGL(k_rope_rows, dim3(T), dim3(256), 0, st, k, kvd, nkv, hd, m->rope_cos, m->rope_sin);
        AttnArgs a;
        a.mode = 1; a.qkv = q; a.ld_qkv = hid; a.kc = k; a.vc = v; a.S = T; a.pos = m->codes_tmp;
        a.row_b = m->codes_tmp + m->t_cap; a.NH = nh; a.KV = nkv; a.HD = hd; a.out = m->tatt; a.ld_out = hid;
        a.nrows = T; a.win = d.cwin;
        KCK(qtts_attention(a, st));
        const float *ls1 = cw(m, p + "self_attn_layer_scale.scale");
        XGemm o = lin(m->tatt, T, hid, cw(m, p + "self_attn.o_proj.weight"), hid, m->tx, XE_SCALE_RESID_N);
        o.vec = ls1;
        if (!ls1) return -1;
        KCK(xgm(m, o, st));
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, m->tx, hid,
                           cw(m, p + "post_attention_layernorm.weight"), d.ceps, m->txn);
        KCK(xgm(m, lin(m->txn, T, hid, cw(m, p + "mlp.gate_proj.weight"), I, m->tg, XE_STORE), st));
        XGemm u = lin(m->txn, T, hid, cw(m, p + "mlp.up_proj.weight"), I, m->tu, XE_SILU_MUL);
        u.aux = m->tg; u.ldaux = I;
        KCK(xgm(m, u, st));
        const float *ls2 = cw(m, p + "mlp_layer_scale.scale");
        XGemm dn = lin(m->tu, T, I, cw(m, p + "mlp.down_proj.weight"), hid, m->tx, XE_SCALE_RESID_N);
        dn.vec = ls2;
        if (!ls2) return -1;
        KCK(xgm(m, dn, st));
    }
    const float *fn = cw(m, P + "norm.weight");
    const float *xin = m->tx;
    if (fn) {
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, m->tx, hid, fn, d.ceps, m->txn);
        xin = m->txn;
    }
    XGemm og = lin(xin, T, hid, cw(m, P + "output_proj.weight"), lat, out, XE_BIAS_T);
    og.bias = cw(m, P + "output_proj.bias");
    og.ldc = T;
    if (!og.bias) return -1;
    return xgm(m, og, st);
}

// the whole decode enqueued on m->st; the clamped waveform stays in m's
// scratch (*wav, *L samples) until the next use of m
static int codec_decode_enqueue(CodecModel *m, const int *codes, int T, float **wav_out, int *L_out) {
    const qtts_dims_t &d = m->d;
    if (ensure_codec_state(m, T)) return -1;
    hipStream_t st = m->st;
    const int lat = d.clat, vq = d.ccbdim / 2, half = lat / 2;
    float *A = m->bufA, *B = m->bufB, *Cb = m->bufC, *D = m->bufD;
#define DCK(x) do { if ((x) != 0) { fprintf(stderr, "qtts codec: stage failed at %s:%d\n", __FILE__, __LINE__); return -1; } } while (0)
    m->timed = false;
    if (m->timing && !m->tev[0])
        for (hipEvent_t &e : m->tev)
            if (hipEventCreate(&e) != hipSuccess) { e = nullptr; m->timing = false; }
    auto mark = [&](int i) { if (m->timing) hipEventRecord(m->tev[i], st); };
    mark(0);
    // 1. RVQ dequantise -> A [half][T]
    hipLaunchKernelGGL(k_rvq_sum, dim3(T), dim3(vq < 64 ? 64 : (vq + 63) / 64 * 64), 0, st, codes, T, d.cq, d.ccb, vq,
                       m->cb, B, Cb);
    hipLaunchKernelGGL(k_rvq_proj, dim3((half * T + 3) / 4), dim3(256), 0, st,
                       cw(m, "decoder.quantizer.rvq_first.output_proj.weight"),
                       cw(m, "decoder.quantizer.rvq_rest.output_proj.weight"), B, Cb, vq, half, T, T, A);
    mark(1);
    // 2. pre-conv k=3 -> B [lat][T]
    DCK(conv(m, A, d.ccbdim, T, "decoder.pre_conv.conv.weight", "decoder.pre_conv.conv.bias", lat, 3, 1, B, XE_BIAS_M,
             nullptr, nullptr, nullptr));
    mark(2);
    // 3. transformer -> A [lat][T]
    DCK(codec_transformer(m, B, T, A));
    mark(3);
    // 4. upsample: transposed conv + ConvNeXt, x2
    int L = T;
    float *cur = A;
    for (int s = 0; s < 2; ++s) {
        const int f = d.ratios[s];
        const std::string p = "decoder.upsample." + std::to_string(s) + ".";
        float *up = cur == A ? B : A;
        DCK(tconv(m, cur, lat, L, cw(m, p + "0.conv.weight"), cw(m, p + "0.conv.bias"), lat, f, f, up, nullptr, nullptr,
                  st));
        L *= f;
        cur = up;
        // ConvNeXt: dwconv -> LN (time-major) -> pw1+GELU -> pw2*gamma (+res, channel-major)
        hipLaunchKernelGGL(k_dwconv, dim3((unsigned)(((size_t)lat * L + 255) / 256)), dim3(256), 0, st, cur, L, 0,
                           cw(m, p + "1.dwconv.conv.weight"), cw(m, p + "1.dwconv.conv.bias"), lat, L, 7, Cb, L);
        hipLaunchKernelGGL(k_ln_t, dim3(L), dim3(256), 0, st, Cb, L, lat, cw(m, p + "1.norm.weight"),
                           cw(m, p + "1.norm.bias"), 1e-6f, D);
        XGemm g1 = lin(D, L, lat, cw(m, p + "1.pwconv1.weight"), 4 * lat, Cb, XE_BIAS_N_GELU);
        g1.bias = cw(m, p + "1.pwconv1.bias");
        DCK(xgm(m, g1, st));
        XGemm g2 = lin(Cb, L, 4 * lat, cw(m, p + "1.pwconv2.weight"), lat, cur, XE_BIAS_GAMMA_RES_T);
        g2.bias = cw(m, p + "1.pwconv2.bias");
        g2.vec = cw(m, p + "1.gamma");
        g2.res = cur; g2.ldres = L; g2.ldc = L;
        DCK(xgm(m, g2, st));
    }
    mark(4);
    // 5. vocoder
    float *voc = cur == A ? B : A;
    DCK(conv(m, cur, lat, L, "decoder.decoder.0.conv.weight", "decoder.decoder.0.conv.bias", d.cdec, 7, 1, voc,
             XE_BIAS_M, nullptr, nullptr, nullptr));
    int C = d.cdec;
    static const int dil[3] = {1, 3, 9};
    for (int b = 0; b < 4; ++b) {
        const int r = d.rates[b], co = C / 2;
        const std::string p = "decoder.decoder." + std::to_string(b + 1) + ".block.";
        float *nx = voc == A ? B : A;
        DCK(tconv(m, voc, C, L, cw(m, p + "1.conv.weight"), cw(m, p + "1.conv.bias"), co, 2 * r, r, nx,
                  cw(m, p + "0.alpha"), cw(m, p + "0.beta"), st));
        L *= r;
        C = co;
        voc = nx;
        for (int u = 0; u < 3; ++u) {
            const std::string q = p + std::to_string(u + 2) + ".";
            // conv1(snake1(x)) -> snake2 fused in the epilogue -> Cb
            DCK(conv(m, voc, C, L, q + "conv1.conv.weight", q + "conv1.conv.bias", C, 7, dil[u], Cb, XE_BIAS_M_SNAKE,
                     cw(m, q + "act1.alpha"), cw(m, q + "act1.beta"), nullptr, cw(m, q + "act2.alpha"),
                     cw(m, q + "act2.beta")));
            // conv2 (k=1) + residual, in place on x
            DCK(conv(m, Cb, C, L, q + "conv2.conv.weight", q + "conv2.conv.bias", C, 1, 1, voc, XE_BIAS_M_RES, nullptr,
                     nullptr, voc));
        }
    }
    // final SnakeBeta + conv -> 1 channel, clamp
    float *wav = voc == A ? B : A;
    DCK(conv(m, voc, C, L, "decoder.decoder.6.conv.weight", "decoder.decoder.6.conv.bias", 1, 7, 1, wav, XE_BIAS_M,
             cw(m, "decoder.decoder.5.alpha"), cw(m, "decoder.decoder.5.beta"), nullptr));
    hipLaunchKernelGGL(k_clamp, dim3((L + 255) / 256), dim3(256), 0, st, wav, L);
    mark(5);
    *wav_out = wav;
    *L_out = L;
    return hipGetLastError() == hipSuccess ? 0 : -1;
#undef DCK
}

float *codec_decode(CodecModel *m, const int *codes, int T, int *out_samples) {
    if (out_samples) *out_samples = 0;
    float *wav = nullptr;
    int L = 0;
    if (codec_decode_enqueue(m, codes, T, &wav, &L)) return nullptr;
    float *host = (float *)malloc((size_t)L * sizeof(float));
    if (!host) return nullptr;
    if (hipMemcpyAsync(host, wav, (size_t)L * 4, hipMemcpyDeviceToHost, m->st) != hipSuccess ||
        hipStreamSynchronize(m->st) != hipSuccess) {
        free(host);
        return nullptr;
    }
    if (m->timing) {
        for (int i = 0; i < 5; ++i) hipEventElapsedTime(&m->stage_ms[i], m->tev[i], m->tev[i + 1]);
        m->timed = true;
    }
    if (out_samples) *out_samples = L;
    return host;
}

// ---------------------------------------------------------------- independent decodes side by side
// A batch's utterances are decoded by independent codec passes (one per slot,
// as qwen_tts_generate decodes its one utterance, Cd.c:581-749).  One pass is
// a chain of ~200 launches, most of them latency-bound (the transformer's
// 128-row GEMMs, the small-channel early convs), so several passes run side by
// side: lane k (m itself for k = 0, else a CodecModel that shares m's weights
// and re-laid weights and owns its scratch, split-K workspace and stream)
// decodes jobs k, k + nl, ...; each job's waveform goes device-to-device into
// `dwav` behind its last kernel (the lane's scratch is reused by its next job
// in stream order), and the host waits once for every lane.  The kernels,
// shapes and split decisions are a lone decode's, so the audio is
// bit-identical to codec_decode's.
static void lane_sync_weights(CodecModel *m, CodecModel *ln) {
    ln->d = m->d;
    ln->cb = m->cb;
    ln->w = m->w;
    ln->wt = m->wt;
    ln->timing = false;
}

CodecModel *codec_lane_new(CodecModel *m, hipStream_t st) {
    CodecModel *ln = new CodecModel;
    lane_sync_weights(m, ln);
    ln->st = st;
    return ln;
}

// (every re-laid weight a lane made was adopted by m or freed by
// codec_decode_many, so the lane owns only its scratch)
void codec_lane_delete(CodecModel *ln) {
    if (!ln) return;
    ln->wt.clear();
    ln->w.clear();
    codec_free_state(ln);
    delete ln;
}

int codec_decode_many(CodecModel *m, CodecModel *const *lanes, int nl, int n, const int *const *codes,
                      const int *T, float *dwav, const size_t *dwav_off, int *out_samples) {
    if (nl < 1 || n < 0) return -1;
    if (nl > n) nl = n;
    for (int k = 1; k < nl; ++k) lane_sync_weights(m, lanes[k]);
    hipEvent_t ready = nullptr;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess) return -1;
    int rc = hipEventRecord(ready, m->st) == hipSuccess ? 0 : -1;   // the codes were written on m->st
    for (int k = 1; k < nl && !rc; ++k)
        if (hipStreamWaitEvent(lanes[k]->st, ready, 0) != hipSuccess) rc = -1;
    for (int i = 0; i < n && !rc; ++i) {
        CodecModel *ln = i % nl == 0 ? m : lanes[i % nl];
        float *wav = nullptr;
        int L = 0;
        if (codec_decode_enqueue(ln, codes[i], T[i], &wav, &L) ||
            hipMemcpyAsync(dwav + dwav_off[i], wav, (size_t)L * 4, hipMemcpyDeviceToDevice, ln->st) != hipSuccess) {
            rc = -1;
            break;
        }
        out_samples[i] = L;
    }
    for (int k = 0; k < nl; ++k) {
        CodecModel *ln = k == 0 ? m : lanes[k];
        if (hipStreamSynchronize(ln->st) != hipSuccess) rc = -1;
    }
    hipEventDestroy(ready);
    // adopt the re-laid weights a lane made (the first decode of a shape on
    // it); a key made by two lanes keeps the first copy, the other is freed
    // (every stream has drained)
    for (int k = 1; k < nl; ++k) {
        for (auto &kv : lanes[k]->wt) {
            auto it = m->wt.find(kv.first);
            if (it == m->wt.end()) m->wt[kv.first] = kv.second;
            else if (it->second != kv.second) hipFree(kv.second);
        }
        lanes[k]->wt = m->wt;
    }
    return rc;
}

// ===================================================================== kernel-level C-ABI
extern "C" int qtts_hip_causal_conv1d(float *out, const float *in, const float *w, const float *b, int ci, int co,
                                      int k, int L, int dilation, int groups, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (groups == ci && ci == co) {
        if (dilation != 1) return -1;
        hipLaunchKernelGGL(k_dwconv, dim3((unsigned)(((size_t)co * L + 255) / 256)), dim3(256), 0, st, in, L, 0, w, b, co,
                           L, k, out, L);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (groups != 1) return -1;
    XGemm g;
    g.M = co; g.N = L; g.K = ci * k;
    g.amode = XA_ROWS; g.A = w; g.lda = ci * k;
    g.bmode = XB_CONV; g.B = in; g.ldb = L; g.Kw = k; g.dil = dilation; g.pad = (k - 1) * dilation; g.L = L;
    g.C = out; g.ldc = L; g.emode = XE_BIAS_M; g.bias = b;
    float *t = nullptr;
    const size_t cnt = (size_t)co * ci * k;
    if (hipMalloc(&t, cnt * 10) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_wt_relayout, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, w, co, ci, k, t);
    wt_planes(t, cnt, st);
    g.wt = t;
    const int rc = qtts_xgemm(g, st);
    if (hipStreamSynchronize(st) != hipSuccess) { hipFree(t); return -1; }
    hipFree(t);
    return rc;
}

extern "C" int qtts_hip_transposed_conv1d(float *out, const float *in, const float *w, const float *b, int ci, int co,
                                          int k, int stride, int L, void *stream) {
    if (k % stride) return -1;
    CodecModel dummy;
    int rc = tconv(&dummy, in, ci, L, w, b, co, k, stride, out, nullptr, nullptr, (hipStream_t)stream);
    if (!dummy.wt.empty()) {
        if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) rc = -1;
        for (auto &kv : dummy.wt) hipFree(kv.second);
        dummy.wt.clear();
    }
    return rc;
}

extern "C" int qtts_hip_snake_beta(float *out, const float *x, const float *alpha, const float *inv_beta, int channels,
                                   int length, void *stream) {
    hipLaunchKernelGGL(k_snake, dim3((unsigned)(((size_t)channels * length + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, x, alpha, inv_beta, channels, length, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int qtts_hip_expf_glibc(float *out, const float *in, int n, void *stream) {
    hipLaunchKernelGGL(k_expf_glibc, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ===================================================================== streaming decode
// Exact incremental decode.  Channel-major activations live
// in buffers with a left margin of `hm` columns; before a convolution runs,
// its history slot ((K-1)*dil input columns, or the last input frame of a
// K = 2s transposed conv) is copied into the margin and read through
// XGemm::tmin < 0; right after it, the last H columns of [history | new] are
// saved back.  The transformer keeps the last window-1 K/V rows per layer and
// continues the absolute positions (RoPE table offset by pos0).
namespace {
constexpr int kStreamChunk = 16;      // frames per internal chunk
constexpr int kStreamChunkMax = 128;  // largest chunk a begin may ask for

void *salloc(CodecStream &S, size_t bytes) {
    void *p = nullptr;
    const hipError_t prior = hipPeekAtLastError();
    const hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        fprintf(stderr, "qtts codec stream: hipMalloc(%zu) failed: %s (last error before it: %s)\n", bytes,
                hipGetErrorName(e), hipGetErrorName(prior));
        return nullptr;
    }
    hipMemset(p, 0, bytes ? bytes : 16);
    S.allocs.push_back(p);
    return p;
}

void copy2d(hipStream_t st, float *dst, int ldd, const float *src, int lds, int rows, int cols) {
    const size_t n = (size_t)rows * cols;
    if (n) hipLaunchKernelGGL(k_copy2d, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, ldd, src, lds, rows, cols);
}

// history in: slot -> margin of x;  history out: last H columns of [margin | x[0, L)) -> slot
void hist_in(CodecModel *m, int slot, float *x, int ldx) {
    CodecStream &S = m->cs;
    const int H = S.hist_h[slot];
    copy2d(m->st, x - H, ldx, S.hist[slot], H, S.hist_c[slot], H);
}
void hist_out(CodecModel *m, int slot, const float *x, int ldx, int L) {
    CodecStream &S = m->cs;
    const int H = S.hist_h[slot];
    copy2d(m->st, S.hist[slot], H, x + L - H, ldx, S.hist_c[slot], H);
}

int sconv(CodecModel *m, int slot, float *x, int ldx, int ci, int L, const std::string &wn, const std::string &bn,
          int co, int K, int dil, float *out, int ldo, int emode, const float *sa, const float *sb, const float *res,
          const float *ea = nullptr, const float *eb = nullptr) {
    const int H = (K - 1) * dil;
    if (H > 0) hist_in(m, slot, x, ldx);
    XGemm g;
    g.M = co; g.N = L; g.K = ci * K;
    g.amode = XA_ROWS; g.A = cw(m, wn); g.lda = ci * K; g.wt = cwt(m, wn, co, ci, K);
    g.bmode = XB_CONV; g.B = x; g.ldb = ldx; g.Kw = K; g.dil = dil; g.pad = H; g.L = L; g.tmin = -H;
    g.sa = sa; g.sb = sb;
    g.C = out; g.ldc = ldo; g.emode = emode; g.bias = bn.empty() ? nullptr : cw(m, bn); g.res = res; g.ldres = ldo;
    g.ea = ea; g.eb = eb;
    if (!g.A) return -1;
    KCK(xgm(m, g, m->st));
    if (H > 0) hist_out(m, slot, x, ldx, L);
    return 0;
}

int stconv(CodecModel *m, int slot, float *x, int ldx, int ci, int L, const float *w, const float *bias, int co, int Kw,
           int s, float *out, int ldo, const float *sa, const float *sb) {
    const int H = Kw / s - 1;
    if (H > 0) hist_in(m, slot, x, ldx);
    XGemm g;
    g.M = co; g.N = L; g.K = ci * (Kw / s);
    g.amode = XA_TCONV_W; g.A = w; g.co = co; g.Kw = Kw; g.stride = s;
    g.bmode = XB_TCONV; g.B = x; g.ldb = ldx; g.L = L; g.tmin = -H; g.sa = sa; g.sb = sb;
    g.C = out; g.ldc = ldo; g.emode = XE_BIAS_M; g.bias = bias;
    KCK(tconv_run(m, g, m->st));
    if (H > 0) hist_out(m, slot, x, ldx, L);
    return 0;
}

int stransformer(CodecModel *m, const float *pc, int ldp, int T, float *out, int ldo) {
    CodecStream &S = m->cs;
    const qtts_dims_t &d = m->d;
    const int lat = d.clat, hid = d.chid, nh = d.cheads, nkv = d.ckv, hd = hid / nh, kvd = nkv * hd, I = d.cinter;
    const int keepmax = d.cwin - 1;
    hipStream_t st = m->st;
    const std::string P = "decoder.pre_transformer.";
    XGemm g;
    g.M = T; g.N = hid; g.K = lat; g.amode = XA_TRANS; g.A = pc; g.lda = ldp; g.bmode = XB_WT;
    g.B = cw(m, P + "input_proj.weight"); g.ldb = lat; g.C = S.tx; g.ldc = hid;
    g.bias = cw(m, P + "input_proj.bias");
    g.emode = g.bias ? XE_BIAS_N : XE_STORE;
    KCK(xgm(m, g, st));
    const float *cs = S.rope_cos + (size_t)S.pos0 * hd, *sn = S.rope_sin + (size_t)S.pos0 * hd;
    const int hl = S.hl;
    for (int l = 0; l < d.clayers; ++l) {
        const std::string p = P + "layers." + std::to_string(l) + ".";
        float *kcl = S.kc[l], *vcl = S.vc[l];
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, S.tx, hid, cw(m, p + "input_layernorm.weight"),
                           d.ceps, S.txn);
        KCK(xgm(m, lin(S.txn, T, hid, cw(m, p + "self_attn.q_proj.weight"), hid, S.tq, XE_STORE), st));
        KCK(xgm(m, lin(S.txn, T, hid, cw(m, p + "self_attn.k_proj.weight"), kvd, kcl + (size_t)hl * kvd, XE_STORE), st));
        KCK(xgm(m, lin(S.txn, T, hid, cw(m, p + "self_attn.v_proj.weight"), kvd, vcl + (size_t)hl * kvd, XE_STORE), st));
        hipLaunchKernelGGL(k_rope_rows, dim3(T), dim3(256), 0, st, S.tq, hid, nh, hd, cs, sn);
        hipLaunchKernelGGL(k_rope_rows, dim3(T), dim3(256), 0, st, kcl + (size_t)hl * kvd, kvd, nkv, hd, cs, sn);
        AttnArgs a;
        a.mode = 1; a.qkv = S.tq; a.ld_qkv = hid; a.kc = kcl; a.vc = vcl; a.S = hl + T; a.pos = S.iota + hl;
        a.row_b = S.zeros; a.NH = nh; a.KV = nkv; a.HD = hd; a.out = S.tatt; a.ld_out = hid;
        a.nrows = T; a.win = d.cwin;
        KCK(qtts_attention(a, st));
        const float *ls1 = cw(m, p + "self_attn_layer_scale.scale");
        if (!ls1) return -1;
        XGemm o = lin(S.tatt, T, hid, cw(m, p + "self_attn.o_proj.weight"), hid, S.tx, XE_SCALE_RESID_N);
        o.vec = ls1;
        KCK(xgm(m, o, st));
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, S.tx, hid,
                           cw(m, p + "post_attention_layernorm.weight"), d.ceps, S.txn);
        KCK(xgm(m, lin(S.txn, T, hid, cw(m, p + "mlp.gate_proj.weight"), I, S.tg, XE_STORE), st));
        XGemm u = lin(S.txn, T, hid, cw(m, p + "mlp.up_proj.weight"), I, S.tu, XE_SILU_MUL);
        u.aux = S.tg; u.ldaux = I;
        KCK(xgm(m, u, st));
        const float *ls2 = cw(m, p + "mlp_layer_scale.scale");
        if (!ls2) return -1;
        XGemm dn = lin(S.tu, T, I, cw(m, p + "mlp.down_proj.weight"), hid, S.tx, XE_SCALE_RESID_N);
        dn.vec = ls2;
        KCK(xgm(m, dn, st));
        // keep the last window-1 rows for the next chunk
        const int tot = hl + T, keep = tot < keepmax ? tot : keepmax;
        if (keep > 0 && tot > keep) {
            copy2d(st, S.kvtmp, kvd, kcl + (size_t)(tot - keep) * kvd, kvd, keep, kvd);
            copy2d(st, kcl, kvd, S.kvtmp, kvd, keep, kvd);
            copy2d(st, S.kvtmp, kvd, vcl + (size_t)(tot - keep) * kvd, kvd, keep, kvd);
            copy2d(st, vcl, kvd, S.kvtmp, kvd, keep, kvd);
        }
    }
    {
        const int tot = hl + T;
        S.hl = tot < keepmax ? tot : keepmax;
    }
    const float *fn = cw(m, P + "norm.weight");
    const float *xin = S.tx;
    if (fn) {
        hipLaunchKernelGGL(k_rms_rows, dim3(T), dim3(256), 0, st, S.tx, hid, fn, d.ceps, S.txn);
        xin = S.txn;
    }
    XGemm og = lin(xin, T, hid, cw(m, P + "output_proj.weight"), lat, out, XE_BIAS_T);
    og.bias = cw(m, P + "output_proj.bias");
    og.ldc = ldo;
    if (!og.bias) return -1;
    return xgm(m, og, st);
}

int add_slot(CodecStream &S, int c, int h) {
    S.hist_c.push_back(c);
    S.hist_h.push_back(h);
    S.hist.push_back((float *)salloc(S, (size_t)c * (h > 0 ? h : 1) * 4));
    return S.hist.back() ? (int)S.hist.size() - 1 : -1;
}
}  // namespace

void codec_stream_free(CodecModel *m) {
    CodecStream &S = m->cs;
    for (void *p : S.allocs) hipFree(p);
    S = CodecStream();
}

int codec_stream_begin(CodecModel *m, int max_frames, int chunk) {
    const qtts_dims_t &d = m->d;
    CodecStream &S0 = m->cs;
    // frames per internal chunk: kStreamChunk, or up to kStreamChunkMax when a
    // caller pushes long runs at once (the voice-clone reference frames: one
    // chunk of T frames runs ~T/16 times fewer, larger kernels)
    const int tc_want = chunk > kStreamChunk ? (chunk < kStreamChunkMax ? chunk : kStreamChunkMax) : kStreamChunk;
    // the codec GEMMs' split-K workspace belongs to the (non-streaming) codec
    // state, which the decode state's re-allocation frees (free_state ->
    // codec_free_state): re-create it before a stream reuses its own buffers
    if (ensure_codec_state(m, 1)) return -1;
    if (S0.active && max_frames + S0.tc <= S0.rope_cap && S0.tc >= tc_want) {
        // reuse the buffers: only the carried state restarts (zero histories =
        // the causal left padding, no K/V rows, position 0), on the codec stream
        for (size_t i = 0; i < S0.hist.size(); ++i)
            if (hipMemsetAsync(S0.hist[i], 0, (size_t)S0.hist_c[i] * (S0.hist_h[i] > 0 ? S0.hist_h[i] : 1) * 4,
                               m->st) != hipSuccess)
                return -1;
        S0.pos0 = 0;
        S0.hl = 0;
        return 0;
    }
    codec_stream_free(m);
    // (ensure_codec_state ran above: the split-K workspace exists)
    CodecStream &S = m->cs;
    S.tc = tc_want;
    const int hm = S.hm, tc = S.tc;
    // activation buffers: largest C x (hm + L) over the stages at tc frames
    size_t L = (size_t)tc * d.ratios[0] * d.ratios[1];
    size_t mx = (size_t)d.clat * L * 4 + (size_t)4 * d.clat * hm;
    if ((size_t)d.cdec * (L + hm) > mx) mx = (size_t)d.cdec * (L + hm);
    int C = d.cdec;
    for (int b = 0; b < 4; ++b) {
        L *= d.rates[b];
        C /= 2;
        if ((size_t)C * (L + hm) > mx) mx = (size_t)C * (L + hm);
    }
    if ((size_t)d.clat * (tc + hm) > mx) mx = (size_t)d.clat * (tc + hm);
    S.buf_elems = mx + hm;
    S.bufA = (float *)salloc(S, S.buf_elems * 4);
    S.bufB = (float *)salloc(S, S.buf_elems * 4);
    S.bufC = (float *)salloc(S, S.buf_elems * 4);
    S.bufD = (float *)salloc(S, S.buf_elems * 4);
    const int hid = d.chid, hd = hid / d.cheads, kvd = d.ckv * hd, keep = d.cwin - 1;
    S.tx = (float *)salloc(S, (size_t)tc * hid * 4);
    S.txn = (float *)salloc(S, (size_t)tc * hid * 4);
    S.tq = (float *)salloc(S, (size_t)tc * hid * 4);
    S.tatt = (float *)salloc(S, (size_t)tc * hid * 4);
    S.tg = (float *)salloc(S, (size_t)tc * d.cinter * 4);
    S.tu = (float *)salloc(S, (size_t)tc * d.cinter * 4);
    const int vq = d.ccbdim / 2;
    S.rvq_s = (float *)salloc(S, (size_t)vq * tc * 4);
    S.rvq_a = (float *)salloc(S, (size_t)vq * tc * 4);
    for (int l = 0; l < d.clayers; ++l) {
        S.kc.push_back((float *)salloc(S, (size_t)(keep + tc) * kvd * 4));
        S.vc.push_back((float *)salloc(S, (size_t)(keep + tc) * kvd * 4));
    }
    S.kvtmp = (float *)salloc(S, (size_t)(keep > 0 ? keep : 1) * kvd * 4);
    // RoPE table for absolute positions [0, max_frames + tc) (theta 1e4, Cd.c:309)
    S.rope_cap = max_frames + tc;
    const int half = hd / 2;
    std::vector<float> c((size_t)S.rope_cap * hd), s((size_t)S.rope_cap * hd);
    for (int p = 0; p < S.rope_cap; ++p)
        for (int i = 0; i < half; ++i) {
            float freq = 1.0f / powf(10000.0f, (float)(2 * i) / (float)hd);
            float ang = (float)p * freq;
            c[(size_t)p * hd + i] = c[(size_t)p * hd + i + half] = cosf(ang);
            s[(size_t)p * hd + i] = s[(size_t)p * hd + i + half] = sinf(ang);
        }
    S.rope_cos = (float *)salloc(S, c.size() * 4);
    S.rope_sin = (float *)salloc(S, s.size() * 4);
    std::vector<int> io(keep + tc + 1);
    for (size_t i = 0; i < io.size(); ++i) io[i] = (int)i;
    S.iota = (int *)salloc(S, io.size() * 4);
    S.zeros = (int *)salloc(S, (size_t)tc * 4);
    for (void *p : S.allocs)
        if (!p) return -1;
    if (!S.bufA || !S.bufB || !S.bufC || !S.bufD || !S.rope_cos || !S.rope_sin || !S.iota || !S.zeros) return -1;
    if (hipMemcpy(S.rope_cos, c.data(), c.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (hipMemcpy(S.rope_sin, s.data(), s.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (hipMemcpy(S.iota, io.data(), io.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    // history slots, in the order codec_stream_push consumes them
    add_slot(S, d.ccbdim, 2);                  // 0 pre-conv k3
    add_slot(S, d.clat, 6);                    // 1 upsample 0 dwconv k7
    add_slot(S, d.clat, 6);                    // 2 upsample 1 dwconv k7
    add_slot(S, d.clat, 6);                    // 3 vocoder conv0 k7
    C = d.cdec;
    static const int dil[3] = {1, 3, 9};
    for (int b = 0; b < 4; ++b) {
        add_slot(S, C, 1);                     // block tconv (K = 2r): last input frame
        for (int u = 0; u < 3; ++u) add_slot(S, C / 2, 6 * dil[u]);   // ResUnit conv1 k7 dil
        C /= 2;
    }
    add_slot(S, C, 6);                         // final conv k7
    for (float *h : S.hist)
        if (!h) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    S.active = true;
    return 0;
}

int codec_stream_push(CodecModel *m, const int *codes, int ldc_codes, int Ttot, float *host_out) {
    return codec_stream_push_to(m, codes, ldc_codes, Ttot, host_out, true);
}

int codec_stream_push_to(CodecModel *m, const int *codes, int ldc_codes, int Ttot, float *out, bool host) {
    CodecStream &S = m->cs;
    const qtts_dims_t &d = m->d;
    if (!S.active || ldc_codes != d.cq) return -1;
    if (!m->xg_part) {   // freed with the codec state and not re-created (codec_stream_begin re-creates it)
        fprintf(stderr, "qtts codec stream: split-K workspace missing (stream not begun after a state re-allocation)\n");
        return -1;
    }
    if (S.pos0 + Ttot > S.rope_cap - S.tc) {
        fprintf(stderr, "qtts codec stream: %d frames exceed the stream capacity\n", S.pos0 + Ttot);
        return -1;
    }
    hipStream_t st = m->st;
    const int lat = d.clat, vq = d.ccbdim / 2, half = lat / 2, hm = S.hm;
    int written = 0;
    for (int t0 = 0; t0 < Ttot; t0 += S.tc) {
        const int T = Ttot - t0 < S.tc ? Ttot - t0 : S.tc;
        float *A = S.bufA + hm, *B = S.bufB + hm, *Cb = S.bufC, *D = S.bufD;
        int L = T, ld = hm + L;
        // 1. RVQ dequantise -> A [half][T]
        hipLaunchKernelGGL(k_rvq_sum, dim3(T), dim3(vq < 64 ? 64 : (vq + 63) / 64 * 64), 0, st,
                           codes + (size_t)t0 * d.cq, T, d.cq, d.ccb, vq, m->cb, S.rvq_s, S.rvq_a);
        hipLaunchKernelGGL(k_rvq_proj, dim3((half * T + 3) / 4), dim3(256), 0, st,
                           cw(m, "decoder.quantizer.rvq_first.output_proj.weight"),
                           cw(m, "decoder.quantizer.rvq_rest.output_proj.weight"), S.rvq_s, S.rvq_a, vq, half, T, ld, A);
        // 2. pre-conv k3 -> B
        KCK(sconv(m, 0, A, ld, d.ccbdim, L, "decoder.pre_conv.conv.weight", "decoder.pre_conv.conv.bias", lat, 3, 1, B,
                  ld, XE_BIAS_M, nullptr, nullptr, nullptr));
        // 3. transformer -> A
        KCK(stransformer(m, B, ld, T, A, ld));
        // 4. upsample x2: tconv (K = s, no history) + ConvNeXt
        float *cur = A;
        for (int s = 0; s < 2; ++s) {
            const int f = d.ratios[s];
            const std::string p = "decoder.upsample." + std::to_string(s) + ".";
            float *up = cur == A ? B : A;
            const int ldu = hm + L * f;
            KCK(stconv(m, -1, cur, ld, lat, L, cw(m, p + "0.conv.weight"), cw(m, p + "0.conv.bias"), lat, f, f, up, ldu,
                       nullptr, nullptr));
            L *= f;
            ld = ldu;
            cur = up;
            hist_in(m, 1 + s, cur, ld);
            hipLaunchKernelGGL(k_dwconv, dim3((unsigned)(((size_t)lat * L + 255) / 256)), dim3(256), 0, st, cur, ld, -6,
                               cw(m, p + "1.dwconv.conv.weight"), cw(m, p + "1.dwconv.conv.bias"), lat, L, 7, Cb, L);
            hist_out(m, 1 + s, cur, ld, L);
            hipLaunchKernelGGL(k_ln_t, dim3(L), dim3(256), 0, st, Cb, L, lat, cw(m, p + "1.norm.weight"),
                               cw(m, p + "1.norm.bias"), 1e-6f, D);
            XGemm g1 = lin(D, L, lat, cw(m, p + "1.pwconv1.weight"), 4 * lat, Cb, XE_BIAS_N_GELU);
            g1.bias = cw(m, p + "1.pwconv1.bias");
            KCK(xgm(m, g1, st));
            XGemm g2 = lin(Cb, L, 4 * lat, cw(m, p + "1.pwconv2.weight"), lat, cur, XE_BIAS_GAMMA_RES_T);
            g2.bias = cw(m, p + "1.pwconv2.bias");
            g2.vec = cw(m, p + "1.gamma");
            g2.res = cur; g2.ldres = ld; g2.ldc = ld;
            KCK(xgm(m, g2, st));
        }
        // 5. vocoder
        float *voc = cur == A ? B : A;
        KCK(sconv(m, 3, cur, ld, lat, L, "decoder.decoder.0.conv.weight", "decoder.decoder.0.conv.bias", d.cdec, 7, 1,
                  voc, ld, XE_BIAS_M, nullptr, nullptr, nullptr));
        int C = d.cdec, slot = 4;
        static const int dil[3] = {1, 3, 9};
        for (int b = 0; b < 4; ++b) {
            const int r = d.rates[b], co = C / 2;
            const std::string p = "decoder.decoder." + std::to_string(b + 1) + ".block.";
            float *nx = voc == A ? B : A;
            const int ldn = hm + L * r;
            KCK(stconv(m, slot++, voc, ld, C, L, cw(m, p + "1.conv.weight"), cw(m, p + "1.conv.bias"), co, 2 * r, r, nx,
                       ldn, cw(m, p + "0.alpha"), cw(m, p + "0.beta")));
            L *= r;
            ld = ldn;
            C = co;
            voc = nx;
            for (int u = 0; u < 3; ++u) {
                const std::string q = p + std::to_string(u + 2) + ".";
                KCK(sconv(m, slot++, voc, ld, C, L, q + "conv1.conv.weight", q + "conv1.conv.bias", C, 7, dil[u], Cb, L,
                          XE_BIAS_M_SNAKE, cw(m, q + "act1.alpha"), cw(m, q + "act1.beta"), nullptr,
                          cw(m, q + "act2.alpha"), cw(m, q + "act2.beta")));
                KCK(sconv(m, -1, Cb, L, C, L, q + "conv2.conv.weight", q + "conv2.conv.bias", C, 1, 1, voc, ld,
                          XE_BIAS_M_RES, nullptr, nullptr, voc));
            }
        }
        float *wav = voc == A ? B : A;
        KCK(sconv(m, slot, voc, ld, C, L, "decoder.decoder.6.conv.weight", "decoder.decoder.6.conv.bias", 1, 7, 1, wav,
                  ld, XE_BIAS_M, cw(m, "decoder.decoder.5.alpha"), cw(m, "decoder.decoder.5.beta"), nullptr));
        hipLaunchKernelGGL(k_clamp, dim3((L + 255) / 256), dim3(256), 0, st, wav, L);
        if (hipMemcpyAsync(out + written, wav, (size_t)L * 4, host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice,
                           st) != hipSuccess)
            return -1;
        written += L;
        S.pos0 += T;
    }
    if (host && hipStreamSynchronize(st) != hipSuccess) return -1;
    return written;
}
