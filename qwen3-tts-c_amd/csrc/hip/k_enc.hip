// k_enc.hip - voice-clone audio encoders on gfx950.
//
//   speaker x-vector  mel_spectrogram + ECAPA-TDNN   modeling_qwen3_tts.py:90-464, 1941-1954
//   12 Hz codes       MimiModel encoder + split RVQ  modeling_qwen3_tts_tokenizer_v2.py:899-991
//                     (transformers/models/mimi/modeling_mimi.py, the published algorithm)
//
// One kernel carries every dense contraction: k_econv, a batched implicit-GEMM
// conv1d (out[b][m][n] = sum_k W[m][k] * x'[b][k][n], k = ci * kw + tap,
// x' = the input column ci at n * stride + tap * dil - padl, remapped by the
// padding mode) on v_mfma_f32_32x32x16_bf16.  Weights are split once at load
// into three exact bf16 planes, inputs when a K-step is staged into LDS, and
// the six plane products with i + j <= 4 give fp32-equivalent products
// (dropped terms < 2^-24 |w x|) at 3/8 of the fp32-input MFMA's issue time.
// The same kernel is the STFT (one input channel, kw = n_fft, stride = hop,
// reflect padding, a Hann-windowed DFT basis as weights), every TDNN
// ("same" reflect padding, dilation), every SEANet conv (causal zero
// padding, strides 4/5/6/8, ELU prologue), the replicate-padded downsample
// and the transformer's linears (kw = 1 over time-major rows).  Epilogues:
// bias, per-utterance bias, ReLU / tanh(ReLU) / exact GELU, LayerScale,
// residual.  Tile 64 (out channels) x 64 (time) per 256-thread workgroup,
// 2 x 2 waves of 32 x 32, K-steps of 32 double-buffered through registers,
// LDS rows of 64 B with an XOR swizzle (conflict-free 16-B fragment reads).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "qtts_common.h"
#include "qtts_enc.h"
#include "qtts_kernels.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define ECK(x)                                                                        \
    do {                                                                              \
        if ((x) != 0) {                                                               \
            fprintf(stderr, "qtts enc: step failed at %s:%d: %s\n", __FILE__, __LINE__, #x); \
            return -1;                                                                \
        }                                                                             \
    } while (0)

namespace {

enum { PAD_ZERO = 0, PAD_REFLECT = 1, PAD_REPLICATE = 2 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU_TANH = 2, ACT_GELU = 3, ACT_SIGMOID = 4 };

struct EConv {
    const unsigned short *w = nullptr;  // [3][M][Kp] bf16 planes
    size_t wplane = 0;                  // M * Kp
    int M = 0, K = 0, Kp = 0, kw = 1, stride = 1, dil = 1, padl = 0, pmode = PAD_ZERO, act_in = ACT_NONE;
    const float *x = nullptr, *x2 = nullptr;   // x'(ci, t) = x[b*xb + ci*xc + t*xt] (+ x2, same strides)
    size_t xb = 0;
    int xc = 0, xt = 1;
    int lin[ENC_MAXB], lout[ENC_MAXB];
    float *y = nullptr;                 // y[b*yb + m*yc + n*yt]
    size_t yb = 0;
    int yc = 0, yt = 1;
    const float *bias = nullptr;        // [M]
    const float *bias2 = nullptr;       // [b][bias2_b] per-utterance bias
    int bias2_b = 0;
    int act_out = ACT_NONE;
    const float *vec = nullptr;         // LayerScale [M] (after the activation)
    const float *res = nullptr;         // residual, res[b*rb + m*rc + n*rt]
    size_t rb = 0;
    int rc = 0, rt = 1;
    // split-K (set by launch_econv): blockIdx.z = b * kz + split; raw partial
    // tiles to part[split][b][M][pn], k_econv_reduce sums them in split order
    float *part = nullptr;
    int kz = 1, pn = 0, nb = 1;
};

__device__ __forceinline__ void econv_store(const EConv &g, int b, int m, int n, float v) {
    const float *bias2 = g.bias2 ? g.bias2 + (size_t)b * g.bias2_b : nullptr;
    if (g.bias) v += g.bias[m];
    if (bias2) v += bias2[m];
    switch (g.act_out) {
        case 1: v = fmaxf(v, 0.f); break;
        case 2: v = tanhf(fmaxf(v, 0.f)); break;
        case 3: v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); break;
        case 4: v = 1.0f / (1.0f + expf(-v)); break;
        default: break;
    }
    if (g.vec) v *= g.vec[m];
    if (g.res) v += g.res[(size_t)b * g.rb + (size_t)m * g.rc + (size_t)n * g.rt];
    g.y[(size_t)b * g.yb + (size_t)m * g.yc + (size_t)n * g.yt] = v;
}

__device__ __forceinline__ int eswz(int r, int c) { return r * 32 + ((c ^ ((r >> 2) & 3)) << 3); }

__device__ __forceinline__ uint32_t e_pk(float lo, float hi) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    const bf2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float e_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float e_hi(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

// 8 floats -> three exact bf16 planes (16 B each)
__device__ __forceinline__ void e_split8(const float (&v)[8], uint4 &p1, uint4 &p2, uint4 &p3) {
    uint32_t a[4], b[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = e_pk(v[2 * i], v[2 * i + 1]);
        const float e0 = v[2 * i] - e_lo(a[i]), e1 = v[2 * i + 1] - e_hi(a[i]);
        b[i] = e_pk(e0, e1);
        c[i] = e_pk(e0 - e_lo(b[i]), e1 - e_hi(b[i]));
    }
    p1 = make_uint4(a[0], a[1], a[2], a[3]);
    p2 = make_uint4(b[0], b[1], b[2], b[3]);
    p3 = make_uint4(c[0], c[1], c[2], c[3]);
}

__device__ __forceinline__ float act_apply(int act, float v) {
    switch (act) {
        case ACT_RELU: return fmaxf(v, 0.f);
        case ACT_RELU_TANH: return tanhf(fmaxf(v, 0.f));
        case ACT_GELU: return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
        case ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
        default: return v;
    }
}

// ROWS: the input is time-major rows with k contiguous (kw = 1, xc = 1,
// stride 1, no padding): each thread's 8 k values are two float4 loads.
template <bool ROWS>
__global__ __launch_bounds__(256) void k_econv(EConv g) {
    __shared__ __attribute__((aligned(16))) unsigned short As[3][64 * 32];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[3][64 * 32];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int kz = g.kz, b = blockIdx.z / kz, kzi = blockIdx.z - b * kz;
    const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int lout = g.lout[b], lin = g.lin[b];
    if (n0 >= lout) return;   // uniform per workgroup, before any barrier
    const float *x = g.x + (size_t)b * g.xb;
    const float *x2 = g.x2 ? g.x2 + (size_t)b * g.xb : nullptr;
    // weight tile loader: row ar, 16-B chunk ac of the 64-B K-step row, one per plane
    const int ar = tid >> 2, ac = tid & 3;
    const bool arow = m0 + ar < g.M;
    const unsigned short *wa = g.w + (size_t)(m0 + ar) * g.Kp + ac * 8;
    // input tile loader: column bn, k group bq (8 consecutive k)
    const int bn = tid & 63, bq = tid >> 6;
    const bool bcol = n0 + bn < lout;
    const int tcol = (n0 + bn) * g.stride - g.padl;
    uint4 ra[3];
    float rb[8];
    auto load = [&](int k0) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
            ra[p] = arow ? *reinterpret_cast<const uint4 *>(wa + p * g.wplane + k0) : make_uint4(0u, 0u, 0u, 0u);
        const int k = k0 + 8 * bq;
        if (ROWS) {
            if (bcol && k < g.K) {
                const float4 *src = reinterpret_cast<const float4 *>(x + (size_t)(n0 + bn) * g.xt + k);
                const float4 u = src[0], v = src[1];
                rb[0] = u.x; rb[1] = u.y; rb[2] = u.z; rb[3] = u.w;
                rb[4] = v.x; rb[5] = v.y; rb[6] = v.z; rb[7] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) rb[j] = 0.f;
            }
            return;
        }
        int ci = k / g.kw, tap = k - ci * g.kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float v = 0.f;
            if (bcol && k + j < g.K) {
                int t = tcol + tap * g.dil;
                bool ok = true;
                if (t < 0 || t >= lin) {
                    if (g.pmode == PAD_REFLECT) t = t < 0 ? -t : 2 * (lin - 1) - t;
                    else if (g.pmode == PAD_REPLICATE) t = t < 0 ? 0 : lin - 1;
                    else ok = false;
                }
                if (ok) {
                    const size_t o = (size_t)ci * g.xc + (size_t)t * g.xt;
                    v = x[o];
                    if (x2) v += x2[o];
                    if (g.act_in == 1) v = v > 0.f ? v : expm1f(v);   // ELU (alpha 1), before the padding
                }
            }
            rb[j] = v;
            if (++tap == g.kw) { tap = 0; ++ci; }
        }
    };
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const int nk = g.Kp / 32, s0 = nk * kzi / kz, s1 = nk * (kzi + 1) / kz;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32, r = lane & 31, hh = lane >> 5;
    load(s0 * 32);
    for (int s = s0; s < s1; ++s) {
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4 *>(&As[p][eswz(ar, ac)]) = ra[p];
        {
            uint4 p1, p2, p3;
            e_split8(rb, p1, p2, p3);
            const int o = eswz(bn, bq);
            *reinterpret_cast<uint4 *>(&Bs[0][o]) = p1;
            *reinterpret_cast<uint4 *>(&Bs[1][o]) = p2;
            *reinterpret_cast<uint4 *>(&Bs[2][o]) = p3;
        }
        __syncthreads();
        if (s + 1 < s1) load((s + 1) * 32);
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
            const int c = kg * 2 + hh;
            const int oa = eswz(wm + r, c), ob = eswz(wn + r, c);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8 *>(&As[0][oa]);
            const bf16x8 a2 = *reinterpret_cast<const bf16x8 *>(&As[1][oa]);
            const bf16x8 a3 = *reinterpret_cast<const bf16x8 *>(&As[2][oa]);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(&Bs[0][ob]);
            const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(&Bs[1][ob]);
            const bf16x8 b3 = *reinterpret_cast<const bf16x8 *>(&Bs[2][ob]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b3, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a3, b1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    const int n = n0 + wn + r;
    if (n >= lout) return;
    if (kz > 1) {
        float *pz = g.part + ((size_t)kzi * g.nb + b) * g.M * g.pn;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (m < g.M) pz[(size_t)m * g.pn + n] = acc[i];
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + 4 * hh;
        if (m < g.M) econv_store(g, b, m, n, acc[i]);
    }
}

// split-K partial sums in split order + the epilogue
__global__ void k_econv_reduce(EConv g) {
    const int n = blockIdx.x * 256 + threadIdx.x, m = blockIdx.y, b = blockIdx.z;
    if (n >= g.lout[b]) return;
    float v = 0.f;
    for (int z = 0; z < g.kz; ++z) v += g.part[(((size_t)z * g.nb + b) * g.M + m) * g.pn + n];
    econv_store(g, b, m, n, v);
}

// fp32 [M][K] -> three exact bf16 planes [3][M][Kp] (zero K padding)
__global__ void k_ewsplit(const float *w, int M, int K, int Kp, unsigned short *planes) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)M * Kp) return;
    const int m = (int)(i / Kp), k = (int)(i - (size_t)m * Kp);
    const float v = k < K ? w[(size_t)m * K + k] : 0.f;
    const uint32_t a = e_pk(v, 0.f);
    const float e1 = v - e_lo(a);
    const uint32_t b = e_pk(e1, 0.f);
    const uint32_t c = e_pk(e1 - e_lo(b), 0.f);
    const size_t pl = (size_t)M * Kp;
    planes[i] = (unsigned short)(a & 0xFFFFu);
    planes[pl + i] = (unsigned short)(b & 0xFFFFu);
    planes[2 * pl + i] = (unsigned short)(c & 0xFFFFu);
}

// |STFT| -> slaney mel -> log (modeling_qwen3_tts.py:459-462): spec
// [b][2*nf][ldt] (cos rows, then sin rows), mel [b][nm][ldt]
__global__ __launch_bounds__(256) void k_mel(const float *spec, int nf, int ldt, const int *T, const float *fb,
                                             const int *flo, const int *fhi, int nm, float *mel) {
    __shared__ float mag[1040];
    const int t = blockIdx.x, b = blockIdx.y;
    if (t >= T[b]) return;
    const float *s = spec + (size_t)b * 2 * nf * ldt;
    for (int f = threadIdx.x; f < nf; f += 256) {
        const float re = s[(size_t)f * ldt + t], im = s[(size_t)(nf + f) * ldt + t];
        mag[f] = sqrtf(re * re + im * im + 1e-9f);
    }
    __syncthreads();
    for (int m = threadIdx.x; m < nm; m += 256) {
        float acc = 0.f;
        for (int f = flo[m]; f < fhi[m]; ++f) acc += fb[(size_t)m * nf + f] * mag[f];
        mel[((size_t)b * nm + m) * ldt + t] = logf(fmaxf(acc, 1e-5f));
    }
}

// per-(b, c) mean over t < len[b] (torch .mean(dim=2)): one wave per row
__global__ __launch_bounds__(256) void k_row_mean(const float *x, size_t xb, int ldt, const int *len, int C,
                                                  float *out) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y, l = threadIdx.x & 63;
    if (c >= C) return;
    const float *r = x + (size_t)b * xb + (size_t)c * ldt;
    const int L = len[b];
    float s = 0.f;
    for (int t = l; t < L; t += 64) s += r[t];
    s = wave_sum(s);
    if (l == 0) out[(size_t)b * C + c] = s / (float)L;
}

// y[b][r] = act(sum_c W[r][c] x[b][c] + bias[r]); one wave per (r, b)
__global__ __launch_bounds__(256) void k_egemv(const float *W, int R, int Cc, const float *x, int ldx,
                                               const float *bias, int act, float *y, int ldy) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y, l = threadIdx.x & 63;
    if (r >= R) return;
    const float *w = W + (size_t)r * Cc, *xv = x + (size_t)b * ldx;
    float s = 0.f;
    for (int c = l; c < Cc; c += 64) s += w[c] * xv[c];
    s = wave_sum(s);
    if (l == 0) y[(size_t)b * ldy + r] = act_apply(act, s + (bias ? bias[r] : 0.f));
}

// SqueezeExcitation output + block residual (modeling_qwen3_tts.py:150-156, 300-308):
// out = h * s[b][c] + res
__global__ void k_se_apply(const float *h, size_t hb, const float *s, int C, const float *res, size_t rb,
                           float *out, size_t ob, int ldt, const int *len) {
    const int t = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y, b = blockIdx.z;
    if (t >= len[b]) return;
    const size_t o = (size_t)c * ldt + t;
    out[(size_t)b * ob + o] = h[(size_t)b * hb + o] * s[(size_t)b * C + c] + res[(size_t)b * rb + o];
}

// attentive statistics pooling, uniform weights m = 1/T (modeling_qwen3_tts.py:209-231):
// st[b][c] = mean, st[b][C + c] = std
__global__ __launch_bounds__(256) void k_asp_stats(const float *x, size_t xb, int ldt, const int *len, int C,
                                                   float *st) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y, l = threadIdx.x & 63;
    if (c >= C) return;
    const float *r = x + (size_t)b * xb + (size_t)c * ldt;
    const int L = len[b];
    const float m = 1.0f / (float)L;
    float s = 0.f;
    for (int t = l; t < L; t += 64) s += m * r[t];
    const float mean = wave_sum(s);
    float v = 0.f;
    for (int t = l; t < L; t += 64) { const float d = r[t] - mean; v += m * d * d; }
    v = wave_sum(v);
    if (l == 0) {
        st[(size_t)b * 2 * C + c] = mean;
        st[(size_t)b * 2 * C + C + c] = sqrtf(fmaxf(v, 1e-12f));
    }
}

// softmax over time of the attention logits, then the attended mean / std
// (modeling_qwen3_tts.py:237-245): pooled[b] = [mean; std]
__global__ __launch_bounds__(256) void k_asp_pool(const float *x, size_t xb, const float *lg, size_t lb, int ldt,
                                                  const int *len, int C, float *pooled) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y, l = threadIdx.x & 63;
    if (c >= C) return;
    const float *xr = x + (size_t)b * xb + (size_t)c * ldt, *a = lg + (size_t)b * lb + (size_t)c * ldt;
    const int L = len[b];
    float mx = -3.402823466e38f;
    for (int t = l; t < L; t += 64) mx = fmaxf(mx, a[t]);
    mx = wave_max(mx);
    float z = 0.f;
    for (int t = l; t < L; t += 64) z += expf(a[t] - mx);
    z = wave_sum(z);
    const float iz = 1.0f / z;
    float s = 0.f;
    for (int t = l; t < L; t += 64) s += expf(a[t] - mx) * iz * xr[t];
    const float mean = wave_sum(s);
    float v = 0.f;
    for (int t = l; t < L; t += 64) { const float d = xr[t] - mean; v += expf(a[t] - mx) * iz * d * d; }
    v = wave_sum(v);
    if (l == 0) {
        pooled[(size_t)b * 2 * C + c] = mean;
        pooled[(size_t)b * 2 * C + C + c] = sqrtf(fmaxf(v, 1e-12f));
    }
}

// LayerNorm over rows [R][D] with weight and bias (nn.LayerNorm, biased variance)
__global__ __launch_bounds__(256) void k_ln_rows(const float *x, int D, const float *w, const float *bb, float eps,
                                                 float *y) {
    __shared__ float red[8];
    const size_t r = blockIdx.x;
    const float *xr = x + r * D;
    float s = 0.f;
    for (int c = threadIdx.x; c < D; c += 256) s += xr[c];
    const float mean = block_sum256(s, red) / (float)D;
    float v = 0.f;
    for (int c = threadIdx.x; c < D; c += 256) { const float d = xr[c] - mean; v += d * d; }
    const float inv = 1.0f / sqrtf(block_sum256(v, red + 4) / (float)D + eps);
    for (int c = threadIdx.x; c < D; c += 256) y[r * D + c] = (xr[c] - mean) * inv * w[c] + bb[c];
}

// rotate-half RoPE in place on rows [R][nh*hd], position = row % T
__global__ void k_rope_bt(float *x, int ld, int nh, int hd, int T, const float *cs, const float *sn) {
    const int row = blockIdx.x, p = row % T, half = hd / 2;
    for (int i = threadIdx.x; i < nh * half; i += blockDim.x) {
        const int h = i / half, e = i - h * half;
        float *q = x + (size_t)row * ld + h * hd;
        const float a = q[e], c = q[e + half];
        q[e] = a * cs[(size_t)p * hd + e] - c * sn[(size_t)p * hd + e];
        q[e + half] = c * cs[(size_t)p * hd + e + half] + a * sn[(size_t)p * hd + e + half];
    }
}

__global__ void k_rows_bt(int *row_b, int *pos, int R, int T) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r < R) { row_b[r] = r / T; pos[r] = r % T; }
}

// Split residual vector quantizer encode (modeling_mimi.py:1050-1126): rows
// (b, t) of the latent [b][hid][T12]; per chain (semantic: codebook 0,
// acoustic: 1..nvalid-1) r = input_proj z, then per codebook the argmin
// squared Euclidean distance (first index on ties) and r -= e[argmin].
// RVQ_ROWS (2) rows per workgroup of 16 waves share every codebook read; the codebooks are
// stored dim-major ([q][vq][CB]) and the projections transposed ([hid][vq]) so
// that consecutive lanes read consecutive codes / outputs (coalesced).
constexpr int RVQ_ROWS = 2, RVQ_NT = 1024;
__global__ __launch_bounds__(RVQ_NT) void k_rvq_enc(const float *lat, int T12, int hid, int R, const float *psemT,
                                                    const float *pacT, const float *cbkT, int CB, int vq, int nvalid,
                                                    int nsem, int *codes, int ldc_t) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr int NW = RVQ_NT / 64;
    float *z = sm;                                  // [ROWS][hid]
    float *rr = z + RVQ_ROWS * hid;                 // [ROWS][vq]
    float *bd = rr + RVQ_ROWS * vq;                 // [NW][ROWS] best distance per wave
    int *bi = reinterpret_cast<int *>(bd + NW * RVQ_ROWS);   // [NW][ROWS]
    int *best = bi + NW * RVQ_ROWS;                 // [ROWS]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r0 = blockIdx.x * RVQ_ROWS;
    const int nr = min(RVQ_ROWS, R - r0);
    for (int i = tid; i < RVQ_ROWS * hid; i += RVQ_NT) {
        const int j = i / hid, c = i - j * hid, row = r0 + j;
        float v = 0.f;
        if (j < nr) {
            const int b = row / T12, t = row - b * T12;
            v = lat[((size_t)b * hid + c) * T12 + t];
        }
        z[i] = v;
    }
    __syncthreads();
    for (int chain = 0; chain < 2; ++chain) {
        const float *PT = chain == 0 ? psemT : pacT;
        const int q0 = chain == 0 ? 0 : nsem, q1 = chain == 0 ? nsem : nvalid;
        for (int i = tid; i < RVQ_ROWS * vq; i += RVQ_NT) {
            const int j = i / vq, o = i - j * vq;
            const float *zz = z + j * hid;
            float s = 0.f;
            for (int c0 = 0; c0 < hid; c0 += 16) {   // 16 loads in flight, then the FMAs in order
                float pv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) pv[u] = PT[(size_t)(c0 + u) * vq + o];
#pragma unroll
                for (int u = 0; u < 16; ++u) s += pv[u] * zz[c0 + u];
            }
            rr[i] = s;
        }
        __syncthreads();
        for (int q = q0; q < q1; ++q) {
            const float *E = cbkT + (size_t)q * vq * CB;   // [vq][CB]
            float bdist[RVQ_ROWS];
            int bidx[RVQ_ROWS];
#pragma unroll
            for (int j = 0; j < RVQ_ROWS; ++j) { bdist[j] = 3.402823466e38f; bidx[j] = 0; }
            for (int code = tid; code < CB; code += RVQ_NT) {
                float d[RVQ_ROWS];
#pragma unroll
                for (int j = 0; j < RVQ_ROWS; ++j) d[j] = 0.f;
                // 16 dims of this code in flight at once (the loop is otherwise
                // one L2 round trip per 4 dims), then 8 rows x 16 dims of FMAs
                for (int k0 = 0; k0 < vq; k0 += 16) {
                    float e[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) e[i] = E[(size_t)(k0 + i) * CB + code];
#pragma unroll
                    for (int i = 0; i < 16; i += 4)
#pragma unroll
                        for (int j = 0; j < RVQ_ROWS; ++j) {
                            const float4 rv = *reinterpret_cast<const float4 *>(rr + j * vq + k0 + i);
                            const float a = rv.x - e[i], bb = rv.y - e[i + 1], c = rv.z - e[i + 2],
                                        dd = rv.w - e[i + 3];
                            d[j] += a * a + bb * bb + c * c + dd * dd;
                        }
                }
#pragma unroll
                for (int j = 0; j < RVQ_ROWS; ++j)
                    if (d[j] < bdist[j]) { bdist[j] = d[j]; bidx[j] = code; }
            }
            // (distance, index) argmin with first index on ties: wave, then the waves
#pragma unroll
            for (int j = 0; j < RVQ_ROWS; ++j) {
                float dv = bdist[j];
                int iv = bidx[j];
                for (int o = 32; o >= 1; o >>= 1) {
                    const float d2 = __shfl_xor(dv, o, 64);
                    const int i2 = __shfl_xor(iv, o, 64);
                    if (d2 < dv || (d2 == dv && i2 < iv)) { dv = d2; iv = i2; }
                }
                if (lane == 0) { bd[wave * RVQ_ROWS + j] = dv; bi[wave * RVQ_ROWS + j] = iv; }
            }
            __syncthreads();
            if (tid < RVQ_ROWS) {
                float dv = bd[tid];
                int iv = bi[tid];
                for (int w = 1; w < NW; ++w) {
                    const float d2 = bd[w * RVQ_ROWS + tid];
                    const int i2 = bi[w * RVQ_ROWS + tid];
                    if (d2 < dv || (d2 == dv && i2 < iv)) { dv = d2; iv = i2; }
                }
                best[tid] = iv;
                if (tid < nr) {
                    const int row = r0 + tid, b = row / T12, t = row - b * T12;
                    codes[((size_t)b * ldc_t + t) * 16 + q] = iv;
                }
            }
            __syncthreads();
            for (int i = tid; i < RVQ_ROWS * vq; i += RVQ_NT) {
                const int j = i / vq, o = i - j * vq;
                rr[i] -= E[(size_t)o * CB + best[j]];
            }
            __syncthreads();
        }
    }
}

// ----------------------------------------------------------------- host helpers
int launch_econv(EncModel *em, const EConv &gin, int nb, int nmax, hipStream_t st) {
    EConv g = gin;
    if (g.M <= 0 || nmax <= 0) return 0;
    if (nb > ENC_MAXB || !g.w || g.Kp % 32 || g.K > g.Kp) {
        fprintf(stderr, "qtts enc: bad conv launch (nb %d, K %d, Kp %d)\n", nb, g.K, g.Kp);
        return -1;
    }
    for (int b = 0; b < nb; ++b) {
        if (g.lout[b] > nmax || g.lout[b] < 0) return -1;
        // every input column a valid output reads, with the padding remap, lies in [0, lin)
        if (g.pmode == PAD_REFLECT && g.lout[b] > 0 && (g.padl >= g.lin[b] || g.lin[b] < 2)) {
            fprintf(stderr, "qtts enc: reflect padding %d needs more than %d input columns\n", g.padl, g.lin[b]);
            return -1;
        }
    }
    const bool rows = g.kw == 1 && g.xc == 1 && g.stride == 1 && g.padl == 0 && !g.x2 && g.act_in == ACT_NONE &&
                      g.K % 8 == 0 && g.xt % 4 == 0 && ((uintptr_t)g.x & 15) == 0;
    // split-K when one utterance's output tiles cannot fill the chip: each
    // K-step waits on its loads (a few steps of MFMA work cannot hide them),
    // so more, shorter workgroups are the latency cover.  The split depends
    // on the shape and the (padded) length only, never on the batch size, so
    // an utterance gets the same sums alone or in a batch of equal padding.
    const int tiles1 = (nmax + 63) / 64 * ((g.M + 63) / 64), nk = g.Kp / 32;
    int kz = 1;
    if (rows) kz = nk >= 8 ? std::min(4, nk / 4) : 1;
    else if (tiles1 < 256 && nk >= 8) kz = std::max(1, std::min(std::min(nk / 4, 16), (512 + tiles1 - 1) / tiles1));
    g.kz = kz; g.nb = nb; g.pn = nmax;
    if (kz > 1) {
        const size_t need = (size_t)kz * nb * g.M * nmax;
        if (need > em->part_cap) {
            hipStreamSynchronize(st);
            if (em->part) hipFree(em->part);
            em->part = nullptr;
            em->part_cap = 0;
            if (hipMalloc(&em->part, need * 4) != hipSuccess) {
                fprintf(stderr, "qtts enc: split-K workspace hipMalloc(%zu) failed\n", need * 4);
                return -1;
            }
            em->part_cap = need;
        }
        g.part = em->part;
    }
    const dim3 grid((nmax + 63) / 64, (g.M + 63) / 64, nb * kz);
    if (rows) hipLaunchKernelGGL((k_econv<true>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((k_econv<false>), grid, dim3(256), 0, st, g);
    if (kz > 1) hipLaunchKernelGGL(k_econv_reduce, dim3((nmax + 255) / 256, g.M, nb), dim3(256), 0, st, g);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

// ===================================================================== model
static void *ewalloc(EncModel *m, size_t n) {
    void *p = nullptr;
    const hipError_t prior = hipPeekAtLastError();
    const hipError_t e = hipMalloc(&p, n ? n : 16);
    if (e != hipSuccess) {
        fprintf(stderr, "qtts enc: hipMalloc(%zu) failed: %s (last error before it: %s)\n", n, hipGetErrorName(e),
                hipGetErrorName(prior));
        return nullptr;
    }
    m->wallocs.push_back(p);
    m->wbytes += n;
    return p;
}

static float *up_f32(EncModel *m, const std::vector<float> &v) {
    float *p = (float *)ewalloc(m, v.size() * 4);
    if (!p || hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

// host [M][K] fp32 -> device planes [3][M][Kp]
static int make_planes(EncModel *m, const float *host, int M, int K, int kw, EncW *out) {
    const int Kp = (K + 31) / 32 * 32;
    float *tmp = nullptr;
    if (hipMalloc(&tmp, (size_t)M * K * 4) != hipSuccess) return -1;
    unsigned short *pl = (unsigned short *)ewalloc(m, (size_t)3 * M * Kp * 2);
    int rc = -1;
    if (pl && hipMemcpy(tmp, host, (size_t)M * K * 4, hipMemcpyHostToDevice) == hipSuccess) {
        const size_t n = (size_t)M * Kp;
        hipLaunchKernelGGL(k_ewsplit, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, tmp, M, K, Kp, pl);
        rc = hipDeviceSynchronize() == hipSuccess ? 0 : -1;
    }
    hipFree(tmp);
    if (rc) return -1;
    out->p = pl; out->M = M; out->K = K; out->Kp = Kp; out->kw = kw;
    return 0;
}

int enc_set_dims(EncModel *m, const qtts_enc_dims_t *d) {
    m->d = *d;
    m->have_dims = true;
    return 0;
}

size_t enc_weight_bytes(const EncModel *m) { return m->wbytes; }

int enc_put_tensor(EncModel *m, const std::string &name, const void *host, int dtype, const int64_t *shape, int ndim,
                   size_t n) {
    const bool spk = name.compare(0, 16, "speaker_encoder.") == 0;
    const bool mimi = name.compare(0, 8, "encoder.") == 0;
    if (!spk && !mimi) return 0;
    if (mimi) {
        // only what encode() reads: no output projections / init flags, and the
        // first encoder_valid_num_quantizers codebooks (the reference slices
        // the codes to them, modeling_qwen3_tts_tokenizer_v2.py:983)
        if (name.find("output_proj") != std::string::npos || name.find(".initialized") != std::string::npos)
            return 1;
        const std::string ac = "encoder.quantizer.acoustic_residual_vector_quantizer.layers.";
        if (name.compare(0, ac.size(), ac) == 0) {
            const int i = atoi(name.c_str() + ac.size());
            const int nac = m->have_dims ? m->d.n_valid - m->d.n_sem : 15;
            if (i >= nac) return 1;
        }
    }
    std::vector<float> v(n);
    if (dtype == 0) memcpy(v.data(), host, n * 4);
    else {
        const uint16_t *h = (const uint16_t *)host;
        for (size_t i = 0; i < n; ++i) {
            if (dtype == 1) {
                const uint32_t u = (uint32_t)h[i] << 16;
                memcpy(&v[i], &u, 4);
            } else {
                _Float16 x;
                memcpy(&x, &h[i], 2);
                v[i] = (float)x;
            }
        }
    }
    m->host[name] = std::move(v);
    m->shape[name] = std::vector<int64_t>(shape, shape + ndim);
    (spk ? m->got_spk : m->got_mimi) = true;
    return 1;
}

// ---- slaney mel filterbank (librosa.filters.mel, htk=False, norm="slaney")
static double hz2mel(double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + log(f / min_log_hz) / logstep : f / f_sp;
}
static double mel2hz(double mm) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
    return mm >= min_log_mel ? min_log_hz * exp(logstep * (mm - min_log_mel)) : f_sp * mm;
}

static int build_mel_front(EncModel *m) {
    const int nfft = 1024, nf = nfft / 2 + 1, nm = m->d.mel_dim;
    const double sr = 24000.0, fmin = 0.0, fmax = 12000.0;
    // Hann-windowed DFT basis: rows f (cos) and nf + f (-sin); angle index f*n mod nfft
    std::vector<float> basis((size_t)2 * nf * nfft);
    for (int f = 0; f < nf; ++f)
        for (int n = 0; n < nfft; ++n) {
            const double w = 0.5 - 0.5 * cos(2.0 * M_PI * n / nfft);
            const double a = 2.0 * M_PI * (double)((long)f * n % nfft) / nfft;
            basis[(size_t)f * nfft + n] = (float)(w * cos(a));
            basis[(size_t)(nf + f) * nfft + n] = (float)(-w * sin(a));
        }
    if (make_planes(m, basis.data(), 2 * nf, nfft, nfft, &m->stft)) return -1;
    std::vector<double> mf(nm + 2);
    const double lo = hz2mel(fmin), hi = hz2mel(fmax);
    for (int i = 0; i < nm + 2; ++i) mf[i] = mel2hz(lo + (hi - lo) * i / (nm + 1));
    std::vector<float> fb((size_t)nm * nf, 0.f);
    std::vector<int> flo(nm, nf), fhi(nm, 0);
    for (int i = 0; i < nm; ++i) {
        const double enorm = 2.0 / (mf[i + 2] - mf[i]);
        for (int f = 0; f < nf; ++f) {
            const double fr = sr / 2.0 * f / (nf - 1);
            const double lower = -(mf[i] - fr) / (mf[i + 1] - mf[i]);
            const double upper = (mf[i + 2] - fr) / (mf[i + 2] - mf[i + 1]);
            const double wv = std::max(0.0, std::min(lower, upper)) * enorm;
            fb[(size_t)i * nf + f] = (float)wv;
            if (fb[(size_t)i * nf + f] != 0.f) { flo[i] = std::min(flo[i], f); fhi[i] = std::max(fhi[i], f + 1); }
        }
        if (fhi[i] < flo[i]) { flo[i] = 0; fhi[i] = 0; }
    }
    m->melfb = up_f32(m, fb);
    int *ib = (int *)ewalloc(m, (size_t)2 * nm * 4);
    if (!m->melfb || !ib) return -1;
    std::vector<int> lh(2 * nm);
    for (int i = 0; i < nm; ++i) { lh[i] = flo[i]; lh[nm + i] = fhi[i]; }
    if (hipMemcpy(ib, lh.data(), lh.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
    m->fw["#melfb_lo"] = reinterpret_cast<float *>(ib);
    return 0;
}

static const std::vector<float> *hget(EncModel *m, const std::string &n) {
    auto it = m->host.find(n);
    if (it == m->host.end()) { fprintf(stderr, "Error: missing encoder tensor: %s\n", n.c_str()); return nullptr; }
    return &it->second;
}

static int conv_w(EncModel *m, const std::string &n, int co, int ci, int kw) {
    const std::vector<float> *h = hget(m, n);
    if (!h) return -1;
    if (h->size() != (size_t)co * ci * kw) {
        fprintf(stderr, "Error: encoder tensor %s has %zu elements, expected %d x %d x %d\n", n.c_str(), h->size(), co,
                ci, kw);
        return -1;
    }
    return make_planes(m, h->data(), co, ci * kw, kw, &m->cw[n]);
}

static int vec_w(EncModel *m, const std::string &n, size_t expect) {
    const std::vector<float> *h = hget(m, n);
    if (!h) return -1;
    if (expect && h->size() != expect) {
        fprintf(stderr, "Error: encoder tensor %s has %zu elements, expected %zu\n", n.c_str(), h->size(), expect);
        return -1;
    }
    return (m->fw[n] = up_f32(m, *h)) ? 0 : -1;
}

static int finalize_speaker(EncModel *m) {
    const qtts_enc_dims_t &d = m->d;
    if (d.n_ch < 3 || d.n_ch > 8 || d.mel_dim != 128 || d.res2net_scale < 2) {
        fprintf(stderr, "Error: unsupported speaker encoder config (channels %d, mel %d)\n", d.n_ch, d.mel_dim);
        return -1;
    }
    const std::string P = "speaker_encoder.";
    const int C = d.ch[0], sc = d.res2net_scale;
    for (int i = 1; i < d.n_ch - 1; ++i)
        if (d.ch[i] != C || C % sc) { fprintf(stderr, "Error: ECAPA channels must be equal\n"); return -1; }
    if (d.ch[d.n_ch - 1] != (d.n_ch - 2) * C) { fprintf(stderr, "Error: ECAPA mfa channels\n"); return -1; }
    ECK(conv_w(m, P + "blocks.0.conv.weight", C, d.mel_dim, d.ks[0]));
    ECK(vec_w(m, P + "blocks.0.conv.bias", C));
    for (int i = 1; i < d.n_ch - 1; ++i) {
        const std::string b = P + "blocks." + std::to_string(i) + ".";
        ECK(conv_w(m, b + "tdnn1.conv.weight", C, C, 1));
        ECK(vec_w(m, b + "tdnn1.conv.bias", C));
        for (int j = 0; j < sc - 1; ++j) {
            const std::string r = b + "res2net_block.blocks." + std::to_string(j) + ".conv.";
            ECK(conv_w(m, r + "weight", C / sc, C / sc, d.ks[i]));
            ECK(vec_w(m, r + "bias", C / sc));
        }
        ECK(conv_w(m, b + "tdnn2.conv.weight", C, C, 1));
        ECK(vec_w(m, b + "tdnn2.conv.bias", C));
        ECK(vec_w(m, b + "se_block.conv1.weight", (size_t)d.se_ch * C));
        ECK(vec_w(m, b + "se_block.conv1.bias", d.se_ch));
        ECK(vec_w(m, b + "se_block.conv2.weight", (size_t)C * d.se_ch));
        ECK(vec_w(m, b + "se_block.conv2.bias", C));
    }
    const int CM = d.ch[d.n_ch - 1];
    ECK(conv_w(m, P + "mfa.conv.weight", CM, CM, d.ks[d.n_ch - 1]));
    ECK(vec_w(m, P + "mfa.conv.bias", CM));
    // asp.tdnn over cat[x, mean, std]: the x columns as MFMA planes, the
    // time-constant mean / std columns as a per-utterance bias GEMV
    {
        const std::vector<float> *h = hget(m, P + "asp.tdnn.conv.weight");
        if (!h || h->size() != (size_t)d.att_ch * 3 * CM) return -1;
        std::vector<float> wx((size_t)d.att_ch * CM), wms((size_t)d.att_ch * 2 * CM);
        for (int a = 0; a < d.att_ch; ++a) {
            memcpy(&wx[(size_t)a * CM], &(*h)[(size_t)a * 3 * CM], (size_t)CM * 4);
            memcpy(&wms[(size_t)a * 2 * CM], &(*h)[(size_t)a * 3 * CM + CM], (size_t)2 * CM * 4);
        }
        ECK(make_planes(m, wx.data(), d.att_ch, CM, 1, &m->cw["#asp_x"]));
        ECK((m->fw["#asp_ms"] = up_f32(m, wms)) ? 0 : -1);
    }
    ECK(vec_w(m, P + "asp.tdnn.conv.bias", d.att_ch));
    ECK(conv_w(m, P + "asp.conv.weight", CM, d.att_ch, 1));
    ECK(vec_w(m, P + "asp.conv.bias", CM));
    ECK(vec_w(m, P + "fc.weight", (size_t)d.enc_dim * 2 * CM));
    ECK(vec_w(m, P + "fc.bias", d.enc_dim));
    return build_mel_front(m);
}

static int finalize_mimi(EncModel *m) {
    const qtts_enc_dims_t &d = m->d;
    if (d.n_valid != 16 || d.n_sem < 1 || d.n_sem >= d.n_valid || d.hidden % 16 || d.vq_dim % 32 ||
        d.head_dim % 8 || d.head_dim > 128 || d.hidden > 1024 || d.vq_dim > 512 || d.compress < 1) {
        fprintf(stderr, "Error: unsupported 12 Hz encoder config (hidden %d, vq %d, head_dim %d, valid %d)\n", d.hidden,
                d.vq_dim, d.head_dim, d.n_valid);
        return -1;
    }
    const std::string P = "encoder.encoder.layers.";
    int li = 0, C = d.n_filters;
    ECK(conv_w(m, P + "0.conv.weight", C, 1, d.kernel));
    ECK(vec_w(m, P + "0.conv.bias", C));
    li = 1;
    for (int ri = 3; ri >= 0; --ri) {
        const int r = d.ratios[ri];
        for (int j = 0; j < d.n_res; ++j) {
            const std::string b = P + std::to_string(li) + ".block.";
            ECK(conv_w(m, b + "1.conv.weight", C / d.compress, C, d.res_kernel));
            ECK(vec_w(m, b + "1.conv.bias", C / d.compress));
            ECK(conv_w(m, b + "3.conv.weight", C, C / d.compress, 1));
            ECK(vec_w(m, b + "3.conv.bias", C));
            li += 1;
        }
        li += 1;   // ELU
        ECK(conv_w(m, P + std::to_string(li) + ".conv.weight", 2 * C, C, 2 * r));
        ECK(vec_w(m, P + std::to_string(li) + ".conv.bias", 2 * C));
        li += 1;
        C *= 2;
    }
    li += 1;
    ECK(conv_w(m, P + std::to_string(li) + ".conv.weight", d.hidden, C, d.last_kernel));
    ECK(vec_w(m, P + std::to_string(li) + ".conv.bias", d.hidden));
    const int H = d.hidden, qd = d.heads * d.head_dim, kd = d.kv_heads * d.head_dim;
    for (int l = 0; l < d.layers; ++l) {
        const std::string p = "encoder.encoder_transformer.layers." + std::to_string(l) + ".";
        ECK(vec_w(m, p + "input_layernorm.weight", H));
        ECK(vec_w(m, p + "input_layernorm.bias", H));
        ECK(vec_w(m, p + "post_attention_layernorm.weight", H));
        ECK(vec_w(m, p + "post_attention_layernorm.bias", H));
        ECK(conv_w(m, p + "self_attn.q_proj.weight", qd, H, 1));
        ECK(conv_w(m, p + "self_attn.k_proj.weight", kd, H, 1));
        ECK(conv_w(m, p + "self_attn.v_proj.weight", kd, H, 1));
        ECK(conv_w(m, p + "self_attn.o_proj.weight", H, qd, 1));
        ECK(conv_w(m, p + "mlp.fc1.weight", d.inter, H, 1));
        ECK(conv_w(m, p + "mlp.fc2.weight", H, d.inter, 1));
        ECK(vec_w(m, p + "self_attn_layer_scale.scale", H));
        ECK(vec_w(m, p + "mlp_layer_scale.scale", H));
    }
    ECK(conv_w(m, "encoder.downsample.conv.weight", H, H, 4));
    for (const char *kind : {"semantic", "acoustic"}) {   // input_proj [vq][H] -> transposed [H][vq]
        const std::string n = std::string("encoder.quantizer.") + kind + "_residual_vector_quantizer.input_proj.weight";
        const std::vector<float> *h = hget(m, n);
        if (!h || h->size() != (size_t)d.vq_dim * H) return -1;
        std::vector<float> t((size_t)H * d.vq_dim);
        for (int o = 0; o < d.vq_dim; ++o)
            for (int c = 0; c < H; ++c) t[(size_t)c * d.vq_dim + o] = (*h)[(size_t)o * H + c];
        ECK((m->fw[n] = up_f32(m, t)) ? 0 : -1);
    }
    // codebooks: embed_sum / max(cluster_usage, 1e-5) (MimiEuclideanCodebook.embed)
    std::vector<float> cb((size_t)d.n_valid * d.cb_size * d.vq_dim);   // [q][vq][CB] (dim-major)
    for (int q = 0; q < d.n_valid; ++q) {
        const std::string p = q < d.n_sem
            ? "encoder.quantizer.semantic_residual_vector_quantizer.layers." + std::to_string(q) + ".codebook."
            : "encoder.quantizer.acoustic_residual_vector_quantizer.layers." + std::to_string(q - d.n_sem) + ".codebook.";
        const std::vector<float> *es = hget(m, p + "embed_sum"), *us = hget(m, p + "cluster_usage");
        if (!es || !us || es->size() != (size_t)d.cb_size * d.vq_dim || us->size() != (size_t)d.cb_size) return -1;
        for (int c = 0; c < d.cb_size; ++c) {
            const float u = std::max((*us)[c], 1e-5f);
            for (int k = 0; k < d.vq_dim; ++k)
                cb[((size_t)q * d.vq_dim + k) * d.cb_size + c] = (*es)[(size_t)c * d.vq_dim + k] / u;
        }
    }
    return (m->cbk = up_f32(m, cb)) ? 0 : -1;
}

// Never fatal: a model whose encoders do not fit still decodes (custom voice,
// voice clone from given codes / x-vectors); the failing encoder stays off
// (spk_ready / mimi_ready false) and its entry points refuse with a message.
int enc_finalize(EncModel *m, int talker_hidden) {
    if ((m->got_spk || m->got_mimi) && !m->have_dims) {
        fprintf(stderr, "Warning: encoder tensors without an encoder config: voice-clone encoders disabled\n");
    } else {
        if (m->got_spk) {
            // the x-vector takes the place of a talker codec-embedding row
            // (modeling_qwen3_tts.py:2104-2125): its width must be the talker's
            if (m->d.enc_dim != talker_hidden)
                fprintf(stderr, "Warning: speaker encoder enc_dim %d != talker hidden %d: speaker encoder disabled\n",
                        m->d.enc_dim, talker_hidden);
            else if (finalize_speaker(m) == 0)
                m->spk_ready = true;
            else
                fprintf(stderr, "Warning: speaker encoder weights rejected: speaker encoder disabled\n");
        }
        if (m->got_mimi) {
            if (finalize_mimi(m) == 0) m->mimi_ready = true;
            else fprintf(stderr, "Warning: 12 Hz encoder weights rejected: reference-audio encoding disabled\n");
        }
    }
    m->host.clear();
    m->shape.clear();
    return 0;
}

void enc_destroy(EncModel *m) {
    for (void *p : m->wallocs) hipFree(p);
    for (void *p : m->sallocs) hipFree(p);
    if (m->part) hipFree(m->part);
    m->part = nullptr;
    m->part_cap = 0;
    m->wallocs.clear();
    m->sallocs.clear();
    m->sbase = nullptr;
    m->scap = 0;
}

// ---- scratch: one device block carved per call (grown on demand)
static char *scratch(EncModel *m, size_t bytes) {
    if (bytes > m->scap) {
        hipStreamSynchronize(m->st);
        for (void *p : m->sallocs) hipFree(p);
        m->sallocs.clear();
        m->scap = 0;
        m->sbase = nullptr;
        void *p = nullptr;
        const hipError_t prior = hipPeekAtLastError();
        const hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            fprintf(stderr, "qtts enc: scratch hipMalloc(%zu) failed: %s (last error before it: %s)\n", bytes,
                    hipGetErrorName(e), hipGetErrorName(prior));
            return nullptr;
        }
        m->sallocs.push_back(p);
        m->sbase = (char *)p;
        m->scap = bytes;
    }
    return m->sbase;
}

struct Carve {
    char *base;
    size_t off = 0;
    template <class T> T *take(size_t n) {
        T *p = reinterpret_cast<T *>(base + off);
        off += (n * sizeof(T) + 255) / 256 * 256;
        return p;
    }
};

static size_t carve_size(const std::vector<size_t> &bytes) {
    size_t s = 0;
    for (size_t b : bytes) s += (b + 255) / 256 * 256;
    return s;
}

static EConv conv_of(const EncW &w) {
    EConv g;
    g.w = w.p;
    g.wplane = (size_t)w.M * w.Kp;
    g.M = w.M; g.K = w.K; g.Kp = w.Kp; g.kw = w.kw;
    return g;
}

static const EncW *W(EncModel *m, const std::string &n) {
    auto it = m->cw.find(n);
    if (it == m->cw.end()) { fprintf(stderr, "qtts enc: no weight %s\n", n.c_str()); return nullptr; }
    return &it->second;
}
static const float *F(EncModel *m, const std::string &n) {
    auto it = m->fw.find(n);
    return it == m->fw.end() ? nullptr : it->second;
}

static int upload_wavs(EncModel *m, int nb, const float *const *wav, const int *n, int nmax, float *dst) {
    hipStream_t st = m->st;
    if (hipMemsetAsync(dst, 0, (size_t)nb * nmax * 4, st) != hipSuccess) return -1;
    for (int b = 0; b < nb; ++b)
        if (hipMemcpyAsync(dst + (size_t)b * nmax, wav[b], (size_t)n[b] * 4, hipMemcpyHostToDevice, st) != hipSuccess)
            return -1;
    return 0;
}

// ===================================================================== speaker x-vector
int enc_speaker(EncModel *m, int nb, const float *const *wav, const int *n, float *out, float *mel_out) {
    if (!m->spk_ready) { fprintf(stderr, "qtts: the model has no speaker encoder (speaker_encoder.*)\n"); return -1; }
    if (nb < 1 || nb > ENC_MAXB) { fprintf(stderr, "qtts: speaker encoder batch %d not in 1..%d\n", nb, ENC_MAXB); return -1; }
    const qtts_enc_dims_t &d = m->d;
    const int hop = 256, nfft = 1024, padr = (nfft - hop) / 2, nf = nfft / 2 + 1, nm = d.mel_dim;
    int nmax = 0, T[ENC_MAXB], Tm = 0;
    for (int b = 0; b < nb; ++b) {
        if (!wav[b] || n[b] <= padr) { fprintf(stderr, "qtts: reference audio %d too short (%d samples)\n", b, n[b]); return -1; }
        nmax = std::max(nmax, n[b]);
        T[b] = (n[b] + 2 * padr - nfft) / hop + 1;
        Tm = std::max(Tm, T[b]);
    }
    hipStream_t st = m->st;
    const int C = d.ch[0], CM = d.ch[d.n_ch - 1], sc = d.res2net_scale, cs = C / sc, A = d.att_ch;
    const int nblk = d.n_ch - 2;
    const size_t fT = (size_t)Tm * 4;
    std::vector<size_t> sz = {(size_t)nb * nmax * 4, (size_t)nb * 2 * nf * fT, (size_t)nb * nm * fT,
                              (size_t)nb * C * fT, (size_t)nb * CM * fT, (size_t)nb * C * fT, (size_t)nb * C * fT,
                              (size_t)nb * C * fT, (size_t)nb * CM * fT, (size_t)nb * A * fT, (size_t)nb * CM * fT,
                              (size_t)nb * C * 4, (size_t)nb * d.se_ch * 4, (size_t)nb * C * 4,
                              (size_t)nb * 2 * CM * 4, (size_t)nb * A * 4, (size_t)nb * 2 * CM * 4,
                              (size_t)nb * d.enc_dim * 4, (size_t)ENC_MAXB * 4};
    char *base = scratch(m, carve_size(sz));
    if (!base) return -1;
    Carve cv{base};
    float *dw = cv.take<float>((size_t)nb * nmax), *spec = cv.take<float>((size_t)nb * 2 * nf * Tm);
    float *mel = cv.take<float>((size_t)nb * nm * Tm), *x0 = cv.take<float>((size_t)nb * C * Tm);
    float *cat = cv.take<float>((size_t)nb * CM * Tm), *h1 = cv.take<float>((size_t)nb * C * Tm);
    float *h2 = cv.take<float>((size_t)nb * C * Tm), *h3 = cv.take<float>((size_t)nb * C * Tm);
    float *mfa = cv.take<float>((size_t)nb * CM * Tm), *a1 = cv.take<float>((size_t)nb * A * Tm);
    float *lg = cv.take<float>((size_t)nb * CM * Tm), *mean = cv.take<float>((size_t)nb * C);
    float *s1 = cv.take<float>((size_t)nb * d.se_ch), *s2 = cv.take<float>((size_t)nb * C);
    float *stats = cv.take<float>((size_t)nb * 2 * CM), *b2 = cv.take<float>((size_t)nb * A);
    float *pooled = cv.take<float>((size_t)nb * 2 * CM), *xv = cv.take<float>((size_t)nb * d.enc_dim);
    int *lens = cv.take<int>(ENC_MAXB);
    ECK(upload_wavs(m, nb, wav, n, nmax, dw));
    ECK(hipMemcpyAsync(lens, T, nb * 4, hipMemcpyHostToDevice, st) != hipSuccess);
    auto setlen = [&](EConv &g) { for (int b = 0; b < nb; ++b) { g.lin[b] = T[b]; g.lout[b] = T[b]; } };
    auto chan = [&](EConv &g, const float *x, int Cx, float *y, int Cy) {   // channel-major [nb][C][Tm] in / out
        g.x = x; g.xb = (size_t)Cx * Tm; g.xc = Tm; g.xt = 1;
        g.y = y; g.yb = (size_t)Cy * Tm; g.yc = Tm; g.yt = 1;
    };
    // 1. STFT: one input channel, kw = n_fft, stride = hop, reflect pad (n_fft - hop) / 2
    {
        EConv g = conv_of(m->stft);
        g.stride = hop; g.padl = padr; g.pmode = PAD_REFLECT;
        g.x = dw; g.xb = nmax; g.xc = 0; g.xt = 1;
        g.y = spec; g.yb = (size_t)2 * nf * Tm; g.yc = Tm; g.yt = 1;
        for (int b = 0; b < nb; ++b) { g.lin[b] = n[b]; g.lout[b] = T[b]; }
        ECK(launch_econv(m, g, nb, Tm, st));
    }
    hipLaunchKernelGGL(k_mel, dim3(Tm, nb), dim3(256), 0, st, spec, nf, Tm, lens, m->melfb,
                       reinterpret_cast<const int *>(F(m, "#melfb_lo")),
                       reinterpret_cast<const int *>(F(m, "#melfb_lo")) + nm, nm, mel);
    const std::string P = "speaker_encoder.";
    auto tdnn = [&](const std::string &name, const float *x, int Cx, const float *x2, float *y, int Cy, int dil,
                    int act) {
        const EncW *w = W(m, name + ".weight");
        if (!w) return -1;
        EConv g = conv_of(*w);
        chan(g, x, Cx, y, Cy);
        g.x2 = x2;
        g.dil = dil;
        g.padl = dil * (w->kw - 1) / 2;
        g.pmode = PAD_REFLECT;
        g.bias = F(m, name + ".bias");
        g.act_out = act;
        setlen(g);
        return launch_econv(m, g, nb, Tm, st);
    };
    // 2. block 0
    ECK(tdnn(P + "blocks.0.conv", mel, nm, nullptr, x0, C, d.dil[0], ACT_RELU));
    // 3. SE-Res2Net blocks, outputs into the channel slices of cat
    for (int i = 1; i <= nblk; ++i) {
        const std::string bp = P + "blocks." + std::to_string(i) + ".";
        const float *in = i == 1 ? x0 : cat + (size_t)(i - 2) * C * Tm;
        const int inC = i == 1 ? C : CM;
        ECK(tdnn(bp + "tdnn1.conv", in, inC, nullptr, h1, C, 1, ACT_RELU));
        ECK(hipMemcpy2DAsync(h2, (size_t)C * fT, h1, (size_t)C * fT, (size_t)cs * fT, nb, hipMemcpyDeviceToDevice, st) !=
            hipSuccess);
        for (int j = 1; j < sc; ++j) {
            const std::string rp = bp + "res2net_block.blocks." + std::to_string(j - 1) + ".conv";
            const float *x2 = j >= 2 ? h2 + (size_t)(j - 1) * cs * Tm : nullptr;
            ECK(tdnn(rp, h1 + (size_t)j * cs * Tm, C, x2, h2 + (size_t)j * cs * Tm, C, d.dil[i], ACT_RELU));
        }
        ECK(tdnn(bp + "tdnn2.conv", h2, C, nullptr, h3, C, 1, ACT_RELU));
        hipLaunchKernelGGL(k_row_mean, dim3((C + 3) / 4, nb), dim3(256), 0, st, h3, (size_t)C * Tm, Tm, lens, C, mean);
        hipLaunchKernelGGL(k_egemv, dim3((d.se_ch + 3) / 4, nb), dim3(256), 0, st, F(m, bp + "se_block.conv1.weight"),
                           d.se_ch, C, mean, C, F(m, bp + "se_block.conv1.bias"), (int)ACT_RELU, s1, d.se_ch);
        hipLaunchKernelGGL(k_egemv, dim3((C + 3) / 4, nb), dim3(256), 0, st, F(m, bp + "se_block.conv2.weight"), C,
                           d.se_ch, s1, d.se_ch, F(m, bp + "se_block.conv2.bias"), (int)ACT_SIGMOID, s2, C);
        hipLaunchKernelGGL(k_se_apply, dim3((Tm + 255) / 256, C, nb), dim3(256), 0, st, h3, (size_t)C * Tm, s2, C, in,
                           (size_t)inC * Tm, cat + (size_t)(i - 1) * C * Tm, (size_t)CM * Tm, Tm, lens);
    }
    // 4. multi-layer feature aggregation
    ECK(tdnn(P + "mfa.conv", cat, CM, nullptr, mfa, CM, d.dil[d.n_ch - 1], ACT_RELU));
    // 5. attentive statistics pooling
    hipLaunchKernelGGL(k_asp_stats, dim3((CM + 3) / 4, nb), dim3(256), 0, st, mfa, (size_t)CM * Tm, Tm, lens, CM, stats);
    hipLaunchKernelGGL(k_egemv, dim3((A + 3) / 4, nb), dim3(256), 0, st, F(m, "#asp_ms"), A, 2 * CM, stats, 2 * CM,
                       F(m, P + "asp.tdnn.conv.bias"), (int)ACT_NONE, b2, A);
    {
        const EncW *w = W(m, "#asp_x");
        if (!w) return -1;
        EConv g = conv_of(*w);
        chan(g, mfa, CM, a1, A);
        g.bias2 = b2; g.bias2_b = A; g.act_out = ACT_RELU_TANH;
        setlen(g);
        ECK(launch_econv(m, g, nb, Tm, st));
    }
    ECK(tdnn(P + "asp.conv", a1, A, nullptr, lg, CM, 1, ACT_NONE));
    hipLaunchKernelGGL(k_asp_pool, dim3((CM + 3) / 4, nb), dim3(256), 0, st, mfa, (size_t)CM * Tm, lg, (size_t)CM * Tm,
                       Tm, lens, CM, pooled);
    // 6. final 1x1 conv on the pooled statistics
    hipLaunchKernelGGL(k_egemv, dim3((d.enc_dim + 3) / 4, nb), dim3(256), 0, st, F(m, P + "fc.weight"), d.enc_dim,
                       2 * CM, pooled, 2 * CM, F(m, P + "fc.bias"), (int)ACT_NONE, xv, d.enc_dim);
    ECK(hipGetLastError() != hipSuccess);
    ECK(hipMemcpyAsync(out, xv, (size_t)nb * d.enc_dim * 4, hipMemcpyDeviceToHost, st) != hipSuccess);
    if (mel_out) {
        size_t off = 0;
        for (int b = 0; b < nb; ++b) {
            ECK(hipMemcpy2DAsync(mel_out + off, (size_t)T[b] * 4, mel + (size_t)b * nm * Tm, fT, (size_t)T[b] * 4, nm,
                                 hipMemcpyDeviceToHost, st) != hipSuccess);
            off += (size_t)nm * T[b];
        }
    }
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

// ===================================================================== 12 Hz codes
static int ensure_mimi_rope(EncModel *m, int T) {
    if (T <= m->rope_cap) return 0;
    const int hd = m->d.head_dim, cap = std::max(T, 512);
    std::vector<float> c((size_t)cap * hd), s((size_t)cap * hd);
    // MimiRotaryEmbedding: float32 inv_freq = 1 / theta^(2i/hd), float32 angle = pos * inv_freq
    for (int i = 0; i < hd / 2; ++i) {
        const float inv = 1.0f / powf(m->d.rope_theta, (float)(2 * i) / (float)hd);
        for (int p = 0; p < cap; ++p) {
            const float a = (float)p * inv;
            c[(size_t)p * hd + i] = c[(size_t)p * hd + i + hd / 2] = (float)cos((double)a);
            s[(size_t)p * hd + i] = s[(size_t)p * hd + i + hd / 2] = (float)sin((double)a);
        }
    }
    m->rope_cos = up_f32(m, c);
    m->rope_sin = up_f32(m, s);
    if (!m->rope_cos || !m->rope_sin) return -1;
    m->rope_cap = cap;
    return 0;
}

int enc_codes(EncModel *m, int nb, const float *const *wav, const int *n, int *codes, int max_frames, int *frames,
              float *latent) {
    if (!m->mimi_ready) { fprintf(stderr, "qtts: the model has no 12 Hz encoder (speech_tokenizer encoder.*)\n"); return -1; }
    if (nb < 1 || nb > ENC_MAXB) { fprintf(stderr, "qtts: audio encoder batch %d not in 1..%d\n", nb, ENC_MAXB); return -1; }
    const qtts_enc_dims_t &d = m->d;
    int nmax = 0;
    for (int b = 0; b < nb; ++b) {
        if (!wav[b] || n[b] < 1) { fprintf(stderr, "qtts: reference audio %d is empty\n", b); return -1; }
        nmax = std::max(nmax, n[b]);
    }
    // lengths through the SEANet strides: ceil(L / r) each (MimiConv1d extra right padding)
    int Ls[5];
    Ls[0] = nmax;
    for (int i = 0; i < 4; ++i) Ls[i + 1] = (Ls[i] + d.ratios[3 - i] - 1) / d.ratios[3 - i];
    const int T25 = Ls[4], T12 = (T25 + 1) / 2;
    for (int b = 0; b < nb; ++b) {
        frames[b] = (n[b] + 1919) / 1920;
        if (frames[b] > max_frames) { fprintf(stderr, "qtts: %d reference frames exceed max_frames %d\n", frames[b], max_frames); return -1; }
    }
    ECK(ensure_mimi_rope(m, T25));
    hipStream_t st = m->st;
    const int H = d.hidden, qd = d.heads * d.head_dim, kd = d.kv_heads * d.head_dim, R = nb * T25;
    size_t big = 0;   // largest [C][L] activation of the conv stack per utterance
    {
        int C = d.n_filters;
        for (int i = 0; i < 4; ++i) { big = std::max(big, (size_t)C * Ls[i]); C *= 2; big = std::max(big, (size_t)C * Ls[i + 1]); }
    }
    std::vector<size_t> sz = {(size_t)nb * nmax * 4, (size_t)nb * big * 4, (size_t)nb * big * 4,
                              (size_t)R * H * 4, (size_t)R * H * 4, (size_t)R * qd * 4, (size_t)R * kd * 4,
                              (size_t)R * kd * 4, (size_t)R * qd * 4, (size_t)R * d.inter * 4,
                              (size_t)nb * H * T12 * 4, (size_t)nb * T12 * 16 * 4, (size_t)R * 4, (size_t)R * 4};
    char *base = scratch(m, carve_size(sz));
    if (!base) return -1;
    Carve cv{base};
    float *dw = cv.take<float>((size_t)nb * nmax), *A = cv.take<float>((size_t)nb * big), *B = cv.take<float>((size_t)nb * big);
    float *x = cv.take<float>((size_t)R * H), *h = cv.take<float>((size_t)R * H), *q = cv.take<float>((size_t)R * qd);
    float *k = cv.take<float>((size_t)R * kd), *v = cv.take<float>((size_t)R * kd), *att = cv.take<float>((size_t)R * qd);
    float *mlp = cv.take<float>((size_t)R * d.inter), *lat = cv.take<float>((size_t)nb * H * T12);
    int *dcodes = cv.take<int>((size_t)nb * T12 * 16), *row_b = cv.take<int>(R), *pos = cv.take<int>(R);
    ECK(upload_wavs(m, nb, wav, n, nmax, dw));
    const std::string P = "encoder.encoder.layers.";
    // causal SEANet conv over channel-major [nb][C][L] (MimiConv1d: left pad k_eff - stride, zero)
    auto sconv = [&](const std::string &name, const float *xin, int Ci, int Lin, float *y, int Co, int Lout,
                     int stride, bool elu, const float *res) {
        const EncW *w = W(m, name + ".weight");
        if (!w) return -1;
        EConv g = conv_of(*w);
        g.x = xin; g.xb = (size_t)Ci * Lin; g.xc = Lin; g.xt = 1;
        g.y = y; g.yb = (size_t)Co * Lout; g.yc = Lout; g.yt = 1;
        g.stride = stride; g.padl = w->kw - stride; g.pmode = PAD_ZERO;
        g.act_in = elu ? 1 : 0;
        g.bias = F(m, name + ".bias");
        if (res) { g.res = res; g.rb = g.yb; g.rc = Lout; g.rt = 1; }
        for (int b = 0; b < nb; ++b) { g.lin[b] = Lin; g.lout[b] = Lout; }
        return launch_econv(m, g, nb, Lout, st);
    };
    ECK(sconv(P + "0.conv", dw, 1, nmax, A, d.n_filters, nmax, 1, false, nullptr));
    int li = 1, C = d.n_filters;
    float *cur = A, *oth = B;
    for (int i = 0; i < 4; ++i) {
        const int r = d.ratios[3 - i], L = Ls[i];
        for (int j = 0; j < d.n_res; ++j) {
            if (j > 0) { fprintf(stderr, "qtts enc: num_residual_layers > 1 unsupported\n"); return -1; }
            const std::string bp = P + std::to_string(li) + ".block.";
            ECK(sconv(bp + "1.conv", cur, C, L, oth, C / d.compress, L, 1, true, nullptr));
            ECK(sconv(bp + "3.conv", oth, C / d.compress, L, cur, C, L, 1, true, cur));
            li += 1;
        }
        li += 1;
        ECK(sconv(P + std::to_string(li) + ".conv", cur, C, L, oth, 2 * C, Ls[i + 1], r, true, nullptr));
        li += 1;
        C *= 2;
        std::swap(cur, oth);
    }
    li += 1;
    // final conv straight into time-major transformer rows x[b*T25 + t][H]
    {
        const std::string name = P + std::to_string(li) + ".conv";
        const EncW *w = W(m, name + ".weight");
        if (!w) return -1;
        EConv g = conv_of(*w);
        g.x = cur; g.xb = (size_t)C * T25; g.xc = T25; g.xt = 1;
        g.y = x; g.yb = (size_t)T25 * H; g.yc = 1; g.yt = H;
        g.padl = w->kw - 1; g.act_in = 1; g.bias = F(m, name + ".bias");
        for (int b = 0; b < nb; ++b) { g.lin[b] = T25; g.lout[b] = T25; }
        ECK(launch_econv(m, g, nb, T25, st));
    }
    // transformer over R = nb * T25 rows (MimiTransformerModel, no final norm)
    hipLaunchKernelGGL(k_rows_bt, dim3((R + 255) / 256), dim3(256), 0, st, row_b, pos, R, T25);
    auto lin = [&](const std::string &name, const float *xin, int K, float *y, int N, int act, const float *vec,
                   bool resid) {
        const EncW *w = W(m, name);
        if (!w) return -1;
        EConv g = conv_of(*w);
        g.x = xin; g.xb = 0; g.xc = 1; g.xt = K;
        g.y = y; g.yb = 0; g.yc = 1; g.yt = N;
        g.act_out = act; g.vec = vec;
        if (resid) { g.res = y; g.rb = 0; g.rc = 1; g.rt = N; }
        g.lin[0] = R; g.lout[0] = R;
        return launch_econv(m, g, 1, R, st);
    };
    for (int l = 0; l < d.layers; ++l) {
        const std::string p = "encoder.encoder_transformer.layers." + std::to_string(l) + ".";
        hipLaunchKernelGGL(k_ln_rows, dim3(R), dim3(256), 0, st, x, H, F(m, p + "input_layernorm.weight"),
                           F(m, p + "input_layernorm.bias"), d.norm_eps, h);
        ECK(lin(p + "self_attn.q_proj.weight", h, H, q, qd, ACT_NONE, nullptr, false));
        ECK(lin(p + "self_attn.k_proj.weight", h, H, k, kd, ACT_NONE, nullptr, false));
        ECK(lin(p + "self_attn.v_proj.weight", h, H, v, kd, ACT_NONE, nullptr, false));
        hipLaunchKernelGGL(k_rope_bt, dim3(R), dim3(256), 0, st, q, qd, d.heads, d.head_dim, T25, m->rope_cos, m->rope_sin);
        hipLaunchKernelGGL(k_rope_bt, dim3(R), dim3(256), 0, st, k, kd, d.kv_heads, d.head_dim, T25, m->rope_cos,
                           m->rope_sin);
        AttnArgs a;
        a.mode = 1; a.qkv = q; a.ld_qkv = qd; a.kc = k; a.vc = v; a.S = T25; a.pos = pos; a.row_b = row_b;
        a.NH = d.heads; a.KV = d.kv_heads; a.HD = d.head_dim; a.out = att; a.ld_out = qd; a.nrows = R;
        a.win = d.window;
        ECK(qtts_attention(a, st));
        ECK(lin(p + "self_attn.o_proj.weight", att, qd, x, H, ACT_NONE, F(m, p + "self_attn_layer_scale.scale"), true));
        hipLaunchKernelGGL(k_ln_rows, dim3(R), dim3(256), 0, st, x, H, F(m, p + "post_attention_layernorm.weight"),
                           F(m, p + "post_attention_layernorm.bias"), d.norm_eps, h);
        ECK(lin(p + "mlp.fc1.weight", h, H, mlp, d.inter, ACT_GELU, nullptr, false));
        ECK(lin(p + "mlp.fc2.weight", mlp, d.inter, x, H, ACT_NONE, F(m, p + "mlp_layer_scale.scale"), true));
    }
    // downsample: k 4, stride 2, replicate padding, no bias -> latent [nb][H][T12]
    {
        const EncW *w = W(m, "encoder.downsample.conv.weight");
        if (!w) return -1;
        EConv g = conv_of(*w);
        g.x = x; g.xb = (size_t)T25 * H; g.xc = 1; g.xt = H;
        g.y = lat; g.yb = (size_t)H * T12; g.yc = T12; g.yt = 1;
        g.stride = 2; g.padl = w->kw - 2; g.pmode = PAD_REPLICATE;
        for (int b = 0; b < nb; ++b) { g.lin[b] = T25; g.lout[b] = T12; }
        ECK(launch_econv(m, g, nb, T12, st));
    }
    // split RVQ encode of the first n_valid codebooks
    {
        const int rows = nb * T12;
        const size_t smem = ((size_t)RVQ_ROWS * (H + d.vq_dim) + 2 * (RVQ_NT / 64) * RVQ_ROWS + RVQ_ROWS) * 4 + 64;
        hipLaunchKernelGGL(k_rvq_enc, dim3((rows + RVQ_ROWS - 1) / RVQ_ROWS), dim3(RVQ_NT), smem, st, lat, T12, H, rows,
                           F(m, "encoder.quantizer.semantic_residual_vector_quantizer.input_proj.weight"),
                           F(m, "encoder.quantizer.acoustic_residual_vector_quantizer.input_proj.weight"), m->cbk,
                           d.cb_size, d.vq_dim, d.n_valid, d.n_sem, dcodes, T12);
    }
    ECK(hipGetLastError() != hipSuccess);
    std::vector<int> hc((size_t)nb * T12 * 16);
    ECK(hipMemcpyAsync(hc.data(), dcodes, hc.size() * 4, hipMemcpyDeviceToHost, st) != hipSuccess);
    std::vector<float> hl;
    if (latent) {
        hl.resize((size_t)nb * H * T12);
        ECK(hipMemcpyAsync(hl.data(), lat, hl.size() * 4, hipMemcpyDeviceToHost, st) != hipSuccess);
    }
    ECK(hipStreamSynchronize(st) != hipSuccess);
    for (int b = 0; b < nb; ++b) {
        for (int t = 0; t < max_frames; ++t)
            for (int g = 0; g < 16; ++g)
                codes[((size_t)b * max_frames + t) * 16 + g] = t < frames[b] ? hc[((size_t)b * T12 + t) * 16 + g] : -1;
        if (latent)
            for (int c = 0; c < H; ++c)
                for (int t = 0; t < max_frames; ++t)
                    latent[((size_t)b * H + c) * max_frames + t] =
                        t < frames[b] ? hl[((size_t)b * H + c) * T12 + t] : 0.f;
    }
    return 0;
}
