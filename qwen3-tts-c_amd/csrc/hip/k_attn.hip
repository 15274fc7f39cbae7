// k_attn.hip - GQA attention for the talker / sub-talker on gfx950.
//
// Decode (mode 0), one workgroup per (query head h, batch row b):
//   q, k, v of the new token come raw from the fused QKV GEMV output;
//   per-head RMSNorm (T.c:150-156) and rotate-half RoPE with a host table
//   (T.c:158-189) are applied in LDS; the workgroup that owns kv head
//   h/(NH/KV)'s first query head writes k, v into the fp32 KV cache
//   (T.c:191-196).  Scores over positions [0, pos] read K rows from the cache
//   (the current position from LDS, so no cross-workgroup hand-off is needed),
//   softmax with max subtraction (K.c:371-378), then P.V with V rows read as
//   coalesced float4 segments.
// Cached (mode 1, prefill): q was normalised/rotated in place and all k/v are
// already in the cache (qtts_qk_prep), positions come per row.
//
// Scores: HD/8 lanes per key (two float4 loads each) -> 256/(HD/8) keys per
// pass; P.V: HD/4 lanes per row -> 256/(HD/4) rows per pass, partial sums
// combined through LDS in a fixed order.
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

__device__ __forceinline__ void rope_lds(const float *x, float *y, const float *cs, const float *sn, int HD, int i) {
    const int half = HD >> 1;
    if (i < half) y[i] = x[i] * cs[i] - x[i + half] * sn[i];
    else y[i] = x[i] * cs[i] + x[i - half] * sn[i];
}

__global__ __launch_bounds__(256) void k_attn(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int tid = threadIdx.x;
    const int h = blockIdx.x, r = blockIdx.y;
    const int HD = a.HD, KVD = a.KV * a.HD, gph = a.NH / a.KV, kvh = h / gph;
    const int b = a.mode == 0 ? r : a.row_b[r];
    const int p = a.pos ? a.pos[r] : a.pos_const;
    const int n = p + 1;
    const int ts = (a.win > 0 && n > a.win) ? n - a.win : 0;  // first key in the window
    float *qr = sm;              // [HD] rotated q
    float *kr = qr + 128;        // [HD] rotated k (decode)
    float *vv = kr + 128;        // [HD] v (decode)
    float *tmp = vv + 128;       // [2*HD] scratch
    float *red = tmp + 256;      // [8]
    float *part = red + 8;       // [8][HD]
    float *sc = part + 8 * 128;  // [n]
    const float *row = a.qkv + (size_t)r * a.ld_qkv;
    const float *Kc = a.kc + (size_t)b * a.S * KVD + kvh * HD;
    const float *Vc = a.vc + (size_t)b * a.S * KVD + kvh * HD;

    if (a.mode == 0) {
        float qv = 0.f, kv = 0.f;
        if (tid < HD) {
            qv = row[h * HD + tid];
            kv = row[a.NH * HD + kvh * HD + tid];
            vv[tid] = row[(a.NH + a.KV) * HD + kvh * HD + tid];
        }
        const float ssq = block_sum256(qv * qv, red);
        const float ssk = block_sum256(kv * kv, red + 4);
        if (tid < HD) {
            tmp[tid] = qv * rms_inv(ssq, HD, a.eps) * a.qn_w[tid];
            tmp[128 + tid] = kv * rms_inv(ssk, HD, a.eps) * a.kn_w[tid];
        }
        __syncthreads();
        if (tid < HD) {
            const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
            rope_lds(tmp, qr, cs, sn, HD, tid);
            rope_lds(tmp + 128, kr, cs, sn, HD, tid);
        }
        __syncthreads();
        if (h % gph == 0 && tid < HD && !(a.skip && a.skip[b])) {
            a.kc[((size_t)b * a.S + p) * KVD + kvh * HD + tid] = kr[tid];
            a.vc[((size_t)b * a.S + p) * KVD + kvh * HD + tid] = vv[tid];
        }
    } else {
        if (tid < HD) qr[tid] = row[h * HD + tid];
        __syncthreads();
    }

    // ---- scores ----
    const float scale = div_rn(1.0f, sqrt_rn((float)HD));
    const int lpk = HD >> 3;        // lanes per key
    const int kpp = 256 / lpk;      // keys per pass
    const int gi = tid / lpk, li = tid - gi * lpk;
    const float4 q0 = *reinterpret_cast<const float4 *>(qr + 8 * li);
    const float4 q1 = *reinterpret_cast<const float4 *>(qr + 8 * li + 4);
    for (int t0 = ts; t0 < n; t0 += kpp) {
        const int t = t0 + gi;
        float s = 0.f;
        if (t < n) {
            const float *kp = (a.mode == 0 && t == p) ? kr + 8 * li : Kc + (size_t)t * KVD + 8 * li;
            const float4 k0 = *reinterpret_cast<const float4 *>(kp);
            const float4 k1 = *reinterpret_cast<const float4 *>(kp + 4);
            s = q0.x * k0.x + q0.y * k0.y + q0.z * k0.z + q0.w * k0.w + q1.x * k1.x + q1.y * k1.y + q1.z * k1.z +
                q1.w * k1.w;
        }
        for (int o = lpk >> 1; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (li == 0 && t < n) sc[t] = s * scale;
    }
    __syncthreads();
    // ---- softmax ----
    float mx = -3.402823466e38f;
    for (int t = ts + tid; t < n; t += 256) mx = fmaxf(mx, sc[t]);
    mx = block_max256(mx, red);
    float sum = 0.f;
    for (int t = ts + tid; t < n; t += 256) {
        const float e = expf(sc[t] - mx);
        sc[t] = e;
        sum += e;
    }
    sum = block_sum256(sum, red + 4);
    const float inv = div_rn(1.0f, sum);
    for (int t = ts + tid; t < n; t += 256) sc[t] *= inv;
    __syncthreads();
    // ---- P.V ----
    const int lpr = HD >> 2;        // lanes per row (float4 each)
    const int rpp = 256 / lpr;      // rows per pass (<= 8 for HD >= 128; tiny HD uses more groups)
    const int g2 = tid / lpr, l2 = tid - g2 * lpr;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t = ts + g2; t < n; t += rpp) {
        const float *vp = (a.mode == 0 && t == p) ? vv + 4 * l2 : Vc + (size_t)t * KVD + 4 * l2;
        const float4 v4 = *reinterpret_cast<const float4 *>(vp);
        const float w = sc[t];
        acc.x += w * v4.x; acc.y += w * v4.y; acc.z += w * v4.z; acc.w += w * v4.w;
    }
    // combine rpp partial rows: fold groups >= 8 into 8 slots first (small HD)
    const int ng = rpp < 8 ? rpp : 8;
    for (int gg = 0; gg < rpp; gg += 8) {
        if (g2 >= gg && g2 < gg + 8) {
            float *dst = part + (g2 - gg) * 128 + 4 * l2;
            if (gg == 0) { dst[0] = acc.x; dst[1] = acc.y; dst[2] = acc.z; dst[3] = acc.w; }
            else { dst[0] += acc.x; dst[1] += acc.y; dst[2] += acc.z; dst[3] += acc.w; }
        }
        __syncthreads();
    }
    if (tid < HD) {
        float s = 0.f;
        for (int gg = 0; gg < ng; ++gg) s += part[gg * 128 + tid];
        a.out[(size_t)r * a.ld_out + h * HD + tid] = s;
    }
}

// prefill: per row, normalise + rotate q heads in place, k heads -> cache, v -> cache
__global__ __launch_bounds__(256) void k_qk_prep(AttnArgs a) {
    __shared__ float buf[4096 + 64];
    const int r = blockIdx.x, tid = threadIdx.x;
    const int HD = a.HD, NH = a.NH, KV = a.KV, KVD = KV * HD;
    const int b = a.row_b[r], p = a.pos[r];
    float *row = const_cast<float *>(a.qkv) + (size_t)r * a.ld_qkv;
    float *x = buf;            // [NH+KV][HD] normalised
    float *red = buf + 4096;   // unused scratch
    const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
    const int nh = NH + KV;
    // one wave per head (loop), lanes stride over HD
    const int w = tid >> 6, l = tid & 63;
    for (int hh = w; hh < nh; hh += 4) {
        const float *src = row + hh * HD;
        float ss = 0.f;
        for (int i = l; i < HD; i += 64) ss += src[i] * src[i];
        ss = wave_sum(ss);
        const float iv = rms_inv(ss, HD, a.eps);
        const float *nw = hh < NH ? a.qn_w : a.kn_w;
        for (int i = l; i < HD; i += 64) x[hh * HD + i] = src[i] * iv * nw[i];
    }
    __syncthreads();
    for (int i = tid; i < nh * HD; i += 256) {
        const int hh = i / HD, e = i - hh * HD;
        float y;
        const int half = HD >> 1;
        const float *xh = x + hh * HD;
        if (e < half) y = xh[e] * cs[e] - xh[e + half] * sn[e];
        else y = xh[e] * cs[e] + xh[e - half] * sn[e];
        if (hh < NH) row[i] = y;
        else a.kc[((size_t)b * a.S + p) * KVD + (hh - NH) * HD + e] = y;
    }
    for (int i = tid; i < KVD; i += 256) a.vc[((size_t)b * a.S + p) * KVD + i] = row[nh * HD + i];
    (void)red;
}

}  // namespace

int qtts_attention(const AttnArgs &a, hipStream_t st) {
    if (a.HD > 128 || a.HD < 8 || (a.HD & 7) || a.NH % a.KV) {
        fprintf(stderr, "qtts_attention: unsupported head config NH=%d KV=%d HD=%d\n", a.NH, a.KV, a.HD);
        return -1;
    }
    size_t smem = (size_t)(128 * 3 + 256 + 8 + 8 * 128 + a.S + 4) * sizeof(float);
    hipLaunchKernelGGL(k_attn, dim3(a.NH, a.nrows), dim3(256), smem, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int qtts_qk_prep(const AttnArgs &a, hipStream_t st) {
    if ((a.NH + a.KV) * a.HD > 4096) {
        fprintf(stderr, "qtts_qk_prep: (NH+KV)*HD=%d exceeds 4096\n", (a.NH + a.KV) * a.HD);
        return -1;
    }
    hipLaunchKernelGGL(k_qk_prep, dim3(a.nrows), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
