// qtts_attn_pro.h - short-context decode attention as a GEMV PROLOGUE.
//
// The sub-talker attends over at most G = 16 keys (its KV is reset every
// frame, positions 0..15: T.c:562-569).  At that size the attention of one
// token over all NH query heads is a few hundred FMAs per thread and n*8 KB
// of cache reads -- far less than a kernel boundary plus a dependent
// launch.  So the O-projection GEMV (k_gemv1_att, k_gemv.hip) computes it in
// every workgroup, straight into the LDS row its weight stream consumes, and
// the attention kernel disappears from the frame graph.
//
// Per workgroup, for the batch-1 token at p = pos (n = p + 1 <= ATT_NMAX keys),
// following ST_FORWARD (T.c:638-672):
//   1. the raw q|k|v row and every cached K / V row t < p are loaded into
//      registers at once (one memory round trip; the caller has already
//      issued its first weight loads);
//   2. per-head RMSNorm of q and k (T.c:646-649, K.c:27-39) over HD/4 float4
//      lanes, rotate-half RoPE from the host table (T.c:650-653,
//      K.c:564-587), the partner half one xor-shuffle away; workgroup 0
//      writes the rotated k and the raw v into the fp32 cache at p
//      (T.c:654-655);
//   3. scores q.k_t * (1/sqrt(HD)) for t <= p (T.c:662-665): LPK = HD/16
//      lanes per (kv head, key), both query heads of the group per K row;
//   4. softmax as kernel_softmax (K.c:371-378): max, expf, sum, x * (1/sum);
//   5. out_h = sum_t p_t v_t in key order (T.c:667-671) -> xs[h*HD + d].
// GQA with NH = 2*KV (both model sizes); anything else takes the separate
// attention kernel (att_pro_ok() is false and the host launches k_attn_dec).
#pragma once
#include "qtts_common.h"
#include "qtts_kernels.h"

constexpr int ATT_NMAX = 16;   // keys held in registers (>= num_code_groups)
constexpr int ATT_KPASS = 4;   // score passes held in registers

// LDS floats the prologue needs besides the GEMV's xs[C] and red[32]
__host__ __device__ constexpr int att_pro_lds_floats(int NH, int KV, int HD) {
    return (NH + 2 * KV) * HD + NH * ATT_NMAX;
}

// Can the prologue serve this attention?  (the host checks before launching)
__host__ __device__ inline bool att_pro_ok(const AttnArgs &t, int C) {
    const int HD = t.HD;
    return t.mode == 0 && t.win == 0 && t.nrows == 1 && (HD == 16 || HD == 32 || HD == 64 || HD == 128) &&
           t.KV > 0 && t.NH == 2 * t.KV && C == t.NH * HD && (t.NH + 2 * t.KV) * HD <= 4096 &&
           t.KV * HD <= 1024 && t.S <= ATT_NMAX && t.KV * t.S * (HD / 16) <= 256 * ATT_KPASS;
}

// xs[NH*HD] <- attention output of the token; lq / sc: LDS scratch of
// att_pro_lds_floats().  All 256 threads; ends with a barrier (xs ready).
template <int HD>
__device__ __forceinline__ void att_prologue(const AttnArgs &t, float *xs, float *lq, float *sc, bool write_cache) {
    constexpr int D4 = HD / 4;       // float4 per head
    constexpr int LPK = HD / 16;     // lanes per (kv head, key) in the scores, 16 dims each
    constexpr int TPP = 256 / LPK;   // score tasks per pass
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int NH = t.NH, KV = t.KV, KVD = KV * HD;
    const int p = t.pos ? t.pos[0] : t.pos_const;
    const int n = p + 1;
    const int NQ4 = NH * D4, NQK4 = (NH + KV) * D4, QR4 = (NH + 2 * KV) * D4;
    const float4 *row4 = reinterpret_cast<const float4 *>(t.qkv);
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

    // ---- 1. every load up front: the q|k|v row, K rows for the scores, V rows for P.V
    float4 rv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int f = tid + 256 * j;
        rv[j] = f < QR4 ? row4[f] : zero4;
    }
    const int sub = tid % LPK;
    float4 kr[ATT_KPASS][4];
#pragma unroll
    for (int i = 0; i < ATT_KPASS; ++i) {
        const int task = tid / LPK + i * TPP;
        const int kvh = task / n, tk = task - kvh * n;
        const bool ld = kvh < KV && tk < p;
        const float4 *kp = reinterpret_cast<const float4 *>(t.kc + (size_t)(ld ? tk : 0) * KVD + (ld ? kvh : 0) * HD +
                                                            16 * sub);
#pragma unroll
        for (int c = 0; c < 4; ++c) kr[i][c] = ld ? kp[c] : zero4;
    }
    const int pv_kvh = tid / D4, pv_d4 = tid - pv_kvh * D4;
    const bool pv_on = pv_kvh < KV;
    float4 vr[ATT_NMAX];
#pragma unroll
    for (int tt = 0; tt < ATT_NMAX; ++tt)
        vr[tt] = (pv_on && tt < p) ? reinterpret_cast<const float4 *>(t.vc + (size_t)tt * KVD + pv_kvh * HD)[pv_d4]
                                   : zero4;

    // ---- 2. per-head RMSNorm + RoPE of q and k, v raw -> lq; k / v of p -> cache
    const float *cs = t.rope_cos + (size_t)p * HD, *sn = t.rope_sin + (size_t)p * HD;
    const bool wr = write_cache && !(t.skip && t.skip[0]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int f = tid + 256 * j;
        const int l = f % D4;        // float4 index inside the head
        float4 v = rv[j];
        float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
#pragma unroll
        for (int o = D4 / 2; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
        const bool qk = f < NQK4;
        if (qk) {
            const float iv = rms_inv(ss, HD, t.eps);
            const float4 nw = reinterpret_cast<const float4 *>(f < NQ4 ? t.qn_w : t.kn_w)[l];
            v.x = v.x * iv * nw.x; v.y = v.y * iv * nw.y; v.z = v.z * iv * nw.z; v.w = v.w * iv * nw.w;
        }
        // rotate-half: the partner float4 (dims +-HD/2) sits D4/2 lanes away
        float4 o4;
        o4.x = __shfl_xor(v.x, D4 / 2, 64); o4.y = __shfl_xor(v.y, D4 / 2, 64);
        o4.z = __shfl_xor(v.z, D4 / 2, 64); o4.w = __shfl_xor(v.w, D4 / 2, 64);
        if (f < QR4) {
            float4 y = v;
            if (qk) {
                const float4 c4 = *reinterpret_cast<const float4 *>(cs + 4 * l);
                const float4 s4 = *reinterpret_cast<const float4 *>(sn + 4 * l);
                if (l < D4 / 2) {   // x[i] c[i] - x[i+half] s[i]
                    y.x = v.x * c4.x - o4.x * s4.x; y.y = v.y * c4.y - o4.y * s4.y;
                    y.z = v.z * c4.z - o4.z * s4.z; y.w = v.w * c4.w - o4.w * s4.w;
                } else {            // x[i+half] c[i] + x[i] s[i]
                    y.x = v.x * c4.x + o4.x * s4.x; y.y = v.y * c4.y + o4.y * s4.y;
                    y.z = v.z * c4.z + o4.z * s4.z; y.w = v.w * c4.w + o4.w * s4.w;
                }
            }
            reinterpret_cast<float4 *>(lq)[f] = y;
            if (wr && f >= NQ4) {
                float *dst = f < NQK4 ? t.kc + (size_t)p * KVD + 4 * (f - NQ4) : t.vc + (size_t)p * KVD + 4 * (f - NQK4);
                *reinterpret_cast<float4 *>(dst) = y;
            }
        }
    }
    __syncthreads();

    // ---- 3. scores, both query heads of a kv head per K row
    const float scale = div_rn(1.0f, sqrt_rn((float)HD));
#pragma unroll
    for (int i = 0; i < ATT_KPASS; ++i) {
        const int task = tid / LPK + i * TPP;
        const int kvh = task / n, tk = task - kvh * n;
        const bool on = kvh < KV;
        float d0 = 0.f, d1 = 0.f;
        if (on) {
            const float4 *kl = reinterpret_cast<const float4 *>(lq + NH * HD + kvh * HD + 16 * sub);
            const float4 *q0 = reinterpret_cast<const float4 *>(lq + (2 * kvh) * HD + 16 * sub);
            const float4 *q1 = reinterpret_cast<const float4 *>(lq + (2 * kvh + 1) * HD + 16 * sub);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 k4 = tk == p ? kl[c] : kr[i][c];
                const float4 a4 = q0[c], b4 = q1[c];
                d0 += a4.x * k4.x + a4.y * k4.y + a4.z * k4.z + a4.w * k4.w;
                d1 += b4.x * k4.x + b4.y * k4.y + b4.z * k4.z + b4.w * k4.w;
            }
        }
#pragma unroll
        for (int o = LPK / 2; o >= 1; o >>= 1) {
            d0 += __shfl_xor(d0, o, 64);
            d1 += __shfl_xor(d1, o, 64);
        }
        if (on && sub == 0) {
            sc[(2 * kvh) * ATT_NMAX + tk] = d0 * scale;
            sc[(2 * kvh + 1) * ATT_NMAX + tk] = d1 * scale;
        }
    }
    __syncthreads();

    // ---- 4. softmax per head (K.c:371-378): one wave per head, one lane per key
    for (int h = w; h < NH; h += 4) {
        const float s = lane < n ? sc[h * ATT_NMAX + lane] : -INFINITY;
        const float m = wave_max(s);
        const float e = lane < n ? expf(s - m) : 0.f;
        const float inv = div_rn(1.0f, wave_sum(e));
        if (lane < n) sc[h * ATT_NMAX + lane] = e * inv;
    }
    __syncthreads();

    // ---- 5. P.V in key order -> xs
    if (pv_on) {
        float4 a0 = zero4, a1 = zero4;
        const float *p0 = sc + (2 * pv_kvh) * ATT_NMAX, *p1 = p0 + ATT_NMAX;
        const float4 vcur = reinterpret_cast<const float4 *>(lq + (NH + KV) * HD + pv_kvh * HD)[pv_d4];
#pragma unroll
        for (int tt = 0; tt < ATT_NMAX; ++tt) {
            if (tt < n) {
                const float4 v4 = tt == p ? vcur : vr[tt];
                const float w0 = p0[tt], w1 = p1[tt];
                a0.x += w0 * v4.x; a0.y += w0 * v4.y; a0.z += w0 * v4.z; a0.w += w0 * v4.w;
                a1.x += w1 * v4.x; a1.y += w1 * v4.y; a1.z += w1 * v4.z; a1.w += w1 * v4.w;
            }
        }
        reinterpret_cast<float4 *>(xs + (2 * pv_kvh) * HD)[pv_d4] = a0;
        reinterpret_cast<float4 *>(xs + (2 * pv_kvh + 1) * HD)[pv_d4] = a1;
    }
    __syncthreads();
}
