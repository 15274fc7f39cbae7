// qtts_attn_dev.h - single-workgroup decode attention for one kv head, as a
// device function: used as the tail of the fused QKV GEMV (k_gemv.hip: the
// last workgroup to finish a kv head's q/k/v rows runs it) so decode
// attention costs no kernel of its own.
//
// For kv head `kvh` of batch row `r` at position p = pos[r] (n = p + 1 keys):
//   per-head RMSNorm of q (GPH heads) and k (T.c:150-156), rotate-half RoPE
//   from the host table (T.c:158-189), k/v of the current token written to
//   the fp32 cache (T.c:191-196), then for each query head
//   softmax(q.K^T / sqrt(HD)) V over all n keys (T.c:198-230, K.c:371-378),
//   in chunks of CH keys merged online (running max / sum, fp32).
// Thread mapping per chunk: LPK lanes per key for the scores (DPL dims each,
// float4 loads, GPH dots per K row), one wave per head for the chunk
// softmax, HD/4 float4 lanes x KG key groups for P.V with an LDS reduction.
#pragma once
#include "qtts_common.h"
#include "qtts_kernels.h"

template <int HD, int GPH>
struct AttnWG {
    static constexpr int LPK = HD >= 32 ? HD / 32 : 1;   // lanes per key
    static constexpr int DPL = HD / LPK;                  // dims per lane
    static constexpr int CH = 256 / LPK;                  // keys per chunk
    static constexpr int D4 = HD / 4;
    static constexpr int KG = 256 / D4;                   // key groups in P.V
    static constexpr int NO = GPH * HD;                   // outputs
    static constexpr int NJ = (NO + 255) / 256;           // outputs per thread
    static constexpr int NV = (CH + KG - 1) / KG;         // V rows per thread per chunk
    // LDS pool layout (floats)
    static constexpr int XN = 0, QK = XN + (GPH + 1) * HD, VV = QK + (GPH + 1) * HD, SC = VV + HD,
                         ML = SC + GPH * CH, RED = ML + 8, POOL = RED + KG * NO;
};

// SC1: the q/k/v row was written by other workgroups of this launch with
// write-through stores; read it with sc1 loads (no acquire fence needed).
template <int HD, int GPH, bool SC1>
__device__ __forceinline__ void attn_full_wg(const AttnArgs &a, int kvh, int r, float *pool) {
    using W = AttnWG<HD, GPH>;
    constexpr int LPK = W::LPK, DPL = W::DPL, CH = W::CH, D4 = W::D4, KG = W::KG, NO = W::NO, NJ = W::NJ,
                  NV = W::NV;
    float *xn = pool + W::XN, *qk = pool + W::QK, *vv = pool + W::VV, *sc = pool + W::SC, *ml = pool + W::ML,
          *red = pool + W::RED;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int KVD = a.KV * HD;
    const int p = a.pos ? a.pos[r] : a.pos_const;
    const int n = p + 1;
    const float *row = a.qkv + (size_t)r * a.ld_qkv;
    const float *Kc = a.kc + (size_t)r * a.S * KVD + kvh * HD;
    const float *Vc = a.vc + (size_t)r * a.S * KVD + kvh * HD;

    // ---- prologue: q heads (waves 0..GPH-1), k head (wave GPH), v ----
    for (int hh = w; hh <= GPH; hh += 4) {
        const float *src = hh < GPH ? row + (kvh * GPH + hh) * HD : row + a.NH * HD + kvh * HD;
        const float *nw = hh < GPH ? a.qn_w : a.kn_w;
        float v[(HD + 63) / 64];
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < (HD + 63) / 64; ++j) {
            const int i = lane + 64 * j;
            v[j] = i < HD ? (SC1 ? ld_sc1(src + i) : src[i]) : 0.f;
            ss += v[j] * v[j];
        }
        ss = wave_sum(ss);
        const float iv = rms_inv(ss, HD, a.eps);
#pragma unroll
        for (int j = 0; j < (HD + 63) / 64; ++j) {
            const int i = lane + 64 * j;
            if (i < HD) xn[hh * HD + i] = v[j] * iv * nw[i];
        }
    }
    if (tid < HD) {
        const float *vp = row + (a.NH + a.KV) * HD + kvh * HD + tid;
        vv[tid] = SC1 ? ld_sc1(vp) : *vp;
    }
    __syncthreads();
    {
        const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
        constexpr int half = HD / 2;
        for (int i = tid; i < (GPH + 1) * HD; i += 256) {
            const int e = i % HD, hb = i - e;
            qk[i] = e < half ? xn[i] * cs[e] - xn[hb + e + half] * sn[e] : xn[i] * cs[e] + xn[hb + e - half] * sn[e];
        }
    }
    __syncthreads();
    if (tid < HD && !(a.skip && a.skip[r])) {
        a.kc[((size_t)r * a.S + p) * KVD + kvh * HD + tid] = qk[GPH * HD + tid];
        a.vc[((size_t)r * a.S + p) * KVD + kvh * HD + tid] = vv[tid];
    }

    const float scale = div_rn(1.0f, sqrt_rn((float)HD));
    const int kl = tid / LPK, ksub = tid - kl * LPK;
    const int d4 = tid % D4, kg = tid / D4;
    float M[GPH], L[GPH], acc[NJ];
#pragma unroll
    for (int g = 0; g < GPH; ++g) { M[g] = -INFINITY; L[g] = 0.f; }
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = 0.f;

    for (int t0 = 0; t0 < n; t0 += CH) {
        const int t1 = min(n, t0 + CH);
        // cache loads of the chunk first
        const int tk = t0 + kl;
        const bool kld = tk < t1 && tk != p;
        float4 kreg[DPL / 4];
        {
            const float4 *kp = reinterpret_cast<const float4 *>(Kc + (size_t)(kld ? tk : 0) * KVD + ksub * DPL);
#pragma unroll
            for (int j = 0; j < DPL / 4; ++j) kreg[j] = kld ? kp[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float4 vreg[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int t = t0 + kg + j * KG;
            const bool ok = kg + j * KG < CH && t < t1 && t != p;
            vreg[j] = ok ? reinterpret_cast<const float4 *>(Vc + (size_t)t * KVD)[d4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        // scores
        {
            float d[GPH];
#pragma unroll
            for (int g = 0; g < GPH; ++g) d[g] = 0.f;
            if (tk < t1) {
                float4 kv[DPL / 4];
#pragma unroll
                for (int j = 0; j < DPL / 4; ++j)
                    kv[j] = (tk == p) ? reinterpret_cast<const float4 *>(qk + GPH * HD + ksub * DPL)[j] : kreg[j];
#pragma unroll
                for (int g = 0; g < GPH; ++g) {
                    const float4 *q4 = reinterpret_cast<const float4 *>(qk + g * HD + ksub * DPL);
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < DPL / 4; ++j) {
                        const float4 q = q4[j];
                        s += q.x * kv[j].x + q.y * kv[j].y + q.z * kv[j].z + q.w * kv[j].w;
                    }
                    d[g] = s;
                }
            }
#pragma unroll
            for (int g = 0; g < GPH; ++g) {
#pragma unroll
                for (int o = LPK >> 1; o >= 1; o >>= 1) d[g] += __shfl_xor(d[g], o, 64);
                if (ksub == 0) sc[g * CH + kl] = tk < t1 ? d[g] * scale : -INFINITY;
            }
        }
        __syncthreads();
        for (int g = w; g < GPH; g += 4) {
            float m = -INFINITY;
            for (int k = lane; k < CH; k += 64) m = fmaxf(m, sc[g * CH + k]);
            m = wave_max(m);
            float l = 0.f;
            for (int k = lane; k < CH; k += 64) {
                const float e = t0 + k < t1 ? expf(sc[g * CH + k] - m) : 0.f;
                sc[g * CH + k] = e;
                l += e;
            }
            l = wave_sum(l);
            if (lane == 0) { ml[2 * g] = m; ml[2 * g + 1] = l; }
        }
        __syncthreads();
        {
            float4 pv[GPH];
#pragma unroll
            for (int g = 0; g < GPH; ++g) pv[g] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const int k = kg + j * KG;
                const int t = t0 + k;
                if (k < CH && t < t1) {
                    const float4 v4 = (t == p) ? reinterpret_cast<const float4 *>(vv)[d4] : vreg[j];
#pragma unroll
                    for (int g = 0; g < GPH; ++g) {
                        const float pw = sc[g * CH + k];
                        pv[g].x += pw * v4.x; pv[g].y += pw * v4.y; pv[g].z += pw * v4.z; pv[g].w += pw * v4.w;
                    }
                }
            }
#pragma unroll
            for (int g = 0; g < GPH; ++g) reinterpret_cast<float4 *>(red + kg * NO + g * HD)[d4] = pv[g];
        }
        __syncthreads();
        // online merge of the chunk into the running (M, L, acc) per head
        float an[GPH], ao[GPH];
#pragma unroll
        for (int g = 0; g < GPH; ++g) {
            const float mc = ml[2 * g], lc = ml[2 * g + 1];
            const float Mn = fmaxf(M[g], mc);
            ao[g] = expf(M[g] - Mn);
            an[g] = expf(mc - Mn);
            L[g] = L[g] * ao[g] + lc * an[g];
            M[g] = Mn;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int o = tid + 256 * j;
            if (o < NO) {
                float s = 0.f;
                for (int k = 0; k < KG; ++k) s += red[k * NO + o];
                const int g = o / HD;
                acc[j] = acc[j] * ao[g] + s * an[g];
            }
        }
        __syncthreads();   // sc / red / ml are rewritten by the next chunk
    }
    float *outr = a.out + (size_t)r * a.ld_out + kvh * GPH * HD;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int o = tid + 256 * j;
        if (o < NO) outr[o] = acc[j] / L[o / HD];
    }
}

// ---------------------------------------------------------------------------
// Short-context decode attention: n = pos + 1 <= 16 keys (the sub-talker,
// whose KV restarts every frame, T.c:562-569; ST_FORWARD T.c:646-671), one
// workgroup per (kv head, row) serving its GQA pair of query heads.  At this
// size the kernel is bound by its own instruction stream and memory round
// trips, so every load is issued up front and each thread does one piece:
//   threads < 4*HD/4  one float4 of q0 | q1 | k | v: per-head RMSNorm over
//                     HD/4-lane shuffles, rotate-half RoPE (partner HD/8
//                     lanes away) -> LDS; k / v of the token -> cache
//   all               scores: HD/16 lanes per (query head, key)
//   wave 0            softmax over the keys of each head (16-lane shuffles),
//                     x * (1/sum) as kernel_softmax (K.c:371-378)
//   threads < 2*HD    P.V: one output each, keys in order (st_axpy order)
// Device function: also the tail of the fused QKV GEMV (k_gemv.hip), where
// the q|k|v row was written by other workgroups of the same launch (SC1:
// read it with write-through loads).  lq: 4*HD floats, scs: 2*16 floats of LDS.
// lout != nullptr: the 2*HD outputs go to LDS lout (the caller barriers);
// wcache = false: the token's k / v are used but not stored (another
// workgroup of the launch stores them).
struct NoIssue { __device__ __forceinline__ void operator()() const {} };
// `issue` runs right after the attention's own loads are issued (k_attn_o
// issues its O-weight fragment there: loads retire in issue order, so the
// attention's inputs must not queue behind the weights)
template <int HD, bool SC1, class Issue = NoIssue>
__device__ __forceinline__ void attn_short_wg(const AttnArgs &a, int kvh, int r, float *lq, float *scs,
                                              float *lout = nullptr, bool wcache = true, Issue issue = Issue()) {
    constexpr int D4 = HD / 4, LPK = HD / 16, NK = 16;
    float (*sc)[NK] = reinterpret_cast<float (*)[NK]>(scs);
    const int tid = threadIdx.x;
    const int KVD = a.KV * HD;
    const int p = a.pos ? a.pos[r] : a.pos_const, n = p + 1;
    const float *row = a.qkv + (size_t)r * a.ld_qkv;
    if (a.qkv_tab) {
        const int *ip = a.tab_ids + (size_t)r * a.tab_bstride + a.tab_off;
        if (a.tab_row_sel) ip += (size_t)a.tab_row_sel[r] * a.tab_rstride;
        row = a.qkv_tab + (size_t)(*ip) * a.ld_qkv;
    }
    const float *Kc = a.kc + (size_t)r * a.S * KVD + kvh * HD;
    const float *Vc = a.vc + (size_t)r * a.S * KVD + kvh * HD;
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

    // ---- every load first: the token's q0|q1|k|v, K rows for the scores, V columns for P.V
    const int seg = tid / D4, l = tid - seg * D4;     // seg 0, 1: query heads, 2: k, 3: v
    float4 x = zero4;
    if (seg < 4) {
        const float *src = seg < 2 ? row + (2 * kvh + seg) * HD
                                   : row + (seg == 2 ? a.NH * HD : (a.NH + a.KV) * HD) + kvh * HD;
        if constexpr (SC1) x = make_float4(ld_sc1(src + 4 * l), ld_sc1(src + 4 * l + 1), ld_sc1(src + 4 * l + 2),
                                           ld_sc1(src + 4 * l + 3));
        else x = reinterpret_cast<const float4 *>(src)[l];
    }
    const int dI = tid / LPK, sub = tid - dI * LPK, gs = dI / NK, ts = dI - gs * NK;
    const bool kld = gs < 2 && ts < p;
    float4 kr[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        kr[c] = kld ? reinterpret_cast<const float4 *>(Kc + (size_t)ts * KVD + 16 * sub)[c] : zero4;
    const int go = tid / HD, dd = tid - go * HD;
    float vr[NK];
#pragma unroll
    for (int t = 0; t < NK; ++t) vr[t] = (go < 2 && t < p) ? Vc[(size_t)t * KVD + dd] : 0.f;
    issue();

    // ---- per-head RMSNorm (T.c:646-649) + RoPE (T.c:650-653) -> LDS; k, v -> cache (T.c:654-655)
    float ss = x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
#pragma unroll
    for (int o = D4 / 2; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if (seg < 3) {
        const float iv = rms_inv(ss, HD, a.eps);
        const float4 w = reinterpret_cast<const float4 *>(seg < 2 ? a.qn_w : a.kn_w)[l];
        x.x = x.x * iv * w.x; x.y = x.y * iv * w.y; x.z = x.z * iv * w.z; x.w = x.w * iv * w.w;
    }
    float4 o4;
    o4.x = __shfl_xor(x.x, D4 / 2, 64); o4.y = __shfl_xor(x.y, D4 / 2, 64);
    o4.z = __shfl_xor(x.z, D4 / 2, 64); o4.w = __shfl_xor(x.w, D4 / 2, 64);
    if (seg < 4) {
        float4 y = x;
        if (seg < 3) {
            const float4 c4 = reinterpret_cast<const float4 *>(a.rope_cos + (size_t)p * HD)[l];
            const float4 s4 = reinterpret_cast<const float4 *>(a.rope_sin + (size_t)p * HD)[l];
            if (l < D4 / 2) {   // x[i] c[i] - x[i+half] s[i]
                y.x = x.x * c4.x - o4.x * s4.x; y.y = x.y * c4.y - o4.y * s4.y;
                y.z = x.z * c4.z - o4.z * s4.z; y.w = x.w * c4.w - o4.w * s4.w;
            } else {            // x[i+half] c[i] + x[i] s[i]
                y.x = x.x * c4.x + o4.x * s4.x; y.y = x.y * c4.y + o4.y * s4.y;
                y.z = x.z * c4.z + o4.z * s4.z; y.w = x.w * c4.w + o4.w * s4.w;
            }
        }
        reinterpret_cast<float4 *>(lq)[tid] = y;
        if (seg >= 2 && wcache && !(a.skip && a.skip[r])) {
            float *dst = (seg == 2 ? a.kc : a.vc) + ((size_t)r * a.S + p) * KVD + kvh * HD;
            reinterpret_cast<float4 *>(dst)[l] = y;
        }
    }
    __syncthreads();

    // ---- scores q.k_t / sqrt(HD) (T.c:662-665)
    {
        float d = 0.f;
        if (gs < 2 && ts < n) {
            const float4 *q4 = reinterpret_cast<const float4 *>(lq + gs * HD + 16 * sub);
            const float4 *k4 = reinterpret_cast<const float4 *>(lq + 2 * HD + 16 * sub);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 k = ts == p ? k4[c] : kr[c], q = q4[c];
                d += q.x * k.x + q.y * k.y + q.z * k.z + q.w * k.w;
            }
        }
#pragma unroll
        for (int o = LPK / 2; o >= 1; o >>= 1) d += __shfl_xor(d, o, 64);
        if (sub == 0 && gs < 2) sc[gs][ts] = ts < n ? d * div_rn(1.0f, sqrt_rn((float)HD)) : -INFINITY;
    }
    __syncthreads();

    // ---- softmax per head over its <= 16 keys
    if (tid < 2 * NK) {
        const int g = tid / NK, t = tid - g * NK;
        const float s = sc[g][t];
        float m = s;
#pragma unroll
        for (int o = NK / 2; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        const float e = t < n ? expf(s - m) : 0.f;
        float sum = e;
#pragma unroll
        for (int o = NK / 2; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
        sc[g][t] = e * div_rn(1.0f, sum);
    }
    __syncthreads();

    // ---- P.V, keys in order (T.c:667-671)
    if (go < 2) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NK; ++t)
            if (t < n) acc += sc[go][t] * (t == p ? lq[3 * HD + dd] : vr[t]);
        if (lout) lout[go * HD + dd] = acc;
        else a.out[(size_t)r * a.ld_out + (2 * kvh + go) * HD + dd] = acc;
    }
}
