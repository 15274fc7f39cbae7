// qtts_attn_dev.h - the sub-talker's short-context decode attention (<= 16
// keys, GQA 2) as a device function (k_attn_o, k_attn_short in k_attn.hip).
// (A one-wave-per-head variant without workgroup barriers measured slower,
// 6.95 vs 6.2 us per k_attn_o launch: the serial per-wave stream of 16 V
// loads and 8 K loads per lane costs more than the barriers it removes.)
#pragma once
#include "qtts_common.h"
#include "qtts_kernels.h"

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
// (stamp builds: phase stamps of the attention inside k_attn_o -- slots 1 / 5 /
// 6 of the gm_dbg record: q|k staged, scores, softmax)
__device__ __forceinline__ void as_stamp(const AttnArgs &a, int k) {
#ifdef QTTS_STAMPS
    if (a.dbg && threadIdx.x == 0)
        a.dbg[(blockIdx.x + (size_t)gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + k] = __builtin_amdgcn_s_memrealtime();
#endif
}
// `issue` runs right after the attention's own loads are issued (k_attn_o
// issues its O-weight fragment there: loads retire in issue order, so the
// attention's inputs must not queue behind the weights)
// rsrc: the q|k|v rows (a.qkv) or the table (a.qkv_tab); ids: a.tab_ids +
// a.tab_off, or nullptr (no table) -- passed separately so a kernel can take
// them as preloaded kernel arguments (k_attn_o)
template <int HD, bool SC1, class Issue = NoIssue>
__device__ __forceinline__ void attn_short_wg(const AttnArgs &a, int kvh, int r, float *lq, float *scs,
                                              float *lout, bool wcache, Issue issue, const float *rsrc,
                                              const int *ids) {
    constexpr int D4 = HD / 4, LPK = HD / 16, NK = 16;
    float (*sc)[NK] = reinterpret_cast<float (*)[NK]>(scs);
    const int tid = threadIdx.x;
    const int KVD = a.KV * HD;
    const int p = a.pos ? a.pos[r] : a.pos_const, n = p + 1;
    const float *row = rsrc + (size_t)r * a.ld_qkv;
    if (ids) {
        const int *ip = ids + (size_t)r * a.tab_bstride;
        if (a.tab_row_sel) ip += (size_t)a.tab_row_sel[r] * a.tab_rstride;
        row = rsrc + (size_t)(*ip) * a.ld_qkv;
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
    // the norm weights and RoPE rows of this lane right behind x: issued after
    // the K / V / W_o loads they would wait for all of them (in-order retire)
    float4 nwq = zero4, c4 = zero4, s4 = zero4;
    if (seg < 3) {
        nwq = reinterpret_cast<const float4 *>(seg < 2 ? a.qn_w : a.kn_w)[l];
        c4 = reinterpret_cast<const float4 *>(a.rope_cos + (size_t)p * HD)[l];
        s4 = reinterpret_cast<const float4 *>(a.rope_sin + (size_t)p * HD)[l];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the K / V / W_o loads behind these
    // K / V rows: unconditional loads from rows clamped below a.S (the slot's
    // cache capacity), whose values are read only for keys t < p below.
    // (Loads under a per-element condition compiled to one branch-wrapped
    // dword load each -- 16 + 16 of them -- and the wait for x counted them
    // all: the q|k|v row was staged 2.2 us into k_attn_o,
    // profiles/r06x_attn_o_phases.txt.)
    const int dI = tid / LPK, sub = tid - dI * LPK, gs = dI / NK, ts = dI - gs * NK;
    float4 kr[4];
    {
        const int tr = gs < 2 && ts < a.S ? ts : 0;
        const float4 *kp = reinterpret_cast<const float4 *>(Kc + (size_t)tr * KVD + 16 * sub);
#pragma unroll
        for (int c = 0; c < 4; ++c) kr[c] = kp[c];
    }
    const int go = tid / HD, dd = tid - go * HD;
    float vr[NK];
#pragma unroll
    for (int t = 0; t < NK; ++t) vr[t] = Vc[(size_t)(t < a.S ? t : a.S - 1) * KVD + dd];
    issue();

    // ---- per-head RMSNorm (T.c:646-649) + RoPE (T.c:650-653) -> LDS; k, v -> cache (T.c:654-655)
    float ss = x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    ss = group_sum<D4>(ss);
    if (seg < 3) {
        const float iv = rms_inv(ss, HD, a.eps);
        const float4 w = nwq;
        x.x = x.x * iv * w.x; x.y = x.y * iv * w.y; x.z = x.z * iv * w.z; x.w = x.w * iv * w.w;
    }
    float4 o4;
    if constexpr (D4 / 2 == 16) {   // the rotate-half partner one row away
        o4.x = xor16_get(x.x); o4.y = xor16_get(x.y); o4.z = xor16_get(x.z); o4.w = xor16_get(x.w);
    } else {
        o4.x = __shfl_xor(x.x, D4 / 2, 64); o4.y = __shfl_xor(x.y, D4 / 2, 64);
        o4.z = __shfl_xor(x.z, D4 / 2, 64); o4.w = __shfl_xor(x.w, D4 / 2, 64);
    }
    if (seg < 4) {
        float4 y = x;
        if (seg < 3) {
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
    as_stamp(a, 1);

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
        d = group_sum<LPK>(d);
        if (sub == 0 && gs < 2) sc[gs][ts] = ts < n ? d * div_rn(1.0f, sqrt_rn((float)HD)) : -INFINITY;
    }
    __syncthreads();
    as_stamp(a, 5);

    // ---- softmax per head over its <= 16 keys
    if (tid < 2 * NK) {
        const int g = tid / NK, t = tid - g * NK;
        const float s = sc[g][t];
        float m = s;
        m = group_max<NK>(m);
        const float e = t < n ? expf(s - m) : 0.f;
        float sum = e;
        sum = group_sum<NK>(sum);
        sc[g][t] = e * div_rn(1.0f, sum);
    }
    __syncthreads();
    as_stamp(a, 6);

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
