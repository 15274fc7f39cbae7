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
#include "qtts_attn_dev.h"
#include "qtts_common.h"
#include "qtts_kernels.h"
#include "qtts_l2pf.h"

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

// prefill, one wave per (row, head): q / k heads normalised + rotated (q in
// place, k -> cache), v heads -> cache; no LDS, no barrier.  grid (rows,
// ceil((NH + 2 KV) / 4)), 256 threads.  HD = 128: a lane holds e and e + 64
// (its own rotate-half partner); HD <= 64: one element, partner one xor away.
__global__ __launch_bounds__(256) void k_qk_prep_w(AttnArgs a) {
    const int r = blockIdx.x, w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int HD = a.HD, NH = a.NH, KV = a.KV, KVD = KV * HD;
    const int hh = blockIdx.y * 4 + w;
    if (hh >= NH + 2 * KV) return;
    const int b = a.row_b[r], p = a.pos[r];
    float *row = const_cast<float *>(a.qkv) + (size_t)r * a.ld_qkv;
    float *kdst = a.kc + ((size_t)b * a.S + p) * KVD, *vdst = a.vc + ((size_t)b * a.S + p) * KVD;
    if (hh >= NH + KV) {   // v head: copy to the cache
        const int vh = hh - NH - KV;
        for (int i = l; i < HD; i += 64) vdst[vh * HD + i] = row[(NH + KV) * HD + vh * HD + i];
        return;
    }
    const float *src = row + hh * HD;
    const float *nw = hh < NH ? a.qn_w : a.kn_w;
    const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
    const int half = HD >> 1;
    float y0, y1 = 0.f;
    if (HD == 128) {
        const float x0 = src[l], x1 = src[l + 64];
        const float iv = rms_inv(wave_sum(x0 * x0 + x1 * x1), HD, a.eps);
        const float n0 = x0 * iv * nw[l], n1 = x1 * iv * nw[l + 64];
        y0 = n0 * cs[l] - n1 * sn[l];
        y1 = n1 * cs[l + 64] + n0 * sn[l + 64];
    } else {
        const float x0 = l < HD ? src[l] : 0.f;
        const float iv = rms_inv(wave_sum(x0 * x0), HD, a.eps);
        const float n0 = l < HD ? x0 * iv * nw[l] : 0.f;
        const float pn = __shfl_xor(n0, half, 64);
        y0 = l < HD ? (l < half ? n0 * cs[l] - pn * sn[l] : n0 * cs[l] + pn * sn[l]) : 0.f;
    }
    float *dst = hh < NH ? row + hh * HD : kdst + (hh - NH) * HD;
    if (HD == 128) { dst[l] = y0; dst[l + 64] = y1; }
    else if (l < HD) dst[l] = y0;
}

// ---------------------------------------------------------------------------
// Decode attention, split over keys (flash-decoding) for one kv head per
// workgroup: grid (KV, nsplit, rows).  A workgroup serves all GPH query heads
// of its kv head (each K/V row is read once for them), keys
// [split*CH, min(n, split*CH + CH)).  Per workgroup:
//   prologue  one wave per head: per-head RMSNorm (T.c:150-156) -> LDS, then
//             rotate-half RoPE from the host table (T.c:158-189); the split
//             that holds the current token writes its k, v to the cache
//             (T.c:191-196) and reads them from LDS.
//   scores    LPK lanes per key (DPL dims each, float4 loads), GPH dots per
//             key, lane-pair shuffles; one pass (CH = 256 / LPK keys).
//   softmax   one wave per head: chunk max, exp, sum (K.c:371-378).
//   P.V       HD/4 lanes x KG key groups, float4 V rows, LDS reduction.
// With one active split the normalised result is written directly; otherwise
// each split leaves (acc, max, sum) in scratch, and the last split to finish
// (agent-scope acq_rel ticket) merges them in split order and resets the
// ticket.  Grid size is fixed at graph capture (nsplit from the cache
// capacity); splits past the live length exit at once.
// (qkv / pos / kc / vc lead the arguments: preloaded into SGPRs, Makefile --
// the position load and the cache loads behind it need no kernarg round trip)
template <int HD, int GPH, int LPK>
__global__ __launch_bounds__(256) void k_attn_dec(const float *qkv_, const int *pos_, float *kc_, float *vc_,
                                                  AttnArgs a) {
    // LPK lanes per key
    constexpr int DPL = HD / LPK;                  // dims per lane
    constexpr int CH = 256 / LPK;                  // keys per workgroup
    constexpr int D4 = HD / 4;
    constexpr int KG = 256 / D4;                   // key groups in P.V
    constexpr int NO = GPH * HD;                   // outputs per workgroup
    __shared__ __attribute__((aligned(16))) float xn[(GPH + 1) * HD];
    __shared__ __attribute__((aligned(16))) float qk[(GPH + 1) * HD];   // rotated q heads, then k
    __shared__ __attribute__((aligned(16))) float vv[HD];
    __shared__ float sc[GPH][CH];
    __shared__ float ml[GPH][2];
    __shared__ __attribute__((aligned(16))) float red[KG * NO];
    __shared__ int last;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kvh = blockIdx.x, split = blockIdx.y, r = blockIdx.z;
    const int KVD = a.KV * HD;
    const int p = pos_ ? pos_[r] : a.pos_const;
    const int n = p + 1;
    const int nact = (n + CH - 1) / CH;
    if (split >= nact) return;
    const int t0 = split * CH;
    const int t1 = min(n, t0 + CH);
    const bool owner = (split == nact - 1);        // holds the current token
    const float *row = qkv_ + (size_t)r * a.ld_qkv;
    const float *Kc = kc_ + (size_t)r * a.S * KVD + kvh * HD;
    const float *Vc = vc_ + (size_t)r * a.S * KVD + kvh * HD;

    // ---- the token's own inputs first (q / k head values, norm weights, RoPE
    // rows, v): issued behind the cache loads they would wait for all of them
    // (loads retire in issue order) ----
    constexpr int HJ = (HD + 63) / 64;
    static_assert(GPH + 1 <= 4, "one wave per q / k head");
    // (every load of the kernel is unconditional, from a clamped valid
    // address: a load under a divergent branch makes the compiler's vmcnt
    // bookkeeping drain everything outstanding at the join)
    const int hh0 = w < GPH ? w : GPH;   // GPH + 1 <= 4 heads: one per wave (wave 3 repeats the k head)
    float hv[HJ], hw[HJ];
    {
        const float *src = hh0 < GPH ? row + (kvh * GPH + hh0) * HD : row + a.NH * HD + kvh * HD;
        const float *nw = hh0 < GPH ? a.qn_w : a.kn_w;
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
            const int i = (lane + 64 * j) % HD;
            hv[j] = src[i];
            hw[j] = nw[i];
        }
    }
    // RoPE rows: HD 128 -- a lane holds elements lane and lane + 64, its own
    // rotate-half partner, so its wave rotates in registers; else by thread
    constexpr bool RREG = HD == 128;
    constexpr int RJ = RREG ? 2 : ((GPH + 1) * HD + 255) / 256;
    float rc[RJ], rs[RJ];
    {
        const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const int e = RREG ? lane + 64 * j : (tid + 256 * j) % HD;
            rc[j] = cs[e];
            rs[j] = sn[e];
        }
    }
    const float vtok = row[(a.NH + a.KV) * HD + kvh * HD + tid % HD];
    __builtin_amdgcn_sched_barrier(0);   // keep the cache loads behind these

    // ---- then every cache load of this split: K rows for the scores, V rows
    // for P.V (the current token's come from LDS later) ----
    const int kl = tid / LPK, ksub = tid - kl * LPK;
    const int tk = t0 + kl;
    // (rows past the split or the current token's own read a valid row and
    // are never used: the scores skip t >= t1 and take t == p from LDS)
    float4 kreg[DPL / 4];
    {
        const float4 *kp = reinterpret_cast<const float4 *>(Kc + (size_t)(tk < t1 ? tk : t0) * KVD + ksub * DPL);
#pragma unroll
        for (int j = 0; j < DPL / 4; ++j) kreg[j] = kp[j];
    }
    const int d4 = tid % D4, kg = tid / D4;
    constexpr int NV = (CH + KG - 1) / KG;
    float4 vreg[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int t = t0 + kg + j * KG;
        const bool ok = kg + j * KG < CH && t < t1;   // (t == p: read, then replaced from LDS)
        vreg[j] = reinterpret_cast<const float4 *>(Vc + (size_t)(ok ? t : t0) * KVD)[d4];
    }

    // ---- prologue: q heads (waves 0..GPH-1), k head (wave GPH), v ----
    if (w <= GPH) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < HJ; ++j) ss += lane + 64 * j < HD ? hv[j] * hv[j] : 0.f;   // (HD < 64: lanes past HD repeat)
        ss = wave_sum(ss);
        const float iv = rms_inv(ss, HD, a.eps);
        if constexpr (RREG) {   // normalise and rotate in registers (T.c:150-189)
            const float n0 = hv[0] * iv * hw[0], n1 = hv[1] * iv * hw[1];
            qk[hh0 * HD + lane] = n0 * rc[0] - n1 * rs[0];
            qk[hh0 * HD + lane + 64] = n1 * rc[1] + n0 * rs[1];
        } else {
#pragma unroll
            for (int j = 0; j < HJ; ++j) {
                const int i = lane + 64 * j;
                if (i < HD) xn[hh0 * HD + i] = hv[j] * iv * hw[j];
            }
        }
    }
    if (owner && tid < HD) vv[tid] = vtok;
    __syncthreads();
    if constexpr (!RREG) {
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const int i = tid + 256 * j;
            if (i < (GPH + 1) * HD) {
                const int e = i % HD, hb = i - e;
                constexpr int half = HD / 2;
                qk[i] = e < half ? xn[i] * rc[j] - xn[hb + e + half] * rs[j] : xn[i] * rc[j] + xn[hb + e - half] * rs[j];
            }
        }
        __syncthreads();
    }
    if (owner && tid < HD && !(a.skip && a.skip[r])) {
        kc_[((size_t)r * a.S + p) * KVD + kvh * HD + tid] = qk[GPH * HD + tid];
        vc_[((size_t)r * a.S + p) * KVD + kvh * HD + tid] = vv[tid];
    }

    // ---- scores ----
    const float scale = div_rn(1.0f, sqrt_rn((float)HD));
    {
        const int sub = ksub;
        const int t = tk;
        float d[GPH];
#pragma unroll
        for (int g = 0; g < GPH; ++g) d[g] = 0.f;
        if (t < t1) {
            float4 kv[DPL / 4];
#pragma unroll
            for (int j = 0; j < DPL / 4; ++j)
                kv[j] = (t == p) ? reinterpret_cast<const float4 *>(qk + GPH * HD + sub * DPL)[j] : kreg[j];
#pragma unroll
            for (int g = 0; g < GPH; ++g) {
                const float4 *q4 = reinterpret_cast<const float4 *>(qk + g * HD + sub * DPL);
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
            d[g] = group_sum<LPK>(d[g]);
            if (sub == 0) sc[g][kl] = t < t1 ? d[g] * scale : -INFINITY;
        }
    }
    __syncthreads();
    // ---- chunk softmax (unnormalised) ----
    for (int g = w; g < GPH; g += 4) {
        float m = -INFINITY;
        for (int k = lane; k < CH; k += 64) m = fmaxf(m, sc[g][k]);
        m = wave_max(m);
        float l = 0.f;
        for (int k = lane; k < CH; k += 64) {
            const float e = t0 + k < t1 ? expf(sc[g][k] - m) : 0.f;
            sc[g][k] = e;
            l += e;
        }
        l = wave_sum(l);
        if (lane == 0) { ml[g][0] = m; ml[g][1] = l; }
    }
    __syncthreads();
    // ---- P.V ----
    {
        float4 acc[GPH];
#pragma unroll
        for (int g = 0; g < GPH; ++g) acc[g] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int k = kg + j * KG;
            const int t = t0 + k;
            if (k < CH && t < t1) {
                const float4 v4 = (t == p) ? reinterpret_cast<const float4 *>(vv)[d4] : vreg[j];
#pragma unroll
                for (int g = 0; g < GPH; ++g) {
                    const float pw = sc[g][k];
                    acc[g].x += pw * v4.x; acc[g].y += pw * v4.y; acc[g].z += pw * v4.z; acc[g].w += pw * v4.w;
                }
            }
        }
#pragma unroll
        for (int g = 0; g < GPH; ++g) reinterpret_cast<float4 *>(red + kg * NO + g * HD)[d4] = acc[g];
    }
    __syncthreads();
    float res[(NO + 255) / 256];
#pragma unroll
    for (int j = 0; j < (NO + 255) / 256; ++j) {
        const int o = tid + 256 * j;
        float s = 0.f;
        if (o < NO)
            for (int k = 0; k < KG; ++k) s += red[k * NO + o];
        res[j] = s;
    }
    float *outr = a.out + (size_t)r * a.ld_out + kvh * GPH * HD;
    const int stride = NO + 2 * GPH;
    float *base = a.part + (size_t)(r * a.KV + kvh) * a.nsplit * stride;
    if (a.defer) {   // every split leaves (acc, max, sum); the O projection merges (GemvArgs::amerge)
        float *mine = base + (size_t)split * stride;
#pragma unroll
        for (int j = 0; j < (NO + 255) / 256; ++j) {
            const int o = tid + 256 * j;
            if (o < NO) mine[o] = res[j];
        }
        if (tid < GPH) { mine[NO + 2 * tid] = ml[tid][0]; mine[NO + 2 * tid + 1] = ml[tid][1]; }
        return;
    }
    if (nact == 1) {
#pragma unroll
        for (int j = 0; j < (NO + 255) / 256; ++j) {
            const int o = tid + 256 * j;
            if (o < NO) outr[o] = res[j] / ml[o / HD][1];
        }
        return;
    }
    // ---- multi-split: publish partials, the last split merges.  Hand-off form
    // R1 of cdna_hip_programming.md Guideline 16 (no fences: a __threadfence()
    // costs ~3.5 us per workgroup): write-through (sc1) stores, every wave
    // drains them, one relaxed ticket add per workgroup, the last arriver
    // reads the partials with sc1 loads ----
    float *mine = base + (size_t)split * stride;
#pragma unroll
    for (int j = 0; j < (NO + 255) / 256; ++j) {
        const int o = tid + 256 * j;
        if (o < NO) st_sc1(mine + o, res[j]);
    }
    if (tid < GPH) { st_sc1(mine + NO + 2 * tid, ml[tid][0]); st_sc1(mine + NO + 2 * tid + 1, ml[tid][1]); }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(a.cnt + r * a.KV + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (old == nact - 1);
    }
    __syncthreads();
    if (!last) return;
    if (nact <= 8) {   // every partial of this thread's outputs in flight at once, then the merge in split order
#pragma unroll
        for (int j = 0; j < (NO + 255) / 256; ++j) {
            const int o = tid + 256 * j;
            const int oc = o < NO ? o : 0, g = oc / HD;
            float mm[8], ll[8], aa[8];
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2) {
                const float *ps = base + (size_t)(s2 < nact ? s2 : 0) * stride;
                mm[s2] = ld_sc1(ps + NO + 2 * g);
                ll[s2] = ld_sc1(ps + NO + 2 * g + 1);
                aa[s2] = ld_sc1(ps + oc);
            }
            float M = -INFINITY;
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2)
                if (s2 < nact) M = fmaxf(M, mm[s2]);
            float num = 0.f, den = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2) {
                if (s2 < nact) {
                    const float f = expf(mm[s2] - M);
                    num = fmaf(f, aa[s2], num);
                    den = fmaf(f, ll[s2], den);
                }
            }
            if (o < NO) outr[o] = num / den;
        }
        if (tid == 0) __hip_atomic_store(a.cnt + r * a.KV + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
#pragma unroll
    for (int j = 0; j < (NO + 255) / 256; ++j) {
        const int o = tid + 256 * j;
        if (o < NO) {
            const int g = o / HD;
            float M = -INFINITY;
            for (int s2 = 0; s2 < nact; ++s2) M = fmaxf(M, ld_sc1(base + (size_t)s2 * stride + NO + 2 * g));
            float num = 0.f, den = 0.f;
            for (int s2 = 0; s2 < nact; ++s2) {
                const float *ps = base + (size_t)s2 * stride;
                const float f = expf(ld_sc1(ps + NO + 2 * g) - M);
                num = fmaf(f, ld_sc1(ps + o), num);
                den = fmaf(f, ld_sc1(ps + NO + 2 * g + 1), den);
            }
            outr[o] = num / den;
        }
    }
    if (tid == 0) __hip_atomic_store(a.cnt + r * a.KV + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int HD>
__global__ __launch_bounds__(256) void k_attn_short(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float lq[4 * HD];   // rotated q0 | q1 | k, raw v
    __shared__ float sc[2 * 16];
    attn_short_wg<HD, false>(a, blockIdx.x, blockIdx.y, lq, sc, nullptr, true, NoIssue(),
                             a.qkv_tab ? a.qkv_tab : a.qkv, a.qkv_tab ? a.tab_ids + a.tab_off : nullptr);
    if (a.xc_dst && blockIdx.x == 0) {   // the input row as the residual (AttnArgs::xc_dst)
        const int r = blockIdx.y;
        const int *ip = a.tab_ids + a.tab_off + (size_t)r * a.tab_bstride;
        if (a.tab_row_sel) ip += (size_t)a.tab_row_sel[r] * a.tab_rstride;
        const size_t row = (size_t)(*ip) * a.xc_n;
        float *dst = a.xc_dst + (size_t)r * a.xc_n;
        for (int c = 4 * (int)threadIdx.x; c < a.xc_n; c += 4 * (int)blockDim.x) {
            float4 v;
            if (a.xc_tab) {
                v = *reinterpret_cast<const float4 *>(a.xc_tab + row + c);
            } else {
                const uint2 u = *reinterpret_cast<const uint2 *>(a.xc_tab16 + row + c);
                v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u),
                                __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xFFFF0000u));
            }
            *reinterpret_cast<float4 *>(dst + c) = v;
        }
    }
}

// Short-context attention + the O projection split by kv head (the
// sub-talker, GQA 2): workgroup (rb, kvh) recomputes kvh's attention (<= 16
// keys, attn_short_wg; only rb == 0 stores the token's k / v) and multiplies
// it with the 2*HD columns of W_o that head pair feeds, for RPW rows:
// part[kvh][row] = W_o[row, 2 HD kvh .. 2 HD (kvh + 1)) . attn_kvh.
// The consumer (the next GEMV's prologue, GemvArgs::xadd) sums the KV
// partials in head order and adds the residual: x + o_proj(attn) of
// T.c:667-676 with o_proj's dot split by head.
// Lanes: LPS per row slot, 8 columns (16 B of bf16) per lane per load.
// (rsrc / ids lead the arguments: the Makefile preloads them into SGPRs)
template <int HD>
__global__ __launch_bounds__(256) void k_attn_o(const float *rsrc, const int *ids, AttnArgs t, const bf16_t *Wo,
                                                int R, float *part) {
    constexpr int W2 = 2 * HD, LPS = W2 / 8 < 8 ? W2 / 8 : 8, NJ = W2 / (8 * LPS), RPW = 256 / LPS;
    __shared__ __attribute__((aligned(16))) float lq[4 * HD];
    __shared__ __attribute__((aligned(16))) float att[W2];
    __shared__ float sc[2 * 16];
    const int tid = threadIdx.x, kvh = blockIdx.y, rb = blockIdx.x, b = blockIdx.z;   // b: batch row
#ifdef QTTS_STAMPS
    // (stamp builds: the in-graph span of this launch, phases 0 start / 2 dot
    // done / 3 end per workgroup, read by qtts_dev_get_codes' gm_dbg print)
    const size_t wgl = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (t.dbg && tid == 0) t.dbg[wgl * 8 + 0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int slot = tid / LPS, sub = tid - slot * LPS;
    const int row = rb * RPW + slot, rowc = row < R ? row : R - 1;
    const int AD = t.NH * HD;
    // the weight fragment (row `row`, columns W2*kvh + 8*(sub + LPS*j)) is
    // issued right behind the attention's own loads
    v4u wv[NJ];
    const bf16_t *wr = Wo + (size_t)rowc * AD + W2 * kvh + 8 * sub;
    L2PfRegs pfr;   // the next launch's weight slice (AttnArgs::pf), behind the W_o fragment
    auto issue = [&]() {
#pragma unroll
        for (int j = 0; j < NJ; ++j) wv[j] = *reinterpret_cast<const v4u *>(wr + 8 * LPS * j);
        qtts_l2pf_issue<256>(t.pf, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), pfr, Wo);
    };
    attn_short_wg<HD, false>(t, kvh, b, lq, sc, att, rb == 0, issue, rsrc, ids);
    __syncthreads();
#ifdef QTTS_STAMPS
    if (t.dbg && tid == 0) t.dbg[wgl * 8 + 4] = __builtin_amdgcn_s_memrealtime();
#endif
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        float f[8];
        unpack8(wv[j], f);
        const float *xp = att + 8 * (sub + LPS * j);
        const float4 x0 = *reinterpret_cast<const float4 *>(xp);
        const float4 x1 = *reinterpret_cast<const float4 *>(xp + 4);
        acc = fmaf(f[0], x0.x, acc); acc = fmaf(f[1], x0.y, acc);
        acc = fmaf(f[2], x0.z, acc); acc = fmaf(f[3], x0.w, acc);
        acc = fmaf(f[4], x1.x, acc); acc = fmaf(f[5], x1.y, acc);
        acc = fmaf(f[6], x1.z, acc); acc = fmaf(f[7], x1.w, acc);
    }
    acc = group_sum<LPS>(acc);
#ifdef QTTS_STAMPS
    if (t.dbg && tid == 0) t.dbg[wgl * 8 + 2] = __builtin_amdgcn_s_memrealtime();
#endif
    if (sub == 0 && row < R) part[((size_t)kvh * gridDim.z + b) * R + row] = acc;
    qtts_l2pf_sink(t.pf, pfr);
#ifdef QTTS_STAMPS
    if (t.dbg && tid == 0) t.dbg[wgl * 8 + 3] = __builtin_amdgcn_s_memrealtime();
#endif
}

}  // namespace

// Sub-talker attention + O projection by kv head, rows b < nrows (grid z):
// part[(kvh * nrows + b) * R + row]; 1 = not covered.
bool qtts_attn_o_covers(const AttnArgs &a, const bf16_t *Wo) {
    const bool hd_ok = a.HD == 128 || a.HD == 64 || a.HD == 32 || a.HD == 16;
    return a.mode == 0 && a.win == 0 && a.KV > 0 && a.NH == 2 * a.KV && hd_ok && a.S <= 16 && a.nrows >= 1 &&
           ((uintptr_t)Wo & 15) == 0 && (a.NH * a.HD) % 8 == 0;
}

int qtts_attn_o(const AttnArgs &a, const bf16_t *Wo, int R, float *part, hipStream_t st) {
    if (!qtts_attn_o_covers(a, Wo)) return 1;
    const int W2 = 2 * a.HD, LPS = W2 / 8 < 8 ? W2 / 8 : 8, RPW = 256 / LPS;
    const dim3 grid((R + RPW - 1) / RPW, a.KV, a.nrows);
    const float *rsrc = a.qkv_tab ? a.qkv_tab : a.qkv;
    const int *ids = a.qkv_tab ? a.tab_ids + a.tab_off : nullptr;
    switch (a.HD) {
        case 128: hipLaunchKernelGGL((k_attn_o<128>), grid, dim3(256), 0, st, rsrc, ids, a, Wo, R, part); qtts_last_kernel = "k_attn_o<128>"; break;
        case 64: hipLaunchKernelGGL((k_attn_o<64>), grid, dim3(256), 0, st, rsrc, ids, a, Wo, R, part); qtts_last_kernel = "k_attn_o<64>"; break;
        case 32: hipLaunchKernelGGL((k_attn_o<32>), grid, dim3(256), 0, st, rsrc, ids, a, Wo, R, part); qtts_last_kernel = "k_attn_o<32>"; break;
        default: hipLaunchKernelGGL((k_attn_o<16>), grid, dim3(256), 0, st, rsrc, ids, a, Wo, R, part); qtts_last_kernel = "k_attn_o<16>"; break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// lanes per key of the talker decode attention: CH = 256 / LPK keys per split
// workgroup.  HD / 32 (64-key splits at HD 128): 16-, 32- and 128-key splits
// measured 29.3, 28.7, 27.9 vs 29.5 audio-s/s (r02m; the merge of more
// partials costs more than the shorter splits save)
// With the merge deferred to the O projection (batch 1) the splits are halved
// at HD 128: 32-key splits, attention 5.7 -> 4.7 us per layer at <= 138 keys
// (the consumer merges 5 partials instead of 3; profiles/r03d_attn_split_ab.txt).
// QTTS_HIP_ATTN_LPK (HD 128: 4, 8 or 16 lanes per key = 64-, 32- or 16-key
// splits) overrides both for split-size A/B runs.  The model latches it ONCE
// at creation (qtts_dev::attn_lpk) and passes it in AttnArgs::lpk, so the
// split scratch it sizes at allocation always covers the launch.
// Round 5: 32-key splits at HD 128 also where the last split merges (the
// lock-step batch): batch 8 153.5 / 153.3 vs 153.2 / 152.4 audio-s/s with
// 64-key splits (profiles/r05h_batch_switch_sweep.txt).
static int attn_lpk(int HD, bool defer, int env) {
    if (HD == 128 && (env == 4 || env == 8 || env == 16)) return env;
    if (HD == 128) return 8;
    return HD >= 32 ? HD / 32 : 1;
}
int qtts_attn_keys_per_split(int HD, bool defer, int lpk) { return 256 / attn_lpk(HD, defer, lpk); }

bool qtts_attn_defer_ok(const AttnArgs &a) {
    const bool hd_ok = a.HD == 128 || a.HD == 64 || a.HD == 32 || a.HD == 16;
    return a.mode == 0 && a.win == 0 && a.KV > 0 && a.NH == 2 * a.KV && hd_ok && a.S > 16 && a.part && a.nsplit >= 1;
}

int qtts_attention(const AttnArgs &a, hipStream_t st) {
    if (a.HD > 128 || a.HD < 8 || (a.HD & 7) || a.NH % a.KV) {
        fprintf(stderr, "qtts_attention: unsupported head config NH=%d KV=%d HD=%d\n", a.NH, a.KV, a.HD);
        return -1;
    }
    const int gph = a.NH / a.KV;
    const bool hd_ok = a.HD == 128 || a.HD == 64 || a.HD == 32 || a.HD == 16;
    if (a.xc_dst && (!(a.mode == 0 && a.win == 0 && gph == 2 && hd_ok && a.S <= 16) || !a.qkv_tab ||
                     (!a.xc_tab && !a.xc_tab16) || a.xc_n % 4 || ((uintptr_t)a.xc_dst & 15))) {
        fprintf(stderr, "qtts_attention: residual copy (xc_dst) only on the short table path\n");
        return -1;
    }
    if (a.mode == 0 && a.win == 0 && gph == 2 && hd_ok && a.S <= 16) {
        const dim3 grid(a.KV, a.nrows);
        switch (a.HD) {
            case 128: hipLaunchKernelGGL((k_attn_short<128>), grid, dim3(256), 0, st, a); qtts_last_kernel = "k_attn_short<128>"; break;
            case 64: hipLaunchKernelGGL((k_attn_short<64>), grid, dim3(256), 0, st, a); qtts_last_kernel = "k_attn_short<64>"; break;
            case 32: hipLaunchKernelGGL((k_attn_short<32>), grid, dim3(256), 0, st, a); qtts_last_kernel = "k_attn_short<32>"; break;
            default: hipLaunchKernelGGL((k_attn_short<16>), grid, dim3(256), 0, st, a); qtts_last_kernel = "k_attn_short<16>"; break;
        }
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (a.mode == 0 && a.win == 0 && gph == 2 && hd_ok) {
        const int ch = qtts_attn_keys_per_split(a.HD, a.defer, a.lpk);
        // one split per ch keys of the cache's capacity (workgroups past the
        // live length exit at once); the scratch must hold all of them, or
        // keys past a.nsplit * ch would never be attended
        const int nsplit = (a.S + ch - 1) / ch;
        if ((nsplit > 1 || a.defer) && (!a.part || !a.cnt || a.nsplit < nsplit)) {
            fprintf(stderr, "qtts_attention: split scratch missing (need %d splits of %d keys, have %d)\n",
                    nsplit, ch, a.part ? a.nsplit : 0);
            return -1;
        }
        const dim3 grid(a.KV, nsplit, a.nrows);
        const int lpk = attn_lpk(a.HD, a.defer, a.lpk);
#define QTTS_AD(H, L)                                                                                      \
        if (a.HD == H && lpk == L) {                                                                       \
            hipLaunchKernelGGL((k_attn_dec<H, 2, L>), grid, dim3(256), 0, st, a.qkv, a.pos, a.kc, a.vc, a); \
            qtts_last_kernel = "k_attn_dec<" #H ", 2, " #L ">";                                            \
            return hipGetLastError() == hipSuccess ? 0 : -1;                                               \
        }
        QTTS_AD(128, 4) QTTS_AD(128, 8) QTTS_AD(128, 16) QTTS_AD(64, 2) QTTS_AD(32, 1) QTTS_AD(16, 1)
#undef QTTS_AD
        fprintf(stderr, "qtts_attention: no decode kernel for HD=%d lpk=%d\n", a.HD, lpk);
        return -1;
    }
    size_t smem = (size_t)(128 * 3 + 256 + 8 + 8 * 128 + a.S + 4) * sizeof(float);
    hipLaunchKernelGGL(k_attn, dim3(a.NH, a.nrows), dim3(256), smem, st, a);
    qtts_last_kernel = "k_attn";
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int qtts_qk_prep(const AttnArgs &a, hipStream_t st) {
    if ((a.NH + a.KV) * a.HD > 4096) {
        fprintf(stderr, "qtts_qk_prep: (NH+KV)*HD=%d exceeds 4096\n", (a.NH + a.KV) * a.HD);
        return -1;
    }
    if ((a.HD == 128 || (a.HD <= 64 && (a.HD & (a.HD - 1)) == 0))) {
        const dim3 grid(a.nrows, (a.NH + 2 * a.KV + 3) / 4);
        hipLaunchKernelGGL(k_qk_prep_w, grid, dim3(256), 0, st, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL(k_qk_prep, dim3(a.nrows), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
