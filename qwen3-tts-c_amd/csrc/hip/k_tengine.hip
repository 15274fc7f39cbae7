// k_tengine.hip - one talker decoder layer at batch 1 as ONE persistent launch
// (T.c:478-533 with the attention of T.c:119-248): the weight stream never
// waits for the layer's hand-offs.
//
// The launch-per-op layer (k_gemvw q|k|v -> k_attn_dec -> k_gemvw O with the
// split merge -> gate|up -> down) leaves HBM idle through the attention
// (~5 us, no weight bytes) and at every kernel boundary; its in-graph period
// is ~33 us for 100.7 MB (profiles/r05v_talker_layer_stamps.txt,
// r06g_graph_spans.json).  Here every workgroup (one per CU, 512 threads)
// runs two roles side by side:
//   GEMV waves 0-3   hold their rows' weights in REGISTERS, issued ahead of
//                    every hand-off they need: q|k|v + O + a third of gate|up
//                    at the start, the next slices as registers free up; they
//                    never touch another workgroup's data (their vmcnt queue
//                    holds weight loads only), so a hand-off never waits
//                    behind the weight stream.  Inputs come from LDS (flag),
//                    outputs go to LDS (counter).
//   comm waves 4-7   gather each op's input vector from 8-byte {tag, value}
//                    granules (cdna_hip_programming.md Guideline 16 R2: sc1
//                    stores, relaxed agent-scope sweeps), apply RMSNorm, and
//                    publish the GEMV waves' outputs as granules; in the
//                    workgroups of a kv head's splits they also run the
//                    decode attention (k_attn_dec's arithmetic, 32-key splits,
//                    partials + ticket, the last split merges in split order
//                    and publishes the head's output).
// Every value is computed with the arithmetic of the launch-per-op path
// (k_gemvw rows: one wave per row, lane chunks l + 64k, wave_sum; its RMS
// statistic: 256 threads x 2 float4 units, wave sums, red[0..3]; k_attn_dec's
// QK-norm / RoPE / scores / softmax / P.V; its last-split merge == k_gemvw's
// deferred merge), so the layer is bit-identical to it.
// Spins are bounded: a hand-off not seen within ~0.5 s sets *err and the
// launch runs to its end (garbage, reported by the host), never hangs.
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

constexpr int H = 2048, NH = 16, KVH = 8, HD = 128, IM = 6144, QKVR = (NH + 2 * KVH) * HD;   // 1.7B talker
constexpr int GPH = NH / KVH;                       // q heads per kv head
constexpr int LPK = 8, CH = 256 / LPK, DPL = HD / LPK, D4 = HD / 4, KG = 256 / D4, NO = GPH * HD;
constexpr int NVC = CH / KG;                        // P.V keys per thread group
constexpr unsigned SPIN_MAX = 1u << 22;

struct TLds {
    float xs[H];                  // the GEMV input row: normed x (q|k|v), attention output (O), normed x' (gate|up)
    float hs[IM];                 // the down projection's input h
    float hq[4 * HD];             // attention: the head's q0 | q1 | k | v from the q|k|v granules
    float qk[(GPH + 1) * HD];     // rotated q heads, then k
    float vv[HD];
    float sc[GPH][CH];
    float ml[GPH][2];
    float red[KG * NO];
    float cred[4];                // comm RMS partials
    float outq[16], outo[8], outh[24];
    int gflag;                    // comm -> GEMV: 1 x staged, 2 attention staged, 3 x' staged, 4 h staged
    int ocnt;                     // GEMV -> comm: 4 per finished op
    int cbar;                     // comm waves' own barrier counter
    int last;
    int full;                     // (ring engine) weight slots landed in the ring, in order
    int done[4];                  // (ring engine) slots released by consumer wave w
};

__device__ __forceinline__ float dot8w(const v4u &w, const float *x) {
    const float4 x0 = *reinterpret_cast<const float4 *>(x);
    const float4 x1 = *reinterpret_cast<const float4 *>(x + 4);
    float s = 0.f;
    s = fmaf(__uint_as_float(w.x << 16), x0.x, s); s = fmaf(__uint_as_float(w.x & 0xFFFF0000u), x0.y, s);
    s = fmaf(__uint_as_float(w.y << 16), x0.z, s); s = fmaf(__uint_as_float(w.y & 0xFFFF0000u), x0.w, s);
    s = fmaf(__uint_as_float(w.z << 16), x1.x, s); s = fmaf(__uint_as_float(w.z & 0xFFFF0000u), x1.y, s);
    s = fmaf(__uint_as_float(w.w << 16), x1.z, s); s = fmaf(__uint_as_float(w.w & 0xFFFF0000u), x1.w, s);
    return s;
}

__device__ __forceinline__ int lds_ld(int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void give_up(int *err, int code) {
    __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// GEMV waves: wait until the comm waves staged input k.  (No global access in
// here: a store on a divergent path makes the compiler's vmcnt bookkeeping
// drain the weight loads in flight; a timeout is reported at the end.)
__device__ __forceinline__ bool gemv_wait(TLds &L, int k) {
    unsigned n = 0;
    bool ok = true;
    while (lds_ld(&L.gflag) < k) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) { ok = false; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return ok;
}
// GEMV waves: this wave's outputs of the op are in LDS
__device__ __forceinline__ void gemv_done(TLds &L, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(&L.ocnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// comm waves: barrier among the 4 comm waves only (the GEMV waves keep streaming)
__device__ __forceinline__ void cbarrier(TLds &L, int &gen, int lane, int *err) {
    gen += 4;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(&L.cbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned n = 0;
    while (lds_ld(&L.cbar) < gen) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) { give_up(err, 2); break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// comm waves: until the GEMV waves finished op k (4 arrivals per op)
__device__ __forceinline__ void comm_wait_out(TLds &L, int k, int *err) {
    unsigned n = 0;
    while (lds_ld(&L.ocnt) < 4 * k) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) { give_up(err, 20 + k); break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// comm waves: every comm wave's LDS writes of input k are done -> the GEMV waves go
__device__ __forceinline__ void comm_stage(TLds &L, int k, int &gen, int lane, int *err) {
    cbarrier(L, gen, lane, err);
    if (threadIdx.x == 256) __hip_atomic_store(&L.gflag, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

typedef unsigned long long u64;
// diagnostic phase stamps (TLayerArgs::dbg, stamp builds only): 100 MHz wall clock
__device__ __forceinline__ void te_stamp(const TLayerArgs &a, int k, bool who) {
#ifdef QTTS_STAMPS
    if (a.dbg && who) a.dbg[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
#endif
}
__device__ __forceinline__ void put_granule(u64 *g, unsigned tag, float v) {
    __hip_atomic_store(g, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// comm thread ct sweeps its N granules g[idx(j)] until every tag of the wave
// is `tag` (the comm waves' vmcnt queue holds no weight loads)
template <int N, typename Idx>
__device__ __forceinline__ void sweep(const u64 *g, unsigned tag, Idx idx, float (&v)[N], int *err, int code) {
    unsigned n = 0;
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const u64 x = __hip_atomic_load(const_cast<u64 *>(g) + idx(j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[j] = __uint_as_float((unsigned)x);
            ok &= (unsigned)(x >> 32) == tag;
        }
        if (__all(ok)) return;
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) { give_up(err, code); return; }
    }
}

// RMSNorm of a 2048-float row held as k_gemvw holds it: comm thread ct has
// units c = 4 (ct + 256 q), q < 2; the statistic in k_gemvw's order
__device__ __forceinline__ void comm_norm_stage(TLds &L, float4 (&xv)[2], const float *nw, float eps, int ct, int lane,
                                                int cw, int &gen, int *err) {
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const float4 v = xv[q];
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = wave_sum(ss);
    if (lane == 0) L.cred[cw] = ss;
    cbarrier(L, gen, lane, err);
    const float inv = rms_inv(L.cred[0] + L.cred[1] + L.cred[2] + L.cred[3], H, eps);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int c = 4 * (ct + 256 * q);
        const float4 n4 = *reinterpret_cast<const float4 *>(nw + c);
        float4 v = xv[q];
        v.x = v.x * inv * n4.x; v.y = v.y * inv * n4.y; v.z = v.z * inv * n4.z; v.w = v.w * inv * n4.w;
        *reinterpret_cast<float4 *>(L.xs + c) = v;
    }
}

// the rows of q|k|v list index i (0..511) of kv head h: q heads 2h, 2h+1, then k h, v h
__device__ __forceinline__ int qkv_row(int h, int i) {
    return i < NO ? GPH * HD * h + i : i < NO + HD ? NH * HD + HD * h + (i - NO) : (NH + KVH) * HD + HD * h + (i - NO - HD);
}

// One decode-attention split of kv head kvh on the comm waves (k_attn_dec<128,
// 2, 8>'s arithmetic; inputs from L.hq; barriers among the comm waves only).
// Returns through granules: the head's merged output, by the last split.
// The split's inputs that do not depend on this step's q|k|v: its cached key
// and value rows, the QK-norm weights and the RoPE row of position p.  Loaded
// at the comm role's start, so the attention after the head gather waits on
// no memory but the gather itself.  (Position p's own row is never read from
// the cache: it comes from LDS.)
struct AttnPre {
    float4 kreg[DPL / 4];
    float4 vreg[NVC];
    float hw[2], rc[2], rs[2];
};
__device__ __forceinline__ void attn_preload(AttnPre &q, const TLayerArgs &a, int kvh, int split, int p, int ct,
                                             int lane, int cw) {
    const int t0 = split * CH, t1 = min(p + 1, t0 + CH);
    const int KVD = KVH * HD;
    const float *Kc = a.kc + kvh * HD;
    const float *Vc = a.vc + kvh * HD;
    const int hh0 = cw < GPH ? cw : GPH;
    const float *nw = hh0 < GPH ? a.qn_w : a.kn_w;
    const float *cs = a.rope_cos + (size_t)p * HD, *sn = a.rope_sin + (size_t)p * HD;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        q.hw[j] = nw[lane + 64 * j];
        q.rc[j] = cs[lane + 64 * j];
        q.rs[j] = sn[lane + 64 * j];
    }
    const int kl = ct / LPK, ksub = ct - kl * LPK;
    const int tk = t0 + kl;
    const float4 *kp = reinterpret_cast<const float4 *>(Kc + (size_t)(tk < t1 ? tk : t0) * KVD + ksub * DPL);
#pragma unroll
    for (int j = 0; j < DPL / 4; ++j) q.kreg[j] = kp[j];
    const int d4 = ct % D4, kg = ct / D4;
#pragma unroll
    for (int j = 0; j < NVC; ++j) {
        const int t = t0 + kg + j * KG;
        const bool ok = kg + j * KG < CH && t < t1;
        q.vreg[j] = reinterpret_cast<const float4 *>(Vc + (size_t)(ok ? t : t0) * KVD)[d4];
    }
}

__device__ void comm_attention(TLds &L, const TLayerArgs &a, int kvh, int split, int nact, int p, unsigned tag,
                               int ct, int lane, int cw, int &gen, const AttnPre &pre) {
    const int n = p + 1;
    const int t0 = split * CH, t1 = min(n, t0 + CH);
    const bool owner = (split == nact - 1);
    const int KVD = KVH * HD;
    // token inputs (from the gathered head); the rest came with the preload
    const int hh0 = cw < GPH ? cw : GPH;
    float hv[2];
    {
        const float *src = L.hq + (hh0 < GPH ? hh0 * HD : NO);
#pragma unroll
        for (int j = 0; j < 2; ++j) hv[j] = src[lane + 64 * j];
    }
    const float *hw = pre.hw, *rc = pre.rc, *rs = pre.rs;
    const float4 *kreg = pre.kreg, *vreg = pre.vreg;
    const float vtok = L.hq[NO + HD + ct % HD];
    const int kl = ct / LPK, ksub = ct - kl * LPK;
    const int tk = t0 + kl;
    const int d4 = ct % D4, kg = ct / D4;
    // QK-norm + RoPE in registers (waves 0..GPH: q heads, then k)
    if (cw <= GPH) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j) ss += hv[j] * hv[j];
        ss = wave_sum(ss);
        const float iv = rms_inv(ss, HD, a.eps);
        const float n0 = hv[0] * iv * hw[0], n1 = hv[1] * iv * hw[1];
        L.qk[hh0 * HD + lane] = n0 * rc[0] - n1 * rs[0];
        L.qk[hh0 * HD + lane + 64] = n1 * rc[1] + n0 * rs[1];
    }
    if (owner && ct < HD) L.vv[ct] = vtok;
    cbarrier(L, gen, lane, a.err);
    if (owner && ct < HD && !(a.skip && a.skip[0])) {
        a.kc[(size_t)p * KVD + kvh * HD + ct] = L.qk[GPH * HD + ct];
        a.vc[(size_t)p * KVD + kvh * HD + ct] = L.vv[ct];
    }
    // scores
    const float scale = div_rn(1.0f, sqrt_rn((float)HD));
    {
        float d[GPH];
#pragma unroll
        for (int g = 0; g < GPH; ++g) d[g] = 0.f;
        if (tk < t1) {
            float4 kv[DPL / 4];
#pragma unroll
            for (int j = 0; j < DPL / 4; ++j)
                kv[j] = (tk == p) ? reinterpret_cast<const float4 *>(L.qk + GPH * HD + ksub * DPL)[j] : kreg[j];
#pragma unroll
            for (int g = 0; g < GPH; ++g) {
                const float4 *q4 = reinterpret_cast<const float4 *>(L.qk + g * HD + ksub * DPL);
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
            if (ksub == 0) L.sc[g][kl] = tk < t1 ? d[g] * scale : -INFINITY;
        }
    }
    cbarrier(L, gen, lane, a.err);
    for (int g = cw; g < GPH; g += 4) {
        float m = -INFINITY;
        for (int k = lane; k < CH; k += 64) m = fmaxf(m, L.sc[g][k]);
        m = wave_max(m);
        float l = 0.f;
        for (int k = lane; k < CH; k += 64) {
            const float e = t0 + k < t1 ? expf(L.sc[g][k] - m) : 0.f;
            L.sc[g][k] = e;
            l += e;
        }
        l = wave_sum(l);
        if (lane == 0) { L.ml[g][0] = m; L.ml[g][1] = l; }
    }
    cbarrier(L, gen, lane, a.err);
    {
        float4 acc[GPH];
#pragma unroll
        for (int g = 0; g < GPH; ++g) acc[g] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < NVC; ++j) {
            const int k = kg + j * KG;
            const int t = t0 + k;
            if (k < CH && t < t1) {
                const float4 v4 = (t == p) ? reinterpret_cast<const float4 *>(L.vv)[d4] : vreg[j];
#pragma unroll
                for (int g = 0; g < GPH; ++g) {
                    const float pw = L.sc[g][k];
                    acc[g].x += pw * v4.x; acc[g].y += pw * v4.y; acc[g].z += pw * v4.z; acc[g].w += pw * v4.w;
                }
            }
        }
#pragma unroll
        for (int g = 0; g < GPH; ++g) reinterpret_cast<float4 *>(L.red + kg * NO + g * HD)[d4] = acc[g];
    }
    cbarrier(L, gen, lane, a.err);
    float res = 0.f;   // NO == 256: one output per comm thread
    for (int k = 0; k < KG; ++k) res += L.red[k * NO + ct];
    u64 *gout = a.g_att + (size_t)kvh * NO;
    if (nact == 1) {
        put_granule(gout + ct, tag, res / L.ml[ct / HD][1]);
        return;
    }
    // partials (write-through), drained by every comm wave, one ticket per split
    const int stride = NO + 2 * GPH;
    float *base = a.part + (size_t)kvh * a.nsplit * stride;
    float *mine = base + (size_t)split * stride;
    st_sc1(mine + ct, res);
    if (ct < GPH) { st_sc1(mine + NO + 2 * ct, L.ml[ct][0]); st_sc1(mine + NO + 2 * ct + 1, L.ml[ct][1]); }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cbarrier(L, gen, lane, a.err);
    if (ct == 0) {
        const int old = __hip_atomic_fetch_add(a.cnt + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.last = (old == nact - 1);
    }
    cbarrier(L, gen, lane, a.err);
    if (!L.last) return;
    // the merge in split order (k_attn_dec's / k_gemvw's deferred merge
    // arithmetic), its loads issued 8 splits at a time (one dependent round
    // trip per 8 splits, not one per split)
    const int g = ct / HD;
    constexpr int MB = 8;
    float M = -INFINITY;
    for (int s0 = 0; s0 < nact; s0 += MB) {
        float mv[MB];
#pragma unroll
        for (int j = 0; j < MB; ++j)
            mv[j] = s0 + j < nact ? ld_sc1(base + (size_t)(s0 + j) * stride + NO + 2 * g) : -INFINITY;
#pragma unroll
        for (int j = 0; j < MB; ++j) M = fmaxf(M, mv[j]);
    }
    float num = 0.f, den = 0.f;
    for (int s0 = 0; s0 < nact; s0 += MB) {
        float mv[MB], pv[MB], lv[MB];
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            const float *ps = base + (size_t)min(s0 + j, nact - 1) * stride;
            mv[j] = ld_sc1(ps + NO + 2 * g);
            pv[j] = ld_sc1(ps + ct);
            lv[j] = ld_sc1(ps + NO + 2 * g + 1);
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            if (s0 + j >= nact) break;
            const float f = expf(mv[j] - M);
            num = fmaf(f, pv[j], num);
            den = fmaf(f, lv[j], den);
        }
    }
    put_granule(gout + ct, tag, num / den);
    if (ct == 0) __hip_atomic_store(a.cnt + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the weight slices of the GEMV waves: NR rows x NV 16-B chunks per lane,
// non-temporal (read once per frame; the sub-talker keeps the Infinity Cache)
template <int NR, int NV>
struct Slice {
    v4u w[NR][NV];
    __device__ __forceinline__ void load(const bf16_t *W, int C, const int (&rows)[NR], int lane) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const v4u *p = reinterpret_cast<const v4u *>(W + (size_t)rows[r] * C) + lane;
#pragma unroll
            for (int k = 0; k < NV; ++k) w[r][k] = __builtin_nontemporal_load(p + 64 * k);
        }
    }
    __device__ __forceinline__ float dot(int r, const float *x, int lane) const {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) s += dot8w(w[r][k], x + 8 * (lane + 64 * k));
        return wave_sum(s);
    }
};

// the comm waves (threads 256..511): input gathers, RMSNorm, the decode
// attention of this workgroup's kv head splits, the output granules
// DIRECT (the ring engine): the consumer waves publish their own output
// granules (no LDS hop through the comm waves); the comm waves still wait for
// the consumers' local done signal before each sweep (see step 2).
template <bool DIRECT>
__device__ __forceinline__ void comm_role(TLds &L, const TLayerArgs &a, int tid, int lane, int wv, int b) {
    const unsigned epoch = (unsigned)a.epoch[0];
    const unsigned tag = epoch * 32u + (unsigned)a.layer + 1u;
    const int h = b >> 5, j32 = b & 31;
    const int ct = tid - 256, cw = wv - 4;
    int gen = 0;
    const int p = a.pos[0];                        // the token's position (kv_len before this step)
    const int nact = (p + 1 + CH - 1) / CH;
    AttnPre pre;                                   // this workgroup's first split's cache rows, ahead of everything
    if (j32 < nact) attn_preload(pre, a, h, j32, p, ct, lane, cw);
    // 1. x (the layer input) -> RMSNorm (input_layernorm) -> LDS
    {
        float4 xv[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) xv[q] = *reinterpret_cast<const float4 *>(a.x_in + 4 * (ct + 256 * q));
        comm_norm_stage(L, xv, a.in_norm, a.eps, ct, lane, cw, gen, a.err);
        comm_stage(L, 1, gen, lane, a.err);
        te_stamp(a, 1, ct == 0);
    }
    // 2. this workgroup's 16 q|k|v rows -> granules (DIRECT: the consumers
    //    published them; waiting for their local signal still keeps the sweep
    //    below from polling the whole phase -- polling beside the weight stream
    //    slows the stream, MI355X_MICROARCH.md polling-cost: gate|up 5 -> 15 us
    //    when the h sweep started at once, profiles/r06r_ring_engine_stamps.txt)
    comm_wait_out(L, 1, a.err);
    if (!DIRECT && ct < 16) put_granule(a.g_qkv + qkv_row(h, 16 * j32 + ct), tag, L.outq[ct]);
    te_stamp(a, 3, ct == 0);
    // 3. the attention splits of kv head h this workgroup runs (split j32, j32 + 32, ...)
    if (j32 < nact) {
        float v[2];   // the head's 512 q|k|v values (index ct + 256 j of the head's list)
        sweep<2>(a.g_qkv, tag, [&](int j) { return qkv_row(h, ct + 256 * j); }, v, a.err, 3);
        L.hq[ct] = v[0];
        L.hq[ct + 256] = v[1];
        cbarrier(L, gen, lane, a.err);
        te_stamp(a, 4, ct == 0);
        for (int s = j32; s < nact; s += 32) {
            if (s != j32) attn_preload(pre, a, h, s, p, ct, lane, cw);   // (beyond 1024 keys)
            comm_attention(L, a, h, s, nact, p, tag, ct, lane, cw, gen, pre);
            cbarrier(L, gen, lane, a.err);
        }
        te_stamp(a, 5, ct == 0);
    }
    // 4. the attention output of every head -> LDS (the O projection's input, no
    //    norm); granule o = kvh * 256 + g * 128 + d is attention element o itself
    {
        float v[8];
        sweep<8>(a.g_att, tag, [&](int j) { return ct + 256 * j; }, v, a.err, 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) L.xs[ct + 256 * j] = v[j];
        comm_stage(L, 2, gen, lane, a.err);
        te_stamp(a, 6, ct == 0);
    }
    // 5. this workgroup's 8 x' rows -> granules
    comm_wait_out(L, 2, a.err);
    if (!DIRECT && ct < 8) put_granule(a.g_x + 8 * b + ct, tag, L.outo[ct]);
    // 6. x' of every row, in k_gemvw's unit mapping (thread ct: elements
    //    4 (ct + 256 q) + e) -> RMSNorm (post_attention_layernorm) -> LDS
    //    (the GEMV waves finished reading xs: this workgroup's O rows are in)
    {
        float v[8];
        sweep<8>(a.g_x, tag, [&](int j) { return 4 * (ct + 256 * (j >> 2)) + (j & 3); }, v, a.err, 5);
        te_stamp(a, 8, ct == 0);
        float4 xv[2];
        xv[0] = make_float4(v[0], v[1], v[2], v[3]);
        xv[1] = make_float4(v[4], v[5], v[6], v[7]);
        comm_norm_stage(L, xv, a.post_norm, a.eps, ct, lane, cw, gen, a.err);
        comm_stage(L, 3, gen, lane, a.err);
        te_stamp(a, 9, ct == 0);
    }
    // 7. this workgroup's 24 h values -> granules (wave w, pair k: gate row 48 b + w + 8 k)
    comm_wait_out(L, 3, a.err);
    if (!DIRECT && ct < 24) {
        const int w = ct / 6, k = ct - 6 * (ct / 6);
        const int r = 48 * b + w + 8 * k;
        put_granule(a.g_h + (r >> 3) * 4 + (r & 3), tag, L.outh[ct]);
    }
    // 8. h of every row -> LDS (the down projection's input)
    {
        float v[24];
        sweep<24>(a.g_h, tag, [&](int j) { return ct + 256 * j; }, v, a.err, 6);
#pragma unroll
        for (int j = 0; j < 24; ++j) L.hs[ct + 256 * j] = v[j];
        comm_stage(L, 4, gen, lane, a.err);
        te_stamp(a, 11, ct == 0);
    }
    // the next talker pass gets new tags (every workgroup read the epoch long ago:
    // this one waited for all of their h granules)
    if (a.last_layer && b == 0 && ct == 0)
        __hip_atomic_store(a.epoch, (int)(epoch + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(512, 1) void k_tlayer(TLayerArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TLds &L = *reinterpret_cast<TLds *>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int b = blockIdx.x;
    te_stamp(a, 0, threadIdx.x == 0);
    if (a.err[0]) return;   // an earlier launch timed out: the pass is garbage already, do not wait again
    if (tid == 0) { L.gflag = 0; L.ocnt = 0; L.cbar = 0; L.last = 0; }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned epoch = (unsigned)a.epoch[0];
    const unsigned tag = epoch * 32u + (unsigned)a.layer + 1u;   // never 0; unique per (talker pass, layer)
    const int h = b >> 5, j32 = b & 31;

    if (wv < 4) {
        // ================= GEMV waves =================
        const int w = wv;
        int rq[4], ro[2], rg[3][4], rd[2];
#pragma unroll
        for (int r = 0; r < 4; ++r) rq[r] = qkv_row(h, 16 * j32 + w + 4 * r);
#pragma unroll
        for (int r = 0; r < 2; ++r) { ro[r] = 8 * b + w + 4 * r; rd[r] = 8 * b + w + 4 * r; }
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) rg[t][r] = 48 * b + w + 4 * (4 * t + r);
        // the residual rows of the O projection (the layer input), ahead of the weights
        float yres[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) yres[r] = a.x_in[ro[r]];
        Slice<4, 4> sq;
        Slice<2, 4> so;
        Slice<4, 4> sg0, sg1, sg2;
        Slice<1, 12> sd0, sd1;
        const int rd0[1] = {rd[0]}, rd1[1] = {rd[1]};
        sq.load(a.wqkv, H, rq, lane);
        so.load(a.wo, H, ro, lane);
        sg0.load(a.wgu, H, rg[0], lane);
        // q|k|v rows
        bool ok = gemv_wait(L, 1);
        float aq[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) aq[r] = sq.dot(r, L.xs, lane);
        te_stamp(a, 2, tid == 0);
        if (lane == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) L.outq[w + 4 * r] = aq[r];
        gemv_done(L, lane);
        sg1.load(a.wgu, H, rg[1], lane);
        // O rows + residual
        ok &= gemv_wait(L, 2);
        float xm[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) xm[r] = yres[r] + so.dot(r, L.xs, lane);
        te_stamp(a, 7, tid == 0);
        if (lane == 0)
#pragma unroll
            for (int r = 0; r < 2; ++r) L.outo[w + 4 * r] = xm[r];
        gemv_done(L, lane);
        sg2.load(a.wgu, H, rg[2], lane);
        // gate|up rows, SwiGLU (gate row r and its up row r + 4 in this wave)
        ok &= gemv_wait(L, 3);
        float hv[6];
        {
            float g0 = sg0.dot(0, L.xs, lane), u0 = sg0.dot(1, L.xs, lane);
            float g1 = sg0.dot(2, L.xs, lane), u1 = sg0.dot(3, L.xs, lane);
            hv[0] = (g0 / (1.0f + expf(-g0))) * u0;
            hv[1] = (g1 / (1.0f + expf(-g1))) * u1;
        }
        sd0.load(a.wdown, IM, rd0, lane);   // (the down rows as registers free up)
        {
            float g0 = sg1.dot(0, L.xs, lane), u0 = sg1.dot(1, L.xs, lane);
            float g1 = sg1.dot(2, L.xs, lane), u1 = sg1.dot(3, L.xs, lane);
            hv[2] = (g0 / (1.0f + expf(-g0))) * u0;
            hv[3] = (g1 / (1.0f + expf(-g1))) * u1;
        }
        sd1.load(a.wdown, IM, rd1, lane);
        {
            float g0 = sg2.dot(0, L.xs, lane), u0 = sg2.dot(1, L.xs, lane);
            float g1 = sg2.dot(2, L.xs, lane), u1 = sg2.dot(3, L.xs, lane);
            hv[4] = (g0 / (1.0f + expf(-g0))) * u0;
            hv[5] = (g1 / (1.0f + expf(-g1))) * u1;
        }
        te_stamp(a, 10, tid == 0);
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 6; ++k) L.outh[6 * w + k] = hv[k];
        gemv_done(L, lane);
        // down rows + residual -> the layer output (read by the next launch)
        ok &= gemv_wait(L, 4);
        float xo[2];
        xo[0] = xm[0] + sd0.dot(0, L.hs, lane);
        xo[1] = xm[1] + sd1.dot(0, L.hs, lane);
        if (lane == 0) {
#pragma unroll
            for (int r = 0; r < 2; ++r) a.x_out[rd[r]] = xo[r];
            if (!ok) give_up(a.err, 10);
        }
        te_stamp(a, 12, tid == 0);
        return;
    }

    comm_role<false>(L, a, tid, lane, wv, b);
}

// ---------------------------------------------------------------------------
// The ring engine (QTTS_HIP_TENGINE=2|3): the same layer with the weight stream
// moved off the GEMV waves' registers onto one LDS-DMA loader wave.
//
// r06l's stamps of the register form (profiles/r06l_tengine_stamps.txt) show
// where it lost: the GEMV waves issue ~160 KB of weight loads per CU at launch
// start, and every load the comm waves issue after that (the layer input, the
// granule sweeps, the K/V rows) waits behind them in the CU's memory queue --
// x staged 7.6 us into the launch, each gather 2.3-5.8 us.  Here the loader
// keeps at most INFL 16-KB slots in flight (MI355X_MICROARCH.md gather-pass /
// ldsdma-fill: thin the loader so the gathers are not queued behind it) and
// runs up to RING slots ahead of the consumers, through every hand-off
// (prefetch-credit).  A CU's 24 slots per layer, in consumption order:
//   0-3    q|k|v   4 rows x 4 KB each (the head-grouped rows of k_tlayer)
//   4-5    O       rows 8b + 4s + w
//   6-17   gate|up rows 48b + 4m + w (m even: gate, m odd: its up row)
//   18-23  down    columns [1024 j, 1024 j + 1024) of rows 8b..8b+7, 2 KB each
// Consumer wave w (0..3) takes row w of every H-wide slot and rows w, w + 4 of
// the down slots: lane l's chunks l + 64 k in k order, so every row is summed
// exactly as k_gemvw / k_tlayer sum it (bit-identical outputs).
constexpr int RING = 6, SLOT = 16384, NSLOT = 24;
constexpr int RING_THREADS = 576;   // 4 consumer + 4 comm + 1 loader waves

__device__ __forceinline__ unsigned char *ring_base(unsigned char *smem) {
    return smem + ((sizeof(TLds) + 15) & ~size_t(15));
}
// The loader's own LDS words go through inline asm: the compiler counts an
// LDS-DMA as a pending LDS write, so any LDS access it sees in the loader wave
// gets an s_waitcnt vmcnt(0) first -- which would drain the stream at every
// publish.  (The consumers and comm waves issue no LDS-DMA; their LDS accesses
// stay plain.)
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ int min_done(TLds &L) {
    int d0, d1, d2, d3;
    asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\tds_read_b32 %2, %4 offset:8\n\t"
                 "ds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3)
                 : "v"(lds_addr(&L.done[0]))
                 : "memory");
    return min(min(d0, d1), min(d2, d3));
}
__device__ __forceinline__ void publish_full(TLds &L, int n) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(&L.full)), "v"(n) : "memory");
}
template <int INFL>
__device__ __forceinline__ void loader_role(TLds &L, unsigned char *ring, const TLayerArgs &a, int b, int lane) {
    const int h = b >> 5, j32 = b & 31;
    bool ok = true;
    for (int i = 0; i < NSLOT; ++i) {
        if (i >= RING && min_done(L) < i - RING + 1) {
            // the ring is full: publish what landed, then wait for slot i - RING's release
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            publish_full(L, i);
            unsigned n = 0;
            while (min_done(L) < i - RING + 1) {
                __builtin_amdgcn_s_sleep(1);
                if (++n > SPIN_MAX) { ok = false; break; }
            }
        }
        unsigned char *dst = ring + (i % RING) * SLOT;
        if (i < 18) {
            // 4 whole H-wide rows, 4 KB each: piece p = quarter p & 3 of row p >> 2
            const bf16_t *rb[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                rb[r] = i < 4 ? a.wqkv + (size_t)qkv_row(h, 16 * j32 + 4 * i + r) * H
                      : i < 6 ? a.wo + (size_t)(8 * b + 4 * (i - 4) + r) * H
                              : a.wgu + (size_t)(48 * b + 4 * (i - 6) + r) * H;
#pragma unroll
            for (int p = 0; p < 16; ++p)
                __builtin_amdgcn_global_load_lds((const void *)(rb[p >> 2] + 512 * (p & 3) + 8 * lane),
                                                 (__attribute__((address_space(3))) void *)(dst + 1024 * p), 16, 0, 2);
        } else {
            // columns [1024 j, 1024 j + 1024) of the 8 down rows: piece p = half p & 1 of row p >> 1
            const bf16_t *db = a.wdown + (size_t)(8 * b) * IM + 1024 * (i - 18);
#pragma unroll
            for (int p = 0; p < 16; ++p)
                __builtin_amdgcn_global_load_lds((const void *)(db + (size_t)(p >> 1) * IM + 512 * (p & 1) + 8 * lane),
                                                 (__attribute__((address_space(3))) void *)(dst + 1024 * p), 16, 0, 2);
        }
        if (i >= INFL - 1) {
            // slots <= i - INFL + 1 landed: at most INFL - 1 slots stay in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 * (INFL - 1)) : "memory");
            publish_full(L, i - INFL + 2);
        }
    }
    te_stamp(a, 13, lane == 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    publish_full(L, NSLOT);
    if (!ok && lane == 0) give_up(a.err, 11);
}

__device__ __forceinline__ bool slot_wait(TLds &L, int i) {
    unsigned n = 0;
    while (lds_ld(&L.full) <= i) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) return false;
    }
    asm volatile("" ::: "memory");
    return true;
}
// the slot's reads have returned to registers: the loader may refill it
__device__ __forceinline__ void slot_release(TLds &L, int w, int i, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&L.done[w], i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ float dot8r(const v4u &w, const float *x) {   // x: 8 floats in registers
    float s = 0.f;
    s = fmaf(__uint_as_float(w.x << 16), x[0], s); s = fmaf(__uint_as_float(w.x & 0xFFFF0000u), x[1], s);
    s = fmaf(__uint_as_float(w.y << 16), x[2], s); s = fmaf(__uint_as_float(w.y & 0xFFFF0000u), x[3], s);
    s = fmaf(__uint_as_float(w.z << 16), x[4], s); s = fmaf(__uint_as_float(w.z & 0xFFFF0000u), x[5], s);
    s = fmaf(__uint_as_float(w.w << 16), x[6], s); s = fmaf(__uint_as_float(w.w & 0xFFFF0000u), x[7], s);
    return s;
}
// x chunks l + 64 k (k < 4) of a 2048-float LDS row into registers
__device__ __forceinline__ void load_xr(const float *xs, float (&xr)[32], int lane) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 a0 = *reinterpret_cast<const float4 *>(xs + 8 * (lane + 64 * k));
        const float4 a1 = *reinterpret_cast<const float4 *>(xs + 8 * (lane + 64 * k) + 4);
        xr[8 * k + 0] = a0.x; xr[8 * k + 1] = a0.y; xr[8 * k + 2] = a0.z; xr[8 * k + 3] = a0.w;
        xr[8 * k + 4] = a1.x; xr[8 * k + 5] = a1.y; xr[8 * k + 6] = a1.z; xr[8 * k + 7] = a1.w;
    }
}
// row w of the H-wide slot i, dotted with x
__device__ __forceinline__ float ring_row(TLds &L, const unsigned char *ring, int i, int w, const float (&xr)[32], int lane,
                                          bool &ok) {
    ok &= slot_wait(L, i);
    const v4u *row = reinterpret_cast<const v4u *>(ring + (i % RING) * SLOT + 4096 * w);
    v4u wr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) wr[k] = row[lane + 64 * k];
    slot_release(L, w, i, lane);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += dot8r(wr[k], xr + 8 * k);
    return wave_sum(s);
}

template <int INFL>
__global__ __launch_bounds__(RING_THREADS, 1) void k_tlayer_ring(TLayerArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TLds &L = *reinterpret_cast<TLds *>(smem);
    unsigned char *ring = ring_base(smem);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int b = blockIdx.x;
    te_stamp(a, 0, threadIdx.x == 0);
    if (a.err[0]) return;   // an earlier launch timed out: the pass is garbage already, do not wait again
    if (tid == 0) {
        L.gflag = 0; L.ocnt = 0; L.cbar = 0; L.last = 0; L.full = 0;
        L.done[0] = L.done[1] = L.done[2] = L.done[3] = 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wv == 8) {
        loader_role<INFL>(L, ring, a, b, lane);
        te_stamp(a, 14, lane == 0);
        return;
    }
    if (wv >= 4) {
        comm_role<true>(L, a, tid, lane, wv, b);
        return;
    }
    // ================= consumer waves =================
    const int w = wv;
    const unsigned tag = (unsigned)a.epoch[0] * 32u + (unsigned)a.layer + 1u;   // (comm_role's tag)
    const int h = b >> 5, j32 = b & 31;
    float yres[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) yres[r] = a.x_in[8 * b + w + 4 * r];
    float xr[32];
    // q|k|v rows
    bool ok = gemv_wait(L, 1);
    load_xr(L.xs, xr, lane);
    float aq[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) aq[s] = ring_row(L, ring, s, w, xr, lane, ok);
    // (lane s publishes row 4 s + w of the workgroup's q|k|v list)
    if (lane < 4) {
        const float v = lane == 0 ? aq[0] : lane == 1 ? aq[1] : lane == 2 ? aq[2] : aq[3];
        put_granule(a.g_qkv + qkv_row(h, 16 * j32 + 4 * lane + w), tag, v);
    }
    gemv_done(L, lane);
    te_stamp(a, 2, tid == 0);
    // O rows + residual
    ok &= gemv_wait(L, 2);
    load_xr(L.xs, xr, lane);
    float xm[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) xm[s] = yres[s] + ring_row(L, ring, 4 + s, w, xr, lane, ok);
    if (lane < 2) put_granule(a.g_x + 8 * b + w + 4 * lane, tag, lane == 0 ? xm[0] : xm[1]);
    gemv_done(L, lane);
    te_stamp(a, 7, tid == 0);
    // gate|up rows, SwiGLU: pair k = (gate slot 6 + 2k, up slot 7 + 2k)
    ok &= gemv_wait(L, 3);
    load_xr(L.xs, xr, lane);
    float hv[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const float g = ring_row(L, ring, 6 + 2 * k, w, xr, lane, ok);
        const float u = ring_row(L, ring, 7 + 2 * k, w, xr, lane, ok);
        hv[k] = (g / (1.0f + expf(-g))) * u;
    }
    // (lane k publishes pair k: gate row 48 b + w + 8 k)
    if (lane < 6) {
        float v = hv[0];
#pragma unroll
        for (int k = 1; k < 6; ++k) v = lane == k ? hv[k] : v;
        const int r = 48 * b + w + 8 * lane;
        put_granule(a.g_h + (r >> 3) * 4 + (r & 3), tag, v);
    }
    gemv_done(L, lane);
    te_stamp(a, 10, tid == 0);
    // down rows w, w + 4 + residual -> the layer output (read by the next launch)
    ok &= gemv_wait(L, 4);
    float sd[2] = {0.f, 0.f};
#pragma unroll 1
    for (int j = 0; j < 6; ++j) {
        const int i = 18 + j;
        ok &= slot_wait(L, i);
        const unsigned char *sl = ring + (i % RING) * SLOT;
        v4u wr[2][2];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int k = 0; k < 2; ++k) wr[r][k] = reinterpret_cast<const v4u *>(sl + 2048 * (w + 4 * r))[lane + 64 * k];
        slot_release(L, w, i, lane);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const float *hx = L.hs + 8 * (lane + 64 * (2 * j + k));
            float x8[8];
            const float4 a0 = *reinterpret_cast<const float4 *>(hx), a1 = *reinterpret_cast<const float4 *>(hx + 4);
            x8[0] = a0.x; x8[1] = a0.y; x8[2] = a0.z; x8[3] = a0.w; x8[4] = a1.x; x8[5] = a1.y; x8[6] = a1.z; x8[7] = a1.w;
#pragma unroll
            for (int r = 0; r < 2; ++r) sd[r] += dot8r(wr[r][k], x8);
        }
    }
    float xo[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) xo[r] = xm[r] + wave_sum(sd[r]);
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < 2; ++r) a.x_out[8 * b + w + 4 * r] = xo[r];
        if (!ok) give_up(a.err, 12);
    }
    te_stamp(a, 12, tid == 0);
}

}  // namespace

bool qtts_tlayer_dims_ok(int H_, int NH_, int KV_, int HD_, int I_) {
    return H_ == H && NH_ == NH && KV_ == KVH && HD_ == HD && I_ == IM;
}
size_t qtts_tlayer_lds() { return sizeof(TLds); }
static size_t ring_lds() { return ((sizeof(TLds) + 15) & ~size_t(15)) + (size_t)RING * SLOT; }

// mode 1: the register form (k_tlayer); 2 / 3: the ring engine with 1 / 2
// slots left in flight after each issue (k_tlayer_ring<2> / <3>)
int qtts_tlayer(const TLayerArgs &a, hipStream_t st, int mode) {
    static bool attr[4] = {false, false, false, false};
    const void *fn = mode == 1 ? (const void *)k_tlayer : mode == 2 ? (const void *)k_tlayer_ring<2>
                                                                    : (const void *)k_tlayer_ring<3>;
    const size_t lds = mode == 1 ? sizeof(TLds) : ring_lds();
    if (mode < 1 || mode > 3) return -1;
    if (!attr[mode]) {
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -1;
        attr[mode] = true;
    }
    if (mode == 1) {
        hipLaunchKernelGGL(k_tlayer, dim3(256), dim3(512), lds, st, a);
        qtts_last_kernel = "k_tlayer";
    } else if (mode == 2) {
        hipLaunchKernelGGL(k_tlayer_ring<2>, dim3(256), dim3(RING_THREADS), lds, st, a);
        qtts_last_kernel = "k_tlayer_ring<2>";
    } else {
        hipLaunchKernelGGL(k_tlayer_ring<3>, dim3(256), dim3(RING_THREADS), lds, st, a);
        qtts_last_kernel = "k_tlayer_ring<3>";
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
