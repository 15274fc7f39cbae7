// k_gemvm.hip - lock-step batch decode GEMV (2..16 utterances) on the bf16
// matrix cores.
//
// y[b, r] = epilogue( sum_c W[r, c] * xin[b, c] ),  b < nb <= 16
//
// Replaces, for the batched decode of SURVEY.md 8e (B utterances per GPU in
// lock step), the per-utterance kernel_matvec_bf16 / kernel_swiglu_matvec_bf16
// calls (K.c:95-149, 213-233) and the rms_norm / residual passes around them
// (T.c:142-247): one weight read per frame serves every utterance.
//
// Why the matrix cores: at batch B a weight element costs B multiply-adds.
// On the VALU with x in LDS that is 2·B bytes of LDS reads per weight byte
// and 8·B FMAs per 16-B load (k_gemv<NB> ran at 250 GB/s for B = 8).  One
// v_mfma_f32_16x16x32_bf16 instead applies a 16-row x 32-column weight
// fragment to all 16 batch rows at once.
//
// Exact products ("3 x bf16", as k_mgemm.hip): x = x1 + x2 + x3 with
// x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2); bf16 x bf16
// products are exact in fp32, so the sum differs from an fp32 GEMV only in
// summation order (the GEMV bar of tests/test_gpu_kernels.py).
//
// Mapping: one workgroup = 16 weight rows (the MFMA B/N side) x all nb batch
// rows (A/M side, padded to 16 with zeros).  The 4 waves take 32-column K
// steps round-robin; lane l loads W[r0 + (l & 15)][32 s + 8 (l >> 4) .. +7]
// (one 16-B load = the B fragment) and reads x[l & 15][same columns] of the
// three planes from LDS (the A fragments).  Weight loads run U steps ahead in
// registers, the first group issued right behind the prologue's own loads.
// The KS partial 16x16 tiles are summed in wave order through LDS; the
// tile's first wave applies the epilogue.
//
// Load order (loads retire in issue order, so a load waits for every load
// issued before it): x rows / table rows, split-K partials and norm weights
// first, then the weight group, all through buffer descriptors (32-bit
// offsets) and with no branch between them -- the kernel is specialised on
// the source kind (GM_SRC_*), because a branch between differently-loading
// paths makes the compiler drain every outstanding load, the weights
// included, at the join.  (The former per-unit loader did exactly that for
// every x unit: batch 8 117.1 -> 123.4 audio-s/s.)
//
// Prologue: the nb x rows (fp32 rows, or bf16 / fp32 table rows gathered by
// device-side ids) are RMS-normalised (K.c:27-39, x * inv * w), split once and
// stored as three bf16 planes in LDS, so the K loop is loads + MFMAs only.
// Whole rows up to 16 float4 per thread go through registers (one barrier
// for the statistics); longer ones (the down projections at B >= 8) are staged
// in column chunks after a statistics pre-pass.
#include <algorithm>

#include "qtts_gemvm_dev.h"

namespace {

using qtts_gm::lo_f;
using qtts_gm::hi_f;
#define gm_rsrc qtts_gm::rsrc
#define gm_ld4 qtts_gm::ld4

// id of the table row that batch row b reads
__device__ __forceinline__ int gm_row_id(const GemvArgs &a, int b) {
    const int *p = a.ids + (size_t)b * a.ids_bstride + a.ids_off;
    if (a.row_sel) p += (size_t)a.row_sel[b] * a.ids_rstride;
    return *p;
}

// x = x1 + x2 + x3 (each bf16, exact) for 4 values -> the three planes
__device__ __forceinline__ void split_store(float4 v, unsigned short *hp, int plane_stride) {
    uint2 p1, p2, p3;
    qtts_gm::split4(v, p1, p2, p3);
    *reinterpret_cast<uint2 *>(hp) = p1;
    *reinterpret_cast<uint2 *>(hp + plane_stride) = p2;
    *reinterpret_cast<uint2 *>(hp + 2 * plane_stride) = p3;
}

struct NoIssue { __device__ __forceinline__ void operator()() const {} };

// Source loads of N float4 units (unit i: batch row i / n4, columns c0 +
// 4 (i % n4); a unit at or past nu reads unit 0's address and is ignored by
// the caller).  Every load of the batch is issued before any is used: loads
// retire in issue order, so a load issued behind another waits for it (the
// former per-unit loader, branching on the source kind around each load,
// waited for the whole previous load -- the weight group included -- before
// every unit).  Order: x / table rows, the split-K partials p < PM (held in
// registers), the norm weights (NW), then `issue` (the weight stream); then
// the partials are summed in order p = 0, 1, ... (p >= PM read from memory)
// and added to the residual, as GemvArgs::xadd prescribes.
// (buffer-descriptor loads: qtts_gm::rsrc / ld4, 32-bit offsets, cdna_hip_programming.md T8 / T20)

// Source kinds (GM_SRC_*): a kernel specialised on one has no branch between
// its loads, so the compiler's vmcnt bookkeeping stays exact (a uniform
// branch between source kinds that issue different loads into different
// registers makes it wait for every outstanding load -- the weights
// included -- at the join); GM_SRC_ANY decides at run time (generic path).
enum { GM_SRC_X = 0, GM_SRC_XADD = 1, GM_SRC_TAB = 2, GM_SRC_TABF = 3, GM_SRC_ANY = 4 };

template <int SRC>
__device__ __forceinline__ bool gm_is(const GemvArgs &a, int kind) {
    if constexpr (SRC != GM_SRC_ANY) return SRC == kind;
    switch (kind) {
        case GM_SRC_TAB: return a.table != nullptr;
        case GM_SRC_TABF: return a.table == nullptr && a.table_f32 != nullptr;
        case GM_SRC_XADD: return !a.table && !a.table_f32 && a.xadd != nullptr;
        default: return !a.table && !a.table_f32 && a.xadd == nullptr;
    }
}

template <int SRC, int N, int PM, bool NW, class Issue>
__device__ __forceinline__ void gm_fetch(const GemvArgs &a, int i0, int step, int nu, int n4, int c0,
                                         float4 (&v)[N], float4 (&nw)[N], Issue issue) {
    // element offsets (every source here is far below 2^29 elements)
    unsigned b[N], c[N];
#pragma unroll
    for (int u = 0; u < N; ++u) {
        int i = i0 + step * u;
        i = i < nu ? i : 0;
        b[u] = (unsigned)(i / n4);
        c[u] = (unsigned)(c0 + 4 * (i - (int)b[u] * n4));
    }
    const bool tab = gm_is<SRC>(a, GM_SRC_TAB), tabf = gm_is<SRC>(a, GM_SRC_TABF), xadd = gm_is<SRC>(a, GM_SRC_XADD);
    const int np = xadd ? a.n_xadd : 0;
    float4 pv[N][PM];
    uint2 tq[N];
    if (tab || tabf) {
        // ids: the row selectors of all units, then the ids (two round trips)
        unsigned id[N];
        const int *ip = a.ids + a.ids_off;
        if (a.row_sel) {
            int rs[N];
#pragma unroll
            for (int u = 0; u < N; ++u) rs[u] = a.row_sel[b[u]];
#pragma unroll
            for (int u = 0; u < N; ++u)
                id[u] = (unsigned)ip[b[u] * (unsigned)a.ids_bstride + (unsigned)rs[u] * (unsigned)a.ids_rstride];
        } else {
#pragma unroll
            for (int u = 0; u < N; ++u) id[u] = (unsigned)ip[b[u] * (unsigned)a.ids_bstride];
        }
        if (tab) {
            const auto rt = gm_rsrc(a.table);
#pragma unroll
            for (int u = 0; u < N; ++u) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b64(rt, (id[u] * (unsigned)a.C + c[u]) * 2u, 0, 0);
                tq[u] = make_uint2(q[0], q[1]);
            }
        } else {
            const auto rt = gm_rsrc(a.table_f32);
#pragma unroll
            for (int u = 0; u < N; ++u) v[u] = gm_ld4(rt, id[u] * (unsigned)a.C + c[u]);
        }
    } else {
        const auto rx = gm_rsrc(a.x);
#pragma unroll
        for (int u = 0; u < N; ++u) v[u] = gm_ld4(rx, b[u] * (unsigned)a.ldx + c[u]);
        if (xadd) {
            // partials p < PM: unconditional loads (p clamped to the last one),
            // only the sum below looks at np
            const auto rp = gm_rsrc(a.xadd);
#pragma unroll
            for (int p = 0; p < PM; ++p) {
                const unsigned pp = (unsigned)(p < np ? p : np - 1);
#pragma unroll
                for (int u = 0; u < N; ++u)
                    pv[u][p] = gm_ld4(rp, pp * (unsigned)a.ld_xadd + b[u] * (unsigned)a.ldb_xadd + c[u]);
            }
        }
    }
    if constexpr (NW) {
        if (a.norm_w) {
            const auto rn = gm_rsrc(a.norm_w);
#pragma unroll
            for (int u = 0; u < N; ++u) nw[u] = gm_ld4(rn, c[u]);
        }
    }
    issue();
    if (tab) {
#pragma unroll
        for (int u = 0; u < N; ++u) v[u] = make_float4(lo_f(tq[u].x), hi_f(tq[u].x), lo_f(tq[u].y), hi_f(tq[u].y));
    } else if (xadd) {   // (tables carry no partials: host check)
        const auto rp = gm_rsrc(a.xadd);
#pragma unroll
        for (int u = 0; u < N; ++u) {
            float4 s = pv[u][0];
#pragma unroll
            for (int p = 1; p < PM; ++p)
                if (p < np) { s.x += pv[u][p].x; s.y += pv[u][p].y; s.z += pv[u][p].z; s.w += pv[u][p].w; }
            for (int p = PM; p < np; ++p) {
                const float4 t = gm_ld4(rp, (unsigned)p * (unsigned)a.ld_xadd + b[u] * (unsigned)a.ldb_xadd + c[u]);
                s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
            }
            v[u].x += s.x; v[u].y += s.y; v[u].z += s.z; v[u].w += s.w;
        }
    }
}

// normalise (inv / norm weights nw), copy out (workgroup 0), split into the planes
__device__ __forceinline__ void gm_put(const GemvArgs &a, float4 v, float4 nw, int b, int c, int cl, float iv,
                                       unsigned short *hp, int LDH, int PS) {
    if (a.xcopy && blockIdx.x == 0 && !a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + (size_t)b * a.ldxc + c) = v;
    if (a.norm_w) {
        v.x = v.x * iv * nw.x; v.y = v.y * iv * nw.y; v.z = v.z * iv * nw.z; v.w = v.w * iv * nw.w;
        if (a.xcopy && blockIdx.x == 0 && a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + (size_t)b * a.ldxc + c) = v;
    }
    split_store(v, hp + b * LDH + cl, PS);
}

// stage columns [c0, c0 + CCH) of the nb rows (chunked / generic path), 2
// units per thread in flight (the chunked stage runs with a weight group live)
__device__ __forceinline__ void gm_stage(const GemvArgs &a, const float *inv, unsigned short *hp, int LDH, int PS,
                                         int c0, int CCH) {
    const int n4 = CCH / 4, nu = a.nb * n4, nt = blockDim.x;
    for (int i0 = threadIdx.x; i0 < nu; i0 += 2 * nt) {
        float4 v[2], nw[2];
        gm_fetch<GM_SRC_ANY, 2, 1, true>(a, i0, nt, nu, n4, c0, v, nw, NoIssue());
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = i0 + nt * u;
            if (i < nu) {
                const int b = i / n4, cl = 4 * (i - b * n4);
                gm_put(a, v[u], nw[u], b, c0 + cl, cl, a.norm_w ? inv[b] : 1.f, hp, LDH, PS);
            }
        }
    }
}

// A workgroup = TPW row tiles of 16 rows x KS waves per tile (the K steps of a
// tile dealt round-robin to its KS waves).
// XU > 0: register prologue (whole rows, C % 256 == 0, <= XU float4 units per
// thread: unit i = tid + blockDim*q, wave-uniform batch row); the per-64-unit
// partial sums of squares of a row are adjacent and summed in order.
// XU == 0: statistics pre-pass + (chunked) staging.
template <int U, int XU, int KS, int SRC>
__global__ __launch_bounds__(1024) void k_gemvm(GemvArgs a, int tpw) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nthr = blockDim.x, nw = nthr >> 6;
    // split-K producer: this workgroup column takes K columns [off, off + C / kz)
    const int ldw = a.C;
    int woff = 0;
    if (gridDim.y > 1) {
        const int ce = a.C / gridDim.y;
        woff = blockIdx.y * ce;
        a.x += woff;
        if (a.xadd) a.xadd += woff;
        a.C = ce;
    }
    const int nb = a.nb, C = a.C, CCH = a.cch, LDH = CCH + 8, PS = nb * LDH;
    const bool chunked = CCH < C;
    unsigned short *hp = reinterpret_cast<unsigned short *>(smem);        // [3][nb][LDH] bf16 planes
    floatx4 *red = reinterpret_cast<floatx4 *>(smem);                     // [nw][64] (after the K loop)
    const int region = max(3 * PS * 2, nw * 64 * 16) / 4;                 // floats
    float *inv = smem + region;                                           // [16]
    float *part = inv + 16;                                               // [nb * C / 256]

    const int tw = w / KS, ksl = w - tw * KS;                             // tile, K slice of this wave
    const int tile = blockIdx.x * tpw + tw;
    const int r0 = tile * 16, rl = lane & 15, kq = 8 * (lane >> 4);
    const int row = r0 + rl < a.R ? r0 + rl : a.R - 1;
    // weights through a buffer descriptor: one 32-bit offset per lane (host: R * C * 2 < 2^31)
    const auto rw = gm_rsrc(a.W);

    const int nsteps = C / 32;
    const int J = r0 < a.R ? (nsteps - ksl + KS - 1) / KS : 0;   // this wave's K steps: s = ksl + KS * j
    const int ng = (J + U - 1) / U;
    // (a wave with no K step, J == 0, still issues its loads unconditionally:
    // they read the row's first step)
    const unsigned wb = ((unsigned)row * (unsigned)ldw + (unsigned)(woff + kq + (J > 0 ? 32 * ksl : 0))) * 2u;
    const int spc = CCH / 32 / KS;                    // steps per wave per chunk (chunked mode)

    v4u wv[U];
    auto load = [&](int g) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int j = g * U + u;
            j = j < J ? j : (J > 0 ? J - 1 : 0);     // clamp: loads stay unconditional (row is clamped too)
            // default policy: non-temporal loads of these 64-B row fragments measured 5-20 % slower
            wv[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rw, wb + (unsigned)(64 * KS * j), 0, 0));
        }
    };
    // ---- prologue
    if constexpr (XU > 0) {
        const int n4 = C / 4, nu = nb * n4;
        // the x rows, their partials and norm weights first, then the weights
        // (partials in registers: XU * PM <= 8 float4; above 4 units the norm
        // weights come behind the weights, so x, partials and weights fit)
        constexpr int PM = XU <= 2 ? 4 : 2;
        constexpr bool NWE = XU <= 4;
        float4 xv[XU], nwv[XU];
        // (load(0) unconditional: a divergent branch around it would make the
        // compiler's vmcnt bookkeeping wait for the weights at every x use)
        gm_fetch<SRC, XU, PM, NWE>(a, tid, nthr, nu, n4, 0, xv, nwv, [&]() { load(0); });
        if constexpr (!NWE) {
            if (a.norm_w) {
                // offsets recomputed from an opaque copy of tid: reusing the
                // fetch's (spilled) ones would reload them from scratch, and a
                // scratch load makes the next wait drain the weights too
                int t = tid;
                asm volatile("" : "+v"(t));
#pragma unroll
                for (int q = 0; q < XU; ++q) {
                    int i = t + nthr * q;
                    i = i < nu ? i : 0;
                    nwv[q] = gm_ld4(gm_rsrc(a.norm_w), 4u * (unsigned)(i % n4));
                }
            }
        }
        if (a.norm_w) {
#pragma unroll
            for (int q = 0; q < XU; ++q) {
                const int i = tid + nthr * q;
                const float4 v = xv[q];
                const float ss = wave_sum(i < nu ? v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w : 0.f);
                if (lane == 0 && i < nu) part[(i >> 6)] = ss;
            }
            __syncthreads();
            if (tid < nb) {   // row tid: its C / 256 adjacent partials, in order
                const int np = C / 256;
                float ss = 0.f;
                for (int k = 0; k < np; ++k) ss += part[tid * np + k];
                inv[tid] = rms_inv(ss, C, a.eps);
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < XU; ++q) {
            const int i = tid + nthr * q;
            if (i < nu) {
                const int bb = i / n4, c = 4 * (i % n4);
                gm_put(a, xv[q], nwv[q], bb, c, c, a.norm_w ? inv[bb] : 1.f, hp, LDH, PS);
            }
        }
    } else {
        load(0);
        if (a.norm_w) {
            const int n4 = C / 4;
            for (int bb = w; bb < nb; bb += nw) {
                float ss = 0.f;
                for (int k0 = lane; k0 < n4; k0 += 4 * 64) {   // columns 4 k, k = k0 + 64 u, in order
                    float4 v[4], nwd[4];
                    gm_fetch<GM_SRC_ANY, 4, 1, false>(a, bb * n4 + k0, 64, bb * n4 + n4, n4, 0, v, nwd, NoIssue());
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (k0 + 64 * u < n4) ss += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
                }
                ss = wave_sum(ss);
                if (lane == 0) inv[bb] = rms_inv(ss, C, a.eps);
            }
            __syncthreads();
        }
        gm_stage(a, inv, hp, LDH, PS, 0, CCH);
    }
    __syncthreads();

    // ---- weight stream x MFMA (A = the x planes, B = the weight fragment)
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    const int tb = lane & 15;        // batch row of this lane's A fragment
    int cur_ch = 0;
    const int ngm = chunked ? (nsteps / KS + U - 1) / U : ng;   // chunked: every wave runs the same groups
    for (int g = 0; g < ngm; ++g) {
        v4u cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = wv[u];
        if (g + 1 < ng) load(g + 1);
        int cbase = 0;
        if constexpr (XU == 0) {
            if (chunked) {   // spc steps per wave per chunk, spc % U == 0 (host)
                const int ch = (g * U) / spc;
                if (ch != cur_ch) {
                    __syncthreads();
                    gm_stage(a, inv, hp, LDH, PS, ch * CCH, CCH);
                    __syncthreads();
                    cur_ch = ch;
                }
                cbase = cur_ch * CCH;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = g * U + u;
            if (j < J) {
                bf16x8 h1, h2, h3;
                if (tb < nb) {
                    const unsigned short *xp = hp + tb * LDH + 32 * (ksl + KS * j) - cbase + kq;
                    h1 = *reinterpret_cast<const bf16x8 *>(xp);
                    h2 = *reinterpret_cast<const bf16x8 *>(xp + PS);
                    h3 = *reinterpret_cast<const bf16x8 *>(xp + 2 * PS);
                } else {
                    h1 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
                    h2 = h1;
                    h3 = h1;
                }
                const bf16x8 bw = __builtin_bit_cast(bf16x8, cur[u]);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h1, bw, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h2, bw, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h3, bw, acc, 0, 0, 0);
            }
        }
    }

    // ---- a tile's KS partials, summed in wave order; epilogue by its first wave
    __syncthreads();   // the planes are dead: red aliases them
    red[w * 64 + lane] = acc;
    __syncthreads();
    if (a.tick) {      // self-reducing split-K producer (every thread reaches the ticket barrier)
        if (ksl == 0 && r0 < a.R) {
            floatx4 v = red[w * 64 + lane];
#pragma unroll
            for (int k = 1; k < KS; ++k) v += red[(w + k) * 64 + lane];
            const int r = r0 + rl;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int bb = 4 * (lane >> 4) + i;
                if (bb < nb && r < a.R) st_sc1(a.ypart + blockIdx.y * a.ld_ypart + (size_t)bb * a.R + r, v[i]);
            }
        }
        qtts_gm::reduce_last(a, 16 * tpw, reinterpret_cast<int *>(inv));
        return;
    }
    if (ksl != 0 || r0 >= a.R) return;
    floatx4 v = red[w * 64 + lane];
#pragma unroll
    for (int k = 1; k < KS; ++k) v += red[(w + k) * 64 + lane];
    const int r = r0 + rl;   // D: column = lane & 15 (weight row), row = 4 (lane >> 4) + i (batch row)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int bb = 4 * (lane >> 4) + i;
        const float val = v[i];
        // lane + 4 within the 16-lane row (row_shl:4; lanes 12-15 keep their own, unused)
        const float up = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(val), __float_as_int(val), 0x104, 0xF, 0xF, false));
        if (bb >= nb || r >= a.R) continue;
        if (a.ypart) {
            a.ypart[blockIdx.y * a.ld_ypart + (size_t)bb * a.R + r] = val;
            continue;
        }
        qtts_gm::epilogue(a, bb, r, val, up);
    }
}

}  // namespace

// LDS budget for the three bf16 planes of the staged x rows (bytes): one
// workgroup per CU at the largest.
static constexpr int GM_PLANES_MAX = 150 * 1024;
static int gm_planes(int nb, int cch) { return 3 * nb * (cch + 8) * 2; }

// Returns 1 when the shape is not covered (the caller uses k_gemv), 0 ok,
// -1 launch error.
int qtts_gemvm(const GemvArgs &in, hipStream_t st) {
    GemvArgs a = in;
    if (a.nb < 2 || a.nb > 16 || a.R % 16 || a.C % 32 || (size_t)a.R * a.C * 2 >= ((size_t)1 << 31)) return 1;
    if (a.table) {
        if (a.C % 4) return 1;
    } else if (a.table_f32) {
        if ((uintptr_t)a.table_f32 & 15) return 1;
    } else if (!a.x || a.ldx % 4 || ((uintptr_t)a.x & 15)) {
        return 1;
    }
    if (a.norm_w && ((uintptr_t)a.norm_w & 15)) return 1;
    if (a.xcopy && (a.ldxc % 4 || ((uintptr_t)a.xcopy & 15))) return 1;
    if (a.xadd && (a.table || a.table_f32 || ((uintptr_t)a.xadd & 15) || a.ld_xadd % 4 || a.ldb_xadd % 4 ||
                   a.n_xadd < 1))
        return 1;
    const int kz = a.ypart ? a.kz : 1;
    if (a.ypart && (kz < 2 || (a.tick && kz > 4) || a.norm_w || a.table || a.table_f32 || a.xcopy || a.C % (32 * kz) ||
                    ((uintptr_t)a.ypart & 3)))
        return 1;
    const int Cfull = a.C;
    a.C /= kz;   // the K extent one workgroup column takes (host-side configuration only)
    // 16 waves per workgroup where the shape allows (one workgroup per CU):
    // KS waves per tile keep >= 2 K steps each; TPW tiles per workgroup bring
    // the grid to about one round over the 256 CUs (the x prologue is paid
    // once per workgroup)
    const int nsteps = a.C / 32, T = a.R / 16;
    int tpw = (T + 255) / 256;
    if (tpw > 4) tpw = 4;
    int KS = 16 / (tpw == 3 ? 4 : tpw);
    while (KS > 4 && nsteps < 2 * KS) KS /= 2;
    if (tpw * KS > 16) tpw = 16 / KS;
    // three tiles x 4 waves leave 768 threads, so > 4 x units per thread at
    // batch >= 8 (whose registers, with the partials and the weight group in
    // flight, spill): four tiles per 1024-thread workgroup instead
    if (tpw == 3 && (a.nb * a.C / 4 + 767) / 768 > 4) { tpw = 4; KS = 4; }
    // column chunk: the whole row when it fits, else the fewest equal chunks
    // of whole 32 x KS-column step rounds with an even step count per wave
    int cch = a.C;
    if (gm_planes(a.nb, a.C) > GM_PLANES_MAX) {
        const int unit = 32 * KS;
        if (a.C % unit) return 1;
        int n = 2;
        for (; n <= a.C / unit; ++n)
            if ((a.C / unit) % n == 0 && gm_planes(a.nb, a.C / n) <= GM_PLANES_MAX && (a.C / unit / n) % 2 == 0)
                break;
        if (n > a.C / unit) return 1;
        cch = a.C / n;
    }
    a.cch = cch;
    int U;
    if (cch < a.C) {
        const int spc = cch / 32 / KS;
        U = spc % 8 == 0 ? 8 : spc % 4 == 0 ? 4 : 2;
    } else {
        const int J = (nsteps + KS - 1) / KS;
        U = J <= 2 ? 2 : J <= 4 ? 4 : 8;
    }
    const int nthr = 64 * KS * tpw, nu = a.nb * a.C / 4;
    const int xu = (cch == a.C && a.C % 256 == 0) ? (nu + nthr - 1) / nthr : 0;
    const int XU = xu == 0 || xu > 8 ? 0 : xu <= 1 ? 1 : xu <= 2 ? 2 : xu <= 4 ? 4 : xu <= 6 ? 6 : 8;
    const int region = std::max(gm_planes(a.nb, cch), nthr / 64 * 64 * 16);
    const size_t smem = (size_t)region + (16 + (a.nb * a.C / 256 > 64 ? a.nb * a.C / 256 : 64)) * 4;
    const dim3 grid((T + tpw - 1) / tpw, kz);
    a.C = Cfull;
    if (a.tick && (!a.ypart || !a.y || a.epi != EPI_RESID || (int)grid.x > QTTS_GM_TICKS)) {
        fprintf(stderr, "qtts_gemvm: self-reducing split-K needs ypart, y, EPI_RESID and <= %d row blocks\n",
                QTTS_GM_TICKS);
        return -1;
    }
    const int src = a.table ? GM_SRC_TAB : a.table_f32 ? GM_SRC_TABF : a.xadd ? GM_SRC_XADD : GM_SRC_X;
#define QTTS_GMS(UU, XX, KK, SS)                                                                              \
    hipLaunchKernelGGL((k_gemvm<UU, XX, KK, SS>), grid, dim3(nthr), smem, st, a, tpw);                        \
    qtts_last_kernel = "k_gemvm<" #UU ", " #XX ", " #KK ", " #SS ">";
#define QTTS_GM(UU, XX, KK)                                                                                   \
    if (src == GM_SRC_X) { QTTS_GMS(UU, XX, KK, GM_SRC_X) }                                                   \
    else if (src == GM_SRC_XADD) { QTTS_GMS(UU, XX, KK, GM_SRC_XADD) }                                        \
    else if (src == GM_SRC_TAB) { QTTS_GMS(UU, XX, KK, GM_SRC_TAB) }                                          \
    else { QTTS_GMS(UU, XX, KK, GM_SRC_TABF) }
#define QTTS_GMX(UU, KK)                                       \
    if (XU == 1) { QTTS_GM(UU, 1, KK) }                        \
    else if (XU == 2) { QTTS_GM(UU, 2, KK) }                   \
    else if (XU == 4) { QTTS_GM(UU, 4, KK) }                   \
    else if (XU == 6) { QTTS_GM(UU, 6, KK) }                   \
    else if (XU == 8) { QTTS_GM(UU, 8, KK) }                   \
    else { QTTS_GMS(UU, 0, KK, GM_SRC_ANY) }
#define QTTS_GMK(UU)                                           \
    if (KS == 16) { QTTS_GMX(UU, 16) }                         \
    else if (KS == 8) { QTTS_GMX(UU, 8) }                      \
    else { QTTS_GMX(UU, 4) }
    if (U == 8) { QTTS_GMK(8) }
    else if (U == 4) { QTTS_GMK(4) }
    else { QTTS_GMK(2) }
#undef QTTS_GMK
#undef QTTS_GMX
#undef QTTS_GMS
#undef QTTS_GM
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#undef gm_rsrc
#undef gm_ld4
