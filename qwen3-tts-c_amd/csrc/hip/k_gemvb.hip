// k_gemvb.hip - lock-step batch decode GEMV (2..16 utterances) on the bf16
// matrix cores, with the activation rows SLICED PER WAVE.
//
// y[b, r] = epilogue( inv[b] * sum_c W[r, c] * (x[b, c] * nw[c]) ),  b < nb <= 16
//
// Role: the same as k_gemvm (the per-utterance kernel_matvec_bf16 /
// kernel_swiglu_matvec_bf16 calls and the rms_norm / residual passes around
// them, K.c:27-39, 95-149, 213-233, T.c:142-247, batched so that one weight
// read per frame serves all B utterances), with the prologue taken off the
// critical path.  k_gemvm stages all nb rows of x in every workgroup as three
// bf16 planes in LDS: a full-row load, the RMS statistic, the split and three
// barriers before the first MFMA -- the part of the launch that made the
// batch-8 GEMVs 1.5-2.9x their batch-1 time (profiles/r02r_batch_gemvm_decomp.txt).
//
// Mapping: a workgroup = TPW tiles of 16 weight rows x W waves; wave w owns the
// contiguous K slice [32 SPW w, 32 SPW (w + 1)) for ALL the workgroup's tiles,
// so its slice of x is private to it:
//   1. every load is issued at once, in retire order: the slice of x (nb rows
//      x 32 SPW columns, coalesced float4 units) or the table rows by id,
//      the split-K partials, the norm weights, then the weight fragments of
//      the first half of the steps; then the second half once x is staged
//      (its registers are the partials' by then);
//   2. x (+ partials, in order) * nw goes to the wave's own LDS rows as fp32
//      (no barrier: one wave writes and reads it), the per-row sum of squares
//      of the slice to an LDS table;
//   3. per 32-column step the wave reads its MFMA A fragments (row lane & 15,
//      columns 8 (lane >> 4) .. +7), splits them into three exact bf16 planes
//      in registers and runs v_mfma_f32_16x16x32_bf16 against each tile's
//      weight fragment (B: weight row lane & 15);
//   4. ONE barrier; wave t sums tile t's W partial tiles in wave order, scales
//      batch row b by inv[b] = 1 / sqrt(sum_w ss[w][b] / C + eps) and applies
//      the epilogue.
// RMSNorm is applied after the dot product: sum_c W (x inv nw) = inv sum_c W
// (x nw), so the statistic is off the path to the first MFMA.  The rounding
// differs from the reference's (x * inv) * w by that reassociation only
// (fp32, within the GEMV bar of tests/test_gpu_kernels.py); the products are
// exact (3 x bf16 planes, as k_gemvm / k_mgemm).
#include <algorithm>

#include "qtts_gemvm_dev.h"

namespace {

using namespace qtts_gm;

enum { GB_SRC_X = 0, GB_SRC_XADD = 1, GB_SRC_TAB = 2, GB_SRC_TABF = 3 };

// id of the table row that batch row b reads (ids: a.ids + a.ids_off)
__device__ __forceinline__ unsigned gb_row_id(const GemvArgs &a, const int *ids, int b) {
    const int *p = ids + (size_t)b * a.ids_bstride;
    if (a.row_sel) p += (size_t)a.row_sel[b] * a.ids_rstride;
    return (unsigned)*p;
}

// SPW: 32-column K steps per wave; TPW: 16-row tiles per workgroup; NBC: 8 or
// 16 (batch rows covered: the x units per lane are SPW * NBC / 8); PM:
// split-K partials added to x (0, 2 or 4; n_xadd <= PM); SRC: x source kind
// (the kernel is specialised on it: a branch between loads of different kinds
// makes the compiler wait for every outstanding load at the join).
// diagnostic phase stamps (GemvArgs::dbg, QTTS_HIP_GM_DBG; compiled in only
// with `make EXTRA=-DQTTS_STAMPS`: the stores cost registers): 100 MHz wall
// clock, one lane
__device__ __forceinline__ void gb_stamp(const GemvArgs &a, int k) {
#ifdef QTTS_STAMPS
    if (a.dbg && threadIdx.x == 0) a.dbg[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + k] = __builtin_amdgcn_s_memrealtime();
#endif
}

// (src -- a.x, a.table or a.table_f32 by SRC --, ids, W and xadd lead the
// arguments: preloaded into SGPRs, Makefile)
template <int SPW, int TPW, int NBC, int PM, int SRC>
__global__ __launch_bounds__(1024) void k_gemvb(const void *src, const int *ids, const bf16_t *Wt, const float *xadd,
                                                GemvArgs a) {
    gb_stamp(a, 0);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int SC = 32 * SPW;                 // columns of a wave's slice
    constexpr int U4 = SC / 4;                   // float4 units per slice row (8 SPW, divides 64)
    constexpr int XQ = SPW * NBC / 8;            // x units per lane
    constexpr int RPQ = 64 / U4;                 // slice rows per unit index q
    constexpr int LDX = SC + 4;                  // staged row stride (floats; +4: fragment reads spread over banks)
    // steps whose weights go before the staging (the rest reuse the partials'
    // registers).  Issuing every step before the staging where the registers
    // allow measured slower at batch 8 (139.8 / 140.2 vs 142.3 / 142.0
    // audio-s/s, same box) although the stamps show q|k|v's last wave
    // finishing 3.5 us after its first (profiles/r03i_batch8_gemvb_stamps.txt)
    // (SPW <= 2, the sub-talker's shapes: every step before the staging --
    // batch 8 152.5 / 153.2 / 152.6 vs 151.1 / 151.0 / 150.8 audio-s/s with
    // only the first, alternating processes, profiles/r05e_ab_prefetch_modes.txt)
    // (also every step of the partial-free SPW 4 / 8 shapes -- the talker's --
    // measured slower: batch 8 150.4-150.7 vs 152.0-152.6, batch 16 237.2 vs
    // 238.5, profiles/r05f_ab_batch_allw.txt)
    // (a quarter of the talker shapes' steps first measured slower too: batch 8
    // 155.6-155.7 vs 157.2-157.8, profiles/r05aa_ab_batch_steps_first.txt)
    constexpr int SA = SPW <= 2 ? SPW : (SPW + 1) / 2;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
    const int nb = a.nb;
    const int kz = gridDim.y, Ck = a.C / kz, woff = blockIdx.y * Ck;
    const int c0 = woff + w * SC;                // first column of this wave's slice
    const int r0 = blockIdx.x * (16 * TPW);
    const int wreg = max(nb * LDX, TPW * 256);   // floats per wave region (x rows, then the partial tiles)
    float *xs = smem + w * wreg;
    float *ssq = smem + W * wreg;                // [W][16] per-wave row sums of squares

    // ---- unit coordinates: unit q of this lane = slice row lane / U4 + RPQ q, float4 column lane % U4
    const int ucol = 4 * (lane % U4);            // column within the slice
    int urow[XQ];
    bool uok[XQ];
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
        const int b = lane / U4 + RPQ * q;
        uok[q] = b < nb;
        urow[q] = b < nb ? b : 0;                // clamped: every load is unconditional
    }
    const bool norm = a.norm_w != nullptr;

    // ---- 1. loads, in retire order
    float4 xv[XQ];
    float4 pv[XQ][PM > 0 ? PM : 1];
    uint2 tq[XQ];
    if constexpr (SRC == GB_SRC_TAB || SRC == GB_SRC_TABF) {
        unsigned id[XQ];
#pragma unroll
        for (int q = 0; q < XQ; ++q) id[q] = gb_row_id(a, ids, urow[q]);
        if constexpr (SRC == GB_SRC_TAB) {
            const auto rt = rsrc(src);
#pragma unroll
            for (int q = 0; q < XQ; ++q) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rt, (id[q] * (unsigned)a.C + (unsigned)(c0 + ucol)) * 2u, 0, 0);
                tq[q] = make_uint2(v[0], v[1]);
            }
        } else {
            const auto rt = rsrc(src);
#pragma unroll
            for (int q = 0; q < XQ; ++q) xv[q] = ld4(rt, id[q] * (unsigned)a.C + (unsigned)(c0 + ucol));
        }
    } else {
        const auto rx = rsrc(src);
#pragma unroll
        for (int q = 0; q < XQ; ++q) xv[q] = ld4(rx, (unsigned)urow[q] * (unsigned)a.ldx + (unsigned)(c0 + ucol));
        if constexpr (SRC == GB_SRC_XADD) {
            const auto rp = rsrc(xadd);
            const int np = a.n_xadd;
#pragma unroll
            for (int p = 0; p < PM; ++p) {
                const unsigned pp = (unsigned)(p < np ? p : np - 1);
#pragma unroll
                for (int q = 0; q < XQ; ++q)
                    pv[q][p] = ld4(rp, pp * (unsigned)a.ld_xadd + (unsigned)urow[q] * (unsigned)a.ldb_xadd +
                                           (unsigned)(c0 + ucol));
            }
        }
    }
    float4 nwv = make_float4(1.f, 1.f, 1.f, 1.f);
    if (norm) nwv = ld4(rsrc(a.norm_w), (unsigned)(c0 + ucol));
    // weight fragments: tile t, step j -> W[r0 + 16 t + (lane & 15)][c0 + 32 j + 8 (lane >> 4) .. +7]
    const auto rw = rsrc(Wt);
    v4u wv[TPW][SPW];
    unsigned wo[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        int row = r0 + 16 * t + (lane & 15);
        row = row < a.R ? row : a.R - 1;
        wo[t] = ((unsigned)row * (unsigned)a.C + (unsigned)(c0 + 8 * (lane >> 4))) * 2u;
    }
#pragma unroll
    for (int j = 0; j < SA; ++j)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
            wv[t][j] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rw, wo[t] + 64u * j, 0, 0));

    // ---- 2. x (+ partials) -> raw copy, x * nw -> the wave's LDS rows; sums of squares
    const bool copier = a.xcopy && blockIdx.x == 0 && blockIdx.y == 0;
    float ss[XQ];
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
        float4 v;
        if constexpr (SRC == GB_SRC_TAB) v = make_float4(lo_f(tq[q].x), hi_f(tq[q].x), lo_f(tq[q].y), hi_f(tq[q].y));
        else v = xv[q];
        if constexpr (SRC == GB_SRC_XADD) {   // x + (p0 + p1 + ...), as GemvArgs::xadd prescribes
            const int np = a.n_xadd;
            float4 s = pv[q][0];
#pragma unroll
            for (int p = 1; p < PM; ++p)
                if (p < np) { s.x += pv[q][p].x; s.y += pv[q][p].y; s.z += pv[q][p].z; s.w += pv[q][p].w; }
            v.x += s.x; v.y += s.y; v.z += s.z; v.w += s.w;
        }
        float4 *xc = reinterpret_cast<float4 *>(a.xcopy + (size_t)urow[q] * a.ldxc + c0 + ucol);
        if (copier && uok[q] && !a.xcopy_normed) *xc = v;
        ss[q] = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        v.x *= nwv.x; v.y *= nwv.y; v.z *= nwv.z; v.w *= nwv.w;
        if (copier && uok[q] && a.xcopy_normed) *xc = v;   // x * nw; scaled by inv after the barrier
        if (uok[q]) *reinterpret_cast<float4 *>(xs + urow[q] * LDX + ucol) = v;
    }
    if (norm) {
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const float s = group_sum<U4>(ss[q]);   // the U4 lanes of slice row lane / U4 + RPQ q
            if (lane % U4 == 0 && uok[q]) ssq[w * 16 + urow[q]] = s;
        }
    }
    // the second half of the weight fragments (registers of the partials, now summed)
#pragma unroll
    for (int j = SA; j < SPW; ++j)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
            wv[t][j] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rw, wo[t] + 64u * j, 0, 0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // one wave writes and reads its rows: LDS is in order
    gb_stamp(a, 1);

    // ---- 3. per step: A fragments (three exact planes) x each tile's weight fragment
    const int tb = lane & 15, kq = 8 * (lane >> 4);
    const float *xf = xs + (tb < nb ? tb : 0) * LDX + kq;   // rows >= nb: row 0 (D rows >= nb are not stored)
    floatx4 acc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const float4 f0 = *reinterpret_cast<const float4 *>(xf + 32 * j);
        const float4 f1 = *reinterpret_cast<const float4 *>(xf + 32 * j + 4);
        uint2 a1, a2, a3, b1, b2, b3;
        split4(f0, a1, a2, a3);
        split4(f1, b1, b2, b3);
        const bf16x8 h1 = __builtin_bit_cast(bf16x8, v4u{a1.x, a1.y, b1.x, b1.y});
        const bf16x8 h2 = __builtin_bit_cast(bf16x8, v4u{a2.x, a2.y, b2.x, b2.y});
        const bf16x8 h3 = __builtin_bit_cast(bf16x8, v4u{a3.x, a3.y, b3.x, b3.y});
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h1, __builtin_bit_cast(bf16x8, wv[t][j]), acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h2, __builtin_bit_cast(bf16x8, wv[t][j]), acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h3, __builtin_bit_cast(bf16x8, wv[t][j]), acc[t], 0, 0, 0);
    }
    gb_stamp(a, 2);
    // the wave's partial tiles over its own (dead) x rows
    floatx4 *red = reinterpret_cast<floatx4 *>(xs);
#pragma unroll
    for (int t = 0; t < TPW; ++t) red[t * 64 + lane] = acc[t];

    // ---- 4. one barrier; tile t: the W partial tiles in wave order, inv, epilogue
    __syncthreads();
    gb_stamp(a, 3);
    if (copier && norm && a.xcopy_normed) {   // the normalised copy: (x * nw) * inv[b]
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            if (!uok[q]) continue;
            float sq[16];   // (all W slice sums in flight, then added in wave order)
#pragma unroll
            for (int k = 0; k < 16; ++k) sq[k] = ssq[(k < W ? k : 0) * 16 + urow[q]];
            float s2 = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < W) s2 += sq[k];
            const float iv = rms_inv(s2, a.C, a.eps);
            float4 *xc = reinterpret_cast<float4 *>(a.xcopy + (size_t)urow[q] * a.ldxc + c0 + ucol);
            float4 v = *xc;
            v.x *= iv; v.y *= iv; v.z *= iv; v.w *= iv;
            *xc = v;
        }
    }
    const bool tile_wave = w < TPW && r0 + 16 * w < a.R;
    floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
    if (tile_wave) {
        // every wave's partial tile read at once (W <= 16; clamped, unconditional
        // reads), then summed in wave order: the sums of a loop that waited for
        // each read (that loop and the one below -- 16 and 64 dependent LDS
        // round trips -- were 1.3-1.9 us of every normed batch launch's
        // epilogue, profiles/r05a_b8_subtalker_stamps.txt)
        floatx4 pt[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) pt[k] = reinterpret_cast<const floatx4 *>(smem + (k < W ? k : 0) * wreg)[w * 64 + lane];
        v = pt[0];
#pragma unroll
        for (int k = 1; k < 16; ++k)
            if (k < W) v += pt[k];
        gb_stamp(a, 5);
        if (norm) {
            // lane l < 16 forms batch row l's statistic (the W slice sums in wave
            // order) and its 1 / rms once; the D fragment's rows 4 (lane >> 4) + i
            // fetch theirs by ds_bpermute
            const int lb = lane & 15, lr = lb < nb ? lb : 0;
            float sq[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) sq[k] = ssq[(k < W ? k : 0) * 16 + lr];
            float s2 = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (k < W) s2 += sq[k];
            const float iv = rms_inv(s2, a.C, a.eps);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int bb = 4 * (lane >> 4) + i;
                v[i] *= __shfl(iv, bb < nb ? bb : 0, 64);
            }
        }
        gb_stamp(a, 6);
    }
    const int r = r0 + 16 * w + (lane & 15);   // D: column = lane & 15 (weight row), row = 4 (lane >> 4) + i (batch row)
    if (a.tick) {      // self-reducing split-K producer (every thread reaches the ticket barrier)
        if (tile_wave) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int bb = 4 * (lane >> 4) + i;
                if (bb < nb && r < a.R) st_sc1(a.ypart + blockIdx.y * a.ld_ypart + (size_t)bb * a.R + r, v[i]);
            }
        }
        reduce_last(a, 16 * TPW, reinterpret_cast<int *>(ssq));
        return;
    }
    if (!tile_wave) return;
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
        epilogue(a, bb, r, val, up);
    }
    gb_stamp(a, 4);
}

}  // namespace

// Returns 1 when the shape is not covered (the caller uses k_gemvm), 0 ok,
// -1 launch error.  QTTS_HIP_GEMVB=0 keeps k_gemvm for every shape (A/B).
struct GbGeom { int SPW, TPW, W, NBC, PM, src; size_t smem; dim3 grid; };
static bool gemvb_geom(const GemvArgs &a, GbGeom &g) {
    if (a.nb < 2 || a.nb > 16 || a.R % 16 || a.C % 32 || (size_t)a.R * a.C * 2 >= ((size_t)1 << 31)) return false;
    const bool tab = a.table != nullptr, tabf = !tab && a.table_f32 != nullptr;
    if (tab) {
        if (a.C % 4) return false;
    } else if (tabf) {
        if ((uintptr_t)a.table_f32 & 15 || a.C % 4) return false;
    } else if (!a.x || a.ldx % 4 || ((uintptr_t)a.x & 15)) {
        return false;
    }
    if (a.norm_w && ((uintptr_t)a.norm_w & 15)) return false;
    if (a.xcopy && (a.ldxc % 4 || ((uintptr_t)a.xcopy & 15))) return false;
    const bool xadd = !tab && !tabf && a.xadd != nullptr;
    if (a.xadd && (tab || tabf || ((uintptr_t)a.xadd & 15) || a.ld_xadd % 4 || a.ldb_xadd % 4 || a.n_xadd < 1 ||
                   a.n_xadd > 4))
        return false;
    const int kz = a.ypart ? a.kz : 1;
    if (a.ypart && (kz < 2 || (a.tick && kz > 4) || a.norm_w || tab || tabf || a.xcopy || a.C % (32 * kz) ||
                    ((uintptr_t)a.ypart & 3)))
        return false;
    if (a.tick && (!a.ypart || !a.y || a.epi != EPI_RESID)) return false;
    // K slice per wave: the fewest steps that keep <= wmax waves (16; the
    // QTTS_HIP_GB_W=8 A/B switch: 512-thread workgroups, two per CU, one tile each)
    const char *gbw = getenv("QTTS_HIP_GB_W");
    const int wmax = gbw && atoi(gbw) == 8 ? 8 : 16;
    const int S = a.C / kz / 32;
    int SPW = 1;
    while (SPW < 8 && (S / SPW > wmax || S % SPW)) SPW *= 2;
    if (S % SPW || S / SPW > 16) return false;
    const int W = S / SPW;
    const int NBC = a.nb <= 8 ? 8 : 16;
    const int PM = xadd ? (a.n_xadd <= 2 ? 2 : 4) : 0;
    // tiles per workgroup: about one round of workgroups over the 256 CUs,
    // within the register file (estimate below) and W >= TPW epilogue waves
    const int T = a.R / 16;
    int TPW = wmax == 8 && W <= 8 ? 1 : (T * kz + 128) / 256;
    TPW = std::max(1, std::min(TPW, 3));
    if (SPW == 8 && TPW > 2) TPW = 2;
    if (SPW <= 2 && TPW > 2) TPW = 2;
    if (SPW == 1) TPW = 1;
    // instantiations whose partials would not fit the 128 registers of a
    // 1024-thread workgroup (hipcc -Rpass-analysis=kernel-resource-usage
    // reports scratch for exactly these): k_gemvm takes those shapes
    auto spills = [&](int tpw) {
        if (PM == 0) return false;
        if (NBC == 16) return SPW >= 4;
        if (SPW == 8) return !(tpw == 1 && PM == 2);
        return SPW == 4 && tpw == 3 && PM == 4;
    };
    while (TPW > 1 && (spills(TPW) || W < TPW)) --TPW;
    if (spills(TPW) || W < TPW) return false;
    const int wreg = std::max(a.nb * (32 * SPW + 4), TPW * 256);
    const size_t smem = ((size_t)W * wreg + (size_t)W * 16) * sizeof(float);
    if (smem > 160 * 1024) return false;
    const dim3 grid((T + TPW - 1) / TPW, kz);
    if (a.tick && (int)grid.x > QTTS_GM_TICKS) return false;
    const int src = tab ? GB_SRC_TAB : tabf ? GB_SRC_TABF : xadd ? GB_SRC_XADD : GB_SRC_X;
    g.SPW = SPW; g.TPW = TPW; g.W = W; g.NBC = NBC; g.PM = PM; g.src = src; g.smem = smem; g.grid = grid;
    return true;
}

template <int SP, int TP, int NC, int PP, int SS>
static void launch_gb(dim3 grid, dim3 block, size_t smem, hipStream_t st, const void *srcp, const int *idsp,
                      const GemvArgs &a) {
    hipLaunchKernelGGL((k_gemvb<SP, TP, NC, PP, SS>), grid, block, smem, st, srcp, idsp, a.W, a.xadd, a);
    // (rocprofv3's spelling of the instantiation: the bench looks its profile rows up by it)
    static char nm[64];
    snprintf(nm, sizeof nm, "k_gemvb<%d, %d, %d, %d, %d>", SP, TP, NC, PP, SS);
    qtts_last_kernel = nm;
}

int qtts_gemvb(const GemvArgs &in, hipStream_t st) {
    // (read per call: launches happen at graph capture, and tests switch it
    // per model instance)
    const char *ge = getenv("QTTS_HIP_GEMVB");
    if (ge && !atoi(ge)) return 1;
    const GemvArgs &a = in;
    GbGeom g;
    if (!gemvb_geom(a, g)) return 1;
    const int SPW = g.SPW, TPW = g.TPW, W = g.W, NBC = g.NBC, PM = g.PM, src = g.src;
    const size_t smem = g.smem;
    const dim3 grid = g.grid;
    const bool tab = a.table != nullptr, tabf = !tab && a.table_f32 != nullptr;
    const void *srcp = tab ? (const void *)a.table : tabf ? (const void *)a.table_f32 : (const void *)a.x;
    const int *idsp = (tab || tabf) ? a.ids + a.ids_off : nullptr;
    const dim3 block(64 * W);
#define QTTS_GB(SP, TP, NC, PP, SS) launch_gb<SP, TP, NC, PP, SS>(grid, block, smem, st, srcp, idsp, a);
#define QTTS_GB_SRC(SP, TP, NC)                                                                        \
    if (src == GB_SRC_X) QTTS_GB(SP, TP, NC, 0, GB_SRC_X)                                              \
    else if (src == GB_SRC_TAB) QTTS_GB(SP, TP, NC, 0, GB_SRC_TAB)                                     \
    else if (src == GB_SRC_TABF) QTTS_GB(SP, TP, NC, 0, GB_SRC_TABF)                                   \
    else if (PM == 2) QTTS_GB(SP, TP, NC, 2, GB_SRC_XADD)                                              \
    else QTTS_GB(SP, TP, NC, 4, GB_SRC_XADD)
#define QTTS_GB_NB(SP, TP)                                                                             \
    if (NBC == 8) QTTS_GB_SRC(SP, TP, 8) else QTTS_GB_SRC(SP, TP, 16)
    const int key = SPW * 10 + TPW;
    switch (key) {
        case 11: QTTS_GB_NB(1, 1) break;
        case 21: QTTS_GB_NB(2, 1) break;
        case 22: QTTS_GB_NB(2, 2) break;
        case 41: QTTS_GB_NB(4, 1) break;
        case 42: QTTS_GB_NB(4, 2) break;
        case 43: QTTS_GB_NB(4, 3) break;
        case 81: QTTS_GB_NB(8, 1) break;
        case 82: QTTS_GB_NB(8, 2) break;
        default: return 1;
    }
#undef QTTS_GB_NB
#undef QTTS_GB_SRC
#undef QTTS_GB
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
