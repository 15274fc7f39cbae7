// k_gemvw.hip - batch-1 GEMV for the latency-bound sub-talker chain (gfx950).
//
// y[r] = epilogue( sum_c W[r, c] * xin[c] ),  the role of kernel_matvec_bf16 /
// kernel_swiglu_matvec_bf16 (K.c:95-149, :213-233) with the rms_norm and
// residual passes around them (T.c:142-247), for matrices that stay resident
// in the Infinity Cache (the sub-talker's 224 MB, read 16 times per frame).
//
// Why a second batch-1 GEMV: each sub-talker op moves only 4-12.6 MB, so its
// time is the kernel boundary plus one dependent read of x plus the weight
// latency, not bandwidth.  profiles/r02a_mb_persist.txt measures the floor:
// an empty kernel 1.6 us, a kernel that only reads a 4 KB vector 2.0 us, and
// this kernel's shape (whole weight slice in flight before x is read, one
// wave per row, no LDS reduction) 4.2 us per op over the sub-talker chain,
// against ~6 us for k_gemv1 (two workgroups per CU, KSPLIT partials through
// LDS and a third barrier).  A persistent launch with 8-byte granule
// hand-offs between the ops measured 5.1 us per op in the same benchmark:
// the all-to-all vector exchange costs more than the boundary it removes.
//
// Mapping: one 256-thread workgroup per 4*RW rows (grid 256 = one per CU, or
// 512 for the 1.7B talker's gate|up and down);
// wave w owns rows row0 + w + 4i (i < RW); lane l covers the 8-column chunks
// l + 64k (k < NV), so C = 512 NV and every wave load is 1 KB contiguous.
// The x loads are issued first, then all RW*NV 16-B weight loads of a lane;
// the prologue (x or a gathered table row, + the O projection's per-head
// partials, RMSNorm) overlaps the weights; one barrier publishes the
// normalised x in LDS; each row is a dot of the lane's chunks in order + a
// 6-step xor-shuffle sum.
// SwiGLU rows come as interleaved gate|up quads (qtts_runtime.hip layout):
// with 4 | row0 / 8 even RW, a wave's rows i = 2j, 2j+1 are the gate row and
// its up row (r + 4), so the product is formed in registers.
#include "qtts_common.h"
#include "qtts_kernels.h"
#include "qtts_l2pf.h"

namespace {

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

// AM: x is the talker decode attention's output, merged here from its split
// partials (GemvArgs::amerge, AttnArgs::defer) -- the merge the attention's
// last split would do (k_attn.hip), in the same order and arithmetic:
// M = max_s m_s, f_s = expf(m_s - M), x = (sum_s f_s acc_s) / (sum_s f_s l_s).
// (AM_MS: splits whose partials are loaded before the weights, >= the live
// splits of the common case; more come after them, serially)
// Dynamic LDS: [xs: C floats][red: 4 floats] (16-B aligned, Guideline 17).
// diagnostic phase stamps (GemvArgs::dbg, QTTS_HIP_GM_DBG; compiled in only
// with `make EXTRA=-DQTTS_STAMPS`): 100 MHz wall clock, one lane per workgroup
__device__ __forceinline__ void gw_stamp(const GemvArgs &a, int k) {
#ifdef QTTS_STAMPS
    if (a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
#endif
}

// The first arguments are what the kernel's first loads need -- the x (or
// table) base, the weights, the id pointer (ids + ids_off) and the source
// kind (0 x, 1 bf16 table, 2 fp32 table, + 4: a.row_sel set) -- ahead of the
// GemvArgs block: the Makefile builds this file with kernarg preloading, so
// the CP hands them over in SGPRs and the x / id / weight loads issue
// without waiting for a kernarg round trip (the rest of `a` arrives by
// s_load meanwhile).
enum { GW_SRC_X = 0, GW_SRC_TAB = 1, GW_SRC_TABF = 2, GW_SRC_ROWSEL = 4 };

#ifndef QTTS_GW_WSD
#define QTTS_GW_WSD 2   // the talker shapes issue RW / QTTS_GW_WSD weight rows before x is staged (2. below)
#endif
template <int RW, int NV, bool NT, int AM_MS = 0>
__global__ __launch_bounds__(256) void k_gemvw(const void *src, const bf16_t *W, const int *ids, int src_kind,
                                               GemvArgs a) {
    gw_stamp(a, 0);
    constexpr bool AM = AM_MS > 0;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int C = 512 * NV, XQ = C / 1024 > 0 ? (C + 1023) / 1024 : 1;   // float4 of x per thread
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int row0 = blockIdx.x * 4 * RW;
    float *xs = smem, *red = smem + C;

    // 1. x (and the partials it adds) first: the weight loads issued after
    //    them do not hold back the prologue (vmcnt retires loads in issue
    //    order, so x issued behind 12 weight loads would wait for all of them)
    const bf16_t *trow = nullptr;
    const float *xrow = reinterpret_cast<const float *>(src);
    if (src_kind & 3) {
        const int *ip = ids + blockIdx.y;
        if (src_kind & GW_SRC_ROWSEL) ip += (size_t)a.row_sel[0] * a.ids_rstride;
        const size_t off = (size_t)(*ip) * C;
        if ((src_kind & 3) == GW_SRC_TAB) trow = reinterpret_cast<const bf16_t *>(src) + off;
        else xrow += off;
    }
    // partials held in registers (the sub-talker's 8 per-head O partials at
    // C = 1024); wider rows sum them from memory below
    constexpr int PMAX = XQ == 1 ? 8 : 0;
    // (a bf16 table row stays packed until the weights are in flight:
    // converting it here would wait for it before the weight loads issue)
    float4 xv[XQ], pv[XQ][PMAX > 0 ? PMAX : 1], nwv[XQ];
    uint2 tv[XQ];
    const int np = a.xadd ? a.n_xadd : 0;
    // AM: the first AM_MS splits' partials of every unit (their addresses need
    // no live length: slots past it hold stale values, masked below), and the
    // position, all in one round trip
    float4 am_a[AM ? XQ : 1][AM ? AM_MS : 1];
    float am_m[AM ? XQ : 1][AM ? AM_MS : 1], am_l[AM ? XQ : 1][AM ? AM_MS : 1];
    int am_p = 0;
    // (AM: src / ids carry the preloaded amerge / am_pos pointers)
    const float *amerge = AM ? reinterpret_cast<const float *>(src) : nullptr;
    if constexpr (AM) {
        am_p = ids[0];
        const int HDm = a.am_hd, GP = a.am_gph, NO = GP * HDm, stride = NO + 2 * GP;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int c = 4 * (tid + 256 * q);
            const int cc = c < C ? c : 0;
            const int h = cc / HDm, kvh = h / GP, g = h - kvh * GP;
            const float *mb = amerge + (size_t)kvh * a.am_nsplit * stride;
#pragma unroll
            for (int s2 = 0; s2 < AM_MS; ++s2) {
                const int sc = s2 < a.am_nsplit ? s2 : 0;
                am_a[q][s2] = *reinterpret_cast<const float4 *>(mb + (size_t)sc * stride + (cc - h * HDm) + g * HDm);
                am_m[q][s2] = mb[(size_t)sc * stride + NO + 2 * g];
                am_l[q][s2] = mb[(size_t)sc * stride + NO + 2 * g + 1];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
        if constexpr (AM) break;
        const int c = 4 * (tid + 256 * q);
        const int cc = c < C ? c : 0;
        if (trow) tv[q] = *reinterpret_cast<const uint2 *>(trow + cc);
        else xv[q] = *reinterpret_cast<const float4 *>(xrow + cc);
#pragma unroll
        for (int p = 0; p < PMAX; ++p)
            if (p < np) pv[q][p] = *reinterpret_cast<const float4 *>(a.xadd + (size_t)p * a.ld_xadd + cc);
        if (a.norm_w) nwv[q] = *reinterpret_cast<const float4 *>(a.norm_w + cc);
    }

    // 1b. the residual rows of an EPI_RESID epilogue, also ahead of the weights
    //     (read after the dot they were one more dependent round trip at the
    //     end of every O / down projection); rows are owned by this workgroup,
    //     so the early read sees the same values.  Unconditional load from a
    //     clamped address: a branch here would make the compiler wait for it.
    float *y = a.y + blockIdx.y * a.ldy_rep;
    const bool resid = a.epi == EPI_RESID;
    float yres[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) yres[i] = y[resid ? row0 + w + 4 * i : 0];

#ifdef QTTS_STAMPS
    if (a.dbg_xfirst) __builtin_amdgcn_s_waitcnt(0);   // (diagnostics: x alone, no weight traffic behind it)
#endif
    // 2. the weight slice of this lane in flight -- for the talker's HBM
    //    shapes only its first RW1 rows here, the rest once x is staged: x is
    //    an L2 / Infinity-Cache read, but it queues behind every weight request
    //    the chip's workgroups issued before it (in-graph stamps, the 1.7B
    //    gate|up: x lands 3.1-8.1 us into the launch behind the 50 MB stream,
    //    profiles/r05v_talker_layer_stamps.txt).  Half the rows first: x
    //    staged 2.5 -> 1.1 us (q|k|v), 3.7 -> 1.8 (down), 5.8 -> 4.4 (gate|up),
    //    +1.7 % audio-s/s in 4 alternating rounds; a third first, or the split
    //    for the sub-talker's Infinity-Cache shapes too, gave it back
    //    (profiles/r05wx_ab_split_issue.txt)
    // (the O projection with the attention merge in its prologue keeps every
    // row first: split, 33.25-33.46 vs 33.76-33.94 audio-s/s)
    // (and the 0.6B talker's 1024-wide rows keep every row first: split,
    // C2 38.33-38.52 vs 38.45-38.54 audio-s/s, profiles/r05wx_ab_split_issue.txt)
    constexpr bool WS = NT && !AM && RW >= 2 && NV >= 4;
    constexpr int RW1 = WS ? (RW / QTTS_GW_WSD > 0 ? RW / QTTS_GW_WSD : 1) : RW;
    v4u wv[RW][NV];
#pragma unroll
    for (int i = 0; i < RW1; ++i) {
        const v4u *p = reinterpret_cast<const v4u *>(W + (size_t)(row0 + w + 4 * i) * C) + lane;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            if constexpr (NT) wv[i][k] = __builtin_nontemporal_load(p + 64 * k);
            else wv[i][k] = p[64 * k];
        }
    }
    // 2b. the next launch's weight slice into this XCD's L2 (GemvArgs::pf)
    L2PfRegs pfr;
    qtts_l2pf_issue<256, NT>(a.pf, blockIdx.x + gridDim.x * blockIdx.y, pfr, W);

    if constexpr (AM) gw_stamp(a, 5);
    if constexpr (AM) {   // 3a. the attention merge, split order (k_attn_dec's last-split merge)
        const int HDm = a.am_hd, GP = a.am_gph, NO = GP * HDm, stride = NO + 2 * GP;
        const int nact = (am_p + 1 + a.am_ch - 1) / a.am_ch;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int c = 4 * (tid + 256 * q);
            const int cc = c < C ? c : 0;
            const int h = cc / HDm, kvh = h / GP, g = h - kvh * GP, eo = (cc - h * HDm) + g * HDm;
            const float *mb = amerge + (size_t)kvh * a.am_nsplit * stride;
            float M = -INFINITY;
#pragma unroll
            for (int s2 = 0; s2 < AM_MS; ++s2)
                if (s2 < nact) M = fmaxf(M, am_m[q][s2]);
            for (int s2 = AM_MS; s2 < nact; ++s2) M = fmaxf(M, mb[(size_t)s2 * stride + NO + 2 * g]);
            float4 num = make_float4(0.f, 0.f, 0.f, 0.f);
            float den = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < AM_MS; ++s2) {
                if (s2 < nact) {
                    const float f = expf(am_m[q][s2] - M);
                    num.x = fmaf(f, am_a[q][s2].x, num.x); num.y = fmaf(f, am_a[q][s2].y, num.y);
                    num.z = fmaf(f, am_a[q][s2].z, num.z); num.w = fmaf(f, am_a[q][s2].w, num.w);
                    den = fmaf(f, am_l[q][s2], den);
                }
            }
            for (int s2 = AM_MS; s2 < nact; ++s2) {
                const float *ps = mb + (size_t)s2 * stride;
                const float f = expf(ps[NO + 2 * g] - M);
                const float4 av = *reinterpret_cast<const float4 *>(ps + eo);
                num.x = fmaf(f, av.x, num.x); num.y = fmaf(f, av.y, num.y);
                num.z = fmaf(f, av.z, num.z); num.w = fmaf(f, av.w, num.w);
                den = fmaf(f, ps[NO + 2 * g + 1], den);
            }
            xv[q] = make_float4(num.x / den, num.y / den, num.z / den, num.w / den);
        }
        gw_stamp(a, 6);
    }
    // 3. residual + partials summed in partial order, RMS statistic
    if (trow) {
#pragma unroll
        for (int q = 0; q < XQ; ++q)
            xv[q] = make_float4(__uint_as_float(tv[q].x << 16), __uint_as_float(tv[q].x & 0xFFFF0000u),
                                __uint_as_float(tv[q].y << 16), __uint_as_float(tv[q].y & 0xFFFF0000u));
    }
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
        const int c = 4 * (tid + 256 * q);
        float4 v = xv[q];
        if (np > 0) {
            float4 s = pv[q][0];
#pragma unroll
            for (int p = 1; p < PMAX; ++p)
                if (p < np) { s.x += pv[q][p].x; s.y += pv[q][p].y; s.z += pv[q][p].z; s.w += pv[q][p].w; }
            for (int p = PMAX; p < np; ++p) {
                const float4 t = *reinterpret_cast<const float4 *>(a.xadd + (size_t)p * a.ld_xadd + c);
                s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
            }
            v.x += s.x; v.y += s.y; v.z += s.z; v.w += s.w;
        }
        if (c >= C) v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.norm_w) ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        xv[q] = v;
    }
    float inv = 1.f;
    if (a.norm_w) {
        ss = wave_sum(ss);
        if (lane == 0) red[w] = ss;
        __syncthreads();
        inv = rms_inv(red[0] + red[1] + red[2] + red[3], C, a.eps);
    }
    gw_stamp(a, 1);
    const bool cp = a.xcopy && blockIdx.x == 0;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
        const int c = 4 * (tid + 256 * q);
        if (c < C) {
            float4 v = xv[q];
            if (cp && !a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + c) = v;
            if (a.norm_w) {
                const float4 nw = nwv[q];
                v.x = v.x * inv * nw.x; v.y = v.y * inv * nw.y; v.z = v.z * inv * nw.z; v.w = v.w * inv * nw.w;
            }
            if (cp && a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + c) = v;
            *reinterpret_cast<float4 *>(xs + c) = v;
        }
    }
    __syncthreads();
    if constexpr (WS) {   // the rest of the slice (2. above)
#pragma unroll
        for (int i = RW1; i < RW; ++i) {
            const v4u *p = reinterpret_cast<const v4u *>(W + (size_t)(row0 + w + 4 * i) * C) + lane;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                if constexpr (NT) wv[i][k] = __builtin_nontemporal_load(p + 64 * k);
                else wv[i][k] = p[64 * k];
            }
        }
    }

    // 4. one wave per row: the lane's chunks in order, then the wave sum
    float acc[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) s += dot8w(wv[i][k], xs + 8 * (lane + 64 * k));
        acc[i] = wave_sum(s);
    }
    gw_stamp(a, 2);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            const int r = row0 + w + 4 * i;
            const float v = acc[i];
            switch (a.epi) {
                case EPI_STORE: y[r] = v; break;
                case EPI_BIAS: y[r] = v + a.bias[r]; break;
                case EPI_BIAS_SILU: {
                    const float z = v + a.bias[r];
                    y[r] = z / (1.0f + expf(-z));
                    break;
                }
                case EPI_RESID: y[r] = yres[i] + v; break;
                case EPI_SWIGLU:
                    if ((i & 1) == 0 && i + 1 < RW) y[(r >> 3) * 4 + (r & 3)] = (v / (1.0f + expf(-v))) * acc[i + 1];
                    break;
            }
        }
    }
    gw_stamp(a, 3);
    qtts_l2pf_sink(a.pf, pfr);   // (after the stores: the prefetch is off this launch's own path)
    gw_stamp(a, 4);
}

}  // namespace

// Returns 1 when the shape is not covered (the caller uses k_gemv1), 0 ok,
// -1 on a launch error.  Covers nb == 1, C = 512 NV, R = 1024 RW (grid 256,
// one workgroup per CU) or R = 2048 RW (grid 512) where RW * NV loads per
// lane would not fit one workgroup per CU.
bool qtts_gemvw_amerge_ok(int R, int C) { return C == 2048 && (R == 1024 || R == 2048); }

int qtts_gemvw(const GemvArgs &a, hipStream_t st) {
    if (a.amerge) {   // the talker O projection with the attention merge in its prologue
        if (a.nb != 1 || !qtts_gemvw_amerge_ok(a.R, a.C) || a.xadd || a.table || a.table_f32 || a.norm_w ||
            a.am_gph * a.am_hd * (a.C / (a.am_gph * a.am_hd)) != a.C || a.am_hd % 4 || a.am_nsplit < 1 || a.reps != 1) {
            fprintf(stderr, "qtts_gemvw: attention-merge prologue unsupported (R=%d C=%d)\n", a.R, a.C);
            return -1;
        }
        const dim3 grid(a.R / (4 * (a.R / 1024)));
        const size_t smem = (size_t)(a.C + 4) * sizeof(float);
        // partials of up to 4 / 8 splits ahead of the weights: the capacity's
        // splits when they fit (fixed-length decodes), else 8 and the rest after
#define QTTS_GWA(RW_, MS_)                                                                             \
        { hipLaunchKernelGGL((k_gemvw<RW_, 4, true, MS_>), grid, dim3(256), smem, st, (const void *)a.amerge, \
                             a.W, a.am_pos, (int)GW_SRC_X, a);                                          \
          qtts_last_kernel = "k_gemvw<" #RW_ ", 4, true, " #MS_ ">"; }
        if (a.R == 2048) { if (a.am_nsplit <= 4) QTTS_GWA(2, 4) else if (a.am_nsplit <= 6) QTTS_GWA(2, 6) else QTTS_GWA(2, 8) }
        else { if (a.am_nsplit <= 4) QTTS_GWA(1, 4) else if (a.am_nsplit <= 6) QTTS_GWA(1, 6) else QTTS_GWA(1, 8) }
#undef QTTS_GWA
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (a.nb != 1 || a.C % 512 || a.R % 1024 || a.ypart) return 1;
    if (a.reps < 1 || a.reps > 65535 || (a.reps > 1 && (!a.ids || a.xadd || a.xcopy || a.row_sel))) return 1;
    // sources: an fp32 row, a bf16 / fp32 table row (+ per-head partials too:
    // the sub-talker's layer-0 gate|up reads its residual from the table)
    if (a.xadd && (((uintptr_t)a.xadd & 15) || a.ld_xadd % 4 || a.n_xadd < 1)) return 1;
    if (a.norm_w && ((uintptr_t)a.norm_w & 15)) return 1;
    if (!a.table && ((uintptr_t)(a.table_f32 ? a.table_f32 : a.x) & 15)) return 1;
    if (a.xcopy && ((uintptr_t)a.xcopy & 15)) return 1;
    const int NV = a.C / 512;
    int RW = a.R / 1024;
    // two workgroups per CU where the slice would be large -- except the 1.7B
    // talker's down projection (2048 x 6144): one workgroup of 2 x 12 loads
    // per lane, 32.0 vs 31.96 audio-s/s for k_gemv1's wide config (same box)
    if (RW * NV > 16 && a.R % 2048 == 0 && NV != 12) RW = a.R / 2048;
    if (RW * NV > 24 || (a.epi == EPI_SWIGLU && (RW & 1))) return 1;
    const dim3 grid(a.R / (4 * RW), a.reps);
    const size_t smem = (size_t)(a.C + 4) * sizeof(float);
    const void *src = a.table ? (const void *)a.table : a.table_f32 ? (const void *)a.table_f32 : (const void *)a.x;
    const int kind = (a.table ? GW_SRC_TAB : a.table_f32 ? GW_SRC_TABF : GW_SRC_X) |
                     ((a.table || a.table_f32) && a.row_sel ? GW_SRC_ROWSEL : 0);
    const int *ids = (a.table || a.table_f32) ? a.ids + a.ids_off : nullptr;
#define QTTS_GW(RW_, NV_)                                                                              \
    if (RW == RW_ && NV == NV_) {                                                                      \
        if (a.nt) {                                                                                    \
            hipLaunchKernelGGL((k_gemvw<RW_, NV_, true>), grid, dim3(256), smem, st, src, a.W, ids, kind, a); \
            qtts_last_kernel = "k_gemvw<" #RW_ ", " #NV_ ", true>";                                    \
        } else {                                                                                       \
            hipLaunchKernelGGL((k_gemvw<RW_, NV_, false>), grid, dim3(256), smem, st, src, a.W, ids, kind, a); \
            qtts_last_kernel = "k_gemvw<" #RW_ ", " #NV_ ", false>";                                   \
        }                                                                                              \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                               \
    }
    // sub-talker (Hs 1024) and 0.6B talker (H 1024): q|k|v 4096x1024, gate|up
    // 6144x1024, down 1024x3072, lm heads 2048x1024, O 1024x2048, codec head
    // 3072x1024; 1.7B talker (H 2048): q|k|v 4096x2048, O 2048x2048, gate|up
    // 12288x2048 (grid 512), down 2048x6144 (RW 2, NV 12), codec head
    // 3072x2048.  (The down projection as RW 1, NV 12 on grid 512 measured
    // 6.8 vs 5.9 us on k_gemv1's wide config, profiles/r02h_frame_trace_*.txt.)
    QTTS_GW(4, 2) QTTS_GW(6, 2) QTTS_GW(1, 6) QTTS_GW(2, 2) QTTS_GW(1, 4) QTTS_GW(1, 2) QTTS_GW(3, 2)
    QTTS_GW(2, 4) QTTS_GW(4, 4) QTTS_GW(6, 4) QTTS_GW(3, 4) QTTS_GW(2, 12)
#undef QTTS_GW
    return 1;
}
