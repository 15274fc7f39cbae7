// k_gemv.hip - weight-streaming GEMV / skinny GEMM for gfx950.
//
// y[b, r] = epilogue( sum_c W[r, c] * xin[b, c] ),  b < nb <= NB (1..16)
//   W    bf16 row-major [R, C]  (PyTorch Linear.weight), streamed once from HBM
//   xin  fp32, staged in LDS by the prologue:
//          - source: fp32 rows x[b*ldx + c], or a bf16 table row gathered by an
//            id read from device memory (embedding lookup fused in)
//          - optional RMSNorm (c/qwen_tts_kernels.c:27-39) with the full-row
//            statistics computed per workgroup
//          - optional copy-out (raw or normalised) by workgroup 0
//   epilogue: store / +bias / +bias then SiLU / residual add (x += acc) /
//             SwiGLU over interleaved gate|up row quads.
//
// Replaces kernel_matvec_bf16 (K.c:95-149), kernel_swiglu_matvec_bf16
// (K.c:213-233), kernel_matmul_bf16 (K.c:185-207, small M) and the
// rms_norm / add / silu element-wise passes around them (T.c:142-247).
//
// Mapping (64-wide waves): 256 threads = 32 slots of 8 lanes.  A slot owns one
// row; the row's 64-column blocks are dealt round-robin to KSPLIT slots (each
// lane loads 16 B = 8 bf16 of a block), so one 8-lane slot reads 128 B
// contiguous per block and the final reduction is 3 xor-shuffles + a KSPLIT
// combine through LDS.  KSPLIT is chosen on the host so the grid fills the 256
// CUs.  Weight loads for the first block group are issued before the prologue
// so HBM latency overlaps the norm.  Accumulation is fp32 (exact bf16->f32).
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

constexpr int U = 8;  // blocks per load group (16 B each per lane)

template <int NB, bool NT>
__global__ __launch_bounds__(256) void k_gemv(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, slot = tid >> 3, sub = tid & 7;
    const int ksn = a.ksplit, RPW = 32 / ksn;
    const int rloc = slot % RPW, ks = slot / RPW;
    const int row0 = blockIdx.x * RPW;
    const int row = row0 + rloc;
    const int rowc = row < a.R ? row : a.R - 1;
    const int C = a.C, CCH = a.cch, nb = a.nb;
    float *xs = smem;                 // [NB][CCH]
    float *red = xs + NB * CCH;       // [32][NB]
    float *inv = red + 32 * NB;       // [NB]
    float *bred = inv + NB;           // [4]

    const v4u *Wr = reinterpret_cast<const v4u *>(a.W + (size_t)rowc * C) + sub;
    const int nblk = CCH / 64 / ksn;  // blocks per slot per chunk
    const int ng = (nblk + U - 1) / U;

    float acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0f;

    v4u wv[U];
    auto load_group = [&](int c0, int g) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int j = g * U + u;
            j = j < nblk ? j : nblk - 1;          // clamp: loads stay unconditional
            const v4u *p = Wr + ((c0 + 64 * (ks + j * ksn)) >> 3);
            if constexpr (NT) wv[u] = __builtin_nontemporal_load(p);
            else wv[u] = *p;
        }
    };

    // x source row b (fp32 rows or gathered bf16 table row)
    auto src_row_id = [&](int b) -> int {
        const int *p = a.ids + (size_t)b * a.ids_bstride + a.ids_off;
        if (a.row_sel) p += (size_t)a.row_sel[b] * a.ids_rstride;
        return *p;
    };

    // ---- prologue: per-row RMS statistics over the full row ----
    load_group(0, 0);
    if (a.norm_w) {
        for (int b = 0; b < NB; ++b) {
            float ss = 0.0f;
            if (b < nb) {
                if (a.table) {
                    const bf16_t *t = a.table + (size_t)src_row_id(b) * C;
                    for (int c = tid; c < C; c += 256) { float v = bf2f(t[c]); ss += v * v; }
                } else {
                    const float *xr = a.table_f32 ? a.table_f32 + (size_t)src_row_id(b) * C : a.x + (size_t)b * a.ldx;
                    for (int c = tid; c < C; c += 256) { float v = xr[c]; ss += v * v; }
                }
            }
            ss = block_sum256(ss, bred);
            if (tid == 0) inv[b] = rms_inv(ss, C, a.eps);
        }
    }

    for (int c0 = 0; c0 < C; c0 += CCH) {
        if (c0 > 0) load_group(c0, 0);
        __syncthreads();  // inv[] visible, previous chunk consumed
        // stage the chunk
        for (int i = tid; i < NB * CCH; i += 256) {
            const int b = i / CCH, c = i - b * CCH, cg = c0 + c;
            float v = 0.0f;
            if (b < nb) {
                if (a.table) v = bf2f(a.table[(size_t)src_row_id(b) * C + cg]);
                else if (a.table_f32) v = a.table_f32[(size_t)src_row_id(b) * C + cg];
                else v = a.x[(size_t)b * a.ldx + cg];
                if (a.xcopy && blockIdx.x == 0 && !a.xcopy_normed) a.xcopy[(size_t)b * a.ldxc + cg] = v;
                if (a.norm_w) v = v * inv[b] * a.norm_w[cg];
                if (a.xcopy && blockIdx.x == 0 && a.xcopy_normed) a.xcopy[(size_t)b * a.ldxc + cg] = v;
            }
            xs[i] = v;
        }
        __syncthreads();
        for (int g = 0; g < ng; ++g) {
            v4u cur[U];
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = wv[u];
            if (g + 1 < ng) load_group(c0, g + 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = g * U + u;
                if (j < nblk) {
                    float f[8];
                    unpack8(cur[u], f);
                    const int cl = 64 * (ks + j * ksn) + 8 * sub;
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const float4 x0 = *reinterpret_cast<const float4 *>(xs + b * CCH + cl);
                        const float4 x1 = *reinterpret_cast<const float4 *>(xs + b * CCH + cl + 4);
                        float s = acc[b];
                        s = fmaf(f[0], x0.x, s); s = fmaf(f[1], x0.y, s);
                        s = fmaf(f[2], x0.z, s); s = fmaf(f[3], x0.w, s);
                        s = fmaf(f[4], x1.x, s); s = fmaf(f[5], x1.y, s);
                        s = fmaf(f[6], x1.z, s); s = fmaf(f[7], x1.w, s);
                        acc[b] = s;
                    }
                }
            }
        }
    }

    // ---- reduction: 8 lanes, then KSPLIT slots through LDS ----
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float v = acc[b];
        v = group_sum<8>(v);
        acc[b] = v;
    }
    __syncthreads();  // xs no longer read; red may alias nothing but be safe
    if (sub == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) red[(ks * RPW + rloc) * NB + b] = acc[b];
    }
    __syncthreads();
    // final value per (row, b) -> xs scratch [RPW][NB]
    for (int t = tid; t < RPW * NB; t += 256) {
        const int rl = t / NB, b = t - rl * NB;
        float s = red[rl * NB + b];
        for (int k = 1; k < ksn; ++k) s += red[(k * RPW + rl) * NB + b];
        xs[t] = s;
    }
    __syncthreads();
    for (int t = tid; t < RPW * NB; t += 256) {
        const int rl = t / NB, b = t - rl * NB;
        const int r = row0 + rl;
        if (r >= a.R || b >= nb) continue;
        float v = xs[t];
        switch (a.epi) {
            case EPI_STORE: a.y[(size_t)b * a.ldy + r] = v; break;
            case EPI_BIAS: a.y[(size_t)b * a.ldy + r] = v + a.bias[r]; break;
            case EPI_BIAS_SILU: {
                float z = v + a.bias[r];
                a.y[(size_t)b * a.ldy + r] = z / (1.0f + expf(-z));
                break;
            }
            case EPI_RESID: a.y[(size_t)b * a.ldy + r] += v; break;
            case EPI_SWIGLU: {
                if ((r & 7) < 4) {  // gate row; its up row is r + 4 in the same workgroup
                    const float u = xs[(rl + 4) * NB + b];
                    const int o = (r >> 3) * 4 + (r & 3);
                    a.y[(size_t)b * a.ldy + o] = (v / (1.0f + expf(-v))) * u;
                }
                break;
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Batch-1 weight stream of k_gemv1: the 8-lane slot of
// row `row` streams its KSPLIT share of the row's 64-column blocks in groups of
// U1 x 16 B per lane, double-buffered in registers (the first group is issued
// by the caller before its prologue).
template <int U1, bool NT>
struct G1Stream {
    const v4u *Wr;
    int nblk, ng, ks, ksn, sub;
    v4u wv[U1];
    __device__ __forceinline__ G1Stream(const GemvArgs &a, int row, int ks_, int ksn_, int sub_)
        : ks(ks_), ksn(ksn_), sub(sub_) {
        const int rowc = row < a.R ? row : a.R - 1;
        Wr = reinterpret_cast<const v4u *>(a.W + (size_t)rowc * a.C) + sub;
        nblk = a.C / 64 / ksn;
        ng = (nblk + U1 - 1) / U1;
    }
    __device__ __forceinline__ void load(int g) {
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            int j = g * U1 + u;
            j = j < nblk ? j : nblk - 1;   // clamp: loads stay unconditional
            const v4u *p = Wr + ((64 * (ks + j * ksn)) >> 3);
            if constexpr (NT) wv[u] = __builtin_nontemporal_load(p);
            else wv[u] = *p;
        }
    }
    // dot of this lane's share with xs (LDS), reduced over the slot's 8 lanes
    __device__ __forceinline__ float run(const float *xs) {
        float acc = 0.f;
        if constexpr (U1 >= 16) {   // one group (nblk <= U1, launcher): every load already issued
#pragma unroll
            for (int u = 0; u < U1; ++u) {
                if (u < nblk) {
                    float f[8];
                    unpack8(wv[u], f);
                    const int cl = 64 * (ks + u * ksn) + 8 * sub;
                    const float4 x0 = *reinterpret_cast<const float4 *>(xs + cl);
                    const float4 x1 = *reinterpret_cast<const float4 *>(xs + cl + 4);
                    acc = fmaf(f[0], x0.x, acc); acc = fmaf(f[1], x0.y, acc);
                    acc = fmaf(f[2], x0.z, acc); acc = fmaf(f[3], x0.w, acc);
                    acc = fmaf(f[4], x1.x, acc); acc = fmaf(f[5], x1.y, acc);
                    acc = fmaf(f[6], x1.z, acc); acc = fmaf(f[7], x1.w, acc);
                }
            }
            acc = group_sum<8>(acc);
            return acc;
        }
        for (int g = 0; g < ng; ++g) {
            v4u cur[U1];
#pragma unroll
            for (int u = 0; u < U1; ++u) cur[u] = wv[u];
            if (g + 1 < ng) load(g + 1);
#pragma unroll
            for (int u = 0; u < U1; ++u) {
                const int j = g * U1 + u;
                if (j < nblk) {
                    float f[8];
                    unpack8(cur[u], f);
                    const int cl = 64 * (ks + j * ksn) + 8 * sub;
                    const float4 x0 = *reinterpret_cast<const float4 *>(xs + cl);
                    const float4 x1 = *reinterpret_cast<const float4 *>(xs + cl + 4);
                    acc = fmaf(f[0], x0.x, acc); acc = fmaf(f[1], x0.y, acc);
                    acc = fmaf(f[2], x0.z, acc); acc = fmaf(f[3], x0.w, acc);
                    acc = fmaf(f[4], x1.x, acc); acc = fmaf(f[5], x1.y, acc);
                    acc = fmaf(f[6], x1.z, acc); acc = fmaf(f[7], x1.w, acc);
                }
            }
        }
        acc = group_sum<8>(acc);
        return acc;
    }
};

// Batch-1 epilogue: KSPLIT partials through LDS `red` [32], one barrier, then
// one thread per output row applies the epilogue.
__device__ __forceinline__ void g1_epilogue(const GemvArgs &a, float acc, float *red, int row0, int RPW, int ksn,
                                            int ks, int rloc, int sub) {
    const int tid = threadIdx.x;
    if (sub == 0) red[ks * RPW + rloc] = acc;
    __syncthreads();
    if (tid < RPW) {
        const int r = row0 + tid;
        if (r < a.R) {
            float v = red[tid];
            for (int k = 1; k < ksn; ++k) v += red[k * RPW + tid];
            switch (a.epi) {
                case EPI_STORE: a.y[r] = v; break;
                case EPI_BIAS: a.y[r] = v + a.bias[r]; break;
                case EPI_BIAS_SILU: {
                    const float z = v + a.bias[r];
                    a.y[r] = z / (1.0f + expf(-z));
                    break;
                }
                case EPI_RESID: a.y[r] += v; break;
                case EPI_SWIGLU:
                    if ((r & 7) < 4) {
                        float u = red[tid + 4];
                        for (int k = 1; k < ksn; ++k) u += red[k * RPW + tid + 4];
                        a.y[(r >> 3) * 4 + (r & 3)] = (v / (1.0f + expf(-v))) * u;
                    }
                    break;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Batch-1 decode path.  Same slot mapping; the prologue loads x once as float4
// (XV per thread), reduces the RMS statistic with one barrier, writes the
// normalised row to LDS (second barrier); weights for the first U blocks are
// already in flight.  One barrier in the epilogue: each output thread sums
// the KSPLIT partials it needs (for SwiGLU also its up row's) straight from
// LDS.
// Dynamic LDS: [xs: C][red: nslot][bred: nthr/64], all of it in the dynamic
// region (a static __shared__ would shift every float4 LDS access off its
// 16-B alignment: replayed at 64 cycles each, cdna_hip_programming.md
// Guideline 17).
constexpr int G1_HEAD = 0;   // floats in front of xs

// Block size: 256 threads, or up to 1024 ("wide": one workgroup per CU
// streaming R/256 rows, qtts_gemv) -- nslot = blockDim/8 slots.
template <int U1, int XV, bool NT>
__global__ __launch_bounds__(1024) void k_gemv1(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, slot = tid >> 3, sub = tid & 7, nthr = blockDim.x, nslot = nthr >> 3;
    const int ksn = a.ksplit, RPW = nslot / ksn;
    const int rloc = slot % RPW, ks = slot / RPW;
    const int row0 = blockIdx.x * RPW, row = row0 + rloc;
    const int C = a.C;
    float *xs = smem + G1_HEAD;   // [C]
    float *red = xs + C;          // [nslot]
    float *bred = red + nslot;    // [nthr / 64]
    G1Stream<U1, NT> ws(a, row, ks, ksn, sub);

    // ---- prologue: x (fp32 row or gathered bf16 row) -> optional RMSNorm -> LDS.
    // The x and norm-weight loads go out BEFORE the first weight group: loads
    // retire in issue order, so x behind U1 weight loads would wait for them.
    const bf16_t *trow = nullptr;
    const float *xrow = a.x;
    if (a.table || a.table_f32) {
        const int *p = a.ids + a.ids_off;
        if (a.row_sel) p += (size_t)a.row_sel[0] * a.ids_rstride;
        const size_t off = (size_t)(*p) * C;
        if (a.table) trow = a.table + off;
        else xrow = a.table_f32 + off;
    }
    // (a bf16 table row stays packed until the weights are in flight)
    float4 xv[XV], wn[XV];
    uint2 tv[XV];
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int c = 4 * (tid + nthr * i);
        const int cc = c < C ? c : C - 4;
        if (trow) tv[i] = *reinterpret_cast<const uint2 *>(trow + cc);
        else xv[i] = *reinterpret_cast<const float4 *>(xrow + cc);
        if (a.norm_w) wn[i] = *reinterpret_cast<const float4 *>(a.norm_w + cc);
    }
    ws.load(0);
    if (trow) {
#pragma unroll
        for (int i = 0; i < XV; ++i)
            xv[i] = make_float4(__uint_as_float(tv[i].x << 16), __uint_as_float(tv[i].x & 0xFFFF0000u),
                                __uint_as_float(tv[i].y << 16), __uint_as_float(tv[i].y & 0xFFFF0000u));
    }
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int c = 4 * (tid + nthr * i);
        const int cc = c < C ? c : C - 4;
        float4 v = xv[i];
        if (a.xadd) {   // residual (x or table row) + the O projection's per-head partials, summed in head order
            float4 sacc = *reinterpret_cast<const float4 *>(a.xadd + cc);
            for (int p = 1; p < a.n_xadd; ++p) {
                const float4 t = *reinterpret_cast<const float4 *>(a.xadd + (size_t)p * a.ld_xadd + cc);
                sacc.x += t.x; sacc.y += t.y; sacc.z += t.z; sacc.w += t.w;
            }
            v.x += sacc.x; v.y += sacc.y; v.z += sacc.z; v.w += sacc.w;
        }
        if (c >= C) v = make_float4(0.f, 0.f, 0.f, 0.f);
        xv[i] = v;
        if (a.norm_w) ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    float inv = 1.f;
    if (a.norm_w) {
        ss = wave_sum(ss);
        if ((tid & 63) == 0) bred[tid >> 6] = ss;
        __syncthreads();
        float st = bred[0];
        for (int k = 1; k < (nthr >> 6); ++k) st += bred[k];
        inv = rms_inv(st, C, a.eps);
    }
    const bool cp = a.xcopy && blockIdx.x == 0;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int c = 4 * (tid + nthr * i);
        if (c < C) {
            float4 v = xv[i];
            if (cp && !a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + c) = v;
            if (a.norm_w) {
                v.x = v.x * inv * wn[i].x; v.y = v.y * inv * wn[i].y;
                v.z = v.z * inv * wn[i].z; v.w = v.w * inv * wn[i].w;
            }
            if (cp && a.xcopy_normed) *reinterpret_cast<float4 *>(a.xcopy + c) = v;
            *reinterpret_cast<float4 *>(xs + c) = v;
        }
    }
    __syncthreads();

    // ---- stream the weights, then the epilogue (and the tail) ----
    const float acc = ws.run(xs);
    g1_epilogue(a, acc, red, row0, RPW, ksn, ks, rloc, sub);
}

}  // namespace

thread_local const char *qtts_last_kernel = "";

// KSPLIT: grow until the grid has >= `target` workgroups (>= 2 per CU for
// the latency hiding of a weight stream; fewer, larger blocks leave CUs idle
// in the tail), bounded by the row length and by SwiGLU's 8-row quads.
static int pick_ksplit(int R, int C, int epi, int target) {
    int maxk = C / 64;
    if (maxk > 32) maxk = 32;
    if (epi == EPI_SWIGLU && maxk > 4) maxk = 4;
    int ks = 1;
    while (ks < maxk && (R + (32 / ks) - 1) / (32 / ks) < target) ks *= 2;
    while (ks > 1 && (C / 64) % ks) ks /= 2;
    return ks;
}

// "Wide" batch-1 configuration for the talker's (non-temporal) weights:
// about one workgroup per CU (grid ~ 256), each streaming ceil(R / 256) rows
// with up to 1024 threads, so the grid runs in one round and x is staged 256
// times instead of once per 32-row block.
static void wide_config(int R, int C, int epi, int &ks_out, int &nthr_out) {
    const int nb64 = C / 64, quad = epi == EPI_SWIGLU ? 8 : 1;
    int rows = (R + 255) / 256;
    rows = (rows + quad - 1) / quad * quad;
    for (int ks = 32; ks >= 1; ks /= 2) {
        if (nb64 % ks || (epi == EPI_SWIGLU && ks > 4)) continue;
        int rpw = rows;
        while ((rpw * ks) % 8) rpw += quad;   // whole waves of 8 slots
        if (rpw * ks > 128) continue;
        ks_out = ks;
        nthr_out = rpw * ks * 8;
        return;
    }
}

int qtts_gemv(const GemvArgs &in, hipStream_t st) {
    GemvArgs a = in;
    if (a.C % 64 || a.nb < 1 || a.nb > 16 || a.R < 1) {
        fprintf(stderr, "qtts_gemv: unsupported shape R=%d C=%d nb=%d\n", a.R, a.C, a.nb);
        return -1;
    }
    if (a.nb == 1 && a.ksplit <= 0) {   // the wave-per-row kernel where it covers the shape (k_gemvw.hip)
        const int rc = qtts_gemvw(a, st);
        if (rc != 1) return rc;
    }
    if (a.xadd && a.nb == 1 && !(a.C <= 8192 && a.ldx_ok1())) {
        fprintf(stderr, "qtts_gemv: xadd needs the batch-1 fast path (R=%d C=%d)\n", a.R, a.C);
        return -1;
    }
    if (a.nb == 1 && a.C <= 8192 && a.ldx_ok1()) {
        int nthr = 256;
        // (one CU's share >= 96 KB: below that the 256-thread grid measured faster,
        // profiles/r01x_mb_gemv_wide_u16.txt)
        if (a.ksplit <= 0 && a.nt && (size_t)a.R * a.C * 2 / 256 >= 96 * 1024) {
            wide_config(a.R, a.C, a.epi, a.ksplit, nthr);
        }
        if (a.ksplit <= 0) a.ksplit = pick_ksplit(a.R, a.C, a.epi, 512);
        const int rpw = nthr / 8 / a.ksplit;
        const int grid = (a.R + rpw - 1) / rpw;
        const int nblk = a.C / 64 / a.ksplit;
        const int xq = (a.C + 4 * nthr - 1) / (4 * nthr);
        const int xv = xq <= 1 ? 1 : xq <= 2 ? 2 : xq <= 4 ? 4 : 8;
        const size_t smem = (size_t)(G1_HEAD + a.C + nthr / 8 + 16) * sizeof(float);
#define QTTS_G1(U, X)                                                                                 \
        if (a.nt) {                                                                                   \
            hipLaunchKernelGGL((k_gemv1<U, X, true>), dim3(grid), dim3(nthr), smem, st, a);           \
            qtts_last_kernel = "k_gemv1<" #U ", " #X ", true>";                                       \
        } else {                                                                                      \
            hipLaunchKernelGGL((k_gemv1<U, X, false>), dim3(grid), dim3(nthr), smem, st, a);          \
            qtts_last_kernel = "k_gemv1<" #U ", " #X ", false>";                                      \
        }
        if (nthr != 256 && nblk > 8 && nblk <= 16) {   // wide: every weight load of a lane in one group
            switch (xv) { case 1: QTTS_G1(16, 1) break; case 2: QTTS_G1(16, 2) break;
                          case 4: QTTS_G1(16, 4) break; default: QTTS_G1(8, 8) break; }
        } else if (nblk > 4) {   // (5..8 blocks: one group of 8, not two of 4 -- the second
                                 //  would only issue after the prologue's barrier)
            switch (xv) { case 1: QTTS_G1(8, 1) break; case 2: QTTS_G1(8, 2) break;
                          case 4: QTTS_G1(8, 4) break; default: QTTS_G1(8, 8) break; }
        } else {
            switch (xv) { case 1: QTTS_G1(4, 1) break; case 2: QTTS_G1(4, 2) break;
                          case 4: QTTS_G1(4, 4) break; default: QTTS_G1(4, 8) break; }
        }
#undef QTTS_G1
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (a.nb >= 2) {   // lock-step batch: the matrix-core kernels (k_gemvb.hip, k_gemvm.hip) where they cover the shape
        int rc = qtts_gemvb(a, st);
        if (rc == 1) rc = qtts_gemvm(a, st);
        if (rc != 1) return rc;
    }
    if (a.ypart || (a.xadd && a.nb >= 2)) {
        fprintf(stderr, "qtts_gemv: split-K partials need the batch kernel (R=%d C=%d nb=%d)\n", a.R, a.C, a.nb);
        return -1;
    }
    if (a.ksplit <= 0) a.ksplit = pick_ksplit(a.R, a.C, a.epi, 256);
    int NB = a.nb <= 1 ? 1 : a.nb <= 2 ? 2 : a.nb <= 4 ? 4 : a.nb <= 8 ? 8 : 16;
    const int unit = 64 * a.ksplit;
    int cch = (8192 / NB) / unit * unit;
    if (cch < unit) cch = unit;
    if (cch > a.C) cch = a.C;
    while (a.C % cch) cch -= unit;
    a.cch = cch;
    const int rpw = 32 / a.ksplit;
    const int grid = (a.R + rpw - 1) / rpw;
    size_t smem = (size_t)(NB * cch + 32 * NB + NB + 4) * sizeof(float);
#define QTTS_GEMV_CASE(n)                                                                        \
    case n:                                                                                      \
        if (a.nt) hipLaunchKernelGGL((k_gemv<n, true>), dim3(grid), dim3(256), smem, st, a);     \
        else hipLaunchKernelGGL((k_gemv<n, false>), dim3(grid), dim3(256), smem, st, a);         \
        qtts_last_kernel = a.nt ? "k_gemv<" #n ", true>" : "k_gemv<" #n ", false>";         \
        break;
    switch (NB) {
        QTTS_GEMV_CASE(1)
        QTTS_GEMV_CASE(2)
        QTTS_GEMV_CASE(4)
        QTTS_GEMV_CASE(8)
        QTTS_GEMV_CASE(16)
    }
#undef QTTS_GEMV_CASE
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
