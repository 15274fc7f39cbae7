// k_mgemm.hip - skinny GEMM on the bf16 matrix cores for the multi-row
// projections: talker prefill over the prompt rows (T.c:254-472, the
// reference's kernel_matmul_bf16, K.c:185-207) and the text projection
// (Q.c:823-847).  M <= 64 activation rows x bf16 weights [R, C].
//
// Exact-product "3 x bf16" split: each fp32 activation x is written as
// x1 + x2 + x3 with x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2)
// (24 significand bits = 3 x 8), and y = W.x1 + W.x2 + W.x3 on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation.  bf16 x bf16 products are
// exact in fp32, so the result differs from an fp32 GEMV only in summation
// order (the bar the decode GEMV already meets), at 3/16 of the f32-MFMA
// instruction count.
//
// Mapping: one workgroup = 16 weight rows (the MFMA N side) x all M rows
// (up to 4 tiles of 16 on the MFMA M side); the four waves take K steps of 32
// round-robin, then reduce their partial tiles through LDS in wave order.
// Grids under 1024 workgroups split K over grid.z (partials to scratch,
// summed in column order with the epilogue by k_mgemm_reduce): at one
// workgroup per CU each SIMD holds one wave, which waits out every K step's
// loads alone.
// Lane l of a wave loads W[row l&15][k0 + 8(l>>4) .. +7] (one 16 B load) and
// x[t = l&15][same k] (two float4), which are exactly the B and A operand
// fragments of mfma_f32_16x16x32_bf16 (cdna_hip_programming.md section 3).
// RMSNorm (K.c:27-39) is applied while loading x, with per-row 1/rms from
// k_row_rms.  Epilogues: store / +bias / +bias then SiLU / residual add /
// SwiGLU over the interleaved gate|up row quads (the up value comes from
// lane + 4).
#include "qtts_common.h"
#include "qtts_kernels.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ short f2bf_rn(float f) {
    uint32_t u = __float_as_uint(f);
    u = u + 0x7FFFu + ((u >> 16) & 1u);
    return (short)(u >> 16);
}
__device__ __forceinline__ float bf2f_s(short b) { return __uint_as_float(((uint32_t)(uint16_t)b) << 16); }

// per-row 1/rms of x rows (grid = rows)
__global__ __launch_bounds__(256) void k_row_rms(const float *x, int ldx, int C, float eps, float *inv) {
    __shared__ float red[4];
    const float *xr = x + (size_t)blockIdx.x * ldx;
    float s = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) s += xr[c] * xr[c];
    s = block_sum256(s, red);
    if (threadIdx.x == 0) inv[blockIdx.x] = rms_inv(s, C, eps);
}

// NW > 1 (many activation rows): the workgroup covers NW weight tiles, so the
// activation fragments (and their split) are loaded once per NW tiles -- the
// activation re-reads from L2, R/16 per chunk at NW = 1, bound the > 64-row
// case.  Per-wave K partition and the in-order wave reduction are those of
// NW = 1, so the results are bit-identical.
// part != nullptr (split-K, grid.z = kz column groups of C): workgroup z
// covers K steps [z nsz, (z+1) nsz), its waves round-robin inside them, and
// it stores the raw tile sums to part[z][row][R] for k_mgemm_reduce.
template <int MT, int NW>
__global__ __launch_bounds__(256) void k_mgemm(GemvArgs a, const float *inv, float *part) {
    __shared__ floatx4 red[4][MT][NW][64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r0 = blockIdx.x * 16 * NW;
    const int rl = lane & 15, kq = 8 * (lane >> 4);
    // grid.y walks 64-row chunks of the activations: the workgroups of one
    // weight tile share an XCD's L2 (gridDim.x % 8 == 0 -> same XCD for every y)
    const int t0 = blockIdx.y * 64;
    const int M = a.nb - t0 < 64 ? a.nb - t0 : 64, C = a.C;
    const float *xb = a.x ? a.x + (size_t)t0 * a.ldx : nullptr;
    const int *idb = a.ids ? a.ids + (size_t)t0 * a.ids_bstride : nullptr;
    const float *invb = inv ? inv + t0 : nullptr;
    float *yb = a.y + (size_t)t0 * a.ldy;
    const bf16_t *wr[NW];
#pragma unroll
    for (int n = 0; n < NW; ++n) {
        const int row = r0 + 16 * n + rl < a.R ? r0 + 16 * n + rl : a.R - 1;
        wr[n] = a.W + (size_t)row * C + kq;
    }
    floatx4 acc[MT][NW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int n = 0; n < NW; ++n) acc[mt][n] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nsz = C / 32 / gridDim.z, sz0 = blockIdx.z * nsz;
    for (int s = w; s < nsz; s += 4) {
        const int k0 = 32 * (sz0 + s);
        bf16x8 bw[NW];
#pragma unroll
        for (int n = 0; n < NW; ++n) bw[n] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const v4u *>(wr[n] + k0));
        float nw[8];
        if (a.norm_w) {
            const float4 n0 = *reinterpret_cast<const float4 *>(a.norm_w + k0 + kq);
            const float4 n1 = *reinterpret_cast<const float4 *>(a.norm_w + k0 + kq + 4);
            nw[0] = n0.x; nw[1] = n0.y; nw[2] = n0.z; nw[3] = n0.w;
            nw[4] = n1.x; nw[5] = n1.y; nw[6] = n1.z; nw[7] = n1.w;
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int t = mt * 16 + rl;
            float xv[8];
            if (t < M) {
                if (a.table) {
                    const int id = idb[(size_t)t * a.ids_bstride];
                    const v4u q = *reinterpret_cast<const v4u *>(a.table + (size_t)id * C + k0 + kq);
                    float f[8];
                    unpack8(q, f);
#pragma unroll
                    for (int j = 0; j < 8; ++j) xv[j] = f[j];
                } else {
                    const float *xr = xb + (size_t)t * a.ldx + k0 + kq;
                    const float4 x0 = *reinterpret_cast<const float4 *>(xr);
                    const float4 x1 = *reinterpret_cast<const float4 *>(xr + 4);
                    xv[0] = x0.x; xv[1] = x0.y; xv[2] = x0.z; xv[3] = x0.w;
                    xv[4] = x1.x; xv[5] = x1.y; xv[6] = x1.z; xv[7] = x1.w;
                }
                if (a.norm_w) {
                    const float iv = invb[t];
#pragma unroll
                    for (int j = 0; j < 8; ++j) xv[j] = xv[j] * iv * nw[j];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = 0.f;
            }
            bf16x8 h1, h2, h3;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const short b1 = f2bf_rn(xv[j]);
                const float e1 = xv[j] - bf2f_s(b1);
                const short b2 = f2bf_rn(e1);
                const float e2 = e1 - bf2f_s(b2);
                h1[j] = b1;
                h2[j] = b2;
                h3[j] = f2bf_rn(e2);
            }
#pragma unroll
            for (int n = 0; n < NW; ++n) {
                acc[mt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h1, bw[n], acc[mt][n], 0, 0, 0);
                acc[mt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h2, bw[n], acc[mt][n], 0, 0, 0);
                acc[mt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(h3, bw[n], acc[mt][n], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int n = 0; n < NW; ++n) red[w][mt][n][lane] = acc[mt][n];
    __syncthreads();
    // wave j % 4 finishes output tile j = (mt, n) (sum over waves in order)
    for (int j = w; j < MT * NW; j += 4) {
        const int mt = j / NW, n = j % NW;
        floatx4 v = red[0][mt][n][lane];
        for (int ww = 1; ww < 4; ++ww) v += red[ww][mt][n][lane];
        const int r = r0 + 16 * n + rl;   // C/D: col = lane & 15 (weight row), row = (lane >> 4) * 4 + i (token)
        if (part) {
            float *pz = part + ((size_t)blockIdx.z * a.nb + t0) * a.R;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = mt * 16 + (lane >> 4) * 4 + i;
                if (t < M && r < a.R) pz[(size_t)t * a.R + r] = v[i];
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = mt * 16 + (lane >> 4) * 4 + i;
            float val = v[i];
            const float up = __shfl(val, lane + 4 < 64 ? lane + 4 : lane, 64);
            if (t >= M || r >= a.R) continue;
            float *yr = yb + (size_t)t * a.ldy;
            switch (a.epi) {
                case EPI_STORE: yr[r] = val; break;
                case EPI_BIAS: yr[r] = val + a.bias[r]; break;
                case EPI_BIAS_SILU: {
                    const float z = val + a.bias[r];
                    yr[r] = z / (1.0f + expf(-z));
                    break;
                }
                case EPI_RESID: yr[r] += val; break;
                case EPI_SWIGLU:
                    if ((r & 7) < 4) yr[(r >> 3) * 4 + (r & 3)] = (val / (1.0f + expf(-val))) * up;
                    break;
            }
        }
    }
}

// split-K tail: y[row] = epilogue(sum over z of part[z][row], z in order);
// grid (outputs / 256, rows)
__global__ __launch_bounds__(256) void k_mgemm_reduce(GemvArgs a, const float *part, int kz) {
    const int t = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
    const int nout = a.epi == EPI_SWIGLU ? a.R / 2 : a.R;
    if (j >= nout) return;
    const size_t zs = (size_t)a.nb * a.R;
    const float *p = part + (size_t)t * a.R;
    float *yr = a.y + (size_t)t * a.ldy;
    if (a.epi == EPI_SWIGLU) {
        const int g = (j >> 2) * 8 + (j & 3);
        float vg = p[g], vu = p[g + 4];
        for (int z = 1; z < kz; ++z) { vg += p[z * zs + g]; vu += p[z * zs + g + 4]; }
        yr[j] = (vg / (1.0f + expf(-vg))) * vu;
        return;
    }
    float val = p[j];
    for (int z = 1; z < kz; ++z) val += p[z * zs + j];
    switch (a.epi) {
        case EPI_STORE: yr[j] = val; break;
        case EPI_BIAS: yr[j] = val + a.bias[j]; break;
        case EPI_BIAS_SILU: {
            const float z = val + a.bias[j];
            yr[j] = z / (1.0f + expf(-z));
            break;
        }
        case EPI_RESID: yr[j] += val; break;
    }
}

}  // namespace

// (also the prefill GEMM's, k_pgemm.hip)
int qtts_row_rms(const float *x, int ldx, int rows, int C, float eps, float *inv, hipStream_t st) {
    hipLaunchKernelGGL(k_row_rms, dim3(rows), dim3(256), 0, st, x, ldx, C, eps, inv);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int qtts_mgemm_reduce(const GemvArgs &a, const float *part, int kz, hipStream_t st) {
    const int nout = a.epi == EPI_SWIGLU ? a.R / 2 : a.R;
    hipLaunchKernelGGL(k_mgemm_reduce, dim3((nout + 255) / 256, a.nb), dim3(256), 0, st, a, part, kz);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Multi-row projection on the matrix cores, any number of rows (64-row chunks
// on grid.y of one launch).  `inv_scratch` (>= nb floats) receives the
// per-row 1/rms when a.norm_w is set.  Returns 1 when the shape is not
// covered (caller uses qtts_gemv), 0 ok, -1 error.
// (QTTS_HIP_MGEMM_KZ: 1 = no split, n = at most n columns; QTTS_HIP_MGEMM_WG:
// split while the grid stays within n workgroups)
static int mgemm_kzmax() {
    static const int v = [] { const char *e = getenv("QTTS_HIP_MGEMM_KZ"); const int x = e ? atoi(e) : 8;
                              return x >= 1 && x <= 16 ? x : 8; }();
    return v;
}
static int mgemm_wgmax() {
    static const int v = [] { const char *e = getenv("QTTS_HIP_MGEMM_WG"); const int x = e ? atoi(e) : 1024;
                              return x >= 256 && x <= 8192 ? x : 1024; }();
    return v;
}

// The split-K partials qtts_mgemm can need, from the same rule it splits by:
// kz columns x nb rows x R outputs with kz <= kzmax and
// R / (16 nw) x ceil(nb / 64) x kz <= wgmax, i.e. kz x nb x R <=
// min(kzmax x rows x R_max, 64 x 16 x 4 x wgmax) (nb / ceil(nb / 64) <= 64, nw <= 4).
size_t qtts_mgemm_part_elems(size_t rows, size_t widest) {
    if (mgemm_kzmax() < 2) return 0;
    const size_t by_rows = (size_t)mgemm_kzmax() * rows * widest;
    const size_t by_grid = (size_t)64 * 16 * 4 * mgemm_wgmax();
    return by_rows < by_grid ? by_rows : by_grid;
}

int qtts_mgemm(const GemvArgs &a, float *inv_scratch, hipStream_t st, float *part, size_t part_elems) {
    if (a.nb < 2 || a.C % 32 || a.R % 16 || a.xcopy || a.table_f32 || (a.norm_w && !inv_scratch) ||
        (a.table && a.norm_w) || (!a.table && (a.ldx % 4 || ((uintptr_t)a.x & 15))) || (a.C % 8))
        return 1;
    if (a.norm_w) hipLaunchKernelGGL(k_row_rms, dim3(a.nb), dim3(256), 0, st, a.x, a.ldx, a.C, a.eps, inv_scratch);
    const int nch = (a.nb + 63) / 64;
    // > 64 rows: widest weight tile group that still gives >= 256 workgroups
    const int nw = nch < 2 || a.R % 64 ? 1 : a.R / 64 * nch >= 256 ? 4 : a.R % 32 == 0 && a.R / 32 * nch >= 256 ? 2 : 1;
    // split-K over grid.z while the grid is under 1024 workgroups (one
    // workgroup per CU leaves one wave per SIMD to wait out every K step's
    // loads alone), each column group >= 8 K steps per wave pair
    const int kzmax = mgemm_kzmax(), wgmax = mgemm_wgmax();
    int kz = 1;
    const int wgs = a.R / (16 * nw) * nch;
    while (part && 2 * kz <= kzmax && wgs * 2 * kz <= wgmax && a.C % (32 * 2 * kz) == 0 &&
           a.C / 32 / (2 * kz) >= 8 && (size_t)2 * kz * a.nb * a.R <= part_elems)
        kz *= 2;
    float *pt = kz > 1 ? part : nullptr;
    const dim3 grid(a.R / (16 * nw), nch, kz);
    if (nw == 4) hipLaunchKernelGGL((k_mgemm<4, 4>), grid, dim3(256), 0, st, a, inv_scratch, pt);
    else if (nw == 2) hipLaunchKernelGGL((k_mgemm<4, 2>), grid, dim3(256), 0, st, a, inv_scratch, pt);
    else if (a.nb <= 16) hipLaunchKernelGGL((k_mgemm<1, 1>), grid, dim3(256), 0, st, a, inv_scratch, pt);
    else if (a.nb <= 32) hipLaunchKernelGGL((k_mgemm<2, 1>), grid, dim3(256), 0, st, a, inv_scratch, pt);
    else hipLaunchKernelGGL((k_mgemm<4, 1>), grid, dim3(256), 0, st, a, inv_scratch, pt);
    qtts_last_kernel = nw == 4 ? "k_mgemm<4,4>" : nw == 2 ? "k_mgemm<4,2>"
                     : a.nb <= 16 ? "k_mgemm<1>" : a.nb <= 32 ? "k_mgemm<2>" : "k_mgemm<4>";
    if (kz > 1) {
        const int nout = a.epi == EPI_SWIGLU ? a.R / 2 : a.R;
        hipLaunchKernelGGL(k_mgemm_reduce, dim3((nout + 255) / 256, a.nb), dim3(256), 0, st, a, pt, kz);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
