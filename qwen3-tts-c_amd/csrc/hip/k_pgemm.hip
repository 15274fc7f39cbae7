// k_pgemm.hip - the talker prefill's projections over many prompt rows
// (T.c:254-472, the reference's kernel_matmul_bf16, K.c:185-207) as an
// LDS-tiled GEMM on v_mfma_f32_32x32x16_bf16 over PRE-SPLIT activations.
//
// y[m][n] = sum_k x[m][k] W[n][k], x fp32 (RMS-normalised rows, K.c:27-39),
// W bf16.  Each x is written once as three exact bf16 planes x1 + x2 + x3
// (k_split3: x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2)); bf16 x
// bf16 products are exact in fp32, so the GEMM is an fp32 product up to
// summation order, like the decode GEMVs and k_mgemm.
//
// k_mgemm (the round-1..5 kernel) re-read every 64-row activation chunk from
// L2 and re-did its split once per 64-row weight tile group (at ~800
// voice-clone rows the gate|up projection read ~1.3 GB of L2 and spent ~4 G
// VALU operations on splits per launch; MFMA busy 0.14).  Here:
//   k_split3  one pass: x (+ RMSNorm, its statistic formed in the same
//             launch) -> planes [3][Mp][K] (Mp: rows rounded up to the 128-row
//             tile, pad rows zero).
//   k_pgemm   a 128 x 256 (rows x weight rows) tile per 512-thread workgroup,
//             2 x 4 waves of 64 x 64 (2 x 2 MFMA 32x32 tiles each), or
//             128 x 128 on 2 x 2 waves for a single row tile; 32-deep K
//             stages, the loads of the stage after next (8 16-B loads per
//             thread, two register sets) in flight while this one's 24 MFMAs
//             run; both operands in LDS, rows of 4
//             16-B chunks XOR-swizzled by (row >> 2) & 3 so each 16-lane
//             ds_read_b128 group hits 16 distinct bank quads.  Split-K over
//             grid.z (partials summed in column order with the epilogue by
//             k_mgemm_reduce) where the tiles alone would not fill the chip.
// Epilogues: store / residual add / SwiGLU over the interleaved gate|up row
// quads (the up row n + 4 is lane + 4 of the same 32-wide tile).
#include <type_traits>

#include "qtts_common.h"
#include "qtts_kernels.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

__device__ __forceinline__ unsigned short f2bf_rn_u(float f) {
    uint32_t u = __float_as_uint(f);
    u = u + 0x7FFFu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f_u(unsigned short b) { return __uint_as_float(((uint32_t)b) << 16); }

// x rows (+ RMSNorm, K.c:27-39) -> three bf16 planes; one 256-thread
// workgroup per row (grid Mp), 8 consecutive k per thread and pass.  With a
// norm the row's 1/rms is formed here first, exactly as k_row_rms does it
// (strided squares, block_sum256, rms_inv), then x * inv * w as k_mgemm
// applies it.  Rows >= M are written as zeros.
__global__ __launch_bounds__(256) void k_split3(const float *x, int ldx, int M, int K, const float *norm_w,
                                                float eps, unsigned short *planes, int Mp) {
    __shared__ float red[4];
    const int t = blockIdx.x, tid = threadIdx.x;
    const float *xr = x + (size_t)(t < M ? t : 0) * ldx;
    float iv = 1.f;
    if (norm_w && t < M) {
        float ss = 0.f;
        for (int c = tid; c < K; c += 256) ss += xr[c] * xr[c];
        iv = rms_inv(block_sum256(ss, red), K, eps);
    }
    for (int k = tid * 8; k < K; k += 256 * 8) {
        float v[8];
        if (t < M) {
            const float4 a = *reinterpret_cast<const float4 *>(xr + k);
            const float4 b = *reinterpret_cast<const float4 *>(xr + k + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            if (norm_w) {
                const float4 n0 = *reinterpret_cast<const float4 *>(norm_w + k);
                const float4 n1 = *reinterpret_cast<const float4 *>(norm_w + k + 4);
                const float nw[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = v[j] * iv * nw[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;
        }
        unsigned short h[3][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned short b1 = f2bf_rn_u(v[j]);
            const float e1 = v[j] - bf2f_u(b1);
            const unsigned short b2 = f2bf_rn_u(e1);
            const float e2 = e1 - bf2f_u(b2);
            h[0][j] = b1;
            h[1][j] = b2;
            h[2][j] = f2bf_rn_u(e2);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            v4u q;
            q.x = h[p][0] | ((uint32_t)h[p][1] << 16);
            q.y = h[p][2] | ((uint32_t)h[p][3] << 16);
            q.z = h[p][4] | ((uint32_t)h[p][5] << 16);
            q.w = h[p][6] | ((uint32_t)h[p][7] << 16);
            *reinterpret_cast<v4u *>(planes + ((size_t)p * Mp + t) * K + k) = q;
        }
    }
}

constexpr int BM = 128, BK = 32;
constexpr int A_CH = 3 * BM * (BK / 8);   // 16-B chunks of the three A tiles per stage (1536)

// swizzled 16-B chunk index of (row, chunk) in a [rows][4 chunks] tile
__device__ __forceinline__ int swz(int row, int c) { return row * 4 + (c ^ ((row >> 2) & 3)); }

// WN waves along the weight rows: a 128 x 64 WN tile per workgroup of 2 WN
// waves (WN = 2: 128 x 128, 256 threads; WN = 4: 128 x 256, 512 threads --
// every activation stage staged once serves twice the weight rows, which
// halves the launch's activation-plane reads from L2, the bulk of its traffic
// while the planes are re-read once per weight tile)
template <int WN>
__global__ __launch_bounds__(128 * WN) void k_pgemm(GemvArgs a, const unsigned short *planes, int Mp, float *part) {
    constexpr int NT = 128 * WN, BN = 64 * WN;
    constexpr int W_CH = BN * (BK / 8);   // 16-B chunks of the W tile per stage
    constexpr int A_PT = A_CH / NT, W_PT = W_CH / NT;
    static_assert(A_CH % NT == 0 && W_CH % NT == 0, "k_pgemm: stage chunks per thread");
    __shared__ __attribute__((aligned(16))) v4u As[2][3 * BM * 4];
    __shared__ __attribute__((aligned(16))) v4u Ws[2][BN * 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w & 1, wn = w >> 1;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int K = a.C, N = a.R, M = a.nb;
    const int nst = K / BK / gridDim.z, st0 = blockIdx.z * nst;

    // per-thread global chunk sources of one stage (advanced by BK per stage)
    const v4u *ga[A_PT];
    int la[A_PT];
#pragma unroll
    for (int j = 0; j < A_PT; ++j) {
        const int q = tid + NT * j, p = q / (BM * 4), r = (q / 4) % BM, c = q % 4;
        ga[j] = reinterpret_cast<const v4u *>(planes + ((size_t)p * Mp + m0 + r) * K + (size_t)st0 * BK + 8 * c);
        la[j] = p * BM * 4 + swz(r, c);
    }
    const v4u *gw[W_PT];
    int lw[W_PT];
#pragma unroll
    for (int j = 0; j < W_PT; ++j) {
        const int q = tid + NT * j, r = q / 4, c = q % 4;
        const int row = n0 + r < N ? n0 + r : N - 1;
        gw[j] = reinterpret_cast<const v4u *>(a.W + (size_t)row * K + (size_t)st0 * BK + 8 * c);
        lw[j] = swz(r, c);
    }
    // stage s + 2's loads are issued while stage s computes (two register
    // sets): one stage of MFMAs (~0.3 us per wave) does not cover an L2 / MALL
    // round trip
    v4u ra[2][A_PT], rw[2][W_PT];
#pragma unroll
    for (int j = 0; j < A_PT; ++j) ra[0][j] = ga[j][0];
#pragma unroll
    for (int j = 0; j < W_PT; ++j) rw[0][j] = gw[j][0];
#pragma unroll
    for (int j = 0; j < A_PT; ++j) ra[1][j] = ga[j][BK / 8];
#pragma unroll
    for (int j = 0; j < W_PT; ++j) rw[1][j] = gw[j][BK / 8];
#pragma unroll
    for (int j = 0; j < A_PT; ++j) As[0][la[j]] = ra[0][j];
#pragma unroll
    for (int j = 0; j < W_PT; ++j) Ws[0][lw[j]] = rw[0][j];
    __syncthreads();

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int fr = lane & 31, fh = lane >> 5;
    // (stage s's register set is s & 1; the loop body is unrolled by 2 so the
    // set index is a constant.  No branch around any load or LDS store: at a
    // join of paths with different loads in flight the compiler's wait-count
    // pass assumes the worst and drains every load (vmcnt(0)), serialising the
    // stages -- the tail re-loads stage nst - 1 and stores it to the idle buffer)
    auto stage = [&](int s, auto setc) {
        constexpr int set = decltype(setc)::value;
        const int cur = s & 1;
        const int sn = s + 2 < nst ? s + 2 : nst - 1;   // stage s + 2 into the set stage s came in
#pragma unroll
        for (int j = 0; j < A_PT; ++j) ra[set][j] = ga[j][sn * (BK / 8)];
#pragma unroll
        for (int j = 0; j < W_PT; ++j) rw[set][j] = gw[j][sn * (BK / 8)];
        // (the scheduler would sink these loads behind the MFMAs, next to the
        // LDS stores that wait for the other set: one stage of cover, not two)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = 2 * ks + fh;
            bf16x8 bf[2];
#pragma unroll
            for (int tn = 0; tn < 2; ++tn)
                bf[tn] = __builtin_bit_cast(bf16x8, Ws[cur][swz(64 * wn + 32 * tn + fr, c)]);
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int tm = 0; tm < 2; ++tm) {
                    const bf16x8 af = __builtin_bit_cast(bf16x8, As[cur][p * BM * 4 + swz(64 * wm + 32 * tm + fr, c)]);
#pragma unroll
                    for (int tn = 0; tn < 2; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf[tn], acc[tm][tn], 0, 0, 0);
                }
            }
        }
        // stage s + 1 (the other set) into the other buffer
#pragma unroll
        for (int j = 0; j < A_PT; ++j) As[cur ^ 1][la[j]] = ra[set ^ 1][j];
#pragma unroll
        for (int j = 0; j < W_PT; ++j) Ws[cur ^ 1][lw[j]] = rw[set ^ 1][j];
        __syncthreads();
    };
    for (int s = 0; s < nst; s += 2) {   // (nst is even: qtts_pgemm)
        stage(s, std::integral_constant<int, 0>{});
        stage(s + 1, std::integral_constant<int, 1>{});
    }

    // epilogue: acc[tm][tn][e] is (row m, weight row n) with
    // m = m0 + 64 wm + 32 tm + (e & 3) + 8 (e >> 2) + 4 fh, n = n0 + 64 wn + 32 tn + fr
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
            const int n = n0 + 64 * wn + 32 * tn + fr;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + 64 * wm + 32 * tm + (e & 3) + 8 * (e >> 2) + 4 * fh;
                const float v = acc[tm][tn][e];
                const float up = __shfl(v, lane + 4 < 64 ? lane + 4 : lane, 64);
                if (m >= M || n >= N) continue;
                if (part) {
                    part[((size_t)blockIdx.z * M + m) * N + n] = v;
                    continue;
                }
                float *yr = a.y + (size_t)m * a.ldy;
                switch (a.epi) {
                    case EPI_STORE: yr[n] = v; break;
                    case EPI_RESID: yr[n] += v; break;
                    case EPI_SWIGLU:
                        if ((n & 7) < 4) yr[(n >> 3) * 4 + (n & 3)] = (v / (1.0f + expf(-v))) * up;
                        break;
                }
            }
        }
    }
}

}  // namespace

// The plane scratch qtts_pgemm needs for `rows` activation rows of width <= K.
size_t qtts_pgemm_plane_elems(size_t rows, size_t K) {
    return (size_t)3 * ((rows + BM - 1) / BM * BM) * K;
}

// Returns 1 when the shape is not covered (the caller falls back to
// qtts_mgemm), 0 ok, -1 error.  inv_scratch >= nb floats (per-row 1/rms, by
// k_row_rms in qtts_mgemm's file), planes >= qtts_pgemm_plane_elems(nb, C).
int qtts_pgemm(const GemvArgs &a, float *inv_scratch, unsigned short *planes, size_t plane_elems, hipStream_t st,
               float *part, size_t part_elems) {
    if (a.nb < 17 || a.C % 256 || a.R % 32 || !a.x || a.table || a.table_f32 || a.xadd || a.xcopy || a.bias ||
        a.ldx % 4 || ((uintptr_t)a.x & 15) ||
        (a.epi != EPI_STORE && a.epi != EPI_RESID && a.epi != EPI_SWIGLU) || !planes)
        return 1;
    const int Mp = (a.nb + BM - 1) / BM * BM;
    if ((a.C / BK) % 2) return 1;   // (an even stage count per column: k_pgemm's loop)
    if ((size_t)3 * Mp * a.C > plane_elems) return 1;
    hipLaunchKernelGGL(k_split3, dim3(Mp), dim3(256), 0, st, a.x, a.ldx, a.nb, a.C, a.norm_w, a.eps, planes, Mp);
    // split-K while the tiles would not fill the chip (one workgroup per CU
    // cannot hide its own stage loads), each column >= 8 stages
    // The weight-row width of a workgroup's tile: 256 once there are several
    // 128-row tiles (the plane re-reads dominate: voice-clone batch-8 prefill
    // 10.1 -> 9.15 ms), 128 for one row tile (half the weight tiles would need
    // twice the split-K partials: voice-clone batch-1 prefill 6.87 vs 7.16 ms;
    // profiles/r06q_ab_pgemm_bn.txt).  QTTS_HIP_PGEMM_BN=128|256 forces one
    // (read per call: a test switches it between contexts of one process).
    const char *bne = getenv("QTTS_HIP_PGEMM_BN");
    const int BN = bne && atoi(bne) == 128 ? 128 : bne && atoi(bne) == 256 ? 256 : Mp >= 2 * BM ? 256 : 128;
    const int tiles = (a.R + BN - 1) / BN * (Mp / BM);
    int kz = 1;
    while (part && tiles * kz < 256 && kz < 8 && (a.C / BK) % (4 * kz) == 0 && a.C / BK / (2 * kz) >= 8 &&
           (size_t)2 * kz * a.nb * a.R <= part_elems)
        kz *= 2;
    const dim3 grid((a.R + BN - 1) / BN, Mp / BM, kz);
    if (BN == 256) {
        hipLaunchKernelGGL(k_pgemm<4>, grid, dim3(512), 0, st, a, planes, Mp, kz > 1 ? part : nullptr);
        qtts_last_kernel = "k_pgemm<4>";
    } else {
        hipLaunchKernelGGL(k_pgemm<2>, grid, dim3(256), 0, st, a, planes, Mp, kz > 1 ? part : nullptr);
        qtts_last_kernel = "k_pgemm<2>";
    }
    if (kz > 1 && qtts_mgemm_reduce(a, part, kz, st) != 0) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
