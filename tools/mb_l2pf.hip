// mb_l2pf.hip - micro-benchmark (development tool, not product code): does a
// GEMV chain whose weights live in the Infinity Cache (the sub-talker: 20
// distinct matrices, 157 MB) get faster when every workgroup, right after
// issuing its own weight slice, also loads the slice that the SAME workgroup
// index of the NEXT launch will read?  Workgroup b of a 256-workgroup grid
// runs on XCD b % 8 in every launch, so the next launch's slice lands in the
// L2 its reader will use -- if the L2 keeps it across the kernel boundary.
//
// Variants (HIP graph of 16 passes x 20 ops, us per op):
//   pf 0   no prefetch
//   pf 1   next op's slice, plain loads, folded into a never-true store
//   pf 2   next op's slice through LDS DMA (global_load_lds, no registers)
//   pf 3   the product's form (qtts_l2pf.h): one 4-B load per 64-B chunk,
//          offsets computed by selects first (pf 1's per-lane conditions make
//          the compiler reuse in-flight registers and wait for every load)
//   pf 4   the same with one load per 128 B (one per L2 line)
//   hot    every op reads the SAME weights (L2-resident upper bound)
//
// XCC check: a graph of k_op launches with a stamp kernel between them records
// s_getreg(HW_REG_XCC_ID) per workgroup (the premise above: workgroup b on XCD
// b % 8 in EVERY launch); printed as the share of (launch, workgroup) pairs
// that match b % 8 and the number of workgroups whose XCD changed between
// launches.
//
//   hipcc -O3 --offload-arch=gfx950 -Iqwen3-tts-c_amd/csrc/hip tools/mb_l2pf.hip -o tools/mb_l2pf && tools/mb_l2pf
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "qtts_l2pf.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Op {
    const uint16_t *W; int R, C;
    const uint16_t *nW; int nR, nC;   // the next op's weights (prefetch target)
};

__device__ __forceinline__ float dot8(const v4u &w, const float *x) {
    float s = 0.f;
    s = fmaf(__uint_as_float(w.x << 16), x[0], s); s = fmaf(__uint_as_float(w.x & 0xFFFF0000u), x[1], s);
    s = fmaf(__uint_as_float(w.y << 16), x[2], s); s = fmaf(__uint_as_float(w.y & 0xFFFF0000u), x[3], s);
    s = fmaf(__uint_as_float(w.z << 16), x[4], s); s = fmaf(__uint_as_float(w.z & 0xFFFF0000u), x[5], s);
    s = fmaf(__uint_as_float(w.w << 16), x[6], s); s = fmaf(__uint_as_float(w.w & 0xFFFF0000u), x[7], s);
    return s;
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int RW, int NV, int PF>
__global__ __launch_bounds__(256) void k_op(Op o, const float *in, float *out, unsigned *sink) {
    __shared__ __attribute__((aligned(16))) float xs[512 * NV];
    __shared__ __attribute__((aligned(16))) uint32_t pfl[1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int C = 512 * NV;
    float4 xv[NV / 2 > 0 ? NV / 2 : 1];
#pragma unroll
    for (int q = 0; q < NV / 2; ++q) xv[q] = reinterpret_cast<const float4 *>(in)[threadIdx.x + 256 * q];
    v4u wv[RW][NV];
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int k = 0; k < NV; ++k)
            wv[i][k] = reinterpret_cast<const v4u *>(o.W + (size_t)(blockIdx.x * 4 * RW + w + 4 * i) * C)[lane + 64 * k];
    // the next op's slice of this workgroup index: rows [b * nR / 256, +nR / 256), contiguous
    const size_t nbytes = (size_t)o.nR / gridDim.x * o.nC * 2;
    const uint8_t *np = reinterpret_cast<const uint8_t *>(o.nW) + (size_t)blockIdx.x * nbytes;
    unsigned acc = 0;
    if constexpr (PF == 1) {
        v4u pv[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const size_t off = ((size_t)threadIdx.x + 256 * j) * 16;
            pv[j] = off < nbytes ? *reinterpret_cast<const v4u *>(np + off) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < 12; ++j) acc ^= pv[j].x;
    } else if constexpr (PF == 3 || PF == 4) {
        // (the next op's slice: contiguous nbytes; PF 4: one load per 128 B)
        constexpr int CS = PF == 4 ? 7 : 6;
        L2Prefetch p;
        p.base = reinterpret_cast<const unsigned char *>(o.nW); p.pa = (long long)nbytes; p.pb = 0;
        p.chunks = (int)(nbytes >> CS); p.lg = 30; p.ld = 0; p.sink = sink; p.nwg = gridDim.x;
        L2PfRegs r;
        p.cs = CS;
        qtts_l2pf_issue<256, false>(p, blockIdx.x, r, o.W);
#pragma unroll
        for (int j = 0; j < QTTS_PF_LOADS; ++j) acc ^= r.v[j];
    } else if constexpr (PF == 2) {
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const size_t off = ((size_t)threadIdx.x + 256 * j) * 16;
            if (off < nbytes)
                __builtin_amdgcn_global_load_lds((const void *)(np + off), (__attribute__((address_space(3))) void *)pfl,
                                                 16, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < NV / 2; ++q) reinterpret_cast<float4 *>(xs)[threadIdx.x + 256 * q] = xv[q];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) s += dot8(wv[i][k], xs + 8 * (lane + 64 * k));
        s = wsum(s);
        if (lane == 0) out[blockIdx.x * 4 * RW + w + 4 * i] = s * 1e-3f;
    }
    if constexpr (PF == 1 || PF == 3 || PF == 4)
        if (acc == 0x9E3779B9u && threadIdx.x == 0) sink[0] = acc;
}

// XCD of every workgroup of this launch (a vector store from lane 0)
__global__ __launch_bounds__(256) void k_xcc(unsigned *out) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    if (threadIdx.x == 0) out[blockIdx.x] = x;
}
// the same stamp taken inside a weight-streaming k_op-shaped launch
template <int RW, int NV>
__global__ __launch_bounds__(256) void k_op_xcc(Op o, const float *in, float *out, unsigned *xo) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int C = 512 * NV;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const v4u wv = reinterpret_cast<const v4u *>(o.W + (size_t)(blockIdx.x * 4 * RW + w + 4 * i) * C)[lane + 64 * k];
            s += __uint_as_float(wv.x << 16) * in[lane];
        }
    if (threadIdx.x == 0) xo[blockIdx.x] = x;
    if (s == 1.2345e-30f) out[threadIdx.x] = s;
}

#define DISPATCH(o, PF, ...)                                                                              \
    do {                                                                                                  \
        const int rw_ = (o).R / 256 / 4, nv_ = (o).C / 512;                                                \
        if (rw_ == 4 && nv_ == 2) hipLaunchKernelGGL((k_op<4, 2, PF>), dim3(256), dim3(256), 0, __VA_ARGS__); \
        else if (rw_ == 1 && nv_ == 4) hipLaunchKernelGGL((k_op<1, 4, PF>), dim3(256), dim3(256), 0, __VA_ARGS__); \
        else if (rw_ == 6 && nv_ == 2) hipLaunchKernelGGL((k_op<6, 2, PF>), dim3(256), dim3(256), 0, __VA_ARGS__); \
        else if (rw_ == 1 && nv_ == 6) hipLaunchKernelGGL((k_op<1, 6, PF>), dim3(256), dim3(256), 0, __VA_ARGS__); \
    } while (0)

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int Hs = 1024, QKV = 4096, AD = 2048, I = 3072, L = 5;
    std::vector<Op> ops;
    size_t wtot = 0;
    auto W = [&](int R, int C) {
        uint16_t *p;
        CK(hipMalloc(&p, (size_t)R * C * 2));
        std::vector<uint16_t> h((size_t)R * C);
        for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (uint16_t)(i * 2654435761u >> 28);
        CK(hipMemcpy(p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        wtot += h.size() * 2;
        return p;
    };
    for (int l = 0; l < L; ++l) {
        ops.push_back({W(QKV, Hs), QKV, Hs});
        ops.push_back({W(Hs, AD), Hs, AD});
        ops.push_back({W(2 * I, Hs), 2 * I, Hs});
        ops.push_back({W(Hs, I), Hs, I});
    }
    for (size_t i = 0; i < ops.size(); ++i) {
        const Op &n = ops[(i + 1) % ops.size()];
        ops[i].nW = n.W; ops[i].nR = n.R; ops[i].nC = n.C;
    }
    printf("chain: %zu ops, %.1f MB of weights\n", ops.size(), wtot / 1e6);
    float *va, *vb;
    unsigned *sink;
    CK(hipMalloc(&va, 8192 * 4));
    CK(hipMalloc(&vb, 8192 * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(va, 0, 8192 * 4));
    CK(hipMemset(vb, 0, 8192 * 4));
    const int passes = 16;
    auto timed = [&](auto rec) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        rec();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        const int reps = 10;
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return ms * 1e3f / (reps * passes * ops.size());
    };
    {   // XCC premise: 64 launches alternating the stamp kernel and a gate|up-shaped stamped k_op
        const int NL = 64;
        unsigned *xo;
        CK(hipMalloc(&xo, (size_t)NL * 256 * 4));
        CK(hipMemset(xo, 0xff, (size_t)NL * 256 * 4));
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int l = 0; l < NL; ++l) {
            if (l & 1) hipLaunchKernelGGL(k_xcc, dim3(256), dim3(256), 0, st, xo + (size_t)l * 256);
            else hipLaunchKernelGGL((k_op_xcc<6, 2>), dim3(256), dim3(256), 0, st, ops[2 + 4 * ((l / 2) % L)], va, vb,
                                    xo + (size_t)l * 256);
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        std::vector<unsigned> h((size_t)NL * 256);
        CK(hipMemcpy(h.data(), xo, h.size() * 4, hipMemcpyDeviceToHost));
        int match = 0, changed = 0, bad = 0;
        int hist[8][8] = {};
        for (int l = 0; l < NL; ++l)
            for (int b = 0; b < 256; ++b) {
                const unsigned x = h[(size_t)l * 256 + b];
                if (x > 7) { ++bad; continue; }
                match += x == (unsigned)(b % 8);
                if (l > 0 && h[(size_t)(l - 1) * 256 + b] != x) ++changed;
                if (l == 0) hist[b % 8][x]++;
            }
        printf("xcc: %d launches x 256 workgroups: %d of %d (launch, workgroup) pairs on XCD b %% 8, "
               "%d workgroup XCD changes between consecutive launches, %d unreadable\n",
               NL, match, NL * 256 - bad, changed, bad);
        printf("xcc: launch 0, workgroups b = 0..15 ->");
        for (int b = 0; b < 16; ++b) printf(" %u", h[b]);
        printf("\nxcc: launch 1, workgroups b = 0..15 ->");
        for (int b = 0; b < 16; ++b) printf(" %u", h[256 + b]);
        printf("\n");
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    for (int rep = 0; rep < 2; ++rep) {
        float t0 = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (auto &o : ops) { DISPATCH(o, 0, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        float t1 = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (auto &o : ops) { DISPATCH(o, 1, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        float t2 = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (auto &o : ops) { DISPATCH(o, 2, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        float t3 = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (auto &o : ops) { DISPATCH(o, 3, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        float t4 = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (auto &o : ops) { DISPATCH(o, 4, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        // hot: every launch of a shape reads the first layer's matrix of that shape
        float th = timed([&] { int i = 0; for (int p = 0; p < passes; ++p) for (size_t k = 0; k < ops.size(); ++k) { Op o = ops[k % 4]; DISPATCH(o, 0, st, o, (i & 1) ? vb : va, (i & 1) ? va : vb, sink); ++i; } });
        printf("us per op: pf0 %.2f  pf1 %.2f  pf2 %.2f  pf3 %.2f  pf4 %.2f  hot %.2f\n", t0, t1, t2, t3, t4, th);
    }
    return 0;
}
