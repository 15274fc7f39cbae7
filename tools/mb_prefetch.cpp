// mb_prefetch.cpp - micro-benchmark (development tool): a talker-like chain of
// batch-1 GEMV layers (QKV, O, gate|up, down; distinct weights per layer, so
// they stream from HBM) captured in one HIP graph, with and without a
// parallel graph branch that reads layer l+1's weights (pulling them into the
// Infinity Cache) while layer l computes.  Prints us per layer.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iqwen3-tts-c_amd/csrc/hip tools/mb_prefetch.cpp \
//         -Lqwen3-tts-c_amd/lib -lqwen_tts_amd -Wl,-rpath,'$ORIGIN/../qwen3-tts-c_amd/lib' -o tools/mb_prefetch
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "qtts_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// streams `n16` 16-B words through the caches (the value is never used)
__global__ __launch_bounds__(256) void k_touch(const uint4 *p, size_t n16, unsigned *sink) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
    const int L = 28, H = 2048, I = 6144, QKV = 4096;
    struct M { int R, C, epi; bool norm; };
    const M mats[4] = {{QKV, H, EPI_STORE, true}, {H, 2048, EPI_RESID, false}, {2 * I, H, EPI_SWIGLU, true},
                       {H, I, EPI_RESID, false}};
    std::vector<bf16_t *> W(L * 4);
    size_t layer_bytes = 0;
    for (int m = 0; m < 4; ++m) layer_bytes += (size_t)mats[m].R * mats[m].C * 2;
    bf16_t *pool;
    CK(hipMalloc(&pool, layer_bytes * L));
    CK(hipMemset(pool, 0x3c, layer_bytes * L));
    {
        size_t off = 0;
        for (int l = 0; l < L; ++l)
            for (int m = 0; m < 4; ++m) {
                W[l * 4 + m] = reinterpret_cast<bf16_t *>(reinterpret_cast<char *>(pool) + off);
                off += (size_t)mats[m].R * mats[m].C * 2;
            }
    }
    float *x, *y, *h, *nw;
    unsigned *sink;
    CK(hipMalloc(&x, 16384 * 4));
    CK(hipMalloc(&y, 16384 * 4));
    CK(hipMalloc(&h, 16384 * 4));
    CK(hipMalloc(&nw, 16384 * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(x, 0, 16384 * 4));
    CK(hipMemset(y, 0, 16384 * 4));
    CK(hipMemset(h, 0, 16384 * 4));
    CK(hipMemset(nw, 0, 16384 * 4));
    hipStream_t st, sp;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sp, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(L + 2);
    for (auto &evi : ev) CK(hipEventCreateWithFlags(&evi, hipEventDisableTiming));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grids[] = {0, 32, 64, 128};
    for (int nt = 0; nt < 2; ++nt)
        for (int pg : grids) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            if (pg) {   // fork the prefetch branch
                CK(hipEventRecord(ev[L], st));
                CK(hipStreamWaitEvent(sp, ev[L], 0));
            }
            for (int l = 0; l < L; ++l) {
                if (pg && l + 1 < L) {   // layer l+1's weights, beside layer l
                    CK(hipEventRecord(ev[l], st));
                    CK(hipStreamWaitEvent(sp, ev[l], 0));
                    hipLaunchKernelGGL(k_touch, dim3(pg), dim3(256), 0, sp,
                                       reinterpret_cast<const uint4 *>(W[(l + 1) * 4]), layer_bytes / 16, sink);
                }
                for (int m = 0; m < 4; ++m) {
                    GemvArgs a;
                    a.W = W[l * 4 + m]; a.R = mats[m].R; a.C = mats[m].C; a.epi = mats[m].epi; a.nt = nt; a.nb = 1;
                    a.x = m == 3 ? h : x; a.ldx = a.C; a.y = m == 2 ? h : m == 0 ? y : x; a.ldy = a.R;
                    a.norm_w = mats[m].norm ? nw : nullptr;
                    if (qtts_gemv(a, st)) { printf("launch failed\n"); return 1; }
                }
            }
            if (pg) {   // join
                CK(hipEventRecord(ev[L + 1], sp));
                CK(hipStreamWaitEvent(st, ev[L + 1], 0));
            }
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, st));
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("nt=%d prefetch grid %4d: %7.2f us per layer (%.0f GB/s of weights)\n", nt, pg,
                   ms * 1e3 / (10 * L), layer_bytes / (ms * 1e-3 / (10 * L)) / 1e9);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    return 0;
}
