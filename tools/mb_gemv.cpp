// mb_gemv.cpp - GEMV configuration sweep (development tool): times the batch-1
// weight-streaming GEMV (qtts_gemv) on the 1.7B decode shapes for each KSPLIT,
// NT on/off, back-to-back launches captured in a HIP graph.  MB_BATCH=B times
// the lock-step batch path (qtts_gemv at nb = B: k_gemvm) instead, one line
// per shape (talker weights nt, sub-talker default policy).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iqwen3-tts-c_amd/csrc/hip tools/mb_gemv.cpp \
//         -Lqwen3-tts-c_amd/lib -lqwen_tts_amd -Wl,-rpath,$PWD/qwen3-tts-c_amd/lib -o tools/mb_gemv
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "qtts_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
    struct Shape { const char *name; int R, C, epi; bool norm; };
    const Shape shapes[] = {
        {"talker qkv 4096x2048", 4096, 2048, EPI_STORE, true},
        {"talker o 2048x2048", 2048, 2048, EPI_RESID, false},
        {"talker gate|up 12288x2048", 12288, 2048, EPI_SWIGLU, true},
        {"talker down 2048x6144", 2048, 6144, EPI_RESID, false},
        {"codec head 3072x2048", 3072, 2048, EPI_STORE, true},
        {"sub qkv 4096x1024", 4096, 1024, EPI_STORE, true},
        {"sub o 1024x2048", 1024, 2048, EPI_RESID, false},
        {"sub gate|up 6144x1024", 6144, 1024, EPI_SWIGLU, true},
        {"sub down 1024x3072", 1024, 3072, EPI_RESID, false},
    };
    // distinct weight copies: 24 = the sweep streams from HBM; MB_NW=1 = the
    // weights stay resident in the Infinity Cache across replays
    const int NW = getenv("MB_NW") ? atoi(getenv("MB_NW")) : 24;
    const bool talker_only = getenv("MB_TALKER") != nullptr;
    const int NB = getenv("MB_BATCH") ? atoi(getenv("MB_BATCH")) : 1;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape &s : shapes) {
        if (talker_only && s.name[0] != 't') continue;
        const size_t wn = (size_t)s.R * s.C;
        std::vector<bf16_t *> W(NW);
        for (auto &w : W) {
            CK(hipMalloc(&w, wn * 2));
            CK(hipMemset(w, 0x3c, wn * 2));
        }
        float *x, *y, *nw;
        CK(hipMalloc(&x, (size_t)s.C * 4 * NB));
        CK(hipMalloc(&y, (size_t)s.R * 4 * NB));
        CK(hipMalloc(&nw, s.C * 4));
        CK(hipMemset(x, 0, (size_t)s.C * 4 * NB));
        CK(hipMemset(y, 0, (size_t)s.R * 4 * NB));
        CK(hipMemset(nw, 0, s.C * 4));
        for (int nt = 0; nt < 2; ++nt)
            for (int ks = 0; ks <= 32; ks = ks ? 2 * ks : 1) {   // ks 0: the launcher's own choice
                if (NB > 1 && (ks > 1 || nt != (s.name[0] == 't'))) continue;
                if (getenv("MB_AUTO") && ks != 0) continue;
                if (ks && (s.C / 64) % ks) continue;
                if (s.epi == EPI_SWIGLU && ks > 4) continue;
                GemvArgs a;
                a.R = s.R; a.C = s.C; a.ksplit = ks; a.nt = nt; a.nb = NB; a.x = x; a.ldx = s.C; a.y = y;
                a.ldy = s.R; if (NB > 1) a.ksplit = 0; a.epi = s.epi; a.norm_w = s.norm ? nw : nullptr;
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
                for (int i = 0; i < 96; ++i) {
                    a.W = W[i % NW];
                    if (qtts_gemv(a, st)) { printf("launch failed\n"); exit(1); }
                }
                CK(hipStreamEndCapture(st, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGraphLaunch(ge, st));
                CK(hipStreamSynchronize(st));
                CK(hipEventRecord(e0, st));
                for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / (5 * 96);
                if (NB > 1) printf("B=%-2d %-28s %s nt=%d  %7.2f us  %6.0f GB/s\n", NB, s.name, qtts_last_kernel, nt, us,
                                   wn * 2 / (us * 1e-6) / 1e9);
                else printf("%-28s %-26s ks=%2d nt=%d grid=%5d  %7.2f us  %6.0f GB/s\n", s.name, ks ? "" : qtts_last_kernel,
                            ks, nt, ks ? (s.R + 32 / ks - 1) / (32 / ks) : 0,
                       us, wn * 2 / (us * 1e-6) / 1e9);
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(g));
            }
        for (auto &w : W) CK(hipFree(w));
        CK(hipFree(x));
        CK(hipFree(y));
        CK(hipFree(nw));
    }
    return 0;
}
