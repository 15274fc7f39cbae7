// mb_sample.hip - micro-benchmark (development tool): where the on-device
// sampler's time goes.  Times 200 back-to-back launches (one HIP graph) of
// kernels that stop after successive phases of the fast path on the same
// 2048-logit row (sub-talker shape, top-k 50, T 0.9):
//   0 empty kernel            (launch floor)
//   1 logits loaded            (+ a store of their sum)
//   2 + radix select           (k-th largest key)
//   3 + selection, rank, draw  (= the full fast path, qtts_sample_dev.h)
// and the distance-binned path (sample_dist, k <= 64) cut after its phases:
//   11 + max / eligible count (barrier 1)
//   12 + distance histogram (barrier 2), merged-histogram scan
//   13 + candidate compaction (barrier 3)
//   14 = the whole draw (wave 0 ranks, sums, draws)
// and the same on 1024 threads (sample_dist_nt, 2 ids per thread):
//   21 + max / count (barrier 1)   22 + shared histogram, scan (barrier 2)
//   23 + candidate slots (barrier 3)  24 + rank slices (barrier 4)
//   25 + scatter to rank order, read back   26 + sequential sum
//   29 = the whole draw              30 = k_sample_w's sample_fast_nt
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Iqwen3-tts-c_amd/csrc/hip tools/mb_sample.hip -o tools/mb_sample
#include "qtts_sample_dev.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

using namespace qtts_samp;

template <int PHASE>
__global__ __launch_bounds__(256) void k_phase(SampArgs a, float *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    FastSmem &fs = *reinterpret_cast<FastSmem *>(smraw);
    const int tid = threadIdx.x;
    if constexpr (PHASE == 0) {
        if (tid == 0) sink[0] = 1.f;
        return;
    }
    constexpr int EM = 8;
    const int n = a.n, E = (n + 255) / 256;
    float v[EM];
#pragma unroll
    for (int j = 0; j < EM; ++j) v[j] = (j < E && tid * E + j < n) ? div_rn(ld_sc1(a.logits + tid * E + j), a.temp) : -INFINITY;
    if constexpr (PHASE == 1) {
        float s = 0.f;
        for (int j = 0; j < EM; ++j) s += v[j];
        if (s == 12345.f) sink[0] = s;
        return;
    }
    if constexpr (PHASE == 2) {
        uint32_t kk[EM];
#pragma unroll
        for (int j = 0; j < EM; ++j) kk[j] = (j < E && tid * E + j < n && v[j] > -FLT_MAX) ? okey(v[j]) : 0u;
        uint32_t T, Tm;
        int take_eq, ne;
        radix_select_regs<EM>(fs, kk, E, a.top_k, T, Tm, take_eq, ne);
        if (tid == 0) sink[0] = (float)T + take_eq + ne;
        return;
    }
    uint32_t rng = 0x42280000u;
    const uint64_t etab = kExp2fTab[tid & 31];
    if constexpr (PHASE > 10) {
        uint32_t kk[EM];
#pragma unroll
        for (int j = 0; j < EM; ++j) kk[j] = (j < E && tid * E + j < n && v[j] > -FLT_MAX) ? okey(v[j]) : 0u;
        const int t = sample_dist<EM, PHASE - 10>(fs, v, kk, E, a.top_k, rng, etab);
        if (tid == 0) sink[0] = (float)t;
        return;
    }
    const int t = sample_fast_regs<EM>(fs, v, E, n, a.top_k, rng, etab);
    if (tid == 0) sink[0] = (float)t;
}

template <int PHASE>
__global__ __launch_bounds__(1024) void k_phase_w(SampArgs a, float *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    FastSmemNT<1024> &fs = *reinterpret_cast<FastSmemNT<1024> *>(smraw);
    const int tid = threadIdx.x;
    constexpr int EM = 2;
    const int n = a.n, E = (n + 1023) / 1024;
    float v[EM];
    uint32_t kk[EM];
    int id[EM];
    float raw[EM];
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        id[j] = tid * E + j;
        raw[j] = a.logits[id[j] < n ? id[j] : n - 1];   // every load in flight at once
    }
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        v[j] = (j < E && id[j] < n) ? div_rn(raw[j], a.temp) : -INFINITY;
        kk[j] = (j < E && id[j] < n && v[j] > -FLT_MAX) ? okey(v[j]) : 0u;
    }
    uint32_t rng = 0x42280000u;
    const uint64_t etab = kExp2fTab[tid & 31];
    int t;
    if constexpr (PHASE == 30) t = sample_fast_nt<1024, EM>(fs, v, E, n, a.top_k, rng, etab);
    else t = sample_dist_nt<1024, EM, PHASE - 20>(fs, v, kk, id, a.top_k, rng, etab);
    if (tid == 0) sink[0] = (float)t;
}

template <int PHASE>
static float time_phase(const SampArgs &a, float *sink, hipStream_t st) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 200; ++i) {
        if constexpr (PHASE > 20)
            hipLaunchKernelGGL((k_phase_w<PHASE>), dim3(1), dim3(1024), sizeof(FastSmemNT<1024>), st, a, sink);
        else
            hipLaunchKernelGGL((k_phase<PHASE>), dim3(1), dim3(256), sizeof(FastSmem), st, a, sink);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return ms * 1e3f / 1000.f;
}

int main() {
    const int n = 2048;
    float *lg, *sink;
    CK(hipMalloc(&lg, n * 4));
    CK(hipMalloc(&sink, 64));
    float h[n];
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {   // logits ~ a few units wide, like a sampled head
        s = s * 1664525u + 1013904223u;
        h[i] = ((s >> 8) / 16777216.0f - 0.5f) * 8.0f;
    }
    CK(hipMemcpy(lg, h, n * 4, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    SampArgs a;
    a.logits = lg; a.ld = n; a.n = n; a.nb = 1; a.top_k = 50; a.top_p = 1.f; a.temp = 0.9f;
    printf("phase 0 empty kernel        %6.2f us\n", time_phase<0>(a, sink, st));
    printf("phase 1 + logits loaded     %6.2f us\n", time_phase<1>(a, sink, st));
    printf("phase 2 + radix select      %6.2f us\n", time_phase<2>(a, sink, st));
    printf("phase 3 + select/rank/draw  %6.2f us\n", time_phase<3>(a, sink, st));
    printf("dist 11 + max / count       %6.2f us\n", time_phase<11>(a, sink, st));
    printf("dist 12 + histogram, scan   %6.2f us\n", time_phase<12>(a, sink, st));
    printf("dist 13 + compaction        %6.2f us\n", time_phase<13>(a, sink, st));
    printf("dist 14 = whole draw        %6.2f us\n", time_phase<14>(a, sink, st));
    printf("w1024 21 + max / count      %6.2f us\n", time_phase<21>(a, sink, st));
    printf("w1024 22 + histogram, scan  %6.2f us\n", time_phase<22>(a, sink, st));
    printf("w1024 23 + candidate slots  %6.2f us\n", time_phase<23>(a, sink, st));
    printf("w1024 24 + rank slices      %6.2f us\n", time_phase<24>(a, sink, st));
    printf("w1024 25 + scatter, read    %6.2f us\n", time_phase<25>(a, sink, st));
    printf("w1024 26 + sequential sum   %6.2f us\n", time_phase<26>(a, sink, st));
    printf("w1024 29 = whole draw       %6.2f us\n", time_phase<29>(a, sink, st));
    printf("w1024 30 sample_fast_nt     %6.2f us\n", time_phase<30>(a, sink, st));
    return 0;
}
