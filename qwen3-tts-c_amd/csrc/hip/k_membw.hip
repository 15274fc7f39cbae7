// k_membw.hip - the box's own HBM stream bandwidth, measured beside the
// roofline (achieved bandwidth against a stream-copy figure
// measured on the same GPU as well as the 8 TB/s nominal).
//
// Two kernels over a buffer far larger than the 256 MB Infinity Cache:
//   read  -- every lane keeps 8 non-temporal 16-B loads in flight per
//            iteration and folds them into one register (the weight-stream
//            shape of the decode GEMVs);
//   copy  -- the same loads, each stored to a second buffer (read + write
//            bytes counted, as a stream copy is quoted).
// Grid: 8 workgroups of 256 threads per CU, grid-stride over 128-B-per-lane
// blocks, so every CU has ~32 KB of loads in flight.
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

constexpr int MB_UNROLL = 8;
typedef float f4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_bw_read(const f4v *__restrict__ src, size_t n4, float *sink) {
    const size_t stride = (size_t)gridDim.x * 256 * MB_UNROLL;
    float acc = 0.f;
    for (size_t base = (size_t)blockIdx.x * 256 * MB_UNROLL + threadIdx.x; base < n4; base += stride) {
        f4v v[MB_UNROLL];
#pragma unroll
        for (int u = 0; u < MB_UNROLL; ++u) {
            const size_t i = base + (size_t)u * 256;
            v[u] = i < n4 ? __builtin_nontemporal_load(src + i) : f4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < MB_UNROLL; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    // never true for the finite data the host writes; keeps the loads live
    if (acc == -1.2345e-30f) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_bw_copy(const f4v *__restrict__ src, f4v *__restrict__ dst, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 256 * MB_UNROLL;
    for (size_t base = (size_t)blockIdx.x * 256 * MB_UNROLL + threadIdx.x; base < n4; base += stride) {
        f4v v[MB_UNROLL];
#pragma unroll
        for (int u = 0; u < MB_UNROLL; ++u) {
            const size_t i = base + (size_t)u * 256;
            v[u] = i < n4 ? __builtin_nontemporal_load(src + i) : f4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < MB_UNROLL; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) __builtin_nontemporal_store(v[u], dst + i);
        }
    }
}

}  // namespace

extern "C" int qtts_hip_hbm_bw(size_t bytes, int iters, double *read_gbs, double *copy_gbs) {
    if (bytes < ((size_t)1 << 20) || iters < 1) return -1;
    const size_t n4 = bytes / 16;
    f4v *a = nullptr, *b = nullptr;
    float *sink = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = -1;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 grid(8 * cus), block(256);
    if (hipMalloc((void **)&a, n4 * 16) != hipSuccess || hipMalloc((void **)&b, n4 * 16) != hipSuccess ||
        hipMalloc((void **)&sink, 256 * sizeof(float)) != hipSuccess ||
        hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess)
        goto out;
    if (hipMemsetAsync(a, 0, n4 * 16, st) != hipSuccess || hipMemsetAsync(b, 0, n4 * 16, st) != hipSuccess) goto out;
    for (int pass = 0; pass < 2; ++pass) {
        // one untimed launch, then `iters` timed ones on the stream they run on
        for (int w = 0; w < 2; ++w) {
            if (w == 1) hipEventRecord(e0, st);
            const int n = w == 0 ? 1 : iters;
            for (int i = 0; i < n; ++i) {
                if (pass == 0) hipLaunchKernelGGL(k_bw_read, grid, block, 0, st, a, n4, sink);
                else hipLaunchKernelGGL(k_bw_copy, grid, block, 0, st, a, b, n4);
            }
        }
        hipEventRecord(e1, st);
        if (hipEventSynchronize(e1) != hipSuccess) goto out;
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double moved = (double)n4 * 16.0 * (pass == 0 ? 1.0 : 2.0) * iters;
        const double gbs = ms > 0.f ? moved / (ms * 1e-3) / 1e9 : 0.0;
        if (pass == 0 && read_gbs) *read_gbs = gbs;
        if (pass == 1 && copy_gbs) *copy_gbs = gbs;
    }
    rc = hipGetLastError() == hipSuccess ? 0 : -1;
out:
    if (st) hipStreamSynchronize(st);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (st) hipStreamDestroy(st);
    hipFree(a);
    hipFree(b);
    hipFree(sink);
    return rc;
}
