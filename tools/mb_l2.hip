// mb_l2.hip - micro-benchmark (development tool): does a kernel's read of lines
// the PREVIOUS kernel pulled into the same XCD's L2 beat a read served by the
// Infinity Cache?  (Decides whether a decode GEMV can prefetch its successor's
// weight slice into L2.)
//
// 16 MiB buffer = 8 slices of 2 MiB; workgroup b of a 512-WG grid reads slice
// (b + shift) % 8 part b / 8.  Blocks b and b + 8 share an XCD (round-robin
// dealing, MI355X_MICROARCH.md), so shift 0 twice = same-XCD re-read, shift 1
// after shift 0 = every line in another XCD's L2 (Infinity Cache hit).
//
//   hipcc -O3 --offload-arch=gfx950 tools/mb_l2.hip -o tools/mb_l2 && tools/mb_l2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4 *buf, size_t slice16, int shift, unsigned *sink) {
    const int b = blockIdx.x, x = (b + shift) & 7, part = b >> 3, nparts = gridDim.x >> 3;
    const size_t per = slice16 / nparts;
    const uint4 *p = buf + (size_t)x * slice16 + (size_t)part * per;
    unsigned acc = 0;
    for (size_t i = threadIdx.x; i < per; i += 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;   // keeps the loads; practically never true
}

__global__ void k_flush(const uint4 *buf, size_t n16, unsigned *sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x9E3779B9u) sink[1] = acc;
}

int main() {
    const size_t slice = 2u << 20, total = 8 * slice, flushb = (size_t)1 << 30;
    uint4 *buf, *fl;
    unsigned *sink;
    CK(hipMalloc(&buf, total));
    CK(hipMalloc(&fl, flushb));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, total));
    CK(hipMemset(fl, 2, flushb));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    const size_t s16 = slice / 16;
    auto flush = [&]() { hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, st, fl, flushb / 16, sink); };
    auto rd = [&](int shift) { hipLaunchKernelGGL(k_read, dim3(512), dim3(256), 0, st, buf, s16, shift, sink); };
    struct Case { const char *name; int pre; int shift; };   // pre: -1 flush only, else a read with that shift first
    const Case cases[] = {{"cold (after a 1 GiB sweep)", -1, 0},
                          {"same-XCD re-read (L2)", 0, 0},
                          {"other-XCD re-read (Infinity Cache)", 0, 1}};
    for (const Case &c : cases) {
        std::vector<float> t;
        for (int r = 0; r < 25; ++r) {
            flush();
            if (c.pre >= 0) rd(c.pre);
            CK(hipEventRecord(e0, st));
            rd(c.shift);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("%-38s median %7.2f us  min %7.2f us  (%.1f TB/s at median)\n", c.name, t[t.size() / 2], t[0],
               total / (t[t.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
