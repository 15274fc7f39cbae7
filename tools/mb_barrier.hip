// mb_barrier.hip - micro-benchmark (development tool): cost of a kernel
// boundary inside a HIP graph vs a software grid barrier in a persistent
// kernel, on the same tiny per-step work (every workgroup reads a 4 KB vector
// written by the previous step and writes its own slot).
//
//   hipcc -O3 --offload-arch=gfx950 tools/mb_barrier.hip -o /tmp/mb_barrier && /tmp/mb_barrier
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_step(const float *in, float *out, int n) {
    __shared__ float s[256];
    float acc = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) acc += in[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int i = 0; i < 256; ++i) t += s[i];
        out[blockIdx.x % n] = t * 1e-6f + 1.0f;
    }
}

__device__ __forceinline__ void grid_barrier(unsigned *count, unsigned *gen, unsigned nblk, unsigned &my_gen) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = my_gen;
        const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblk - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > 50000000L) break;   // bounded: never hang the GPU
            }
        }
        my_gen = g + 1;
    }
    __syncthreads();
    __threadfence();
}

__global__ void k_persistent(float *a, float *b, int n, int steps, unsigned *count, unsigned *gen) {
    __shared__ float s[256];
    unsigned my_gen = 0;
    if (threadIdx.x == 0) my_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int it = 0; it < steps; ++it) {
        const float *in = (it & 1) ? b : a;
        float *out = (it & 1) ? a : b;
        float acc = 0.f;
        for (int i = threadIdx.x; i < n; i += 256) acc += __builtin_nontemporal_load(in + i);
        s[threadIdx.x] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int i = 0; i < 256; ++i) t += s[i];
            out[blockIdx.x % n] = t * 1e-6f + 1.0f;
        }
        grid_barrier(count, gen, gridDim.x, my_gen);
    }
}

int main() {
    const int n = 1024, steps = 2000;
    float *a, *b;
    unsigned *cnt;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&cnt, 64));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    CK(hipMemset(cnt, 0, 64));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    for (int grid : {256, 512, 1024}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 200; ++i)
            hipLaunchKernelGGL(k_step, dim3(grid), dim3(256), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, n);
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
        printf("graph of kernels, grid %4d: %.2f us per kernel\n", grid, ms * 1e3 / 2000);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    for (int grid : {ncu, 2 * ncu}) {
        // all workgroups must be co-resident: 1-2 per CU at 256 threads is safe
        CK(hipMemset(cnt, 0, 64));
        hipLaunchKernelGGL(k_persistent, dim3(grid), dim3(256), 0, st, a, b, n, 10, cnt, cnt + 16);
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(k_persistent, dim3(grid), dim3(256), 0, st, a, b, n, steps, cnt, cnt + 16);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("persistent kernel, grid %4d: %.2f us per step (barrier + work)\n", grid, ms * 1e3 / steps);
    }
    return 0;
}
