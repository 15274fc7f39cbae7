// k_sample.hip - the sampler as a kernel of its own: one workgroup per batch
// row (the device code and its derivation are in qtts_sample_dev.h).
#include "qtts_sample_dev.h"

namespace {

__global__ __launch_bounds__(256) void k_sample(SampArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    qtts_samp::sample_row<false>(a, blockIdx.x, smraw);
}

}  // namespace

int qtts_sample(const SampArgs &a, hipStream_t st) {
    if (a.n > qtts_samp::NMAX || a.n < 1) {
        fprintf(stderr, "qtts_sample: vocab %d unsupported (max %d)\n", a.n, qtts_samp::NMAX);
        return -1;
    }
    hipLaunchKernelGGL(k_sample, dim3(a.nb), dim3(256), sizeof(qtts_samp::KSmem), st, a);
    qtts_last_kernel = "k_sample";
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
