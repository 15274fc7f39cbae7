// k_sample.hip - the sampler as a kernel of its own: one workgroup per batch
// row (the device code and its derivation are in qtts_sample_dev.h).  The
// register fast path (top_p >= 1, 0 < top_k < n) gets instantiations of its
// own, sized by the ids per thread (EM = ceil(n / 256) rounded up to 8 or 16),
// so a draw neither carries the full path's code nor iterates unused slots.
#include "qtts_sample_dev.h"

namespace {

template <bool FAST, int EM>
__global__ __launch_bounds__(256) void k_sample(SampArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    qtts_samp::sample_row<FAST, EM>(a, blockIdx.x, smraw, a.logits, a.stopped, a.mode == 1 ? a.rng : a.st_rng,
                                    a.n_gen, a.counts);
}

// the fast path on 1024 threads (qtts_sample_dev.h sample_fast_nt): EM ids per
// thread (2 up to 2048 logits, 4 up to 4096); the row's input pointers lead the
// arguments (preloaded into SGPRs, Makefile)
template <int EM>
__global__ __launch_bounds__(1024) void k_sample_w(const float *logits, const int *stopped, const uint32_t *rng,
                                                   const int *n_gen, const int *counts, SampArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    qtts_samp::sample_row<true, EM, 1024>(a, blockIdx.x, smraw, logits, stopped, rng, n_gen, counts);
}

}  // namespace

int qtts_sample(const SampArgs &a, hipStream_t st) {
    if (a.n > qtts_samp::NMAX || a.n < 1) {
        fprintf(stderr, "qtts_sample: vocab %d unsupported (max %d)\n", a.n, qtts_samp::NMAX);
        return -1;
    }
    // QTTS_HIP_SAMPLE_W=0: the 256-thread fast path (A/B; read per call so a
    // test's setting applies to its own launches)
    const char *sw = getenv("QTTS_HIP_SAMPLE_W");
    if (qtts_samp::fast_path(a) && !(sw && !atoi(sw))) {
        const size_t sm = sizeof(qtts_samp::FastSmemNT<1024>);
        const uint32_t *rng = a.mode == 1 ? a.rng : a.st_rng;
        if (a.n <= 2 * 1024) {
            hipLaunchKernelGGL((k_sample_w<2>), dim3(a.nb), dim3(1024), sm, st, a.logits, (const int *)a.stopped, rng,
                               (const int *)a.n_gen, (const int *)a.counts, a);
            qtts_last_kernel = "k_sample_w<2>";
        } else {
            hipLaunchKernelGGL((k_sample_w<4>), dim3(a.nb), dim3(1024), sm, st, a.logits, (const int *)a.stopped, rng,
                               (const int *)a.n_gen, (const int *)a.counts, a);
            qtts_last_kernel = "k_sample_w<4>";
        }
    } else if (qtts_samp::fast_path(a)) {
        const size_t sm = sizeof(qtts_samp::FastSmem);
        if (a.n <= 8 * 256) {
            hipLaunchKernelGGL((k_sample<true, 8>), dim3(a.nb), dim3(256), sm, st, a);
            qtts_last_kernel = "k_sample<true, 8>";
        } else {
            hipLaunchKernelGGL((k_sample<true, 16>), dim3(a.nb), dim3(256), sm, st, a);
            qtts_last_kernel = "k_sample<true, 16>";
        }
    } else {
        hipLaunchKernelGGL((k_sample<false, qtts_samp::EMAX>), dim3(a.nb), dim3(256), sizeof(qtts_samp::KSmem), st, a);
        qtts_last_kernel = "k_sample<false, 16>";
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
