// qtts_l2pf.h - device side of L2Prefetch (qtts_kernels.h).
#pragma once
#include "qtts_common.h"
#include "qtts_kernels.h"

// The next launch's weight slice into this XCD's L2 (L2Prefetch,
// qtts_kernels.h): QTTS_PF_LOADS 4-B loads per thread (one per 64-B chunk), issued right after
// the kernel's own weight loads, every one unconditional (an absent or short
// slice re-reads its first chunk: a branch between loads would make the
// compiler wait for all of them).  The values are folded into `acc`, which
// qtts_l2pf_sink tests at the end of the kernel.
struct L2PfRegs { unsigned v[QTTS_PF_LOADS]; };
// NTL: non-temporal loads (the talker's read-once weights: they must not
// displace the sub-talker's weights from the Infinity Cache)
// NL loads per thread (<= QTTS_PF_LOADS; the 1024-thread batch GEMV takes 2)
template <int NT, bool NTL = false, int NL = QTTS_PF_LOADS>
__device__ __forceinline__ void qtts_l2pf_issue(const L2Prefetch &p, int b, L2PfRegs &r, const void *fallback,
                                                int nthreads = NT) {
    const unsigned m = (1u << p.lg) - 1u, n = (unsigned)p.chunks;
    const unsigned tot = n * (unsigned)p.ntgt;
    // each offset by selects (no exec-masked branches: those made the compiler
    // reuse an in-flight load's registers and wait for every load)
#pragma unroll
    for (int j = 0; j < QTTS_PF_LOADS; ++j) {
        if (j >= NL) { r.v[j] = 0u; continue; }
        const unsigned c0 = threadIdx.x + (unsigned)nthreads * j;
        const unsigned c1 = c0 < tot ? c0 : 0u;
        const unsigned i = p.ntgt > 1 ? c1 / n : 0u, c = c1 - i * n;
        int t = b + (int)i * p.tstride;
        t = t < p.tmax ? t : 0;   // (past the next grid: its first slice again)
        const unsigned char *st = p.base ? p.base + (long long)(t % p.pm) * p.pa + (long long)(t / p.pm) * p.pb
                                         : reinterpret_cast<const unsigned char *>(fallback);
        const unsigned col = (c & m) < p.cmax ? (c & m) : p.cmax;   // (a row slice of cmax + 1 chunks)
        const unsigned *q = reinterpret_cast<const unsigned *>(st + (c >> p.lg) * (unsigned)p.ld + (col << 6));
        if constexpr (NTL) r.v[j] = __builtin_nontemporal_load(q);
        else r.v[j] = *q;
    }
}
__device__ __forceinline__ void qtts_l2pf_sink(const L2Prefetch &p, const L2PfRegs &r) {
    unsigned acc = 0;
#pragma unroll
    for (int j = 0; j < QTTS_PF_LOADS; ++j) acc ^= r.v[j];
    if (acc == 0x9E3779B9u && p.sink) p.sink[0] = acc;
}
