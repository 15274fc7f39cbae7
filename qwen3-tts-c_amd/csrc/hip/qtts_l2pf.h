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
// Single target (workgroup b's slice of the next launch; the batch-1
// kernels): the slice base is uniform, one scalar division per launch.
// (L2Prefetch::cs: log2 of the bytes one load stands for.  What the next
// launch gains is NOT L2 hits -- round-5 counters show its TCC_HIT unchanged
// and its UTCL1 translation misses cut 6-160x -- but touching only one line
// per page (or per 2 MB of the whole next matrix) measured slower than this
// full 64-B touch, profiles/r05e_ab_prefetch_modes.txt: the data movement
// itself is part of the gain)
template <int NT, bool NTL = false>
__device__ __forceinline__ void qtts_l2pf_issue(const L2Prefetch &p, int b, L2PfRegs &r, const void *fallback) {
    // (b is uniform: a scalar select, no branch between loads)
    const bool tgt = p.base && b < p.nwg;
    const unsigned char *st = tgt ? p.base + (long long)(b % p.pm) * p.pa + (long long)(b / p.pm) * p.pb
                                  : reinterpret_cast<const unsigned char *>(fallback);
    // a workgroup without a target slice (past the next launch's grid, or no
    // prefetch) re-reads the first 4 B of its fallback line n times: chunk
    // count 0 sends every offset to 0, whatever the target's row geometry
    const unsigned m = (1u << p.lg) - 1u, n = tgt ? (unsigned)p.chunks : 0u;
    // offsets first (selects, no exec-masked branches: those made the compiler
    // reuse an in-flight load's registers and wait for every load), then the loads
    unsigned off[QTTS_PF_LOADS];
#pragma unroll
    for (int j = 0; j < QTTS_PF_LOADS; ++j) {
        const unsigned c0 = threadIdx.x + NT * j;
        const unsigned c = c0 < n ? c0 : 0u;
        off[j] = (c >> p.lg) * (unsigned)p.ld + ((c & m) << p.cs);
    }
#pragma unroll
    for (int j = 0; j < QTTS_PF_LOADS; ++j) {
        const unsigned *q = reinterpret_cast<const unsigned *>(st + off[j]);
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
