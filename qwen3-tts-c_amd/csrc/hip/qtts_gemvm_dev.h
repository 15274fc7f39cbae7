// qtts_gemvm_dev.h - device helpers shared by the lock-step batch GEMVs
// (k_gemvm.hip: x planes staged per workgroup; k_gemvb.hip: x slices per
// wave): bf16 packing, the exact 3-plane split, buffer-descriptor loads and
// the self-reducing split-K tail.
#pragma once
#include "qtts_common.h"
#include "qtts_kernels.h"

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace qtts_gm {

// two f32 -> packed bf16 (round to nearest even: v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    const bf2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

// x = x1 + x2 + x3 (each bf16, exact: 24 mantissa bits in three 8-bit pieces)
// for 4 values; p1 / p2 / p3 receive 4 packed bf16 each (8 B)
__device__ __forceinline__ void split4(float4 v, uint2 &p1, uint2 &p2, uint2 &p3) {
    const uint32_t a1 = pk_bf16(v.x, v.y), b1 = pk_bf16(v.z, v.w);
    const float ex = v.x - lo_f(a1), ey = v.y - hi_f(a1), ez = v.z - lo_f(b1), ew = v.w - hi_f(b1);
    const uint32_t a2 = pk_bf16(ex, ey), b2 = pk_bf16(ez, ew);
    const uint32_t a3 = pk_bf16(ex - lo_f(a2), ey - hi_f(a2)), b3 = pk_bf16(ez - lo_f(b2), ew - hi_f(b2));
    p1 = make_uint2(a1, b1);
    p2 = make_uint2(a2, b2);
    p3 = make_uint2(a3, b3);
}

// buffer descriptor over a wave-uniform base (kernel arguments): loads take a
// 32-bit byte offset instead of a 64-bit address per lane (cdna_hip_programming.md T8)
// (readfirstlane makes the uniformity provable: no waterfall loop per load, T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    const uint64_t u = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    void *q = (void *)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, 0x7FFFFFF0, 0x00020000);
}
// float4 at element offset eoff
__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, unsigned eoff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, eoff * 4u, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

// Self-reducing split-K (GemvArgs::tick), hand-off form R1 of
// cdna_hip_programming.md Guideline 16 (as k_attn_dec's split merge): the
// partials went out write-through (sc1), every wave drains them, one relaxed
// ticket add per workgroup; the last column to arrive adds the kz partials of
// its row block (nr rows) in column order to the residual (the order the
// consumer's xadd prologue used) and resets the ticket.
__device__ __forceinline__ void reduce_last(const GemvArgs &a, int nr, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(a.tick + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = old == (int)gridDim.y - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
    const int rb = blockIdx.x * nr, kz = gridDim.y;
    for (int i = threadIdx.x; i < a.nb * nr; i += blockDim.x) {
        const int b = i / nr, r = rb + (i - b * nr);
        if (r >= a.R) continue;
        // every partial (kz <= 4, host) and the residual issued before the sum
        const float *p = a.ypart + (size_t)b * a.R + r;
        float *y = a.y + (size_t)b * a.ldy + r;
        float t[4];
#pragma unroll
        for (int z = 0; z < 4; ++z) t[z] = ld_sc1(p + (size_t)(z < kz ? z : 0) * a.ld_ypart);
        const float y0 = *y;
        float s = t[0];
#pragma unroll
        for (int z = 1; z < 4; ++z)
            if (z < kz) s += t[z];
        *y = y0 + s;
    }
    if (threadIdx.x == 0) __hip_atomic_store(a.tick + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the GEMV epilogue of one output element val = (W x)[b][r]; `up` is the value
// 4 weight rows further (the SwiGLU partner of a gate row, row_shl:4)
__device__ __forceinline__ void epilogue(const GemvArgs &a, int bb, int r, float val, float up) {
    float *yr = a.y + (size_t)bb * a.ldy;
    switch (a.epi) {
        case EPI_STORE: yr[r] = val; break;
        case EPI_BIAS: yr[r] = val + a.bias[r]; break;
        case EPI_BIAS_SILU: {
            const float z = val + a.bias[r];
            yr[r] = z / (1.0f + expf(-z));
            break;
        }
        case EPI_RESID: yr[r] += val; break;
        case EPI_SWIGLU:
            if ((r & 7) < 4) yr[(r >> 3) * 4 + (r & 3)] = (val / (1.0f + expf(-val))) * up;
            break;
    }
}

}  // namespace qtts_gm
