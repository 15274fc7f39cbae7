// k_sample.hip - on-device sampling for the talker (group 0) and sub-talker
// (groups 1..15), one workgroup per batch row.  Keeping this on the device is
// what lets a whole frame run without a host round trip.
//
// Reproduces c/qwen_tts_kernels.c:384-558 and the loop around it
// (c/qwen_tts.c:1302-1340) EXACTLY given identical logits:
//   * suppress ids [V-1024, V) except EOS to -1e9 (Q.c:1272-1305), talker only
//   * repetition penalty once per OCCURRENCE (K.c:395-405, Q.c:1308): an id
//     seen c times is divided / multiplied c times
//   * fast path (top_p >= 1, 0 < top_k < n): v = logit / T, the top-k in
//     (value desc, index asc) order -- the order the reference's strict '>'
//     insertion list produces -- p_j = expf(v_j - v_0) summed sequentially,
//     r = u * sum, first j with cumsum >= r
//   * full path otherwise: softmax, keep p >= k-th largest, nucleus over the
//     stable descending order, renormalise, inverse CDF in index order
//   * xorshift32 over the bits of a float state (K.c:384-393); the sub-talker
//     state is reset to (float)seed at every frame (T.c:718)
//   * fixed-length mode: an EOS draw is masked and redrawn (Q.c:1315-1321)
// Sequential sums run on one lane in the reference's order; expf is the
// glibc-exact replica (qtts_common.h); divisions are correctly rounded.
//
// Top-k selection is a 4-pass MSB radix select over order-preserving u32 keys
// (256-bin LDS histograms, one wave scans the bins), then an exact rank of
// the k selected (value desc, index asc).
#include <float.h>
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

constexpr int NMAX = 4096;

struct SampSmem {
    float lg[NMAX];        // (penalised) logits
    float v[NMAX];         // logits / T  (or probabilities in the full path)
    uint32_t key[NMAX];
    union {
        struct {           // fast path: the k selected, then the k ranked
            float sel_v[NMAX];
            int sel_i[NMAX];
            float top_v[NMAX];
            int top_i[NMAX];
        };
        unsigned long long srt[NMAX];  // full path: sort buffer
    };
    int hist[256];
    int scan[256];
    int misc[16];
    float fmisc[8];
};

__device__ __forceinline__ uint32_t okey(float v) {
    if (v == 0.0f) v = 0.0f;  // -0 == +0 for the comparisons
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float rand_uniform(uint32_t &s) {
#pragma clang fp contract(off)
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return div_rn((float)(s & 0x7FFFFFFFu), (float)0x7FFFFFFF);
}

// Wave 0 finds, scanning bins from high to low, the bin where the running
// count reaches `rem`.  Returns via sm.misc[0] = bin, sm.misc[1] = new rem.
__device__ void pick_bin(SampSmem &sm, int rem) {
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        // lane l holds bins 255-4l .. 252-4l (descending)
        int c[4], tot = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) { c[i] = sm.hist[255 - 4 * l - i]; tot += c[i]; }
        // inclusive prefix over lanes
        int inc = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o, 64);
            if (l >= o) inc += y;
        }
        const int exc = inc - tot;
        const bool hit = exc < rem && inc >= rem;
        if (hit) {
            int cum = exc;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (cum + c[i] >= rem) {
                    sm.misc[0] = 255 - 4 * l - i;
                    sm.misc[1] = rem - cum;
                    break;
                }
                cum += c[i];
            }
        }
    }
    __syncthreads();
}

// block-wide exclusive scan of one int per thread (256 threads)
__device__ int block_excl_scan(SampSmem &sm, int x) {
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    int inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (l >= o) inc += y;
    }
    __syncthreads();
    if (l == 63) sm.scan[w] = inc;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; ++i) base += sm.scan[i];
    return base + inc - x;
}

// Radix select: among keys != 0 (eligible), find the k-th largest key T.
// Returns T in misc[2]; misc[3] = how many elements equal to T are taken.
__device__ void radix_select(SampSmem &sm, int n, int k) {
    const int tid = threadIdx.x;
    uint32_t prefix = 0, mask = 0;
    int rem = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        sm.hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < n; i += 256) {
            const uint32_t kk = sm.key[i];
            if (kk != 0 && (kk & mask) == prefix) atomicAdd(&sm.hist[(kk >> shift) & 255], 1);
        }
        __syncthreads();
        pick_bin(sm, rem);
        prefix |= (uint32_t)sm.misc[0] << shift;
        mask |= 255u << shift;
        rem = sm.misc[1];
        __syncthreads();
    }
    if (tid == 0) { sm.misc[2] = (int)prefix; sm.misc[3] = rem; }
    __syncthreads();
}

// Fast path.  sm.lg holds logits.  Returns sampled id (valid in all threads).
__device__ int sample_fast(SampSmem &sm, int n, int k, float temp, uint32_t &rng /*thread 0*/) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    int elig = 0;
    for (int i = tid; i < n; i += 256) {
        const float v = div_rn(sm.lg[i], temp);
        sm.v[i] = v;
        const bool ok = v > -FLT_MAX;            // the reference list starts at -FLT_MAX
        sm.key[i] = ok ? okey(v) : 0u;
        elig += ok;
    }
    elig = block_excl_scan(sm, elig) + elig;     // inclusive; last thread has the total
    if (tid == 255) sm.misc[4] = elig;
    __syncthreads();
    const int ne = sm.misc[4];
    const int ke = k < ne ? k : ne;
    if (ke == 0) return 0;                       // sum == 0 -> idx[0] < 0 -> 0 (no draw)
    radix_select(sm, n, ke);
    const uint32_t T = (uint32_t)sm.misc[2];
    const int take_eq = sm.misc[3];
    // tie order among key == T by index: contiguous ranges per thread
    const int E = (n + 255) / 256, i0 = tid * E, i1 = min(n, i0 + E);
    int neq = 0;
    for (int i = i0; i < i1; ++i) neq += sm.key[i] == T;
    int off = block_excl_scan(sm, neq);
    if (tid == 0) sm.misc[5] = 0;
    __syncthreads();
    for (int i = i0; i < i1; ++i) {
        const uint32_t kk = sm.key[i];
        bool take = kk > T;
        if (kk == T) { take = off < take_eq; ++off; }
        if (take) {
            const int s = atomicAdd(&sm.misc[5], 1);
            sm.sel_v[s] = sm.v[i];
            sm.sel_i[s] = i;
        }
    }
    __syncthreads();
    // exact rank among the ke selected: (value desc, index asc)
    for (int s = tid; s < ke; s += 256) {
        const float vs = sm.sel_v[s];
        const int is = sm.sel_i[s];
        const uint32_t ks = okey(vs);
        int rk = 0;
        for (int t = 0; t < ke; ++t) {
            const uint32_t kt = okey(sm.sel_v[t]);
            rk += (kt > ks) || (kt == ks && sm.sel_i[t] < is);
        }
        sm.top_v[rk] = vs;
        sm.top_i[rk] = is;
    }
    __syncthreads();
    const float mx = sm.top_v[0];
    for (int j = tid; j < ke; j += 256) sm.sel_v[j] = expf_glibc(sm.top_v[j] - mx);
    __syncthreads();
    if (tid == 0) {
        float sum = 0.0f;
        for (int j = 0; j < ke; ++j) sum += sm.sel_v[j];
        int out = 0;
        if (sum > 0.0f) {
            const float r = rand_uniform(rng) * sum;
            float c = 0.0f;
            for (int j = 0; j < ke; ++j) {
                c += sm.sel_v[j];
                if (c >= r) { out = sm.top_i[j]; break; }
            }
        } else {
            out = sm.top_i[0];
        }
        sm.misc[6] = out;
    }
    __syncthreads();
    return sm.misc[6];
}

// bitonic sort of sm.srt[0..N2) descending
__device__ void bitonic_desc(SampSmem &sm, int N2) {
    const int tid = threadIdx.x;
    for (int size = 2; size <= N2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < N2 / 2; i += 256) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool desc = ((lo & size) == 0);
                const unsigned long long x = sm.srt[lo], y = sm.srt[hi];
                if ((x < y) == desc) { sm.srt[lo] = y; sm.srt[hi] = x; }
            }
            __syncthreads();
        }
    }
}

// Full path (K.c:486-557).
__device__ int sample_full(SampSmem &sm, int n, int k, float top_p, float temp, uint32_t &rng) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += 256) sm.v[i] = div_rn(sm.lg[i], temp);
    __syncthreads();
    // softmax (K.c:371-378): max, e = expf(x - max), sequential sum, scale
    if (tid == 0) {
        float mx = sm.v[0];
        for (int i = 1; i < n; ++i) if (sm.v[i] > mx) mx = sm.v[i];
        sm.fmisc[0] = mx;
    }
    __syncthreads();
    const float mx = sm.fmisc[0];
    for (int i = tid; i < n; i += 256) sm.v[i] = expf_glibc(sm.v[i] - mx);
    __syncthreads();
    if (tid == 0) {
        float s = 0.0f;
        for (int i = 0; i < n; ++i) s += sm.v[i];
        sm.fmisc[1] = div_rn(1.0f, s);
    }
    __syncthreads();
    const float inv = sm.fmisc[1];
    for (int i = tid; i < n; i += 256) sm.v[i] *= inv;
    __syncthreads();
    int N2 = 1;
    while (N2 < n) N2 <<= 1;
    const bool need_sort = (k > 0 && k < n) || top_p < 1.0f;
    if (need_sort) {
        // composite (key desc, index asc): key<<32 | ~index
        for (int i = tid; i < N2; i += 256)
            sm.srt[i] = i < n ? (((unsigned long long)okey(sm.v[i]) << 32) | (0xFFFFFFFFu - (uint32_t)i)) : 0ull;
        __syncthreads();
        bitonic_desc(sm, N2);
    }
    if (k > 0 && k < n) {
        const uint32_t thr_key = (uint32_t)(sm.srt[k - 1] >> 32);
        for (int i = tid; i < n; i += 256)
            if (okey(sm.v[i]) < thr_key) sm.v[i] = 0.0f;   // p < k-th largest -> 0
        __syncthreads();
        if (top_p < 1.0f) {  // re-sort with the zeroed values (ties stay in index order)
            for (int i = tid; i < N2; i += 256)
                sm.srt[i] = i < n ? (((unsigned long long)okey(sm.v[i]) << 32) | (0xFFFFFFFFu - (uint32_t)i)) : 0ull;
            __syncthreads();
            bitonic_desc(sm, N2);
        }
    }
    if (top_p < 1.0f) {
        if (tid == 0) {
            float c = 0.0f;
            int cut = n;
            for (int i = 0; i < n; ++i) {
                c += sm.v[0xFFFFFFFFu - (uint32_t)(sm.srt[i] & 0xFFFFFFFFull)];
                if (c >= top_p) { cut = i + 1; break; }
            }
            sm.misc[7] = cut;
        }
        __syncthreads();
        const int cut = sm.misc[7];
        for (int i = cut + tid; i < n; i += 256) sm.v[0xFFFFFFFFu - (uint32_t)(sm.srt[i] & 0xFFFFFFFFull)] = 0.0f;
        __syncthreads();
    }
    if (tid == 0) {
        float s = 0.0f;
        for (int i = 0; i < n; ++i) s += sm.v[i];
        sm.fmisc[2] = s;
    }
    __syncthreads();
    const float s = sm.fmisc[2];
    if (s > 0.0f) {
        const float iv = div_rn(1.0f, s);
        for (int i = tid; i < n; i += 256) sm.v[i] *= iv;
    }
    __syncthreads();
    if (tid == 0) {
        const float r = rand_uniform(rng);
        float c = 0.0f;
        int out = 0;
        for (int i = 0; i < n; ++i) {
            c += sm.v[i];
            if (c >= r) { out = i; break; }
        }
        sm.misc[8] = out;
    }
    __syncthreads();
    return sm.misc[8];
}

__device__ int sample_any(SampSmem &sm, int n, int k, float top_p, float temp, uint32_t &rng) {
    if (temp <= 0.0f) temp = 1e-5f;
    if (top_p >= 1.0f && k > 0 && k < n) return sample_fast(sm, n, k, temp, rng);
    return sample_full(sm, n, k, top_p, temp, rng);
}

__global__ __launch_bounds__(256) void k_sample(SampArgs a) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    SampSmem &sm = *reinterpret_cast<SampSmem *>(smraw);
    const int b = blockIdx.x, tid = threadIdx.x, n = a.n;
    if (a.stopped && a.stopped[b]) return;
    const float *lg = a.logits + (size_t)b * a.ld;
    for (int i = tid; i < n; i += 256) {
        float v = lg[i];
        if (a.mode == 1) {
            if (i >= a.suppress_lo && i != a.eos) v = -1e9f;
            if (a.rep != 1.0f && a.counts) {
                const int c = a.counts[(size_t)b * n + i];
                for (int j = 0; j < c; ++j) v = v > 0 ? div_rn(v, a.rep) : v * a.rep;
            }
        }
        sm.lg[i] = v;
    }
    __syncthreads();
    uint32_t rng = 0;
    if (tid == 0) rng = a.mode == 1 ? a.rng[b] : a.st_rng[b];
    int tok = sample_any(sm, n, a.top_k, a.top_p, a.temp, rng);
    if (a.mode == 1) {
        const int ng = a.n_gen[b];
        if (a.fixed > 0 && tok == a.eos && ng < a.fixed) {
            if (tid == 0) sm.lg[a.eos] = -1e9f;
            __syncthreads();
            tok = sample_any(sm, n, a.top_k, a.top_p, a.temp, rng);
        }
        if (tid == 0) {
            a.rng[b] = rng;
            if (a.fixed == 0 && tok == a.eos) {
                a.stopped[b] = 1;
                if (a.stop_step) a.stop_step[b] = ng;
            } else {
                a.cur_row[b] = ng;
                a.codes[(size_t)b * a.codes_bstride + (size_t)ng * a.G + 0] = tok;
                if (a.counts) a.counts[(size_t)b * n + tok] += 1;
                a.n_gen[b] = ng + 1;
                a.st_rng[b] = a.seed_bits;
            }
            if (a.out_tok) a.out_tok[b] = tok;
        }
    } else {
        if (tid == 0) {
            a.st_rng[b] = rng;
            if (a.codes) a.codes[(size_t)b * a.codes_bstride + (size_t)a.cur_row[b] * a.G + a.g] = tok;
            if (a.out_tok) a.out_tok[b] = tok;
        }
    }
}

}  // namespace

int qtts_sample(const SampArgs &a, hipStream_t st) {
    if (a.n > NMAX || a.n < 1) {
        fprintf(stderr, "qtts_sample: vocab %d unsupported (max %d)\n", a.n, NMAX);
        return -1;
    }
    hipLaunchKernelGGL(k_sample, dim3(a.nb), dim3(256), sizeof(SampSmem), st, a);
    qtts_last_kernel = "k_sample";
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
