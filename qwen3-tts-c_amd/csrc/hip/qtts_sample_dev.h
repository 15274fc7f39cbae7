// qtts_sample_dev.h - on-device sampling for the talker (group 0) and sub-talker
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
// Fast path: each thread keeps its ids in registers.  For k <= 64 (the
// default 50) one histogram of the key distance from the maximum bounds a
// candidate set of <= 64 keys that one wave ranks exactly (sample_dist, three
// barriers); otherwise, or when the candidates overflow, top-k is an MSB
// radix select over order-preserving u32 keys (per-wave 256-bin LDS
// histograms, one barrier per pass, early exit), then an exact rank of the k
// selected (value desc, index asc).  Full path: bitonic sort in LDS.
#pragma once
#include <float.h>
#include <stddef.h>
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace qtts_samp {

constexpr int NMAX = 4096;

struct SampSmem {
    float lg[NMAX];        // (penalised) logits
    float v[NMAX];         // logits / T  (or probabilities in the full path)
    unsigned long long srt[NMAX];  // sort buffer (key desc, index asc)
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

// bitonic sort of sm.srt[0..N2) descending
__device__ __forceinline__ void bitonic_desc(SampSmem &sm, int N2) {
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
__device__ __forceinline__ int sample_full(SampSmem &sm, int n, int k, float top_p, float temp, uint32_t &rng) {
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

__device__ __forceinline__ int sample_any(SampSmem &sm, int n, int k, float top_p, float temp, uint32_t &rng) {
    if (temp <= 0.0f) temp = 1e-5f;
    return sample_full(sm, n, k, top_p, temp, rng);
}

// ---------------------------------------------------------------------------
// Fast path on registers (top_p >= 1, 0 < k < n): thread t owns the
// contiguous ids [t*E, t*E + E), E = ceil(n / 256) <= EMAX.
constexpr int EMAX = NMAX / 256;
constexpr int KFAST = 1024;   // register path for top_k <= KFAST (the LDS rank buffers are sized by it)
constexpr int KC = 64;        // candidate cap of the distance-binned path (one wave ranks them)

struct FastSmem {
    int hist[2][4][256];   // per-wave radix histograms, double-buffered by pass
    int scan[2][4];
    float sel_v[KFAST];
    int sel_i[KFAST];
    float top_v[KFAST];
    int top_i[KFAST];
    int misc[4];
    // distance-binned path (sample_dist)
    unsigned long long cand[4][KC];   // per-wave candidate keys (value key << 32 | ~index)
    unsigned long long rk[KC];        // wave 0: the candidates, one per lane
    float pv[KC];                     // p in rank order
    int pi[KC];                       // ids in rank order
    float red[4];
    int redn[4];
    int ncw[4];
};

// k-th largest eligible key (value desc): 8-bit MSB radix select over
// per-wave LDS histograms, one barrier per pass, early exit once the bin that
// holds the k-th key fits entirely.  Returns T (threshold key prefix, low
// bits 0 after an early exit), take_eq = how many keys == T to take in index
// order when the select ran to the last digit; ne = number of eligible keys.
template <int EM>
__device__ __forceinline__ void radix_select_regs(FastSmem &fs, const uint32_t (&kk)[EM], int E, int k, uint32_t &T,
                                  uint32_t &Tmask, int &take_eq, int &ne) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) { fs.hist[0][w][lane + 64 * i] = 0; fs.hist[1][w][lane + 64 * i] = 0; }
    uint32_t prefix = 0, mask = 0;
    int rem = k;
    ne = -1;
    int par = 0;
    for (int shift = 24; shift >= 0; shift -= 8, par ^= 1) {
        int *h = fs.hist[par][w];
#pragma unroll
        for (int j = 0; j < EM; ++j)
            if (j < E && kk[j] != 0u && (kk[j] & mask) == prefix) atomicAdd(&h[(kk[j] >> shift) & 255u], 1);
        __syncthreads();
        // every wave scans the merged histogram from the top (same result in all waves)
        int c[4], tot = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int bin = 255 - 4 * lane - i;
            c[i] = fs.hist[par][0][bin] + fs.hist[par][1][bin] + fs.hist[par][2][bin] + fs.hist[par][3][bin];
            tot += c[i];
        }
        const int inc = wave_incl_scan(tot);
        if (ne < 0) {
            ne = __builtin_amdgcn_readlane(inc, 63);
            if (k > ne) k = ne;
            rem = k;
        }
        const int exc = inc - tot;
        int bin = -1, nrem = 0, cbin = 0;
        if (exc < rem && inc >= rem) {
            int cum = exc;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (bin < 0 && cum + c[i] >= rem) { bin = 255 - 4 * lane - i; nrem = rem - cum; cbin = c[i]; }
                cum += c[i];
            }
        }
        const unsigned long long hit = __ballot(bin >= 0);
        const int src = hit ? __ffsll((long long)hit) - 1 : 0;
        bin = __builtin_amdgcn_readlane(bin, src);   // (src is wave-uniform: from the ballot)
        nrem = __builtin_amdgcn_readlane(nrem, src);
        cbin = __builtin_amdgcn_readlane(cbin, src);
        // clear this wave's other buffer for the next pass (its readers finished before this barrier)
#pragma unroll
        for (int i = 0; i < 4; ++i) fs.hist[par ^ 1][w][lane + 64 * i] = 0;
        if (k == 0) { T = 0xFFFFFFFFu; Tmask = 0xFFFFFFFFu; take_eq = 0; return; }
        prefix |= (uint32_t)bin << shift;
        mask |= 255u << shift;
        rem = nrem;
        if (cbin == nrem || shift == 0) {   // the whole bin is taken, or the key is exact
            T = prefix; Tmask = mask; take_eq = nrem;
            return;
        }
    }
}

__device__ __forceinline__ void block_scan2(FastSmem &fs, int x, int y, int &ex, int &ey) {
    // exclusive scans of two small per-thread counts packed in one int (16 | 16 bits)
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int v = x | (y << 16);
    const int inc = wave_incl_scan(v);
    if (l == 63) fs.scan[0][w] = inc;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; ++i) base += fs.scan[0][i];
    const int e = base + inc - v;
    ex = e & 0xFFFF;
    ey = e >> 16;
}

// Wave 0, ke <= 64 selected (sel_v / sel_i in index order).  Lane j ranks its
// (value desc, index asc) key -- the order the reference's strict '>'
// insertion list leaves (K.c:436-449) -- against all ke keys read back from
// LDS by broadcast (8 loads in flight per step), scatters itself to
// top_*[rank]; then p_j = expf(v_j - v_0), the sum in j order, r = u * sum
// and the first j whose running sum reaches r (K.c:451-477), every lane
// walking the same broadcast values.  Lane 0 owns the RNG.  Returns the id
// (all lanes).  (v_readlane per step measured 2-3x slower than the LDS reads.)
template <class FS>
__device__ __forceinline__ int wave_sort_draw(FS &fs, int ke, uint32_t &rng, uint64_t etab) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    unsigned long long *keys = reinterpret_cast<unsigned long long *>(fs.top_v);   // 64 x 8 B scratch
    float vj = 0.f;
    int ij = 0;
    unsigned long long key = 0ull;
    if (lane < ke) {
        vj = fs.sel_v[lane];
        ij = fs.sel_i[lane];
        key = ((unsigned long long)okey(vj) << 32) | (0xFFFFFFFFu - (uint32_t)ij);
    }
    keys[lane] = key;   // lanes >= ke: 0, below every real key
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // one wave: LDS is in order once the writes landed
    int rank = 0;
    for (int t0 = 0; t0 < ke; t0 += 8) {
        unsigned long long kt[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) kt[u] = keys[t0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += kt[u] > key;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float *pv = fs.sel_v;   // reused: [rank] -> p_rank, indices in top_i
    if (lane < ke) fs.top_i[rank] = ij;
    float e = 0.f;
    if (lane < ke) pv[rank] = vj;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float v0 = pv[0];
    {   // every lane active for the table's cross-lane reads
        const float ee = expf_glibc_wave(lane < ke ? pv[lane] - v0 : 0.f, etab);
        if (lane < ke) e = ee;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < ke) pv[lane] = e;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float sum = 0.f;
    for (int j0 = 0; j0 < ke; j0 += 8) {
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = pv[j0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j0 + u < ke) sum += p[u];
    }
    if (!(sum > 0.0f)) return fs.top_i[0];
    float r = 0.f;
    if (lane == 0) r = rand_uniform(rng) * sum;
    r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 0));
    float c = 0.f;
    for (int j0 = 0; j0 < ke; j0 += 8) {
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = pv[j0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (j0 + u < ke) {
                c += p[u];
                if (c >= r) return fs.top_i[j0 + u];
            }
        }
    }
    return 0;
}

// Bin of the key distance d = Kmax - key from the largest eligible key:
// exact below 32, then 16 bins per octave (the 4 bits under the leading one).
// Monotone in d, so the bins ascend from the largest value down; 0..463.
// (8 bins per octave left > KC keys through the k-th key's bin in ~10 % of
// standard-normal logit rows at k 50; 16 in < 1 %.)
constexpr int DBINS = 512;
__device__ __forceinline__ int dist_bin(uint32_t d) {
    if (d < 32u) return (int)d;
    const int e = 31 - __builtin_clz(d);
    return 32 + ((e - 5) << 4) + (int)((d >> (e - 4)) & 15u);
}
// okey's inverse (a -0 comes back as +0, which no comparison or difference
// below tells apart)
__device__ __forceinline__ float key_val(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Top-k draw for k <= KC in three barriers, the common case (top-k 50 over
// 2048 / 3072 logits).  (1) the block max M and the eligible count;
// (2) one histogram of dist_bin(okey(M) - key): the first bin B at which the
// running count reaches k bounds a candidate set -- every key in a bin <= B
// -- that holds the top k; (3) each wave compacts its candidates into LDS.
// Wave 0 then ranks the <= KC candidates by (value desc, index asc) -- the
// order the reference's strict '>' insertion list leaves (K.c:436-449) --
// with p_j = expf(v_j - M) computed beside the rank (M is the list's head,
// K.c:452), sums the first k in rank order sequentially (K.c:456-463), lane j
// keeping the running sum through j, and draws the first j whose running sum
// reaches r = u * sum (K.c:466-474) by a ballot: the same sums, so the same
// id.  Returns the id in wave 0 (the other waves return 0), or -1 in every
// thread when more than KC keys share the bins through B (ties, a very dense
// boundary bin): the caller then runs the radix select after a barrier.
// (STOP < 4: the micro-benchmark's phase cut, tools/mb_sample.hip)
template <int EM, int STOP = 4>
__device__ __forceinline__ int sample_dist(FastSmem &fs, const float (&v)[EM], const uint32_t (&kk)[EM], int E, int k,
                                           uint32_t &rng, uint64_t etab) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float m = -INFINITY;
    int ne = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j)
        if (kk[j] != 0u) { m = fmaxf(m, v[j]); ++ne; }
    m = wave_max(m);
    ne = __builtin_amdgcn_readlane(wave_incl_scan(ne), 63);
    int (*dh)[DBINS] = reinterpret_cast<int (*)[DBINS]>(&fs.hist[0][0][0]);   // [wave][bin]
#pragma unroll
    for (int i = 0; i < DBINS / 64; ++i) dh[w][lane + 64 * i] = 0;
    if (lane == 0) { fs.red[w] = m; fs.redn[w] = ne; }
    __syncthreads();
    const float M = fmaxf(fmaxf(fs.red[0], fs.red[1]), fmaxf(fs.red[2], fs.red[3]));
    const int ne_all = fs.redn[0] + fs.redn[1] + fs.redn[2] + fs.redn[3];
    if (k > ne_all) k = ne_all;
    if (k == 0) return 0;                     // nothing eligible: the reference returns 0
    if constexpr (STOP == 1) return (int)M;
    const uint32_t Kmax = okey(M);
    int bb[EM];
    int *h = dh[w];
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        bb[j] = DBINS;
        if (kk[j] != 0u) { bb[j] = dist_bin(Kmax - kk[j]); atomicAdd(&h[bb[j]], 1); }
    }
    __syncthreads();
    // merged histogram, nearest bins first: lane covers bins 8 lane .. 8 lane + 7
    constexpr int BL = DBINS / 64;
    int c[BL], tot = 0;
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int bin = BL * lane + i;
        c[i] = dh[0][bin] + dh[1][bin] + dh[2][bin] + dh[3][bin];
        tot += c[i];
    }
    const int inc = wave_incl_scan(tot), exc = inc - tot;
    int B = -1, nc = 0;
    if (exc < k && inc >= k) {
        int cum = exc;
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            cum += c[i];
            if (B < 0 && cum >= k) { B = BL * lane + i; nc = cum; }
        }
    }
    if constexpr (STOP == 2) return tot;
    const unsigned long long hit = __ballot(B >= 0);   // non-empty: k <= ne_all
    const int src = __ffsll((long long)hit) - 1;
    B = __builtin_amdgcn_readlane(B, src);
    nc = __builtin_amdgcn_readlane(nc, src);
    if (nc > KC) return -1;
    int mine = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j) mine += bb[j] <= B;
    const int wi = wave_incl_scan(mine);
    int pos = wi - mine;
#pragma unroll
    for (int j = 0; j < EM; ++j)
        if (bb[j] <= B) {
            fs.cand[w][pos] = ((unsigned long long)kk[j] << 32) | (0xFFFFFFFFu - (uint32_t)(tid * E + j));
            ++pos;
        }
    if (lane == 63) fs.ncw[w] = wi;
    __syncthreads();
    if (w != 0) return 0;
    if constexpr (STOP == 3) return fs.ncw[0];
    // wave 0: lane l takes candidate l of the concatenated per-wave lists
    const int n0 = fs.ncw[0], n1 = fs.ncw[1], n2 = fs.ncw[2];
    int ww = 0, off = lane;
    if (off >= n0) { off -= n0; ww = 1; if (off >= n1) { off -= n1; ww = 2; if (off >= n2) { off -= n2; ww = 3; } } }
    if (lane >= nc) { ww = 0; off = 0; }
    const unsigned long long key = lane < nc ? fs.cand[ww][off] : 0ull;   // 0: below every real key
    fs.rk[lane] = key;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // one wave: LDS is in order once the writes landed
    const float e = expf_glibc_wave(lane < nc ? key_val((uint32_t)(key >> 32)) - M : 0.f, etab);
    int rank = 0;
    for (int t0 = 0; t0 < nc; t0 += 8) {
        unsigned long long kt[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) kt[u] = fs.rk[t0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += kt[u] > key;
    }
    if (lane < nc && rank < k) { fs.pv[rank] = e; fs.pi[rank] = (int)(0xFFFFFFFFu - (uint32_t)key); }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float sum = 0.f, cj = 0.f;
    for (int j0 = 0; j0 < k; j0 += 8) {
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = fs.pv[j0 + u];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j0 + u < k) {
                sum += p[u];
                if (lane == j0 + u) cj = sum;
            }
    }
    if (!(sum > 0.0f)) return fs.pi[0];
    float r = 0.f;
    if (lane == 0) r = rand_uniform(rng) * sum;
    r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 0));
    const unsigned long long hit2 = __ballot(lane < k && cj >= r);
    return hit2 ? fs.pi[__ffsll((long long)hit2) - 1] : 0;
}

// Returns the sampled id: in wave 0 (the callers that need it in every wave
// broadcast it).  v[]: logits / temperature.
template <int EM>
__device__ __forceinline__ int sample_fast_regs(FastSmem &fs, const float (&v)[EM], int E, int n, int k, uint32_t &rng,
                                                uint64_t etab) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    uint32_t kk[EM];
#pragma unroll
    for (int j = 0; j < EM; ++j) kk[j] = (j < E && tid * E + j < n && v[j] > -FLT_MAX) ? okey(v[j]) : 0u;
    if (k <= KC) {
        const int t = sample_dist<EM>(fs, v, kk, E, k, rng, etab);
        if (t != -1) return t;
        __syncthreads();   // the radix select below rewrites the histograms the other waves read
    }
    uint32_t T, Tm;
    int take_eq, ne;
    radix_select_regs<EM>(fs, kk, E, k, T, Tm, take_eq, ne);
    const int ke = k < ne ? k : ne;
    if (ke == 0) return 0;                       // nothing eligible: the reference returns 0
    // taken: (key & Tm) > T, or == T for the first take_eq of those in index order
    int ngt = 0, neq = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        if (j < E && kk[j] != 0u) {
            const uint32_t m = kk[j] & Tm;
            ngt += m > T;
            neq += m == T;
        }
    }
    int gt0, eq0;
    block_scan2(fs, ngt, neq, gt0, eq0);
    int pos = gt0 + min(eq0, take_eq);
    int eqc = eq0;
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        if (j < E && kk[j] != 0u) {
            const uint32_t m = kk[j] & Tm;
            bool take = m > T;
            if (m == T) { take = eqc < take_eq; ++eqc; }
            if (take) { fs.sel_v[pos] = v[j]; fs.sel_i[pos] = tid * E + j; ++pos; }
        }
    }
    __syncthreads();
    if (ke <= 64) {   // the common case (top-k 50): one wave sorts and draws
        if (tid < 64) {
            const int t = wave_sort_draw(fs, ke, rng, etab);
            if (tid == 0) fs.misc[0] = t;
        }
        __syncthreads();
        const int out = fs.misc[0];
        __syncthreads();   // fs is reused by a second draw (fixed-mode EOS re-sample)
        return out;
    }
    // exact rank among the ke selected (value desc, index asc); sel_* is in index order
    for (int s2 = tid; s2 < ke; s2 += 256) {
        const float vs = fs.sel_v[s2];
        const uint32_t ks = okey(vs);
        int rk = 0;
        for (int t = 0; t < ke; ++t) {
            const uint32_t kt = okey(fs.sel_v[t]);
            rk += (kt > ks) || (kt == ks && t < s2);
        }
        fs.top_v[rk] = vs;
        fs.top_i[rk] = fs.sel_i[s2];
    }
    __syncthreads();
    const float mx = fs.top_v[0];
    for (int j = tid; j < ke; j += 256) fs.sel_v[j] = expf_glibc(fs.top_v[j] - mx);
    __syncthreads();
    if (tid == 0) {
        float sum = 0.0f;
        for (int j = 0; j < ke; ++j) sum += fs.sel_v[j];
        int out = 0;
        if (sum > 0.0f) {
            const float r = rand_uniform(rng) * sum;
            float c = 0.0f;
            for (int j = 0; j < ke; ++j) {
                c += fs.sel_v[j];
                if (c >= r) { out = fs.top_i[j]; break; }
            }
        } else {
            out = fs.top_i[0];
        }
        fs.misc[0] = out;
    }
    __syncthreads();
    const int out = fs.misc[0];
    __syncthreads();   // fs is reused by a second draw (fixed-mode EOS re-sample)
    return out;
}

// ---------------------------------------------------------------------------
// The same fast path on NT = 1024 threads (16 waves, <= 4 ids per thread):
// a quarter of the per-thread work of every phase, one SHARED distance
// histogram, candidate slots by one LDS atomic per wave, and the rank of the
// <= 64 candidates split over the 16 waves (4 comparisons each) instead of
// one wave's 64.  Wave 0 then holds p_j for rank j in lane j and sums them
// sequentially in rank order with v_readlane (the reference's order,
// K.c:456-463), and draws by ballot -- the same sums, so the same id as the
// 256-thread path and the reference.  Dense ties (> 64 candidates) fall back
// to the radix select over a shared three-buffer histogram.
template <int NT>
struct FastSmemNT {
    static constexpr int NW = NT / 64;
    int hist[3][256];                  // radix fallback, rotating buffers
    int scan[NW];
    float sel_v[KFAST];
    int sel_i[KFAST];
    float top_v[KFAST];
    int top_i[KFAST];
    int misc[4];
    alignas(16) int dh[DBINS];         // (read as int4) distance histogram (shared; 4 copies by wave measured slower, 5.21 vs 4.98 us)
    unsigned long long cand[KC];       // candidate keys (value key << 32 | ~index), slots by atomic
    int crank[KC];                     // candidate ranks, summed over the waves' slices
    alignas(16) float pv[KC];          // (read as float4)
    int pi[KC];
    float red[NW];
    int redn[NW];
    int ncand;
};
// the int4 / float4 LDS reads of dh and pv (ds_read_b128) need 16-B offsets
static_assert(offsetof(FastSmemNT<256>, dh) % 16 == 0 && offsetof(FastSmemNT<256>, pv) % 16 == 0, "FastSmemNT<256>");
static_assert(offsetof(FastSmemNT<1024>, dh) % 16 == 0 && offsetof(FastSmemNT<1024>, pv) % 16 == 0, "FastSmemNT<1024>");

// block-wide exclusive scans of two small per-thread counts (16 | 16 bits)
template <int NT>
__device__ __forceinline__ void block_scan2_nt(FastSmemNT<NT> &fs, int x, int y, int &ex, int &ey) {
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int v = x | (y << 16);
    const int inc = wave_incl_scan(v);
    if (l == 63) fs.scan[w] = inc;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; ++i) base += fs.scan[i];
    const int e = base + inc - v;
    ex = e & 0xFFFF;
    ey = e >> 16;
}

// radix_select_regs over one shared histogram per pass; buffers 0 and 1 are
// zeroed by the caller before a barrier, buffer (p + 2) % 3 after pass p's
// barrier (its readers were pass p - 1, its writers come after pass p + 1's)
template <int NT, int EM>
__device__ __forceinline__ void radix_select_nt(FastSmemNT<NT> &fs, const uint32_t (&kk)[EM], int E, int k,
                                                uint32_t &T, uint32_t &Tmask, int &take_eq, int &ne) {
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t prefix = 0, mask = 0;
    int rem = k;
    ne = -1;
    int p = 0;
    for (int shift = 24; shift >= 0; shift -= 8, ++p) {
        int *h = fs.hist[p % 3];
#pragma unroll
        for (int j = 0; j < EM; ++j)
            if (j < E && kk[j] != 0u && (kk[j] & mask) == prefix) atomicAdd(&h[(kk[j] >> shift) & 255u], 1);
        __syncthreads();
        int c[4], tot = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            c[i] = h[255 - 4 * lane - i];
            tot += c[i];
        }
        const int inc = wave_incl_scan(tot);
        if (ne < 0) {
            ne = __builtin_amdgcn_readlane(inc, 63);
            if (k > ne) k = ne;
            rem = k;
        }
        const int exc = inc - tot;
        int bin = -1, nrem = 0, cbin = 0;
        if (exc < rem && inc >= rem) {
            int cum = exc;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (bin < 0 && cum + c[i] >= rem) { bin = 255 - 4 * lane - i; nrem = rem - cum; cbin = c[i]; }
                cum += c[i];
            }
        }
        const unsigned long long hit = __ballot(bin >= 0);
        const int src = hit ? __ffsll((long long)hit) - 1 : 0;
        bin = __builtin_amdgcn_readlane(bin, src);
        nrem = __builtin_amdgcn_readlane(nrem, src);
        cbin = __builtin_amdgcn_readlane(cbin, src);
        if (tid < 256) fs.hist[(p + 2) % 3][tid] = 0;
        if (k == 0) { T = 0xFFFFFFFFu; Tmask = 0xFFFFFFFFu; take_eq = 0; return; }
        prefix |= (uint32_t)bin << shift;
        mask |= 255u << shift;
        rem = nrem;
        if (cbin == nrem || shift == 0) {
            T = prefix; Tmask = mask; take_eq = nrem;
            return;
        }
    }
}

// Top-k draw for k <= KC (see sample_dist): returns the id in wave 0 (0 in
// the other waves), or -1 in every thread when more than KC keys share the
// bins through the k-th key's.  Four barriers.
template <int NT, int EM, int STOP = 9>
__device__ __forceinline__ int sample_dist_nt(FastSmemNT<NT> &fs, const float (&v)[EM], const uint32_t (&kk)[EM],
                                              const int (&id)[EM], int k, uint32_t &rng, uint64_t etab) {
#pragma clang fp contract(off)
    constexpr int NW = NT / 64;
    static_assert(NW * 4 >= KC, "the rank slices cover KC candidates");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float m = -INFINITY;
    int ne = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j)
        if (kk[j] != 0u) { m = fmaxf(m, v[j]); ++ne; }
    m = wave_max(m);
    ne = __builtin_amdgcn_readlane(wave_incl_scan(ne), 63);
    for (int i = tid; i < DBINS; i += NT) fs.dh[i] = 0;
    if (tid < 256) { fs.hist[0][tid] = 0; fs.hist[1][tid] = 0; }   // (the radix fallback's first buffers)
    if (tid < KC) fs.crank[tid] = 0;
    if (tid == 0) fs.ncand = 0;
    if (lane == 0) { fs.red[w] = m; fs.redn[w] = ne; }
    __syncthreads();                                                   // 1
    const float M = wave_max(lane < NW ? fs.red[lane] : -INFINITY);
    const int ne_all = __builtin_amdgcn_readlane(wave_incl_scan(lane < NW ? fs.redn[lane] : 0), 63);
    if (k > ne_all) k = ne_all;
    if (k == 0) return 0;                     // nothing eligible: the reference returns 0
    if constexpr (STOP == 1) return (int)M;
    const uint32_t Kmax = okey(M);
    // keys 2^31 or more below the maximum in key order (most values of the
    // other sign -- often half the row) all count in bin FARB, one LDS atomic per wave and
    // slot instead of 64 colliding ones; should the k-th key lie there, the
    // bins bound more than KC candidates and the radix select takes over
    constexpr int FARB = 32 + 16 * (31 - 5);
    int bb[EM];
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        bb[j] = DBINS;
        bool far = false;
        if (kk[j] != 0u) {
            const int bn = dist_bin(Kmax - kk[j]);
            far = bn >= FARB;
            bb[j] = far ? FARB : bn;
            if (!far) atomicAdd(&fs.dh[bn], 1);
        }
        const unsigned long long fm = __ballot(far);
        if (lane == 0 && fm) atomicAdd(&fs.dh[FARB], (int)__popcll(fm));
    }
    __syncthreads();                                                   // 2
    constexpr int BL = DBINS / 64;
    int c[BL], tot = 0;
    {
        const int4 h0 = *reinterpret_cast<const int4 *>(&fs.dh[BL * lane]);
        const int4 h1 = *reinterpret_cast<const int4 *>(&fs.dh[BL * lane + 4]);
        c[0] = h0.x; c[1] = h0.y; c[2] = h0.z; c[3] = h0.w; c[4] = h1.x; c[5] = h1.y; c[6] = h1.z; c[7] = h1.w;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) tot += c[i];
    const int inc = wave_incl_scan(tot), exc = inc - tot;
    int B = -1, nc = 0;
    if (exc < k && inc >= k) {
        int cum = exc;
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            cum += c[i];
            if (B < 0 && cum >= k) { B = BL * lane + i; nc = cum; }
        }
    }
    if constexpr (STOP == 2) return tot;
    const unsigned long long hit = __ballot(B >= 0);   // non-empty: k <= ne_all
    const int src = __ffsll((long long)hit) - 1;
    B = __builtin_amdgcn_readlane(B, src);
    nc = __builtin_amdgcn_readlane(nc, src);
    if (nc > KC) return -1;
    // candidates (bin <= B) to slots: one returning LDS atomic per wave
    int mine = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j) mine += bb[j] <= B;
    const int wi = wave_incl_scan(mine);
    const int wtot = __builtin_amdgcn_readlane(wi, 63);
    int base = 0;
    if (wtot > 0) {
        if (lane == 0) base = atomicAdd(&fs.ncand, wtot);
        base = __builtin_amdgcn_readlane(base, 0);
    }
    int pos = base + wi - mine;
#pragma unroll
    for (int j = 0; j < EM; ++j)
        if (bb[j] <= B) {
            fs.cand[pos] = ((unsigned long long)kk[j] << 32) | (0xFFFFFFFFu - (uint32_t)id[j]);
            ++pos;
        }
    __syncthreads();                                                   // 3
    if constexpr (STOP == 3) return nc;
    // rank: candidate `lane` against the 4 of this wave's slice (value desc, index asc)
    const unsigned long long key = lane < nc ? fs.cand[lane] : 0ull;   // 0: below every real key
    {
        // (unconditional reads of the slice -- slots past nc hold stale keys,
        // masked after -- so the four LDS reads are in flight together)
        unsigned long long kt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) kt[u] = fs.cand[4 * w + u];
        int r = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) r += (4 * w + u < nc) && kt[u] > key;
        if (lane < nc && r > 0) atomicAdd(&fs.crank[lane], r);
    }
    float e = 0.f;
    if (w == 0) e = expf_glibc_wave(lane < nc ? key_val((uint32_t)(key >> 32)) - M : 0.f, etab);
    __syncthreads();                                                   // 4
    if (w != 0) return 0;
    if constexpr (STOP == 4) return fs.crank[lane];
    const int rank = fs.crank[lane];
    if (lane < nc && rank < k) { fs.pv[rank] = e; fs.pi[rank] = (int)(0xFFFFFFFFu - (uint32_t)key); }
    if (lane >= k) fs.pv[lane] = 0.f;   // (adding +0 leaves every running sum as it is)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // one wave: LDS is in order once the writes landed
    // every lane holds all 64 p_j (broadcast reads) and walks them in rank
    // order: the sum, then the running sum to the first j with c_j >= r --
    // plain dependent adds in registers (a v_readlane per step cost ~30 ns)
    float4 q[KC / 4];
#pragma unroll
    for (int i = 0; i < KC / 4; ++i) q[i] = reinterpret_cast<const float4 *>(fs.pv)[i];
    if constexpr (STOP == 5) return (int)q[0].x;
    // running sums c_j in rank order (the reference's sequential sum); p_j >= 0,
    // so c_j never decreases and the first j with c_j >= r is the number of
    // j with c_j < r -- counted with independent compares (a uniform
    // first-match chain compiled to ~15 dependent VALU -> SALU steps per j)
    float run[KC];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < KC / 4; ++i) {
        sum += q[i].x; run[4 * i] = sum;
        sum += q[i].y; run[4 * i + 1] = sum;
        sum += q[i].z; run[4 * i + 2] = sum;
        sum += q[i].w; run[4 * i + 3] = sum;
    }
    if constexpr (STOP == 6) return (int)sum;
    if (!(sum > 0.0f)) return fs.pi[0];
    float r = 0.f;
    if (lane == 0) r = rand_uniform(rng) * sum;
    r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 0));
    int n4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < KC; ++j) n4[j & 3] += run[j] < r ? 1 : 0;
    const int jf = n4[0] + n4[1] + n4[2] + n4[3];   // k..KC: no j reached r (the reference returns 0)
    return jf < k ? fs.pi[jf] : 0;
}

// sample_fast_regs on NT threads: thread t owns ids id[j] = t*E + j (j < E).
template <int NT, int EM>
__device__ __forceinline__ int sample_fast_nt(FastSmemNT<NT> &fs, const float (&v)[EM], int E, int n, int k,
                                              uint32_t &rng, uint64_t etab) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    uint32_t kk[EM];
    int id[EM];
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        id[j] = tid * E + j;
        kk[j] = (j < E && id[j] < n && v[j] > -FLT_MAX) ? okey(v[j]) : 0u;
    }
    if (k <= KC) {
        const int t = sample_dist_nt<NT, EM>(fs, v, kk, id, k, rng, etab);
        if (t != -1) return t;
        __syncthreads();   // (every thread returned -1 at the same point; hist 0 / 1 were zeroed before barrier 1)
    } else {
        if (threadIdx.x < 256) { fs.hist[0][threadIdx.x] = 0; fs.hist[1][threadIdx.x] = 0; }
        __syncthreads();
    }
    uint32_t T, Tm;
    int take_eq, ne;
    radix_select_nt<NT, EM>(fs, kk, E, k, T, Tm, take_eq, ne);
    const int ke = k < ne ? k : ne;
    if (ke == 0) return 0;
    int ngt = 0, neq = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        if (j < E && kk[j] != 0u) {
            const uint32_t m = kk[j] & Tm;
            ngt += m > T;
            neq += m == T;
        }
    }
    int gt0, eq0;
    block_scan2_nt<NT>(fs, ngt, neq, gt0, eq0);
    int pos = gt0 + min(eq0, take_eq);
    int eqc = eq0;
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        if (j < E && kk[j] != 0u) {
            const uint32_t m = kk[j] & Tm;
            bool take = m > T;
            if (m == T) { take = eqc < take_eq; ++eqc; }
            if (take) { fs.sel_v[pos] = v[j]; fs.sel_i[pos] = id[j]; ++pos; }
        }
    }
    __syncthreads();
    if (ke <= 64) {
        if (tid < 64) {
            const int t = wave_sort_draw(fs, ke, rng, etab);
            if (tid == 0) fs.misc[0] = t;
        }
        __syncthreads();
        const int out = fs.misc[0];
        __syncthreads();   // fs is reused by a second draw (fixed-mode EOS re-sample)
        return out;
    }
    for (int s2 = tid; s2 < ke; s2 += NT) {
        const float vs = fs.sel_v[s2];
        const uint32_t ks = okey(vs);
        int rk = 0;
        for (int t = 0; t < ke; ++t) {
            const uint32_t kt = okey(fs.sel_v[t]);
            rk += (kt > ks) || (kt == ks && t < s2);
        }
        fs.top_v[rk] = vs;
        fs.top_i[rk] = fs.sel_i[s2];
    }
    __syncthreads();
    const float mx = fs.top_v[0];
    for (int j = tid; j < ke; j += NT) fs.sel_v[j] = expf_glibc(fs.top_v[j] - mx);
    __syncthreads();
    if (tid == 0) {
        float sum = 0.0f;
        for (int j = 0; j < ke; ++j) sum += fs.sel_v[j];
        int out = 0;
        if (sum > 0.0f) {
            const float r = rand_uniform(rng) * sum;
            float c = 0.0f;
            for (int j = 0; j < ke; ++j) {
                c += fs.sel_v[j];
                if (c >= r) { out = fs.top_i[j]; break; }
            }
        } else {
            out = fs.top_i[0];
        }
        fs.misc[0] = out;
    }
    __syncthreads();
    const int out = fs.misc[0];
    __syncthreads();
    return out;
}

union KSmem {
    SampSmem full;
    FastSmem fast;
};

__host__ __device__ inline bool fast_path(const SampArgs &a) {
    return a.top_p >= 1.0f && a.top_k > 0 && a.top_k < a.n && a.top_k <= KFAST && a.n <= NMAX;
}

// One row's draw (all NT threads of the workgroup).  `smraw` >= sizeof(KSmem),
// or sizeof(FastSmem) / sizeof(FastSmemNT<NT>) with FAST_ONLY (the caller
// guarantees fast_path(a)).  Used by k_sample.
// The row's input pointers come as parameters (a.logits, a.stopped, the RNG
// state array of the mode, a.n_gen, a.counts) so that k_sample_w can take
// them as preloaded kernel arguments.
template <bool FAST_ONLY, int EM = EMAX, int NT = 256>
__device__ __forceinline__ void sample_row(const SampArgs &a, int b, unsigned char *smraw, const float *logits,
                                           const int *stopped_p, const uint32_t *rng_p, const int *ngen_p,
                                           const int *counts_p) {
#pragma clang fp contract(off)
    static_assert(NT == 256 || FAST_ONLY, "the full path runs on 256 threads");
    KSmem &U = *reinterpret_cast<KSmem *>(smraw);
    int *misc = NT == 256 ? U.fast.misc : reinterpret_cast<FastSmemNT<NT> *>(smraw)->misc;
    const int tid = threadIdx.x, n = a.n;
    // every global read of this kernel is issued up front, as VECTOR loads
    // from unconditional (clamped) addresses: the logits, the repetition
    // counts, then the row's flags and RNG state (through an opaque zero
    // offset: as scalar loads they were waited for one after another --
    // stopped, then the RNG state -- before the first logit load issued)
    const int E = (n + NT - 1) / NT;
    const float *lg = logits + (size_t)b * a.ld;
    const int i0 = tid * E;
    float x[EM];
    int cnt[EM];
    const bool pen = a.mode == 1 && a.rep != 1.0f && counts_p;
    const int *cbase = pen ? counts_p + (size_t)b * n : reinterpret_cast<const int *>(lg);
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        const int i = i0 + j < n ? i0 + j : n - 1;
        x[j] = lg[i];
        cnt[j] = cbase[i];
    }
    int z0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
    // (an absent flag reads a logit word instead, and is replaced by 0 below)
    const int *sp = stopped_p ? stopped_p + b : reinterpret_cast<const int *>(lg);
    const int *np = a.mode == 1 ? ngen_p + b : reinterpret_cast<const int *>(lg);
    const uint32_t *rp = rng_p + b;
    int stopped = sp[z0];
    int ng = np[z0];
    uint32_t rng = rp[z0];
    const uint64_t etab = kExp2fTab[tid & 31];   // expf_glibc_wave's table, with the first loads
    // one wait for all of them here (the compiler would otherwise sink the
    // flag loads into the branches that use them: another round trip each)
    asm volatile("" :: "v"(stopped), "v"(ng), "v"(rng));
    if (!stopped_p) stopped = 0;
    if (a.mode != 1) ng = 0;
#pragma unroll
    for (int j = 0; j < EM; ++j) {
        const bool ok = j < E && i0 + j < n;
        if (!ok) x[j] = -INFINITY;
        if (!(ok && pen)) cnt[j] = 0;
    }
    if (stopped) return;
    if (a.mode == 1) {
#pragma unroll
        for (int j = 0; j < EM; ++j) {
            const int i = i0 + j;
            float v = x[j];
            if (i >= a.suppress_lo && i != a.eos) v = -1e9f;
            for (int c = 0; c < cnt[j]; ++c) v = v > 0 ? div_rn(v, a.rep) : v * a.rep;
            x[j] = (j < E && i < n) ? v : -INFINITY;
        }
    }
    float temp = a.temp;
    if (temp <= 0.0f) temp = 1e-5f;
    const bool fast = FAST_ONLY || fast_path(a);
    int tok = 0;
    if (fast) {
        float v[EM];
#pragma unroll
        for (int j = 0; j < EM; ++j) v[j] = div_rn(x[j], temp);
        auto draw = [&]() {   // (wave 0's id)
            if constexpr (NT == 256) return sample_fast_regs<EM>(U.fast, v, E, n, a.top_k, rng, etab);
            else return sample_fast_nt<NT, EM>(*reinterpret_cast<FastSmemNT<NT> *>(smraw), v, E, n, a.top_k, rng, etab);
        };
        tok = draw();
        if (a.mode == 1 && a.fixed > 0 && ng < a.fixed) {   // Q.c:1315-1321: an EOS draw is redrawn
            if (tid == 0) misc[3] = tok;
            __syncthreads();
            tok = misc[3];
            if (tok == a.eos) {
#pragma unroll
                for (int j = 0; j < EM; ++j)
                    if (i0 + j == a.eos) v[j] = div_rn(-1e9f, temp);
                tok = draw();
            }
        }
    } else if constexpr (!FAST_ONLY) {
        SampSmem &sm = U.full;
#pragma unroll
        for (int j = 0; j < EM; ++j)
            if (j < E && i0 + j < n) sm.lg[i0 + j] = x[j];
        __syncthreads();
        tok = sample_any(sm, n, a.top_k, a.top_p, a.temp, rng);
        if (a.mode == 1 && a.fixed > 0 && tok == a.eos && ng < a.fixed) {
            if (tid == 0) sm.lg[a.eos] = -1e9f;
            __syncthreads();
            tok = sample_any(sm, n, a.top_k, a.top_p, a.temp, rng);
        }
    }
    if (tid == 0) {
        if (a.mode == 1) {
            a.rng[b] = rng;
            if (a.fixed == 0 && tok == a.eos) {
                a.stopped[b] = 1;
                if (a.host_stopped) a.host_stopped[b] = 1;   // the host's lagged poll (qtts_dev_frame_done)
                if (a.stop_step) a.stop_step[b] = ng;
            } else {
                a.cur_row[b] = ng;
                a.codes[(size_t)b * a.codes_bstride + (size_t)ng * a.G + 0] = tok;
                if (a.counts) a.counts[(size_t)b * n + tok] += 1;
                a.n_gen[b] = ng + 1;
                a.st_rng[b] = a.seed_bits;
            }
            // the sub-talker's table readers take this id (pass 1) and keep it
            // for a stopped row (its samplers return early): EOS (>= Vs) would
            // index past the last pass's table, so a stop leaves id 0
            if (a.out_tok) a.out_tok[b] = (a.fixed == 0 && tok == a.eos) ? 0 : tok;
        } else {
            a.st_rng[b] = rng;
            if (a.codes) a.codes[(size_t)b * a.codes_bstride + (size_t)a.cur_row[b] * a.G + a.g] = tok;
            if (a.out_tok) a.out_tok[b] = tok;
        }
    }
}

}  // namespace qtts_samp
