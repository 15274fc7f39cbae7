// k_misc.hip - small element-wise kernels around the decode loop.
#include "qtts_common.h"
#include "qtts_kernels.h"

namespace {

// next_embed (c/qwen_tts.c:1345-1363), per element in the reference's order:
//   0 + codec_emb[code0] + st_emb[0][code1] + ... + st_emb[G-2][code G-1]
//     + (row < n_trailing ? trailing[row] : tts_pad)
// so the result is bit-identical to the host loop.  Also advances kv_len for
// the frame's talker token.
__global__ __launch_bounds__(256) void k_embed_sum(EmbedSumArgs a) {
#pragma clang fp contract(off)
    const int b = blockIdx.y;
    const int d = blockIdx.x * 256 + threadIdx.x;
    // three dependent round trips, each with all of its loads in flight:
    // (stop flag, row, trailing count) -> (16 codes) -> (16 embedding rows + the text row)
    const int stop = a.stopped ? a.stopped[b] : 0;
    const int row = a.cur_row[b];
    const int ntr = a.n_trailing[b];
    if (stop) return;
    const int *cd = a.codes + (size_t)b * a.codes_bstride + (size_t)row * a.G;
    constexpr int GM = 16;   // code groups (host: G <= 16)
    // (groups past G repeat group G - 1's load and are left out of the sum:
    // no branch around a load)
    int c[GM];
#pragma unroll
    for (int g = 0; g < GM; ++g) c[g] = cd[g < a.G ? g : a.G - 1];
    if (d < a.H) {
        const float *tt = row < ntr ? a.trailing + ((size_t)b * a.tr_cap + row) * a.H : a.pad;
        float e[GM];
        e[0] = bf2f(a.codec_emb[(size_t)c[0] * a.H + d]);
#pragma unroll
        for (int g = 1; g < GM; ++g) {
            const int gg = g < a.G ? g : a.G - 1;
            e[g] = bf2f(a.st_emb[((size_t)(gg - 1) * a.Vs + c[g]) * a.H + d]);
        }
        const float t = tt[d];
        float s = 0.0f;
        s += e[0];
#pragma unroll
        for (int g = 1; g < GM; ++g)
            if (g < a.G) s += e[g];
        s += t;
        a.out[(size_t)b * a.H + d] = s;
    }
    if (a.advance && blockIdx.x == 0 && threadIdx.x == 0) a.kv_len[b] += 1;
}

// prompt rows (c/qwen_tts.c:1192-1243): dst = proj_row (+ codec_emb[id]);
// voice clone (modeling_qwen3_tts.py:1967-2019, 2150-2190): + the speaker
// x-vector, or + a reference frame's group-embedding sum (0 + e_0 + ... + e_15
// in that order, out-of-range codes contribute nothing; oracle ref_frame_sum)
__global__ __launch_bounds__(256) void k_prompt(PromptArgs a) {
#pragma clang fp contract(off)
    const int e = blockIdx.y;
    const int *pl = a.plan + 5 * e;
    const int src = pl[0], cid = pl[1], kind = pl[2], b = pl[3], slot = pl[4];
    float *dst = kind == 0 ? a.prefill + ((size_t)b * a.p_cap + slot) * a.H
                           : a.trailing + ((size_t)b * a.tr_cap + slot) * a.H;
    const int f = -3 - cid;
    const int *fr = cid <= -3 && f < a.n_ref ? a.ref_codes + (size_t)f * a.G : nullptr;
    for (int d = blockIdx.x * 256 + threadIdx.x; d < a.H; d += gridDim.x * 256) {
        float v = a.proj[(size_t)src * a.H + d];
        if (cid >= 0) v += bf2f(a.codec_emb[(size_t)cid * a.H + d]);
        else if (cid == -2 && a.spk) v += a.spk[d];
        else if (fr) {
            float s = 0.0f;
            if (fr[0] >= 0 && fr[0] < a.V) s += bf2f(a.codec_emb[(size_t)fr[0] * a.H + d]);
            for (int g = 1; g < a.G; ++g)
                if (fr[g] >= 0 && fr[g] < a.Vs) s += bf2f(a.st_emb[((size_t)(g - 1) * a.Vs + fr[g]) * a.H + d]);
            v += s;
        }
        dst[d] = v;
    }
}

__global__ void k_copy_rows(float *dst, int ldd, const float *src, int lds, const int *rows, int ncols) {
    const int r = blockIdx.y;
    const int sr = rows ? rows[r] : r;
    for (int c = blockIdx.x * 256 + threadIdx.x; c < ncols; c += gridDim.x * 256)
        dst[(size_t)r * ldd + c] = src[(size_t)sr * lds + c];
}

// one slot's fresh-utterance state (qtts_dev_refill): grid covers max(H, V)
__global__ __launch_bounds__(256) void k_slot_reset(SlotResetArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < a.H) a.x[(size_t)a.b * a.H + i] = a.row[i];
    if (i < a.V) a.counts[(size_t)a.b * a.V + i] = 0;
    if (i == 0) {
        a.kv_len[a.b] = a.pos;
        a.n_gen[a.b] = 0;
        a.cur_row[a.b] = 0;
        a.stop_step[a.b] = 0;
        a.last_tok[a.b] = 0;
        a.rng[a.b] = a.seed_bits;
        a.st_rng[a.b] = a.seed_bits;
        a.stopped[a.b] = 0;
    }
}

}  // namespace

int qtts_slot_reset(const SlotResetArgs &a, hipStream_t st) {
    const int n = a.H > a.V ? a.H : a.V;
    hipLaunchKernelGGL(k_slot_reset, dim3((n + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int qtts_embed_sum(const EmbedSumArgs &a, hipStream_t st) {
    if (a.G < 2 || a.G > 16) {
        fprintf(stderr, "qtts_embed_sum: %d code groups (2..16 supported)\n", a.G);
        return -1;
    }
    hipLaunchKernelGGL(k_embed_sum, dim3((a.H + 255) / 256, a.nb), dim3(256), 0, st, a);
    qtts_last_kernel = "k_embed_sum";
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int qtts_prompt_assemble(const PromptArgs &a, hipStream_t st) {
    if (a.nplan <= 0) return 0;
    hipLaunchKernelGGL(k_prompt, dim3((a.H + 255) / 256, a.nplan), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int qtts_copy_rows(float *dst, int ldd, const float *src, int lds, const int *rows, int nrows, int ncols,
                   hipStream_t st) {
    if (nrows <= 0) return 0;
    hipLaunchKernelGGL(k_copy_rows, dim3((ncols + 255) / 256, nrows), dim3(256), 0, st, dst, ldd, src, lds, rows,
                       ncols);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
