// qtts_kernels.h - internal launch interface of the gfx950 kernels (C++ only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;

constexpr int QTTS_GM_TICKS = 1024;   // self-reducing split-K tickets (row blocks per launch)

enum { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_SILU = 2, EPI_RESID = 3, EPI_SWIGLU = 4 };

// The next launch's weight slice, loaded by the SAME workgroup index of this
// launch right after its own weights (qtts_l2pf below): workgroup b of every
// decode launch runs on XCD b % 8, so the slice lands in the L2 that the next
// launch's workgroup b reads from.  For linear workgroup id b:
//   start = base + (b % pm) * pa + (b / pm) * pb,
//   `chunks` 64-B chunks: chunk c at start + (c >> lg) * ld + (c & (2^lg - 1)) * 64
// (rows of 2^lg chunks at stride ld; chunks <= threads x QTTS_PF_LOADS).  One
// 4-B load per chunk brings its line in.
constexpr int QTTS_PF_LOADS = 4;
struct L2Prefetch {
    const unsigned char *base = nullptr;   // nullptr: none
    int pm = 1 << 30;
    long long pa = 0, pb = 0;
    int chunks = 0, lg = 30, ld = 0;
    int cs = 6;                            // log2 bytes per chunk (64 B; the micro-benchmark also runs 128)
    // slices of the target: a workgroup b >= nwg of a launch wider than the
    // next one's grid has no slice of its own and re-reads its fallback line
    // (the start formula would otherwise run past the target's end)
    int nwg = 0;
    unsigned *sink = nullptr;              // never written (the loads' values are folded into a test)
};

struct GemvArgs {
    const bf16_t *W = nullptr;  // [R, C] bf16 row-major
    int R = 0, C = 0;
    int ksplit = 0;             // 0 = auto
    int cch = 0;                // set by launcher
    int nt = 1;                 // non-temporal weight loads
    int nb = 1;                 // batch rows
    // x source: fp32 rows, or bf16 / fp32 table rows gathered by id
    const float *x = nullptr;
    int ldx = 0;
    const bf16_t *table = nullptr;      // [*, C]
    const float *table_f32 = nullptr;   // [*, C] (precomputed projected embeddings)
    const int *ids = nullptr;       // id(b) = ids[b*ids_bstride + row_sel[b]*ids_rstride + ids_off]
    int ids_bstride = 1, ids_rstride = 0, ids_off = 0;
    const int *row_sel = nullptr;
    // lean kernel (qtts_gemvw) only: reps consecutive ids in one launch
    // (grid.y), rep j reads id ids[ids_off + j] and writes y + j * ldy_rep
    int reps = 1;
    size_t ldy_rep = 0;
    // prologue
    // batch-1 prologue only: x += sum_p xadd[p*ld_xadd + c] (p < n_xadd, summed
    // in order first) -- the O projection's per-head partials (qtts_attn_o)
    const float *xadd = nullptr;
    int n_xadd = 0, ld_xadd = 0;
    int ldb_xadd = 0;               // batch path (k_gemvm): row b of partial p at xadd + p*ld_xadd + b*ldb_xadd
    // batch-1 prologue only: x = the decode attention's output, merged here
    // from its split partials (AttnArgs::defer): amerge [KV][am_nsplit][GPH*HD
    // + 2*GPH], am_ch keys per split, the live key count am_pos[0] + 1
    const float *amerge = nullptr;
    const int *am_pos = nullptr;
    int am_nsplit = 0, am_ch = 0, am_hd = 0, am_gph = 0;
    // batch path split-K producer (k_gemvm): kz > 1 workgroup columns each take
    // C / kz of K and store raw partials ypart[z*ld_ypart + b*R + r] (the
    // consumer adds them with the residual through xadd); y / epi unused
    float *ypart = nullptr;
    size_t ld_ypart = 0;
    int kz = 1;
    // self-reducing split-K (EPI_RESID only): one zeroed ticket per grid.x
    // workgroup; the last of the kz columns to finish a row block adds the
    // partials in order to the residual, y = y + (p0 + p1 + ...), and resets
    // its ticket, so the next GEMV reads y alone (no xadd)
    int *tick = nullptr;            // [QTTS_GM_TICKS]
    const float *norm_w = nullptr;  // RMSNorm weights [C] (nullptr: no norm)
    float eps = 1e-6f;
    float *xcopy = nullptr;         // workgroup 0 writes x rows here
    int ldxc = 0;
    int xcopy_normed = 0;
    // epilogue
    float *y = nullptr;
    int ldy = 0;
    const float *bias = nullptr;
    int epi = EPI_STORE;
    unsigned long long *dbg = nullptr;   // diagnostics (k_gemvb): [workgroup][8] phase stamps, 100 MHz clock
#ifdef QTTS_STAMPS
    int dbg_xfirst = 0;                  // (stamp builds) k_gemvw waits for x before issuing its weights
#endif
    L2Prefetch pf;                      // batch-1 lean kernel (k_gemvw): the next launch's weights
    // the batch-1 fast path needs 16-B aligned fp32 rows (or a bf16 table)
    bool ldx_ok1() const {
        if (xadd && (((uintptr_t)xadd & 15) || ld_xadd % 4 || n_xadd < 1)) return false;
        if (table) return C % 4 == 0;
        const bool nw_ok = !norm_w || ((uintptr_t)norm_w & 15) == 0;
        if (table_f32) return C % 4 == 0 && ((uintptr_t)table_f32 & 15) == 0 && nw_ok;
        return ((uintptr_t)x & 15) == 0 && nw_ok;
    }
};

int qtts_gemv(const GemvArgs &a, hipStream_t st);
// batch-1 wave-per-row GEMV for Infinity-Cache-resident weights (k_gemvw.hip); 1 = not covered
int qtts_gemvw(const GemvArgs &a, hipStream_t st);
// shapes whose batch-1 GEMV takes the decode attention's merge in its prologue (GemvArgs::amerge)
bool qtts_gemvw_amerge_ok(int R, int C);
// lock-step batch (2..16 rows) on the bf16 matrix cores (k_gemvm.hip); 1 = not covered
int qtts_gemvm(const GemvArgs &a, hipStream_t st);
// the same with the x rows sliced per wave (k_gemvb.hip, tried first); 1 = not covered
int qtts_gemvb(const GemvArgs &a, hipStream_t st);
// multi-row (2..64) projection on the bf16 matrix cores (k_mgemm.hip); 1 = not covered
int qtts_mgemm(const GemvArgs &a, float *inv_scratch, hipStream_t st, float *part = nullptr, size_t part_elems = 0);
// split-K partial floats qtts_mgemm may use for `rows` activation rows and outputs <= widest
size_t qtts_mgemm_part_elems(size_t rows, size_t widest);
int qtts_row_rms(const float *x, int ldx, int rows, int C, float eps, float *inv, hipStream_t st);
// split-K tail of qtts_mgemm / qtts_pgemm: y = epilogue(sum_z part[z][row][R], z in order)
int qtts_mgemm_reduce(const GemvArgs &a, const float *part, int kz, hipStream_t st);
// the talker prefill's projections over > 16 rows (k_pgemm.hip): activations
// split once into 3 bf16 planes (scratch: qtts_pgemm_plane_elems), then an
// LDS-tiled 128 x 128 MFMA GEMM; 1 = shape not covered
int qtts_pgemm(const GemvArgs &a, float *inv_scratch, unsigned short *planes, size_t plane_elems, hipStream_t st,
               float *part, size_t part_elems);
size_t qtts_pgemm_plane_elems(size_t rows, size_t K);

// one 1.7B talker decoder layer at batch 1 as one persistent launch
// (k_tengine.hip): 256 workgroups x 512 threads, hand-offs through 8-byte
// {tag, value} granules; x_out may alias x_in
struct TLayerArgs {
    const float *x_in = nullptr;
    float *x_out = nullptr;
    const bf16_t *wqkv = nullptr, *wo = nullptr, *wgu = nullptr, *wdown = nullptr;
    const float *in_norm = nullptr, *post_norm = nullptr, *qn_w = nullptr, *kn_w = nullptr;
    const float *rope_cos = nullptr, *rope_sin = nullptr;
    float *kc = nullptr, *vc = nullptr;          // this layer's cache, [S][KV*HD]
    const int *pos = nullptr;                    // kv_len before the step
    const int *skip = nullptr;                   // stopped: no cache write
    float eps = 1e-6f;
    float *part = nullptr;                       // [KV][nsplit][NO + 2 GPH] split partials
    int *cnt = nullptr;                          // [KV] tickets (0 between launches)
    int nsplit = 0;
    unsigned long long *g_qkv = nullptr, *g_att = nullptr, *g_x = nullptr, *g_h = nullptr;
    int *epoch = nullptr;                        // talker passes so far (tags); bumped by the last layer
    int *err = nullptr;                          // != 0: a hand-off timed out (code)
    int layer = 0, last_layer = 0;
    unsigned long long *dbg = nullptr;           // (QTTS_STAMPS builds) [256][16] phase stamps
};
constexpr int QTTS_TE_GRANULES = 4096 + 2048 + 2048 + 6144;   // q|k|v, attention, x', h
bool qtts_tlayer_dims_ok(int H, int NH, int KV, int HD, int I);
size_t qtts_tlayer_lds();
int qtts_tlayer(const TLayerArgs &a, hipStream_t st, int mode);

struct AttnArgs {
    int mode = 0;                  // 0 decode (fused q/k norm + rope + cache write), 1 cached
    const float *qkv = nullptr;    // row r: [q NH*HD | k KV*HD | v KV*HD]
    int ld_qkv = 0;
    const float *qn_w = nullptr, *kn_w = nullptr;
    float eps = 1e-6f;
    const float *rope_cos = nullptr, *rope_sin = nullptr;  // [pos][HD]
    float *kc = nullptr, *vc = nullptr;                    // layer slice [B][S][KV*HD]
    int S = 0;
    const int *pos = nullptr;      // decode: pos[b]; cached: pos[row]
    int pos_const = 0;             // used when pos == nullptr
    const int *row_b = nullptr;    // cached: batch index of each row
    int NH = 0, KV = 0, HD = 0;
    float *out = nullptr;          // [rows][NH*HD]
    int ld_out = 0;
    int nrows = 0;
    const int *skip = nullptr;     // decode: per-b stop flags (skip the cache write)
    int win = 0;                   // >0: sliding window (keys t > pos - win), c/qwen_tts_codec.c:363-367
    // decode: the q|k|v row of row r read from a table by id instead of qkv
    // (the sub-talker's layer-0 projections of every input id, precomputed):
    // id = tab_ids[r*tab_bstride + tab_row_sel[r]*tab_rstride + tab_off]
    const float *qkv_tab = nullptr;
    const int *tab_ids = nullptr, *tab_row_sel = nullptr;
    int tab_bstride = 0, tab_rstride = 0, tab_off = 0;
    // decode split-K scratch: [rows][KV][nsplit][GPH*HD + 2*GPH] partials, [rows][KV] tickets (zeroed)
    float *part = nullptr;
    int *cnt = nullptr;
    int nsplit = 0;
    // decode: every split (one or more) leaves its (acc, max, sum) in `part`
    // and the merge is the consumer's (GemvArgs::amerge, the O projection's
    // prologue) instead of the last split's
    int defer = 0;
    L2Prefetch pf;                 // k_attn_o: the next launch's weights
#ifdef QTTS_STAMPS
    unsigned long long *dbg = nullptr;   // (stamp builds) k_attn_o: [workgroup][8] start / end, 100 MHz clock
#endif
    // k_attn_short with a q|k|v table (the batch sub-talker's layer 0): kv
    // head 0's workgroup of row r also copies the input row of id(r) (the
    // table ids above) from xc_tab (fp32) or xc_tab16 (bf16) to xc_dst + r
    // xc_n -- the residual the skipped q|k|v GEMV would have copied
    const float *xc_tab = nullptr;
    const bf16_t *xc_tab16 = nullptr;
    float *xc_dst = nullptr;
    int xc_n = 0;
    // lanes per key of the split kernel at HD 128 (4 / 8 / 16), latched by the
    // model at creation (QTTS_HIP_ATTN_LPK); 0 = the default for HD / defer
    int lpk = 0;
};
// keys per split of the talker decode attention (deferred merge or not; lpk
// as AttnArgs::lpk)
int qtts_attn_keys_per_split(int HD, bool defer, int lpk);
// true when the decode attention takes these arguments on its split kernel,
// whose merge AttnArgs::defer hands to the consumer
bool qtts_attn_defer_ok(const AttnArgs &a);
// sub-talker attention + O projection split by kv head: part [KV][nrows][R]
// (GQA 2, <= 16 keys); 1 = not covered
int qtts_attn_o(const AttnArgs &a, const bf16_t *Wo, int R, float *part, hipStream_t st);
// true when qtts_attn_o takes these arguments (it returns 1 otherwise)
bool qtts_attn_o_covers(const AttnArgs &a, const bf16_t *Wo);

// Name of the kernel instantiation the last launcher on this thread chose
// (diagnostics: per-kernel profile rows match rocprofv3's kernel names).
extern thread_local const char *qtts_last_kernel;
int qtts_attention(const AttnArgs &a, hipStream_t st);
// prefill helper: q/k RMSNorm + RoPE in place on qkv rows, k/v -> cache at (row_b, pos)
int qtts_qk_prep(const AttnArgs &a, hipStream_t st);

struct SampArgs {
    const float *logits = nullptr;
    int ld = 0, n = 0, nb = 1;
    int top_k = 50;
    float top_p = 1.0f, temp = 0.9f;
    uint32_t *rng = nullptr;       // [B] float-bit xorshift state
    int mode = 0;                  // 0 sub-talker, 1 talker
    // talker mode
    int suppress_lo = 0, eos = -1;
    float rep = 1.0f;
    int *counts = nullptr;         // [B][n] occurrences of each generated id
    int fixed = 0;
    int *n_gen = nullptr, *stopped = nullptr, *cur_row = nullptr, *stop_step = nullptr;
    int *host_stopped = nullptr;   // pinned host mirror of `stopped` (set when a slot stops)
    uint32_t *st_rng = nullptr;    // sub-talker state reset per frame
    uint32_t seed_bits = 0;
    // outputs: codes[b*codes_bstride + cur_row[b]*G + g]
    int *codes = nullptr;
    int codes_bstride = 0, G = 16, g = 0;
    int *out_tok = nullptr;        // optional plain output [b]
};
int qtts_sample(const SampArgs &a, hipStream_t st);

struct EmbedSumArgs {
    const int *codes = nullptr;
    int codes_bstride = 0, G = 16;
    const int *cur_row = nullptr, *stopped = nullptr;
    const bf16_t *codec_emb = nullptr;   // [V][H]
    const bf16_t *st_emb = nullptr;      // [G-1][Vs][H]
    int Vs = 0, H = 0, nb = 1;
    const float *trailing = nullptr;     // [B][tr_cap][H]
    int tr_cap = 0;
    const int *n_trailing = nullptr;
    const float *pad = nullptr;          // [H]
    float *out = nullptr;                // [B][H]
    int *kv_len = nullptr;
    int advance = 0;
};
int qtts_embed_sum(const EmbedSumArgs &a, hipStream_t st);

// prompt assembly: prefill rows [B][p_cap][H] and trailing rows [B][tr_cap][H]
struct PromptArgs {
    const float *proj = nullptr;   // projected text rows [nrows][H]
    const int *plan = nullptr;     // per output row: {proj_row, codec_id, dest_kind(0 prefill/1 trailing), b, slot}
                                   // codec_id >= 0 codec_emb row, -1 none, -2 spk vector,
                                   // <= -3 reference frame (-3 - id): sum of its G group embeddings
    int nplan = 0, H = 0;
    const bf16_t *codec_emb = nullptr;
    const bf16_t *st_emb = nullptr;   // [G-1][Vs][H] sub-talker input embeddings (reference frames)
    const float *spk = nullptr;       // [H] speaker x-vector (voice clone)
    const int *ref_codes = nullptr;   // [n_ref][G] reference codes (voice clone ICL)
    int n_ref = 0, G = 0, V = 0, Vs = 0;
    float *prefill = nullptr;
    int p_cap = 0;
    float *trailing = nullptr;
    int tr_cap = 0;
};
int qtts_prompt_assemble(const PromptArgs &a, hipStream_t st);

int qtts_copy_rows(float *dst, int ldd, const float *src, int lds, const int *src_rows, int nrows, int ncols,
                   hipStream_t st);

// work-queue refill of one slot inside a live batch: the
// slot's talker input row <- its last prompt row, kv_len <- pos, and a fresh
// utterance's counters (Q.c:1250-1270: n_gen, rows, stop, repetition counts,
// both RNG states at the seed)
struct SlotResetArgs {
    int b = 0, pos = 0, H = 0, V = 0;
    const float *row = nullptr;          // [H] the prompt row the slot's next talker step consumes
    float *x = nullptr;                  // [B][H] talker input
    int *kv_len = nullptr, *n_gen = nullptr, *cur_row = nullptr, *stopped = nullptr, *stop_step = nullptr;
    int *last_tok = nullptr, *counts = nullptr;   // counts [B][V]
    uint32_t *rng = nullptr, *st_rng = nullptr;
    uint32_t seed_bits = 0;
};
int qtts_slot_reset(const SlotResetArgs &a, hipStream_t st);
