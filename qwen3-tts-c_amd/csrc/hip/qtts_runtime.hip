// qtts_runtime.hip - device model, weight layout in HBM, generation state,
// frame HIP graphs and the C-ABI of include/qtts_hip.h.
//
// HBM layout (per device, one model, B slots):
//   talker layer l:  wqkv [(NH+2KV)*HD, H] bf16   fused q|k|v rows
//                    wo   [H, NH*HD]            bf16
//                    wgu  [2I, H]               bf16   gate/up interleaved in row quads
//                                                      (g0..g3 u0..u3 g4..g7 u4..u7 ...)
//                    wdown[H, I]                bf16
//                    q/k norm [HD], in/post norm [H] f32
//   sub-talker: same per layer; codec embeddings [G-1][Vs][H] and lm heads
//               [G-1][Vs][Hs] contiguous so a pass selects its table by offset
//   KV caches fp32 (as the reference, T.c:191-196): talker [L][B][S][KV*HD],
//               sub-talker [Ls][B][G][KVs*HDs]
//   codec: f32 tensors by name (k_codec.hip)
//
// One frame (group-0 sample + 15 sub-talker groups + next embedding) is ONE
// captured HIP graph; position / row / stop state lives in device memory so
// the same graph replays every frame with no host round trip.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <atomic>
#include <vector>

#include "qtts_common.h"
#include "qtts_kernels.h"
#include "qtts_codec.h"
#include "qtts_enc.h"
#include "../../../include/qtts_hip.h"

#define CK(x)                                                                                              \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) {                                                                            \
            fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorName(e_), __FILE__, __LINE__, #x);   \
            return -1;                                                                                     \
        }                                                                                                  \
    } while (0)
#define CKI(x)                                                                                             \
    do {                                                                                                   \
        if ((x) != 0) return -1;                                                                           \
    } while (0)

namespace {

struct Layer {
    bf16_t *wqkv = nullptr, *wo = nullptr, *wgu = nullptr, *wdown = nullptr;
    float *qn = nullptr, *kn = nullptr, *in = nullptr, *post = nullptr;
};

float host_bf16(uint16_t v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
uint16_t host_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + (((u >> 16) & 1) + 0x7FFF)) >> 16);
}
float host_f16(uint16_t h) {
    _Float16 x;
    memcpy(&x, &h, 2);
    return (float)x;
}

}  // namespace

static constexpr int QTTS_MAX_SLOTS = 64;   // row counts with their own tail graph (qtts_dev_set_rows)

struct qtts_dev {
    qtts_dims_t d{};
    int device = 0;
    hipStream_t st = nullptr;
    size_t wbytes = 0, sbytes = 0;
    std::vector<void *> wallocs, sallocs;
    // QTTS_HIP_ARENA=1: small buffers (<= QTTS_ARENA_SMALL) carved from
    // 32 MB blocks (dalloc): one 2 MB-fragment mapping for every activation
    // vector, norm weight and bias instead of one allocation each
    unsigned char *war = nullptr, *sar = nullptr;
    size_t war_off = 0, war_cap = 0, sar_off = 0, sar_cap = 0;
    // talker
    std::vector<Layer> tl, sl;
    bf16_t *codec_emb = nullptr, *text_emb = nullptr, *fc1w = nullptr, *fc2w = nullptr, *head = nullptr;
    float *fc1b = nullptr, *fc2b = nullptr, *tk_norm = nullptr;
    // sub-talker
    bf16_t *st_emb = nullptr, *lm = nullptr, *st_proj = nullptr;
    float *st_projb = nullptr, *st_norm = nullptr;
    // small_to_mtp_projection applied once at load to every embedding row a
    // sub-talker pass g >= 1 can consume (fp32): [V][Hs] of the talker codec
    // embedding (pass 1) and [G-1][Vs][Hs] of the sub-talker ones (passes 2..)
    float *codec_ptab = nullptr, *st_ptab = nullptr;
    // the sub-talker's layer-0 q|k|v of every row a pass g >= 1 can consume
    // (its input is a table row chosen by the previous code alone): fp32
    // [V + (G-2) Vs][QKVs], pass 1 rows first, then pass g at V + (g-2) Vs;
    // computed once at load by the per-frame GEMV itself (bit-identical)
    float *qkv0_tab = nullptr;
    // codec
    CodecModel codec;
    // voice-clone encoders (speaker x-vector, 12 Hz reference codes)
    EncModel enc;
    // rope
    float *rope_cos = nullptr, *rope_sin = nullptr, *rope_cos_s = nullptr, *rope_sin_s = nullptr;
    int rope_max = 0;
    std::set<std::string> got;
    // state
    int nb = 0, nrun = 0, max_frames = 0, S = 0, p_cap = 0, tr_cap = 0, rows_cap = 0;  // nb: allocated slots (strides), nrun: rows launched
    float *x_tk = nullptr, *qkv = nullptr, *att = nullptr, *hbuf = nullptr, *logits = nullptr, *tk_hid = nullptr;
    float *x_st2 = nullptr, *opart = nullptr;   // attn_o: second residual buffer, per-head O partials
    // batch split-K (nb >= 2): second talker residual, O / down partials; the
    // talker's final residual = tk_xfin + sum of tk_npend partials at tk_pend
    float *x_tk2 = nullptr, *bpo = nullptr, *bpd = nullptr;
    float *ppart = nullptr;      // prefill split-K partials (<= 16 rows, kz <= 4)
    float *tk_xfin = nullptr;
    const float *tk_pend = nullptr;
    int tk_npend = 0;
    bool bsplit = true;      // QTTS_HIP_BSPLIT=0: batch O / down projections without split-K
    int bself_min = 9;       // batch split-K producers reduce their own partials from this many rows up
    int bkz_max = 0;         // QTTS_HIP_BKZ_MAX: cap on the batch split-K columns (0: 2 up to 8 rows, else 4)
    int bkz_wide = 1;        // QTTS_HIP_BKZ_WIDE=0: above 8 rows, no extra split-K columns for > 2048-wide slices (bsplit_kz); 2: from 2 rows, up to 4 columns
    float *x_st = nullptr, *qkv_s = nullptr, *att_s = nullptr, *h_s = nullptr, *logits_s = nullptr;
    float *kc = nullptr, *vc = nullptr, *kcs = nullptr, *vcs = nullptr;
    int *codes = nullptr, *counts = nullptr, *n_gen = nullptr, *stopped = nullptr, *cur_row = nullptr;
    // [B] the id each slot's last draw produced (every sampler's out_tok): the
    // next sub-talker pass reads its input row by it -- one dependent load
    // where codes[b][cur_row[b]][g-1] took two (cur_row, then the code)
    int *last_tok = nullptr;
    int *stop_step = nullptr, *kv_len = nullptr, *n_trailing = nullptr;
    float *att_part = nullptr;   // split-K decode attention partials (talker)
    int *att_cnt = nullptr, att_nsplit = 0;
    int *btick = nullptr;        // self-reducing batch split-K tickets [QTTS_GM_TICKS] (zeroed)
    uint32_t *rng = nullptr, *st_rng = nullptr;
    float *trailing = nullptr, *prefill = nullptr, *pad_emb = nullptr;
    // prefill / prompt scratch
    float *px = nullptr, *pqkv = nullptr, *patt = nullptr, *ph = nullptr, *pt1 = nullptr, *pproj = nullptr;
    int *prow_b = nullptr, *ppos = nullptr, *psrc = nullptr, *pids = nullptr, *pplan = nullptr, *plast = nullptr;
    int ids_cap = 0;
    // voice-clone prompt inputs of the next qtts_dev_prompt (qtts_dev_prompt_ref)
    int *pref = nullptr;
    float *pspk = nullptr;
    int pref_cap = 0, n_pref = 0, has_spk = 0;
    std::vector<int> p_len_h, n_tr_h;
    qtts_gen_params_t par{};
    bool have_par = false;
    hipGraphExec_t g0 = nullptr, gN = nullptr;
    // work queue, tail of a run: the talker-first frame graph over the first
    // nrun < nb slots (qtts_dev_set_rows), captured on first use
    hipGraphExec_t gNr[QTTS_MAX_SLOTS + 1] = {};
    int graph_key = -1;
    // EOS-mode lagged poll: the sampler mirrors each slot's stop into pinned
    // host memory; an event after every frame lets the host wait for frame
    // s - 1 while frame s is already queued (qtts_dev_frame_done)
    int *hstop = nullptr;
    int hstop_cap = 0;
    hipEvent_t fev[2] = {nullptr, nullptr};
    // codec overlapped with the decode (qtts_dev_codec_async_*): its own stream,
    // ordered after the frames it decodes by an event; output stays on device
    hipStream_t cst = nullptr;
    hipEvent_t cev = nullptr;
    float *cwav = nullptr;
    size_t cwav_cap = 0;
    // host codes staged for qtts_dev_codec_stream_push_host / _prime (grown on demand)
    int *push_codes = nullptr;
    size_t push_cap = 0;
    bool prime_pending = false;   // a qtts_dev_codec_stream_prime push runs on cst (cev marks its end)
    float *pwav = nullptr;        // the prime's discarded audio (never the codec_async output cwav)
    size_t pwav_cap = 0;
    // a batch's codec passes side by side (qtts_dev_codec_multi): lanes 1.. with
    // their own scratch and stream (lane 0 is `codec`), the waveforms and the
    // host-given codes staged on the device
    std::vector<CodecModel *> clanes;
    std::vector<hipStream_t> clane_st;
    float *mwav = nullptr;
    size_t mwav_cap = 0;
    int *mcodes = nullptr;
    size_t mcodes_cap = 0;
    // per-kernel profiling of one eager frame (qtts_dev_profile_frame)
    struct Prof { int kind; double bytes; hipEvent_t a, b; const char *name; };
    std::vector<Prof> prof;
    bool profiling = false;
    bool attn_o = true;      // QTTS_HIP_ATTN_O=0: sub-talker attention and O projection as two kernels
    bool tab0b = true;       // QTTS_HIP_TAB0B=0: batch layer-0 q|k|v by GEMV instead of the table
    // QTTS_HIP_L2PF=<mask>: which edges of the batch-1 sub-talker chain carry
    // the next-launch weight prefetch (0 none): 1 q|k|v -> attention + O,
    // 2 attention + O -> gate|up, 4 gate|up -> down, 8 down -> next q|k|v or
    // head, 16 head -> the next pass's first launch (two launches ahead);
    // (the same for the batch chain on k_gemvb measured 2 % slower at batch 8
    // and 16, profiles/r04g_ab_l2pf_batch.txt, and was removed)
    int l2pf = 31;
    int l2pf_tk = 0;         // QTTS_HIP_L2PF_TK bits (batch-1 talker, non-temporal): 1 q|k|v -> O's W_o, 2 O -> gate|up
    unsigned *pf_sink = nullptr;
    bool attn_defer = true;  // QTTS_HIP_ATTN_DEFER=0: batch-1 talker attention merges its own splits
    int attn_lpk = 0;        // QTTS_HIP_ATTN_LPK=4|8|16 (HD 128 split size), latched here: sizes att_part
    // QTTS_HIP_GM_DBG=<layer>: phase stamps of that talker layer's batch GEMVs
    // (q|k|v, O, gate|up, down), printed by qtts_dev_get_codes
    int gm_dbg_layer = -1;
    unsigned long long *gm_dbg = nullptr;
    // QTTS_HIP_TENGINE=1: the batch-1 1.7B talker layer as one persistent
    // launch (k_tengine.hip); its {tag, value} granules, [epoch, error]
    int tengine = 0;          // 1 register form, 2 / 3 ring engine (slots in flight 1 / 2)
    unsigned long long *te_g = nullptr;
    int *te_ctl = nullptr;
    float *pinv = nullptr;   // per-row 1/rms scratch of the matrix-core projections
    int pinv_cap = 0;
    float *mpart = nullptr;   // split-K partials of the matrix-core projections (k_mgemm_reduce)
    size_t mpart_elems = 0;
    // the prefill GEMM's activation planes [3][rows][K] bf16 (k_pgemm.hip)
    unsigned short *pplanes = nullptr;
    size_t pplanes_elems = 0;
    bool pgemm = true;       // QTTS_HIP_PGEMM=0: the prefill on k_mgemm (rounds 1-5)

    int QKV() const { return (d.NH + 2 * d.KV) * d.HD; }
    int QKVs() const { return (d.NHs + 2 * d.KVs) * d.HDs; }
};

// ----------------------------------------------------------------- helpers
static constexpr size_t QTTS_ARENA_SMALL = (size_t)1 << 20, QTTS_ARENA_BLOCK = (size_t)32 << 20;
static void *dalloc(qtts_dev *dv, size_t n, bool weight) {
    void *p = nullptr;
    if (n == 0) n = 16;
    // (off by default: +1.2 % in one same-box A/B, -1.3 % in the next,
    // profiles/r04g_ab_arena.txt; read per call: tests switch it per model)
    const char *ae = getenv("QTTS_HIP_ARENA");
    const int arena = ae ? atoi(ae) : 0;
    if (arena && n <= QTTS_ARENA_SMALL) {
        unsigned char *&base = weight ? dv->war : dv->sar;
        size_t &off = weight ? dv->war_off : dv->sar_off, &cap = weight ? dv->war_cap : dv->sar_cap;
        const size_t need = (n + 255) & ~(size_t)255;
        if (!base || off + need > cap) {
            void *blk = dalloc(dv, QTTS_ARENA_BLOCK, weight);   // (recorded in wallocs / sallocs)
            if (!blk) return nullptr;
            base = (unsigned char *)blk; off = 0; cap = QTTS_ARENA_BLOCK;
        }
        p = base + off;
        off += need;
        return p;
    }
    const hipError_t prior = hipPeekAtLastError();
    const hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
        fprintf(stderr, "qtts: hipMalloc(%zu) failed: %s (last error before it: %s)\n", n, hipGetErrorName(e),
                hipGetErrorName(prior));
        return nullptr;
    }
    if (weight) { dv->wallocs.push_back(p); dv->wbytes += n; }
    else { dv->sallocs.push_back(p); dv->sbytes += n; }
    return p;
}

static void drop_row_graphs(qtts_dev *dv) {
    for (auto &g : dv->gNr)
        if (g) { hipGraphExecDestroy(g); g = nullptr; }
}

static void free_state(qtts_dev *dv) {
    if (dv->g0) { hipGraphExecDestroy(dv->g0); dv->g0 = nullptr; }
    if (dv->gN) { hipGraphExecDestroy(dv->gN); dv->gN = nullptr; }
    drop_row_graphs(dv);
    for (void *p : dv->sallocs) hipFree(p);
    dv->sallocs.clear();
    dv->sbytes = 0;
    dv->sar = nullptr; dv->sar_off = dv->sar_cap = 0;
    dv->nb = 0;
    dv->nrun = 0;
    dv->ids_cap = 0;  // prompt scratch lived in sallocs
    dv->pids = dv->pplan = nullptr;
    dv->pt1 = dv->pproj = nullptr;
    dv->graph_key = -1;
    codec_free_state(&dv->codec);
}

static std::vector<float> to_f32(const void *host, int dtype, size_t n) {
    std::vector<float> o(n);
    if (dtype == 0) memcpy(o.data(), host, n * 4);
    else if (dtype == 1) for (size_t i = 0; i < n; ++i) o[i] = host_bf16(((const uint16_t *)host)[i]);
    else for (size_t i = 0; i < n; ++i) o[i] = host_f16(((const uint16_t *)host)[i]);
    return o;
}

static float *upload_f32(qtts_dev *dv, const void *host, int dtype, size_t n) {
    std::vector<float> f = to_f32(host, dtype, n);
    float *p = (float *)dalloc(dv, n * 4, true);
    if (!p || hipMemcpy(p, f.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

static int upload_bf16_at(bf16_t *dst, const void *host, int dtype, size_t n) {
    if (dtype == 1) return hipMemcpy(dst, host, n * 2, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
    std::vector<uint16_t> t(n);
    std::vector<float> f = to_f32(host, dtype, n);
    for (size_t i = 0; i < n; ++i) t[i] = host_to_bf16(f[i]);
    return hipMemcpy(dst, t.data(), n * 2, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

static bf16_t *upload_bf16(qtts_dev *dv, const void *host, int dtype, size_t n) {
    bf16_t *p = (bf16_t *)dalloc(dv, n * 2, true);
    if (!p || upload_bf16_at(p, host, dtype, n)) return nullptr;
    return p;
}

// ----------------------------------------------------------------- weights
static int put_layer(qtts_dev *dv, Layer &ly, const std::string &suf, const void *host, int dtype, size_t n,
                     int H, int NH, int KV, int HD, int I) {
    const size_t qd = (size_t)NH * HD, kd = (size_t)KV * HD;
    const size_t qkv_rows = qd + 2 * kd;
    if (suf == "self_attn.q_proj.weight" || suf == "self_attn.k_proj.weight" || suf == "self_attn.v_proj.weight") {
        if (!ly.wqkv) ly.wqkv = (bf16_t *)dalloc(dv, qkv_rows * H * 2, true);
        if (!ly.wqkv) return -1;
        size_t off = suf[10] == 'q' ? 0 : suf[10] == 'k' ? qd : qd + kd;
        size_t rows = suf[10] == 'q' ? qd : kd;
        if (n != rows * H) { fprintf(stderr, "qtts: %s has %zu elements, expected %zu\n", suf.c_str(), n, rows * H); return -1; }
        return upload_bf16_at(ly.wqkv + off * H, host, dtype, n);
    }
    if (suf == "self_attn.o_proj.weight") {
        if (n != (size_t)H * qd) return -1;
        ly.wo = upload_bf16(dv, host, dtype, n);
        return ly.wo ? 0 : -1;
    }
    if (suf == "mlp.gate_proj.weight" || suf == "mlp.up_proj.weight") {
        if (n != (size_t)I * H || I % 4) return -1;
        if (!ly.wgu) ly.wgu = (bf16_t *)dalloc(dv, (size_t)2 * I * H * 2, true);
        if (!ly.wgu) return -1;
        const bool up = suf[4] == 'u';
        std::vector<uint16_t> tmp;
        const void *src = host;
        if (dtype != 1) {
            tmp.resize(n);
            std::vector<float> f = to_f32(host, dtype, n);
            for (size_t i = 0; i < n; ++i) tmp[i] = host_to_bf16(f[i]);
            src = tmp.data();
        }
        // quad q of gate -> rows 8q..8q+3, of up -> rows 8q+4..8q+7
        const size_t quad = (size_t)4 * H * 2;
        return hipMemcpy2D((char *)ly.wgu + (up ? quad : 0), 2 * quad, src, quad, quad, I / 4,
                           hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
    }
    if (suf == "mlp.down_proj.weight") {
        if (n != (size_t)H * I) return -1;
        ly.wdown = upload_bf16(dv, host, dtype, n);
        return ly.wdown ? 0 : -1;
    }
    float **f = suf == "self_attn.q_norm.weight" ? &ly.qn : suf == "self_attn.k_norm.weight" ? &ly.kn
              : suf == "input_layernorm.weight" ? &ly.in : suf == "post_attention_layernorm.weight" ? &ly.post : nullptr;
    if (f) {
        *f = upload_f32(dv, host, dtype, n);
        return *f ? 0 : -1;
    }
    return 0;  // unused tensor
}

static int parse_idx(const std::string &name, const std::string &pre, std::string *rest) {
    if (name.compare(0, pre.size(), pre) != 0) return -1;
    size_t p = pre.size(), q = p;
    while (q < name.size() && isdigit((unsigned char)name[q])) ++q;
    if (q == p || q >= name.size() || name[q] != '.') return -1;
    *rest = name.substr(q + 1);
    return atoi(name.c_str() + p);
}

extern "C" int qtts_dev_put_tensor(qtts_dev_t *dv, const char *cname, const void *host, int dtype,
                                   const int64_t *shape, int ndim) {
    if (!dv || !cname || !host) return -1;
    hipSetDevice(dv->device);
    std::string name(cname), rest;
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) n *= (size_t)shape[i];
    const qtts_dims_t &d = dv->d;
    int rc = 0, idx;
    const int er = enc_put_tensor(&dv->enc, name, host, dtype, shape, ndim, n);
    if (er < 0) { fprintf(stderr, "qtts: failed to take encoder tensor %s\n", cname); return -1; }
    if (er > 0) return 0;
    if (name.compare(0, 8, "decoder.") == 0) {
        rc = codec_put_tensor(&dv->codec, name, host, dtype, shape, ndim, n);
    } else if (name == "talker.model.codec_embedding.weight") {
        dv->codec_emb = upload_bf16(dv, host, dtype, n); rc = dv->codec_emb ? 0 : -1;
    } else if (name == "talker.model.text_embedding.weight") {
        dv->text_emb = upload_bf16(dv, host, dtype, n); rc = dv->text_emb ? 0 : -1;
    } else if (name == "talker.text_projection.linear_fc1.weight") {
        dv->fc1w = upload_bf16(dv, host, dtype, n); rc = dv->fc1w ? 0 : -1;
    } else if (name == "talker.text_projection.linear_fc1.bias") {
        dv->fc1b = upload_f32(dv, host, dtype, n); rc = dv->fc1b ? 0 : -1;
    } else if (name == "talker.text_projection.linear_fc2.weight") {
        dv->fc2w = upload_bf16(dv, host, dtype, n); rc = dv->fc2w ? 0 : -1;
    } else if (name == "talker.text_projection.linear_fc2.bias") {
        dv->fc2b = upload_f32(dv, host, dtype, n); rc = dv->fc2b ? 0 : -1;
    } else if (name == "talker.model.norm.weight") {
        dv->tk_norm = upload_f32(dv, host, dtype, n); rc = dv->tk_norm ? 0 : -1;
    } else if (name == "talker.codec_head.weight") {
        dv->head = upload_bf16(dv, host, dtype, n); rc = dv->head ? 0 : -1;
    } else if (name == "talker.code_predictor.small_to_mtp_projection.weight") {
        dv->st_proj = upload_bf16(dv, host, dtype, n); rc = dv->st_proj ? 0 : -1;
    } else if (name == "talker.code_predictor.small_to_mtp_projection.bias") {
        dv->st_projb = upload_f32(dv, host, dtype, n); rc = dv->st_projb ? 0 : -1;
    } else if (name == "talker.code_predictor.model.norm.weight") {
        dv->st_norm = upload_f32(dv, host, dtype, n); rc = dv->st_norm ? 0 : -1;
    } else if ((idx = parse_idx(name, "talker.code_predictor.model.codec_embedding.", &rest)) >= 0 && rest == "weight") {
        if (idx >= d.G - 1 || n != (size_t)d.Vs * d.H) { fprintf(stderr, "qtts: bad %s\n", cname); return -1; }
        if (!dv->st_emb) dv->st_emb = (bf16_t *)dalloc(dv, (size_t)(d.G - 1) * d.Vs * d.H * 2, true);
        rc = dv->st_emb ? upload_bf16_at(dv->st_emb + (size_t)idx * d.Vs * d.H, host, dtype, n) : -1;
    } else if ((idx = parse_idx(name, "talker.code_predictor.lm_head.", &rest)) >= 0 && rest == "weight") {
        if (idx >= d.G - 1 || n != (size_t)d.Vs * d.Hs) { fprintf(stderr, "qtts: bad %s\n", cname); return -1; }
        if (!dv->lm) dv->lm = (bf16_t *)dalloc(dv, (size_t)(d.G - 1) * d.Vs * d.Hs * 2, true);
        rc = dv->lm ? upload_bf16_at(dv->lm + (size_t)idx * d.Vs * d.Hs, host, dtype, n) : -1;
    } else if ((idx = parse_idx(name, "talker.code_predictor.model.layers.", &rest)) >= 0) {
        if (idx >= d.Ls) return 0;
        rc = put_layer(dv, dv->sl[idx], rest, host, dtype, n, d.Hs, d.NHs, d.KVs, d.HDs, d.Is);
    } else if ((idx = parse_idx(name, "talker.model.layers.", &rest)) >= 0) {
        if (idx >= d.L) return 0;
        rc = put_layer(dv, dv->tl[idx], rest, host, dtype, n, d.H, d.NH, d.KV, d.HD, d.I);
    } else {
        return 0;
    }
    if (rc) {
        fprintf(stderr, "qtts: failed to upload tensor %s\n", cname);
        return -1;
    }
    dv->got.insert(name);
    return 0;
}

extern "C" qtts_dev_t *qtts_dev_create(const qtts_dims_t *dims, int device) {
    if (hipSetDevice(device) != hipSuccess) {
        fprintf(stderr, "qtts: cannot select HIP device %d\n", device);
        return nullptr;
    }
    qtts_dev *dv = new qtts_dev();
    dv->d = *dims;
    dv->device = device;
    if (hipStreamCreateWithFlags(&dv->st, hipStreamNonBlocking) != hipSuccess) {
        delete dv;
        return nullptr;
    }
    dv->tl.resize(dims->L);
    dv->sl.resize(dims->Ls);
    // debug switches: QTTS_HIP_BSPLIT=0 batch O / down
    // projections without split-K; QTTS_HIP_ATTN_O=0 sub-talker attention and
    // O projection as two kernels
    const char *bs = getenv("QTTS_HIP_BSPLIT");
    dv->bsplit = !(bs && !atoi(bs));
    const char *bk = getenv("QTTS_HIP_BKZ_MAX");
    if (bk) dv->bkz_max = atoi(bk) < 1 ? 1 : atoi(bk) > 4 ? 4 : atoi(bk);
    const char *bw = getenv("QTTS_HIP_BKZ_WIDE");
    dv->bkz_wide = bw ? atoi(bw) : 1;
    const char *bm = getenv("QTTS_HIP_BSELF_MIN");
    if (bm) dv->bself_min = atoi(bm);
    const char *ad = getenv("QTTS_HIP_ATTN_DEFER");
    dv->attn_defer = !(ad && !atoi(ad));
    const char *lk = getenv("QTTS_HIP_ATTN_LPK");
    dv->attn_lpk = lk ? atoi(lk) : 0;
    const char *ao = getenv("QTTS_HIP_ATTN_O");
    dv->attn_o = !(ao && !atoi(ao));
    const char *pg = getenv("QTTS_HIP_PGEMM");
    dv->pgemm = !(pg && !atoi(pg));
    const char *te = getenv("QTTS_HIP_TENGINE");
    if (te && atoi(te)) {
        // every workgroup of the launch must be resident at once: one per CU, 256 of them
        int dev = 0, ncu = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu >= 256)
            dv->tengine = std::min(3, std::max(1, atoi(te)));
    }
    const char *tb = getenv("QTTS_HIP_TAB0B");
    dv->tab0b = !(tb && !atoi(tb));
    const char *pf = getenv("QTTS_HIP_L2PF");
    if (pf) dv->l2pf = atoi(pf);
    const char *pft = getenv("QTTS_HIP_L2PF_TK");
    if (pft) dv->l2pf_tk = atoi(pft);
    const char *gd = getenv("QTTS_HIP_GM_DBG");
    if (gd) dv->gm_dbg_layer = atoi(gd);
    codec_init(&dv->codec, dims, dv->st);
    dv->enc.st = dv->st;
    dv->enc.device = device;
    return dv;
}

extern "C" void qtts_dev_destroy(qtts_dev_t *dv) {
    if (!dv) return;
    hipSetDevice(dv->device);
    hipStreamSynchronize(dv->st);
    free_state(dv);
    codec_destroy(&dv->codec);
    enc_destroy(&dv->enc);
    if (dv->cst) hipStreamSynchronize(dv->cst);
    if (dv->hstop) hipHostFree(dv->hstop);
    for (hipEvent_t e : dv->fev)
        if (e) hipEventDestroy(e);
    for (CodecModel *ln : dv->clanes) codec_lane_delete(ln);
    for (hipStream_t st : dv->clane_st) hipStreamDestroy(st);
    if (dv->mwav) hipFree(dv->mwav);
    if (dv->mcodes) hipFree(dv->mcodes);
    if (dv->cwav) hipFree(dv->cwav);
    if (dv->pwav) hipFree(dv->pwav);
    if (dv->push_codes) hipFree(dv->push_codes);
    if (dv->cev) hipEventDestroy(dv->cev);
    if (dv->cst) hipStreamDestroy(dv->cst);
    for (void *p : dv->wallocs) hipFree(p);
    hipStreamDestroy(dv->st);
    delete dv;
}

extern "C" size_t qtts_dev_bytes(const qtts_dev_t *dv, int which) {
    if (!dv) return 0;
    return which == 0 ? dv->wbytes + codec_weight_bytes(&dv->codec) + enc_weight_bytes(&dv->enc) : dv->sbytes;
}

// RoPE tables with the reference's exact libm arithmetic (T.c:97-113)
static int build_rope(qtts_dev *dv, int npos, int hd, float theta, float **cs, float **sn) {
    std::vector<float> c((size_t)npos * hd), s((size_t)npos * hd);
    const int half = hd / 2;
    for (int p = 0; p < npos; ++p)
        for (int i = 0; i < half; ++i) {
            float freq = 1.0f / powf(theta, (float)(2 * i) / (float)hd);
            float ang = (float)p * freq;
            c[(size_t)p * hd + i] = c[(size_t)p * hd + i + half] = cosf(ang);
            s[(size_t)p * hd + i] = s[(size_t)p * hd + i + half] = sinf(ang);
        }
    *cs = (float *)dalloc(dv, c.size() * 4, true);
    *sn = (float *)dalloc(dv, s.size() * 4, true);
    if (!*cs || !*sn) return -1;
    CK(hipMemcpy(*cs, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(*sn, s.data(), s.size() * 4, hipMemcpyHostToDevice));
    return 0;
}

static int build_proj_tables(qtts_dev *dv);
static int build_qkv0_table(qtts_dev *dv);

extern "C" int qtts_dev_finalize(qtts_dev_t *dv) {
    const qtts_dims_t &d = dv->d;
    hipSetDevice(dv->device);
    auto need = [&](const std::string &n) {
        if (!dv->got.count(n)) { fprintf(stderr, "Error: missing required tensor: %s\n", n.c_str()); return false; }
        return true;
    };
    bool ok = need("talker.model.codec_embedding.weight") && need("talker.model.text_embedding.weight") &&
              need("talker.text_projection.linear_fc1.weight") && need("talker.text_projection.linear_fc2.weight") &&
              need("talker.model.norm.weight") && need("talker.codec_head.weight") &&
              need("talker.code_predictor.model.norm.weight");
    static const char *lsuf[] = {"self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
                                 "self_attn.o_proj.weight", "self_attn.q_norm.weight", "self_attn.k_norm.weight",
                                 "input_layernorm.weight", "post_attention_layernorm.weight", "mlp.gate_proj.weight",
                                 "mlp.up_proj.weight", "mlp.down_proj.weight"};
    for (int l = 0; ok && l < d.L; ++l)
        for (const char *s : lsuf) ok = ok && need("talker.model.layers." + std::to_string(l) + "." + s);
    for (int l = 0; ok && l < d.Ls; ++l)
        for (const char *s : lsuf) ok = ok && need("talker.code_predictor.model.layers." + std::to_string(l) + "." + s);
    for (int g = 0; ok && g < d.G - 1; ++g) {
        ok = ok && need("talker.code_predictor.model.codec_embedding." + std::to_string(g) + ".weight");
        ok = ok && need("talker.code_predictor.lm_head." + std::to_string(g) + ".weight");
    }
    if (ok && d.H != d.Hs) ok = need("talker.code_predictor.small_to_mtp_projection.weight");
    if (!ok) return -1;
    if (d.HD > 128 || d.HDs > 128 || d.G > 32) {
        fprintf(stderr, "Error: unsupported head_dim (talker=%d subtalker=%d) or code groups %d\n", d.HD, d.HDs, d.G);
        return -1;
    }
    // every decode GEMV's reduction width (qtts_gemv streams 64-column blocks)
    const int widths[] = {d.H, d.I, d.NH * d.HD, d.Hs, d.Is, d.NHs * d.HDs, d.TH};
    for (int c : widths)
        if (c % 64) {
            fprintf(stderr, "Error: unsupported layer width %d (hidden / intermediate / heads x head_dim must be "
                            "multiples of 64)\n", c);
            return -1;
        }
    if (d.V > 4096 || d.Vs > 4096) {
        fprintf(stderr, "Error: vocab > 4096 unsupported by the device sampler\n");
        return -1;
    }
    const char *pt = getenv("QTTS_HIP_PTAB");
    const bool ptab_on = !(pt && !atoi(pt));
    if (dv->st_proj && ptab_on) CKI(build_proj_tables(dv));
    if (ptab_on) CKI(build_qkv0_table(dv));
    CKI(codec_finalize(&dv->codec));
    // the streaming codec's state for up to 4096 frames, allocated now so the
    // first streaming request of a process does not pay for it (its buffers
    // are reused by every later stream of <= 4096 frames; longer ones re-grow)
    if (codec_stream_begin(&dv->codec, 4096) != 0)
        fprintf(stderr, "qtts: streaming codec state not pre-allocated (allocated on first use)\n");
    return enc_finalize(&dv->enc, d.H);
}

// ----------------------------------------------------------------- voice-clone encoders
static int join_prime(qtts_dev *dv);

extern "C" int qtts_dev_enc_config(qtts_dev_t *dv, const qtts_enc_dims_t *dims) {
    if (!dv || !dims) return -1;
    return enc_set_dims(&dv->enc, dims);
}

extern "C" int qtts_dev_enc_available(qtts_dev_t *dv) {
    if (!dv) return 0;
    return (dv->enc.spk_ready ? 1 : 0) | (dv->enc.mimi_ready ? 2 : 0);
}

extern "C" int qtts_dev_speaker_embed(qtts_dev_t *dv, int nb, const float *const *wav, const int *n, float *out,
                                      float *mel_out) {
    if (!dv || !wav || !n || !out) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    return enc_speaker(&dv->enc, nb, wav, n, out, mel_out);
}

extern "C" int qtts_dev_encode_audio(qtts_dev_t *dv, int nb, const float *const *wav, const int *n, int *codes,
                                     int max_frames, int *frames, float *latent) {
    if (!dv || !wav || !n || !codes || !frames) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    return enc_codes(&dv->enc, nb, wav, n, codes, max_frames, frames, latent);
}

// ----------------------------------------------------------------- state
static int alloc_state(qtts_dev *dv, int nb, int max_frames, int max_prefill) {
    const qtts_dims_t &d = dv->d;
    free_state(dv);
    dv->nb = nb;
    dv->nrun = nb;
    dv->max_frames = max_frames;
    dv->p_cap = max_prefill;
    dv->S = max_prefill + max_frames + 1;
    dv->tr_cap = 4096;  // trailing rows per slot (text length bound)
    dv->rows_cap = nb * max_prefill;
    const size_t B = nb;
#define A(ptr, type, cnt)                                                 \
    do {                                                                  \
        dv->ptr = (type *)dalloc(dv, (size_t)(cnt) * sizeof(type), false); \
        if (!dv->ptr) return -1;                                          \
    } while (0)
    A(x_tk, float, B * d.H);
    A(qkv, float, B * dv->QKV());
    A(att, float, B * d.NH * d.HD);
    A(hbuf, float, B * d.I);
    A(logits, float, B * d.V);
    A(tk_hid, float, B * d.H);
    A(x_st, float, B * d.Hs);
    A(x_st2, float, B * d.Hs);
    A(x_tk2, float, B * d.H);
    A(bpo, float, (size_t)4 * B * (d.H > d.Hs ? d.H : d.Hs));
    A(bpd, float, (size_t)4 * B * (d.H > d.Hs ? d.H : d.Hs));
    A(ppart, float, (size_t)4 * 16 * (d.H > d.Hs ? d.H : d.Hs));
    A(opart, float, (size_t)B * ((size_t)d.KVs * d.Hs > (size_t)d.KV * d.H ? (size_t)d.KVs * d.Hs : (size_t)d.KV * d.H));
    A(qkv_s, float, B * dv->QKVs());
    A(att_s, float, B * d.NHs * d.HDs);
    A(h_s, float, B * d.Is);
    A(logits_s, float, B * d.Vs);
    A(kc, float, (size_t)d.L * B * dv->S * d.KV * d.HD);
    A(vc, float, (size_t)d.L * B * dv->S * d.KV * d.HD);
    A(kcs, float, (size_t)d.Ls * B * d.G * d.KVs * d.HDs);
    A(vcs, float, (size_t)d.Ls * B * d.G * d.KVs * d.HDs);
    A(codes, int, B * (max_frames + 1) * d.G);
    A(counts, int, B * d.V);
    A(n_gen, int, B);
    A(stopped, int, B);
    A(cur_row, int, B);
    A(last_tok, int, B);
    CK(hipMemsetAsync(dv->last_tok, 0, B * sizeof(int), dv->st));
    A(stop_step, int, B);
    A(kv_len, int, B);
    A(n_trailing, int, B);
    A(rng, uint32_t, B);
    A(st_rng, uint32_t, B);
    A(trailing, float, B * 64 * d.H);  // grown on demand in qtts_dev_prompt
    dv->tr_cap = 64;
    A(prefill, float, B * max_prefill * d.H);
    A(pad_emb, float, d.H);
    const size_t R = dv->rows_cap;
    A(px, float, R * d.H);
    A(pqkv, float, R * dv->QKV());
    A(patt, float, R * d.NH * d.HD);
    A(ph, float, R * d.I);
    A(prow_b, int, R);
    A(ppos, int, R);
    A(psrc, int, R);
    A(plast, int, B);
    dv->pinv_cap = dv->rows_cap > 64 ? dv->rows_cap : 64;
    A(pinv, float, dv->pinv_cap);
    {
        // the prefill GEMM's split-K partials, sized by the rule its split
        // follows (qtts_mgemm_part_elems: 4 M floats = 16 MB at the defaults, fewer
        // for short prompts); QTTS_HIP_MGEMM_KZ=0: no scratch, no split
        const size_t wide = std::max<size_t>({(size_t)dv->QKV(), (size_t)2 * d.I, (size_t)d.H, (size_t)d.TH});
        const char *e = getenv("QTTS_HIP_MGEMM_KZ");
        dv->mpart_elems = e && !strcmp(e, "0") ? 0 : qtts_mgemm_part_elems(std::max<size_t>(R, 64), wide);
        // (k_pgemm splits K while its 128 x 128 tiles x columns stay under 512:
        // at most 512 x 128 x 128 partials, 8 columns of every row)
        if (dv->mpart_elems)
            dv->mpart_elems = std::max(dv->mpart_elems, std::min<size_t>((size_t)512 * 128 * 128, (size_t)8 * R * wide));
        if (dv->mpart_elems) A(mpart, float, dv->mpart_elems);
        const size_t kmax = std::max<size_t>({(size_t)d.H, (size_t)d.I, (size_t)d.NH * d.HD});
        dv->pplanes_elems = dv->pgemm ? qtts_pgemm_plane_elems(R, kmax) : 0;
        if (dv->pplanes_elems) A(pplanes, unsigned short, dv->pplanes_elems);
    }
    {
        const int gph = d.NH / d.KV;
        // partial slots for the smaller split size of the two launch forms
        const int ch = std::min(qtts_attn_keys_per_split(d.HD, false, dv->attn_lpk),
                                qtts_attn_keys_per_split(d.HD, true, dv->attn_lpk));
        dv->att_nsplit = (dv->S + ch - 1) / ch;
        A(att_part, float, B * d.KV * dv->att_nsplit * (gph * d.HD + 2 * gph));
        const int kvmax = d.KV > d.KVs ? d.KV : d.KVs;
        A(att_cnt, int, B * kvmax);
        CK(hipMemsetAsync(dv->att_cnt, 0, B * kvmax * sizeof(int), dv->st));
        A(pf_sink, unsigned, 1);
        A(btick, int, QTTS_GM_TICKS);
        if (dv->tengine) {
            A(te_g, unsigned long long, QTTS_TE_GRANULES);
            CK(hipMemsetAsync(dv->te_g, 0, QTTS_TE_GRANULES * 8, dv->st));
            A(te_ctl, int, 2);
            CK(hipMemsetAsync(dv->te_ctl, 0, 2 * sizeof(int), dv->st));
        }
        CK(hipMemsetAsync(dv->btick, 0, QTTS_GM_TICKS * sizeof(int), dv->st));
        if (dv->gm_dbg_layer >= 0) {
            A(gm_dbg, unsigned long long, 4 * 2048 * 8);
            CK(hipMemsetAsync(dv->gm_dbg, 0, 4 * 2048 * 8 * 8, dv->st));
        }
    }
#undef A
    dv->p_len_h.assign(nb, 0);
    dv->n_tr_h.assign(nb, 0);
    CK(hipMemsetAsync(dv->codes, 0, B * (max_frames + 1) * d.G * sizeof(int), dv->st));
    CK(hipMemsetAsync(dv->kcs, 0, (size_t)d.Ls * B * d.G * d.KVs * d.HDs * 4, dv->st));
    CK(hipMemsetAsync(dv->vcs, 0, (size_t)d.Ls * B * d.G * d.KVs * d.HDs * 4, dv->st));
    // RoPE tables sized to the KV capacity
    if (dv->rope_max < dv->S) {
        dv->rope_max = dv->S;
        CKI(build_rope(dv, dv->S, d.HD, d.theta, &dv->rope_cos, &dv->rope_sin));
        if (d.HDs != d.HD) CKI(build_rope(dv, d.G + 2, d.HDs, d.theta, &dv->rope_cos_s, &dv->rope_sin_s));
        else { dv->rope_cos_s = dv->rope_cos; dv->rope_sin_s = dv->rope_sin; }
    }
    dv->graph_key = -1;
    return 0;
}

static uint32_t seed_bits(int seed) {
    float f = (float)seed;
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static int reset_counters(qtts_dev *dv) {
    const size_t B = dv->nb;
    hipStream_t st = dv->st;
    if (dv->hstop_cap < (int)B) {   // (a new pointer: the frame graphs are re-captured)
        if (dv->hstop) CK(hipHostFree(dv->hstop));
        dv->hstop = nullptr;
        CK(hipHostMalloc((void **)&dv->hstop, B * sizeof(int), hipHostMallocDefault));
        dv->hstop_cap = (int)B;
        dv->graph_key = -1;
    }
    if (!dv->fev[0]) {
        CK(hipEventCreateWithFlags(&dv->fev[0], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&dv->fev[1], hipEventDisableTiming));
    }
    CK(hipStreamSynchronize(st));   // no frame of a previous run still writes the mirror
    memset(dv->hstop, 0, B * sizeof(int));
    CK(hipMemsetAsync(dv->counts, 0, B * dv->d.V * sizeof(int), st));
    CK(hipMemsetAsync(dv->n_gen, 0, B * sizeof(int), st));
    CK(hipMemsetAsync(dv->stopped, 0, B * sizeof(int), st));
    CK(hipMemsetAsync(dv->cur_row, 0, B * sizeof(int), st));
    CK(hipMemsetAsync(dv->stop_step, 0, B * sizeof(int), st));
    std::vector<uint32_t> r(B, seed_bits(dv->par.seed));
    CK(hipMemcpyAsync(dv->rng, r.data(), B * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(dv->st_rng, r.data(), B * 4, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    return 0;
}

// ----------------------------------------------------------------- kernels of one frame
enum { PK_GEMV_TALKER = 0, PK_GEMV_SUB = 1, PK_ATTN = 2, PK_SAMPLE = 3, PK_EMBED = 4 };
struct ProfScope {  // brackets one launch with events when profiling is on
    qtts_dev *dv;
    size_t idx;
    ProfScope(qtts_dev *d, int kind, double bytes) : dv(d), idx((size_t)-1) {
        if (!dv->profiling) return;
        qtts_dev::Prof p{kind, bytes, nullptr, nullptr, ""};
        // no system-scope fence per event: a default event's cache write-back /
        // invalidate would be timed as part of every short kernel
        hipEventCreateWithFlags(&p.a, hipEventDisableSystemFence);
        hipEventCreateWithFlags(&p.b, hipEventDisableSystemFence);
        hipEventRecord(p.a, dv->st);
        dv->prof.push_back(p);
        idx = dv->prof.size() - 1;
    }
    void cancel() {
        if (idx == (size_t)-1) return;
        hipEventDestroy(dv->prof[idx].a);
        hipEventDestroy(dv->prof[idx].b);
        dv->prof.pop_back();
        idx = (size_t)-1;
    }
    ~ProfScope() {
        if (idx == (size_t)-1) return;
        hipEventRecord(dv->prof[idx].b, dv->st);
        dv->prof[idx].name = qtts_last_kernel;
    }
};
static double gemv_bytes(const GemvArgs &a) {
    return (double)a.R * a.C * 2 + (double)a.nb * a.C * 4 + (double)a.nb * a.R * 4 + (a.norm_w ? a.C * 4.0 : 0.0);
}
static int pgemv(qtts_dev *dv, const GemvArgs &a, int kind) {
    ProfScope ps(dv, kind, gemv_bytes(a));
    return qtts_gemv(a, dv->st);
}
// Multi-row projection over `rows` activation rows (prefill, text
// projection): > 64 rows in one matrix-core launch (64-row chunks on its
// grid.y), else the matrix-core kernel / batch GEMV / GEMV in chunks of 64 /
// 16.  Row r of x / y / ids is at r*ldx / r*ldy / r*ids_bstride.
static int rows_proj(qtts_dev *dv, GemvArgs a, int rows, bool prefill = false) {
    const int xs = a.ldx, ys = a.ldy;
    // the talker prefill over > 16 rows (voice-clone prompts, long prefills):
    // activations split once, LDS-tiled MFMA GEMM (k_pgemm.hip;
    // QTTS_HIP_PGEMM=0: k_mgemm as before)
    if (prefill && dv->pgemm && rows > 16 && (!a.norm_w || rows <= dv->pinv_cap)) {
        GemvArgs c = a;
        c.nb = rows;
        const int rc = qtts_pgemm(c, dv->pinv, dv->pplanes, dv->pplanes_elems, dv->st, dv->mpart, dv->mpart_elems);
        if (rc <= 0) return rc;
    }
    if (rows > 64 && (!a.norm_w || rows <= dv->pinv_cap)) {
        GemvArgs c = a;
        c.nb = rows;
        const int rc = qtts_mgemm(c, dv->pinv, dv->st, dv->mpart, dv->mpart_elems);
        if (rc <= 0) return rc;
    }
    for (int r0 = 0; r0 < rows;) {
        GemvArgs c = a;
        int nr = rows - r0 < 64 ? rows - r0 : 64;
        if (c.x) c.x = a.x + (size_t)r0 * xs;
        if (c.ids) c.ids = a.ids + (size_t)r0 * a.ids_bstride;
        c.y = a.y + (size_t)r0 * ys;
        c.nb = nr;
        int rc = 1;
        // <= 16 rows (a custom-voice prompt): the batch decode kernels (k_gemvb,
        // x sliced per wave, else k_gemvm, x split once per workgroup; ~1
        // round over the CUs) stream the weights faster than the 64-row
        // prefill GEMM.  (QTTS_HIP_PREFILL_GEMVB=0: k_gemvm only, the round-4
        // path: 72 us of prefill per talker layer at the P128 prompt's rows,
        // profiles/r05af_first_packet.txt)
        static const bool pgb = [] { const char *e = getenv("QTTS_HIP_PREFILL_GEMVB"); return !(e && !atoi(e)); }();
        // the residual projections (O, down: R / 16 row tiles, too few for
        // the chip) split over K in two columns that reduce their own
        // partials, as the talker's decode does (QTTS_HIP_PREFILL_SPLIT=kz,
        // 2 or 4; 0: none)
        static const int psk = [] { const char *e = getenv("QTTS_HIP_PREFILL_SPLIT");
                                    int v = e ? atoi(e) : 2; return v == 4 ? 4 : v ? 2 : 0; }();
        if (nr >= 2 && nr <= 16 && pgb && psk && c.epi == EPI_RESID && !c.norm_w && c.R / 16 < 256 &&
            c.C % (32 * psk) == 0 && c.R <= (dv->d.H > dv->d.Hs ? dv->d.H : dv->d.Hs)) {
            GemvArgs k = c;
            k.ypart = dv->ppart; k.kz = psk; k.ld_ypart = (size_t)nr * k.R; k.tick = dv->btick;
            rc = qtts_gemvb(k, dv->st);
        }
        if (rc == 1 && nr >= 2 && nr <= 16 && pgb) rc = qtts_gemvb(c, dv->st);
        if (rc == 1 && nr >= 2 && nr <= 16) rc = qtts_gemvm(c, dv->st);
        if (rc == 1 && nr >= 2) rc = qtts_mgemm(c, dv->pinv, dv->st, dv->mpart, dv->mpart_elems);
        if (rc < 0) return -1;
        if (rc == 1) {
            nr = nr < 16 ? nr : 16;
            c.nb = nr;
            CKI(qtts_gemv(c, dv->st));
        }
        r0 += nr;
    }
    return 0;
}

// ST_PROJECT_INPUT (T.c:693-702) of every embedding row a pass g >= 1 can
// read, once at load: the per-frame input projection GEMV of those passes
// becomes a row gather (the row a pass needs is fixed by the code id alone).
static int build_proj_tables(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    const int nid = d.V > d.Vs ? d.V : d.Vs;
    std::vector<int> io(nid);
    for (int i = 0; i < nid; ++i) io[i] = i;
    int *ids = (int *)dalloc(dv, (size_t)nid * 4, false);
    dv->codec_ptab = (float *)dalloc(dv, (size_t)d.V * d.Hs * 4, true);
    dv->st_ptab = (float *)dalloc(dv, (size_t)(d.G - 1) * d.Vs * d.Hs * 4, true);
    if (!ids || !dv->codec_ptab || !dv->st_ptab) return -1;
    CK(hipMemcpy(ids, io.data(), (size_t)nid * 4, hipMemcpyHostToDevice));
    GemvArgs a;
    a.W = dv->st_proj; a.R = d.Hs; a.C = d.H; a.y = dv->codec_ptab; a.ldy = d.Hs;
    a.epi = dv->st_projb ? EPI_BIAS : EPI_STORE;
    a.bias = dv->st_projb;
    a.nt = 0;
    a.table = dv->codec_emb; a.ids = ids; a.ids_bstride = 1;
    CKI(rows_proj(dv, a, d.V));
    for (int g = 0; g < d.G - 1; ++g) {
        a.table = dv->st_emb + (size_t)g * d.Vs * d.H;
        a.y = dv->st_ptab + (size_t)g * d.Vs * d.Hs;
        CKI(rows_proj(dv, a, d.Vs));
    }
    CK(hipStreamSynchronize(dv->st));
    return 0;
}

// QKV projection, then the decode attention
static int qkv_attn(qtts_dev *dv, const GemvArgs &a, const AttnArgs &t, int kind) {
    CKI(pgemv(dv, a, kind));
    ProfScope ps(dv, PK_ATTN, 0);
    return qtts_attention(t, dv->st);
}
static GemvArgs gv(const bf16_t *W, int R, int C, const float *x, int ldx, float *y, int ldy, int nb, int epi) {
    GemvArgs a;
    a.W = W; a.R = R; a.C = C; a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.nb = nb; a.epi = epi;
    return a;
}

// The layer-0 q|k|v table (qtts_dev::qkv0_tab): row r of group g's block is
// exactly what the per-frame GEMV computes for input id r (same lean kernel,
// same arguments but the output row), so reading it is bit-identical.  One
// launch per group, the ids on grid.y (GemvArgs::reps); a per-row launch for
// each of ~32k ids took ~0.2 s and crashed rocprofv3's counter collection.
static int build_qkv0_table(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    if (d.G < 2 || d.Ls < 1) return 0;
    if (d.NHs != 2 * d.KVs) return 0;   // read only by the fused attention + O kernel (qtts_attn_o_covers)
    const int QKV = dv->QKVs();
    const size_t rows = (size_t)d.V + (size_t)(d.G - 2) * d.Vs;
    const int nid = d.V > d.Vs ? d.V : d.Vs;
    std::vector<int> io(nid);
    for (int i = 0; i < nid; ++i) io[i] = i;
    int *ids = (int *)dalloc(dv, (size_t)nid * 4, true);
    dv->qkv0_tab = (float *)dalloc(dv, rows * QKV * 4, true);
    if (!ids || !dv->qkv0_tab) return -1;
    CK(hipMemcpy(ids, io.data(), (size_t)nid * 4, hipMemcpyHostToDevice));
    const bool proj = dv->st_proj != nullptr;
    for (int g = 1; g < d.G; ++g) {
        GemvArgs a = gv(dv->sl[0].wqkv, QKV, d.Hs, nullptr, d.Hs, nullptr, QKV, 1, EPI_STORE);
        a.norm_w = dv->sl[0].in; a.eps = d.eps; a.nt = 0;
        if (proj) a.table_f32 = g == 1 ? dv->codec_ptab : dv->st_ptab + (size_t)(g - 2) * d.Vs * d.Hs;
        else a.table = g == 1 ? dv->codec_emb : dv->st_emb + (size_t)(g - 2) * d.Vs * d.H;
        a.ids = ids; a.ids_bstride = 1;
        a.reps = g == 1 ? d.V : d.Vs;
        a.ldy_rep = QKV;
        a.y = dv->qkv0_tab + (g == 1 ? 0 : (size_t)d.V + (size_t)(g - 2) * d.Vs) * QKV;
        const int rc = qtts_gemvw(a, dv->st);
        if (rc < 0) return -1;
        if (rc == 0) continue;
        // shapes the lean kernel does not cover (small test models): the
        // per-frame path runs k_gemv1, so the table does too, one row a launch
        const int n = a.reps;
        float *base = a.y;
        a.reps = 1;
        for (int r = 0; r < n; ++r) {
            a.ids_off = r;
            a.y = base + (size_t)r * QKV;
            CKI(qtts_gemv(a, dv->st));
        }
    }
    CK(hipStreamSynchronize(dv->st));
    return 0;
}


// Batch split-K (nb >= 2, k_gemvm): the O and down projections of R rows take
// kz workgroup columns when R / 16 tiles would not fill the chip; they store
// partials, and the next GEMV that reads the residual adds them (xadd) and
// writes the new residual to the other buffer (xcopy).  0 = no split.
static int bsplit_kz(const qtts_dev *dv, int R, int C) {
    if (!dv->bsplit || dv->nrun < 2) return 0;
    int kz = R / 16 >= 256 ? 1 : 256 / (R / 16);
    // (up to 8 rows the consumers add the partials: 2 columns measured +0.8 %
    // at batch 8 over 4, gpurun_out/kz1, profiles/r03b_batch_kz_ab.txt)
    const int cap = dv->bkz_max > 0 ? dv->bkz_max : dv->nrun <= 8 ? 2 : 4;
    if (kz > cap) kz = cap;
    // above 8 rows, a column slice wider than 2048 (the 1.7B talker's down
    // projection: 6144 / 2) gives k_gemvb's waves 8 steps of 16 staged rows,
    // over the 160 KB of LDS, and the launch fell back to k_gemvm (17.5 us at
    // batch 16 against 10.1 us for batch 8's k_gemvb); more columns keep the
    // slices at <= 4 steps a wave
    if ((dv->nrun > 8 && dv->bkz_wide) || dv->bkz_wide == 2) {
        const int wcap = dv->bkz_wide == 2 ? 4 : cap;
        while (2 * kz <= wcap && C / kz > 2048 && C % (64 * kz) == 0) kz *= 2;
    }
    while (kz > 1 && C % (32 * kz)) kz /= 2;
    return kz > 1 ? kz : 0;
}
// Above 8 rows the producer reduces its own partials (GemvArgs::tick: its
// last column adds them to the residual) and nothing is pending; up to 8 the
// consumer adds them (returns true).  Measured (profiles/r02r_bsplit_self_ab.txt):
// batch 16 174.3 vs 169.5 audio-s/s self-reducing, batch 8 109.9 vs 113.9;
// again after the loads of both sides were unserialised (gpurun_out ab5, same
// box): self-reducing at every batch size gave batch 2 38.7 vs 42.6, 4 70.5
// vs 76.0, 8 123.6 vs 126.3, 16 193.3 vs 189.0.
static bool split_out(qtts_dev *dv, GemvArgs &g, float *part, int kz, int self_min = 0) {
    g.ypart = part; g.kz = kz; g.ld_ypart = (size_t)dv->nrun * g.R;
    if (dv->nrun >= (self_min > 0 ? self_min : dv->bself_min)) { g.tick = dv->btick; return false; }
    g.y = nullptr;
    return true;
}
static void add_in(GemvArgs &g, const float *part, int n, int R, int nrun, float *xnew) {
    g.xadd = part; g.n_xadd = n; g.ld_xadd = nrun * R; g.ldb_xadd = R;
    if (xnew) { g.xcopy = xnew; g.ldxc = R; g.xcopy_normed = 0; }
}

// Next-launch weight slices (L2Prefetch): what workgroup b of the NEXT launch
// reads, for the two launch shapes of the batch-1 sub-talker chain
//   k_gemvw (grid 256): rows [b R / 256, (b + 1) R / 256), contiguous
//   (a next launch of `grid` workgroups, 256 or 512: this launch's workgroup b
//   < 256 takes the first cap bytes of the next one's workgroup b -- b and
//   b + 256 share an XCD, so a 512 grid is half covered)
static L2Prefetch pf_gemvw(const qtts_dev *dv, const bf16_t *W, int R, int C, int grid = 256, bool on = true) {
    L2Prefetch p;
    if (!on || R % grid) return p;
    long long bytes = (long long)(R / grid) * C * 2;
    if (bytes > 64LL * 256 * QTTS_PF_LOADS) bytes = 64LL * 256 * QTTS_PF_LOADS;
    if (bytes % 64) return p;
    p.base = reinterpret_cast<const unsigned char *>(W);
    p.pa = (long long)(R / grid) * C * 2; p.pb = 0; p.chunks = (int)(bytes / 64); p.lg = 30; p.ld = 0;
    p.nwg = grid;
    p.sink = dv->pf_sink;
    return p;
}
#ifdef QTTS_STAMPS
#define DBG_XFIRST(a) do { const char *e_ = getenv("QTTS_HIP_DBG_XFIRST"); (a).dbg_xfirst = e_ ? atoi(e_) : 0; } while (0)
#else
#define DBG_XFIRST(a) do { } while (0)
#endif
//   k_attn_o (grid (R / RPW, KV), linear b = rb + (R / RPW) kvh): rows
//   [RPW rb, +RPW) x columns [2 HD kvh, +2 HD) of W_o [R][NH HD]
static L2Prefetch pf_attn_o(const qtts_dev *dv, const bf16_t *Wo, int R, int NH, int HD) {
    L2Prefetch p;
    const int W2 = 2 * HD, LPS = W2 / 8 < 8 ? W2 / 8 : 8, RPW = 256 / LPS;
    const int cpr = W2 * 2 / 64;   // 64-B chunks per row slice
    if (R % RPW || (cpr & (cpr - 1)) || cpr < 1 || RPW * cpr > 256 * QTTS_PF_LOADS) return p;
    p.base = reinterpret_cast<const unsigned char *>(Wo);
    p.pm = R / RPW; p.pa = (long long)RPW * NH * HD * 2; p.pb = W2 * 2;
    p.chunks = RPW * cpr; p.lg = __builtin_ctz(cpr); p.ld = NH * HD * 2; p.sink = dv->pf_sink;
    p.nwg = (R / RPW) * (NH / 2);   // (R / RPW) row blocks x the kv heads of a GQA-2 W_o
    return p;
}

// the talker layers at batch 1 as persistent launches (k_tengine.hip), each
// bit-identical to the launch-per-op layer below
static bool tengine_ok(qtts_dev *dv, int kzo, int kzd) {
    const qtts_dims_t &d = dv->d;
    // (the launch's 32-key splits need nsplit * 32 >= S partial slots; any S)
    return dv->tengine && dv->te_g && dv->nrun == 1 && !kzo && !kzd && dv->attn_defer &&
           qtts_tlayer_dims_ok(d.H, d.NH, d.KV, d.HD, d.I) && dv->S > 16 && dv->att_nsplit * 32 >= dv->S;
}
// layer launches enqueued (or captured) on the engine since the library
// loaded: a test's proof that the engine, not the launch-per-op layer, ran
static std::atomic<long long> g_tengine_layers{0};
extern "C" long long qtts_hip_tengine_layers(void) { return g_tengine_layers.load(); }
static int talker_layers_te(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    const int NBA = dv->nb, KVD = d.KV * d.HD;
    for (int l = 0; l < d.L; ++l) {
        Layer &ly = dv->tl[l];
        TLayerArgs a;
        a.x_in = dv->x_tk; a.x_out = dv->x_tk;
        a.wqkv = ly.wqkv; a.wo = ly.wo; a.wgu = ly.wgu; a.wdown = ly.wdown;
        a.in_norm = ly.in; a.post_norm = ly.post; a.qn_w = ly.qn; a.kn_w = ly.kn;
        a.rope_cos = dv->rope_cos; a.rope_sin = dv->rope_sin;
        a.kc = dv->kc + (size_t)l * NBA * dv->S * KVD; a.vc = dv->vc + (size_t)l * NBA * dv->S * KVD;
        a.pos = dv->kv_len; a.skip = dv->stopped; a.eps = d.eps;
        a.part = dv->att_part; a.cnt = dv->att_cnt; a.nsplit = dv->att_nsplit;
        a.g_qkv = dv->te_g; a.g_att = dv->te_g + 4096; a.g_x = a.g_att + 2048; a.g_h = a.g_x + 2048;
        a.epoch = dv->te_ctl; a.err = dv->te_ctl + 1;
        a.layer = l; a.last_layer = l == d.L - 1;
        if (dv->gm_dbg && (l == dv->gm_dbg_layer || l == dv->gm_dbg_layer + 1))
            a.dbg = dv->gm_dbg + (size_t)(l - dv->gm_dbg_layer) * 256 * 16;
        ProfScope ps(dv, PK_GEMV_TALKER, 2.0 * ((double)dv->QKV() * d.H + (double)d.H * d.NH * d.HD + 3.0 * d.I * d.H));
        CKI(qtts_tlayer(a, dv->st, dv->tengine));
        g_tengine_layers.fetch_add(1);
    }
    dv->tk_xfin = dv->x_tk; dv->tk_pend = nullptr; dv->tk_npend = 0;
    return 0;
}

static int talker_layers(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    const int nb = dv->nrun, NBA = dv->nb, QKV = dv->QKV(), AD = d.NH * d.HD, KVD = d.KV * d.HD;
    hipStream_t st = dv->st;
    // (the talker's O without split-K at batch 8: 142.0 / 142.6 vs 140.7 / 142.1
    // audio-s/s, within noise; its down without: 135.9 / 135.6, gpurun_out/tkz)
    const int kzo = bsplit_kz(dv, d.H, AD), kzd = bsplit_kz(dv, d.H, d.I);
    if (tengine_ok(dv, kzo, kzd)) return talker_layers_te(dv);
    float *xa = dv->x_tk, *xb = dv->x_tk2;
    const float *pend = nullptr;
    int npend = 0;
    for (int l = 0; l < d.L; ++l) {
        Layer &ly = dv->tl[l];
        GemvArgs a = gv(ly.wqkv, QKV, d.H, xa, d.H, dv->qkv, QKV, nb, EPI_STORE);
        a.norm_w = ly.in; a.eps = d.eps;
        if (pend) add_in(a, pend, npend, d.H, nb, xb);
        AttnArgs t;
        t.mode = 0; t.qkv = dv->qkv; t.ld_qkv = QKV; t.qn_w = ly.qn; t.kn_w = ly.kn; t.eps = d.eps;
        t.rope_cos = dv->rope_cos; t.rope_sin = dv->rope_sin;
        t.kc = dv->kc + (size_t)l * NBA * dv->S * KVD; t.vc = dv->vc + (size_t)l * NBA * dv->S * KVD; t.S = dv->S;
        t.pos = dv->kv_len; t.NH = d.NH; t.KV = d.KV; t.HD = d.HD; t.out = dv->att; t.ld_out = AD; t.nrows = nb;
        t.skip = dv->stopped;
        t.part = dv->att_part; t.cnt = dv->att_cnt; t.nsplit = dv->att_nsplit; t.lpk = dv->attn_lpk;
        // batch 1: the attention's split merge moves into the O projection's
        // prologue (one dependent hand-off fewer per layer)
        const bool defer = dv->attn_defer && nb == 1 && qtts_attn_defer_ok(t) && qtts_gemvw_amerge_ok(d.H, AD);
        t.defer = defer;
        const bool dbg = dv->gm_dbg && l == dv->gm_dbg_layer;
        if (dbg) a.dbg = dv->gm_dbg;
        // (batch 1: the O projection's slices two launches ahead, the attention in between)
        if (nb == 1 && (dv->l2pf_tk & 1)) a.pf = pf_gemvw(dv, ly.wo, d.H, AD);
        CKI(qkv_attn(dv, a, t, PK_GEMV_TALKER));
        if (pend) { std::swap(xa, xb); pend = nullptr; }
        GemvArgs o = gv(ly.wo, d.H, AD, dv->att, AD, xa, d.H, nb, EPI_RESID);
        if (dbg) o.dbg = dv->gm_dbg + 2048 * 8;
        if (defer) {
            o.amerge = dv->att_part; o.am_pos = dv->kv_len; o.am_nsplit = dv->att_nsplit;
            o.am_ch = qtts_attn_keys_per_split(d.HD, true, dv->attn_lpk); o.am_hd = d.HD; o.am_gph = d.NH / d.KV;
        }
        // the talker's O / down reduce their own partials at every batch size:
        // its q|k|v and gate|up prologues (2048-wide x rows) then read x alone
        // (batch 8: 141.1 / 143.1 vs 138.9 / 141.2 audio-s/s adding the partials
        // there, same box, gpurun_out/bstk; the sub-talker keeps the consumer
        // add up to 8 rows, where self-reduction measured slower)
        const int tk_self = 2;
        const bool opend = kzo && split_out(dv, o, dv->bpo, kzo, tk_self);
        if (nb == 1 && (dv->l2pf_tk & 2)) o.pf = pf_gemvw(dv, ly.wgu, 2 * d.I, d.H, 512);
        CKI(pgemv(dv, o, PK_GEMV_TALKER));
        a = gv(ly.wgu, 2 * d.I, d.H, xa, d.H, dv->hbuf, d.I, nb, EPI_SWIGLU);
        a.norm_w = ly.post; a.eps = d.eps;
        if (dbg) a.dbg = dv->gm_dbg + 2 * 2048 * 8;
        if (opend) add_in(a, dv->bpo, kzo, d.H, nb, xb);
        CKI(pgemv(dv, a, PK_GEMV_TALKER));
        if (opend) std::swap(xa, xb);
        GemvArgs dn = gv(ly.wdown, d.H, d.I, dv->hbuf, d.I, xa, d.H, nb, EPI_RESID);
        if (dbg) dn.dbg = dv->gm_dbg + 3 * 2048 * 8;
        if (kzd && split_out(dv, dn, dv->bpd, kzd, tk_self)) { pend = dv->bpd; npend = kzd; }
        CKI(pgemv(dv, dn, PK_GEMV_TALKER));
    }
    dv->tk_xfin = xa; dv->tk_pend = pend; dv->tk_npend = npend;
    return 0;
}

// logit head, then the sampler
static int head_sample(qtts_dev *dv, const GemvArgs &a, const SampArgs &s, int kind) {
    CKI(pgemv(dv, a, kind));
    ProfScope ps(dv, PK_SAMPLE, 0);
    return qtts_sample(s, dv->st);
}

// final norm + codec head; normed hidden -> tk_hid (T.c:526-530, Q.c:1295)
static GemvArgs talker_head_args(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    GemvArgs a = gv(dv->head, d.V, d.H, dv->tk_xfin ? dv->tk_xfin : dv->x_tk, d.H, dv->logits, d.V, dv->nrun,
                    EPI_STORE);
    a.norm_w = dv->tk_norm; a.eps = d.eps; a.xcopy = dv->tk_hid; a.ldxc = d.H; a.xcopy_normed = 1;
    if (dv->tk_pend) add_in(a, dv->tk_pend, dv->tk_npend, d.H, dv->nrun, nullptr);
    return a;
}
static int talker_tail(qtts_dev *dv) { return pgemv(dv, talker_head_args(dv), PK_GEMV_TALKER); }

// codec head, then the group-0 draw with suppression / repetition penalty / EOS rules
static int talker_head_sample(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    const GemvArgs a = talker_head_args(dv);
    SampArgs s;
    s.logits = dv->logits; s.ld = d.V; s.n = d.V; s.nb = dv->nrun;
    s.top_k = dv->par.top_k; s.top_p = dv->par.top_p; s.temp = dv->par.temperature;
    s.rng = dv->rng; s.mode = 1; s.suppress_lo = d.V - 1024; s.eos = d.eos_id;
    s.rep = dv->par.repetition_penalty; s.counts = dv->counts; s.fixed = dv->par.fixed_codec_tokens;
    s.n_gen = dv->n_gen; s.stopped = dv->stopped; s.cur_row = dv->cur_row; s.stop_step = dv->stop_step;
    s.host_stopped = dv->hstop;
    s.st_rng = dv->st_rng; s.seed_bits = seed_bits(dv->par.seed);
    s.codes = dv->codes; s.codes_bstride = (dv->max_frames + 1) * d.G; s.G = d.G; s.out_tok = dv->last_tok;
    return head_sample(dv, a, s, PK_GEMV_TALKER);
}

// 16 sub-talker passes (T.c:539-736)
static int subtalker(qtts_dev *dv) {
    const qtts_dims_t &d = dv->d;
    const int nb = dv->nrun, NBA = dv->nb, QKV = dv->QKVs(), AD = d.NHs * d.HDs, KVD = d.KVs * d.HDs;
    const int cstride = (dv->max_frames + 1) * d.G;
    hipStream_t st = dv->st;
    const bool proj = dv->st_proj != nullptr;
    // batch 1, fused attention + O: each launch also pulls the next launch's
    // weight slice into its XCD's L2 (GemvArgs::pf / AttnArgs::pf)
    const bool pfon = nb == 1 && dv->attn_o && dv->l2pf;
    const int pfm = pfon ? dv->l2pf : 0;
    const bool tab0_ok = nb == 1 && dv->attn_o && dv->qkv0_tab && (!proj || dv->st_ptab);
    auto first_op_pf = [&](int gn) {   // pass gn's first launch (layer 0: the table attention or q|k|v)
        if (gn >= d.G) return L2Prefetch();
        if (gn >= 1 && tab0_ok) return pf_attn_o(dv, dv->sl[0].wo, d.Hs, d.NHs, d.HDs);
        return pf_gemvw(dv, dv->sl[0].wqkv, QKV, d.Hs);
    };
    for (int g = 0; g < d.G; ++g) {
        // input source for this pass
        GemvArgs src;  // x / table description only
        src.nb = nb;
        // passes >= 1 of a projecting model gather their already-projected row
        const bool ptab = proj && g >= 1 && dv->st_ptab;
        if (g == 0) { src.x = dv->tk_hid; src.ldx = d.H; }
        else {
            if (ptab) src.table_f32 = g == 1 ? dv->codec_ptab : dv->st_ptab + (size_t)(g - 2) * d.Vs * d.Hs;
            else src.table = g == 1 ? dv->codec_emb : dv->st_emb + (size_t)(g - 2) * d.Vs * d.H;
            // the previous draw's id (group g - 1: the talker's for g = 1)
            src.ids = dv->last_tok; src.ids_bstride = 1; src.row_sel = nullptr; src.ids_rstride = 0;
            src.ids_off = 0;
        }
        auto set_src = [&](GemvArgs &a) {
            a.x = src.x; a.ldx = src.ldx; a.table = src.table; a.table_f32 = src.table_f32; a.ids = src.ids;
            a.ids_bstride = src.ids_bstride; a.row_sel = src.row_sel; a.ids_rstride = src.ids_rstride;
            a.ids_off = src.ids_off;
        };
        if (proj && !ptab) {  // ST_PROJECT_INPUT (T.c:693-702)
            GemvArgs a = gv(dv->st_proj, d.Hs, d.H, nullptr, 0, dv->x_st, d.Hs, nb, dv->st_projb ? EPI_BIAS : EPI_STORE);
            set_src(a);
            a.bias = dv->st_projb;
            a.nt = 0;
            CKI(pgemv(dv, a, PK_GEMV_SUB));
        }
        // attn_o (batch 1): attention + O projection by kv head into per-head
        // partials, summed with the residual in the gate|up GEMV's prologue,
        // which writes the new residual to the other buffer (xa -> xb)
        // batch (nb >= 2): O / down split-K partials added by the next
        // residual reader (bsplit_kz)
        float *xa = dv->x_st, *xb = dv->x_st2;
        const int kzo = bsplit_kz(dv, d.Hs, AD), kzd = bsplit_kz(dv, d.Hs, d.Is);
        const float *pend = nullptr;
        int npend = 0;
        for (int l = 0; l < d.Ls; ++l) {
            Layer &ly = dv->sl[l];
            // pass 0 produces no logits: its last layer only has to store its k / v
            // (ST_FORWARD of pass 1 restarts from its own input, T.c:704-714)
            const bool kv_only = g == 0 && l == d.Ls - 1;
            GemvArgs a = gv(ly.wqkv, QKV, d.Hs, xa, d.Hs, dv->qkv_s, QKV, nb, EPI_STORE);
            a.norm_w = ly.in; a.eps = d.eps; a.nt = 0;
            // QTTS_HIP_GM_DBG=99: stamps of pass 5, layer 2's q|k|v / (batch: O) / gate|up / down
            const bool sdbg = dv->gm_dbg && dv->gm_dbg_layer == 99 && g == 5 && l == 2;
            if (sdbg) { a.dbg = dv->gm_dbg; DBG_XFIRST(a); }
            if (l == 0 && (!proj || ptab)) { set_src(a); a.xcopy = dv->x_st; a.ldxc = d.Hs; a.xcopy_normed = 0; }
            else if (pend) add_in(a, pend, npend, d.Hs, nb, xb);
            AttnArgs t;
            t.mode = 0; t.qkv = dv->qkv_s; t.ld_qkv = QKV; t.qn_w = ly.qn; t.kn_w = ly.kn; t.eps = d.eps;
            t.rope_cos = dv->rope_cos_s; t.rope_sin = dv->rope_sin_s;
            t.kc = dv->kcs + (size_t)l * NBA * d.G * KVD; t.vc = dv->vcs + (size_t)l * NBA * d.G * KVD; t.S = d.G;
            t.pos = nullptr; t.pos_const = g; t.NH = d.NHs; t.KV = d.KVs; t.HD = d.HDs; t.out = dv->att_s;
            t.ld_out = AD; t.nrows = nb; t.skip = dv->stopped;
            t.cnt = dv->att_cnt;
            // batch 1, pass g >= 1, layer 0: q|k|v come from the load-time table
            // by the input id (no GEMV); the gate|up GEMV reads the residual
            // from the input table row itself.  Only where the fused attention +
            // O kernel runs: it alone reads the table, and the skipped GEMV is
            // also what copies the residual (the generic paths would read a
            // stale qkv_s and an unwritten x_st)
            const bool tab0 = l == 0 && g >= 1 && nb == 1 && dv->attn_o && dv->qkv0_tab && (!proj || ptab) &&
                              qtts_attn_o_covers(t, ly.wo);
            GemvArgs o = gv(ly.wo, d.Hs, AD, dv->att_s, AD, xa, d.Hs, nb, EPI_RESID);
            o.nt = 0;
            bool fused_o = false, opend = false;
            // (batch 1 only: at batch 8 / 16 the per-row recompute measured slower than
            // the separate attention + split-K O projection, 98 vs 107 / 132 vs 155
            // audio-s/s, profiles/r01av_bench_batch_attn_o.txt)
            // batch, pass g >= 1, layer 0: the same table, read by the short
            // attention kernel, which also copies the input row to the
            // residual (AttnArgs::xc_dst; the skipped GEMV's xcopy)
            const bool hd_ok = d.HDs == 128 || d.HDs == 64 || d.HDs == 32 || d.HDs == 16;
            const bool tab0b = l == 0 && g >= 1 && nb >= 2 && dv->tab0b && dv->qkv0_tab && (!proj || ptab) &&
                               d.NHs == 2 * d.KVs && d.G <= 16 && hd_ok;
            if (tab0 || tab0b) {
                t.qkv_tab = dv->qkv0_tab + (g == 1 ? 0 : (size_t)d.V + (size_t)(g - 2) * d.Vs) * QKV;
                t.tab_ids = src.ids; t.tab_bstride = src.ids_bstride; t.tab_row_sel = src.row_sel;
                t.tab_rstride = src.ids_rstride; t.tab_off = src.ids_off;
            }
            if (tab0b) { t.xc_tab = src.table_f32; t.xc_tab16 = src.table; t.xc_dst = xa; t.xc_n = d.Hs; }
            if (pfm & 1) a.pf = pf_attn_o(dv, ly.wo, d.Hs, d.NHs, d.HDs);
            if (pfm & 2) t.pf = kv_only ? first_op_pf(g + 1) : pf_gemvw(dv, ly.wgu, 2 * d.Is, d.Hs);
#ifdef QTTS_STAMPS
            if (sdbg) t.dbg = dv->gm_dbg + 2048 * 8;   // (batch 1: the attention + O launch in the "O / -" slot)
#endif
            if (dv->attn_o && nb == 1) {
                if (!tab0) CKI(pgemv(dv, a, PK_GEMV_SUB));
                if (pend) { std::swap(xa, xb); pend = nullptr; }   // the QKV GEMV wrote xa + partials to xb
                ProfScope ps(dv, PK_ATTN, (double)d.Hs * AD * 2);
                const int rc = qtts_attn_o(t, ly.wo, d.Hs, dv->opart, st);
                if (rc < 0) return -1;
                if (rc == 1) {   // not covered: the attention kernel, then the O GEMV below
                    ps.cancel();
                    { ProfScope pa(dv, PK_ATTN, 0); CKI(qtts_attention(t, st)); }
                    o.y = xa;
                    if (kzo) opend = split_out(dv, o, dv->bpo, kzo);
                    if (!kv_only) CKI(pgemv(dv, o, PK_GEMV_SUB));
                } else {
                    fused_o = true;
                }
            } else {
                if (tab0b) {
                    ProfScope pa(dv, PK_ATTN, 0);
                    CKI(qtts_attention(t, st));
                } else {
                    CKI(qkv_attn(dv, a, t, PK_GEMV_SUB));
                }
                if (pend) { std::swap(xa, xb); pend = nullptr; }   // the QKV GEMV wrote xa + partials to xb
                o.y = xa;
                if (kzo) opend = split_out(dv, o, dv->bpo, kzo);
                if (sdbg) o.dbg = dv->gm_dbg + 2048 * 8;
                if (!kv_only) CKI(pgemv(dv, o, PK_GEMV_SUB));
            }
            if (kv_only) break;
            a = gv(ly.wgu, 2 * d.Is, d.Hs, xa, d.Hs, dv->h_s, d.Is, nb, EPI_SWIGLU);
            a.norm_w = ly.post; a.eps = d.eps; a.nt = 0;
            if (pfm & 4) a.pf = pf_gemvw(dv, ly.wdown, d.Hs, d.Is);
            if (sdbg) { a.dbg = dv->gm_dbg + 2 * 2048 * 8; DBG_XFIRST(a); }
            if (tab0) set_src(a);   // the residual is the input table row (x_st was not written)
            if (fused_o) {
                add_in(a, dv->opart, d.KVs, d.Hs, nb, xb);
            } else if (opend) {
                add_in(a, dv->bpo, kzo, d.Hs, nb, xb);
            }
            CKI(pgemv(dv, a, PK_GEMV_SUB));
            if (fused_o || opend) std::swap(xa, xb);
            a = gv(ly.wdown, d.Hs, d.Is, dv->h_s, d.Is, xa, d.Hs, nb, EPI_RESID);
            a.nt = 0;
            if (pfm & 8) {
                if (l + 1 < d.Ls) a.pf = pf_gemvw(dv, dv->sl[l + 1].wqkv, QKV, d.Hs);
                else if (g >= 1) a.pf = pf_gemvw(dv, dv->lm + (size_t)(g - 1) * d.Vs * d.Hs, d.Vs, d.Hs);
            }
            if (sdbg) { a.dbg = dv->gm_dbg + 3 * 2048 * 8; DBG_XFIRST(a); }
            if (kzd && split_out(dv, a, dv->bpd, kzd)) { pend = dv->bpd; npend = kzd; }
            CKI(pgemv(dv, a, PK_GEMV_SUB));
        }
        if (g == 0) continue;  // pass 0 produces no logits
        GemvArgs a = gv(dv->lm + (size_t)(g - 1) * d.Vs * d.Hs, d.Vs, d.Hs, xa, d.Hs, dv->logits_s, d.Vs, nb,
                        EPI_STORE);
        a.norm_w = dv->st_norm; a.eps = d.eps; a.nt = 0;
        if (pend) add_in(a, pend, npend, d.Hs, nb, nullptr);
        if (pfm & 16) a.pf = first_op_pf(g + 1);   // (two launches ahead: the sampler runs in between)
        SampArgs s;
        s.logits = dv->logits_s; s.ld = d.Vs; s.n = d.Vs; s.nb = nb;
        s.top_k = dv->par.st_top_k; s.top_p = dv->par.st_top_p; s.temp = dv->par.st_temperature;
        s.mode = 0; s.st_rng = dv->st_rng; s.stopped = dv->stopped; s.cur_row = dv->cur_row;
        s.codes = dv->codes; s.codes_bstride = cstride; s.G = d.G; s.g = g; s.out_tok = dv->last_tok;
        CKI(head_sample(dv, a, s, PK_GEMV_SUB));
    }
    return 0;
}

static int embed_sum(qtts_dev *dv, int advance) {
    const qtts_dims_t &d = dv->d;
    EmbedSumArgs e;
    e.codes = dv->codes; e.codes_bstride = (dv->max_frames + 1) * d.G; e.G = d.G;
    e.cur_row = dv->cur_row; e.stopped = dv->stopped; e.codec_emb = dv->codec_emb; e.st_emb = dv->st_emb;
    e.Vs = d.Vs; e.H = d.H; e.nb = dv->nrun; e.trailing = dv->trailing; e.tr_cap = dv->tr_cap;
    e.n_trailing = dv->n_trailing; e.pad = dv->pad_emb; e.out = dv->x_tk; e.kv_len = dv->kv_len; e.advance = advance;
    ProfScope ps(dv, PK_EMBED, 0);
    return qtts_embed_sum(e, dv->st);
}

static int record_frame(qtts_dev *dv, bool with_talker) {
    // step 0 starts from the prefill's hidden in x_tk (no pending partials)
    dv->tk_xfin = dv->x_tk; dv->tk_pend = nullptr; dv->tk_npend = 0;
    if (with_talker) CKI(talker_layers(dv));
    CKI(talker_head_sample(dv));
    CKI(subtalker(dv));
    CKI(embed_sum(dv, with_talker ? 1 : 0));
    return 0;
}

static int capture(qtts_dev *dv, bool with_talker, hipGraphExec_t *out) {
    hipGraph_t g = nullptr;
    CK(hipStreamBeginCapture(dv->st, hipStreamCaptureModeThreadLocal));
    int rc = record_frame(dv, with_talker);
    hipError_t e = hipStreamEndCapture(dv->st, &g);
    if (rc || e != hipSuccess) {
        fprintf(stderr, "qtts: frame graph capture failed\n");
        if (g) hipGraphDestroy(g);
        return -1;
    }
    e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    CK(e);
    return 0;
}

// One graph for step 0 (no talker) and one for every later frame, its talker
// attention grid sized from the KV capacity (splits past the live length exit
// at once).  Graphs per power-of-two bucket of the live key count measured no
// faster, also in EOS mode (4096-frame capacity, 65 splits): 31.0 / 31.3 vs
// 31.1 / 30.5 audio-s/s (profiles/r03c_eos_ab.txt).
static int ensure_graphs(qtts_dev *dv) {
    if (dv->g0 && dv->gN && dv->graph_key == 1) return 0;
    if (dv->g0) { hipGraphExecDestroy(dv->g0); dv->g0 = nullptr; }
    if (dv->gN) { hipGraphExecDestroy(dv->gN); dv->gN = nullptr; }
    drop_row_graphs(dv);
    if (getenv("QTTS_HIP_NO_GRAPH")) { dv->graph_key = 0; return 0; }
    // (the two main graphs always cover every slot)
    const int nrun = dv->nrun;
    dv->nrun = dv->nb;
    int rc = capture(dv, false, &dv->g0);
    if (!rc) rc = capture(dv, true, &dv->gN);
    dv->nrun = nrun;
    CKI(rc);
    dv->graph_key = 1;
    return 0;
}

static bool same_params(const qtts_gen_params_t &a, const qtts_gen_params_t &b) {
    return memcmp(&a, &b, sizeof a) == 0;
}

extern "C" int qtts_dev_begin(qtts_dev_t *dv, int nb, int max_frames, int max_prefill, const qtts_gen_params_t *p) {
    if (!dv || nb < 1 || max_frames < 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));   // a prime left pending by a run that pushed no frames
    if (max_prefill < 16) max_prefill = 16;
    const bool realloc_ = nb != dv->nb || max_frames > dv->max_frames || max_prefill > dv->p_cap;
    if (realloc_) {
        if (dv->cst) CK(hipStreamSynchronize(dv->cst));   // a prime still reading the codec scratch
        dv->prime_pending = false;
        CKI(alloc_state(dv, nb, max_frames, max_prefill));
    }
    if (!dv->have_par || !same_params(dv->par, *p)) {
        dv->par = *p;
        dv->have_par = true;
        dv->graph_key = -1;
    }
    dv->nrun = dv->nb;
    CKI(reset_counters(dv));
    return 0;
}

// ----------------------------------------------------------------- prompt + prefill
static int ensure_trailing(qtts_dev *dv, int n_tr) {
    if (n_tr <= dv->tr_cap) return 0;
    const qtts_dims_t &d = dv->d;
    int cap = dv->tr_cap;
    while (cap < n_tr) cap *= 2;
    float *nt = (float *)dalloc(dv, (size_t)dv->nb * cap * d.H * 4, false);
    if (!nt) return -1;
    CK(hipStreamSynchronize(dv->st));
    for (int b = 0; b < dv->nb; ++b)
        CK(hipMemcpy(nt + (size_t)b * cap * d.H, dv->trailing + (size_t)b * dv->tr_cap * d.H,
                     (size_t)dv->tr_cap * d.H * 4, hipMemcpyDeviceToDevice));
    dv->trailing = nt;  // old block stays in sallocs until free_state
    dv->tr_cap = cap;
    dv->graph_key = -1;
    return 0;
}

// voice-clone inputs for the next qtts_dev_prompt: reference codes
// [n_ref][G] (plan codec ids <= -3) and the speaker x-vector [H] (id -2)
extern "C" int qtts_dev_prompt_ref(qtts_dev_t *dv, const int *ref_codes, int n_ref, const float *spk) {
    if (!dv || n_ref < 0 || (n_ref > 0 && !ref_codes)) return -1;
    hipSetDevice(dv->device);
    const qtts_dims_t &d = dv->d;
    if (!dv->pspk) {
        dv->pspk = (float *)dalloc(dv, (size_t)d.H * 4, true);
        if (!dv->pspk) return -1;
    }
    if (n_ref > dv->pref_cap) {
        const int cap = n_ref < 512 ? 512 : n_ref;
        dv->pref = (int *)dalloc(dv, (size_t)cap * d.G * 4, true);   // lives with the weights (freed at destroy)
        if (!dv->pref) return -1;
        dv->pref_cap = cap;
    }
    CK(hipStreamSynchronize(dv->st));
    if (n_ref > 0) CK(hipMemcpy(dv->pref, ref_codes, (size_t)n_ref * d.G * 4, hipMemcpyHostToDevice));
    if (spk) CK(hipMemcpy(dv->pspk, spk, (size_t)d.H * 4, hipMemcpyHostToDevice));
    dv->n_pref = n_ref;
    dv->has_spk = spk != nullptr;
    return 0;
}

extern "C" int qtts_dev_prompt(qtts_dev_t *dv, int b, const int *text_ids, int n_text, const int *plan, int nplan,
                               int p_len, int n_trailing, int pad_row) {
    if (!dv || b < 0 || b >= dv->nb || p_len > dv->p_cap || n_text < 1) return -1;
    hipSetDevice(dv->device);
    const qtts_dims_t &d = dv->d;
    CKI(ensure_trailing(dv, n_trailing));
    CK(hipStreamSynchronize(dv->st));
    if (n_text > dv->ids_cap || nplan > 4 * dv->ids_cap) {
        int cap = n_text < 256 ? 256 : n_text;
        if (4 * cap < nplan) cap = (nplan + 3) / 4;
        dv->pids = (int *)dalloc(dv, (size_t)cap * 4, false);
        dv->pplan = (int *)dalloc(dv, (size_t)4 * cap * 5 * 4, false);   // 4 * cap plan rows of 5 ints
        dv->pt1 = (float *)dalloc(dv, (size_t)cap * d.TH * 4, false);
        dv->pproj = (float *)dalloc(dv, (size_t)cap * d.H * 4, false);
        if (!dv->pids || !dv->pplan || !dv->pt1 || !dv->pproj) return -1;
        dv->ids_cap = cap;
    }
    if (nplan > 4 * dv->ids_cap) return -1;
    CK(hipMemcpy(dv->pids, text_ids, (size_t)n_text * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv->pplan, plan, (size_t)nplan * 5 * 4, hipMemcpyHostToDevice));
    // text_embedding -> fc1 (+b, SiLU) -> fc2 (+b), 16 rows per launch (Q.c:823-847)
    {
        if (!dv->fc1b) { fprintf(stderr, "qtts: text projection without fc1 bias unsupported\n"); return -1; }
        GemvArgs a = gv(dv->fc1w, d.TH, d.TH, nullptr, 0, dv->pt1, d.TH, 1, EPI_BIAS_SILU);
        a.table = dv->text_emb; a.ids = dv->pids; a.ids_bstride = 1; a.bias = dv->fc1b;
        CKI(rows_proj(dv, a, n_text));
        a = gv(dv->fc2w, d.H, d.TH, dv->pt1, d.TH, dv->pproj, d.H, 1, dv->fc2b ? EPI_BIAS : EPI_STORE);
        a.bias = dv->fc2b;
        CKI(rows_proj(dv, a, n_text));
    }
    PromptArgs pa;
    pa.proj = dv->pproj; pa.plan = dv->pplan; pa.nplan = nplan; pa.H = d.H; pa.codec_emb = dv->codec_emb;
    pa.prefill = dv->prefill; pa.p_cap = dv->p_cap; pa.trailing = dv->trailing; pa.tr_cap = dv->tr_cap;
    pa.st_emb = dv->st_emb; pa.G = d.G; pa.V = d.V; pa.Vs = d.Vs;
    pa.spk = dv->has_spk ? dv->pspk : nullptr;
    pa.ref_codes = dv->n_pref > 0 ? dv->pref : nullptr; pa.n_ref = dv->n_pref;
    CKI(qtts_prompt_assemble(pa, dv->st));
    dv->n_pref = 0; dv->has_spk = 0;   // consumed
    if (pad_row >= 0) CK(hipMemcpyAsync(dv->pad_emb, dv->pproj + (size_t)pad_row * d.H, (size_t)d.H * 4,
                                        hipMemcpyDeviceToDevice, dv->st));
    CK(hipMemcpyAsync(dv->n_trailing + b, &n_trailing, 4, hipMemcpyHostToDevice, dv->st));
    CK(hipStreamSynchronize(dv->st));
    dv->p_len_h[b] = p_len;
    dv->n_tr_h[b] = n_trailing;
    return 0;
}

// talker prefill (T.c:254-472) of prompt rows [0, nrows[i]) of slots[i];
// last[i] = the row index (in px) of slot i's last row
static int prefill_rows(qtts_dev *dv, const std::vector<int> &slots, const std::vector<int> &nrows,
                        std::vector<int> &last) {
    const qtts_dims_t &d = dv->d;
    hipStream_t st = dv->st;
    std::vector<int> rb, pp, src;
    last.assign(slots.size(), 0);
    for (size_t i = 0; i < slots.size(); ++i) {
        const int b = slots[i];
        for (int t = 0; t < nrows[i]; ++t) {
            rb.push_back(b);
            pp.push_back(t);
            src.push_back(b * dv->p_cap + t);
        }
        last[i] = (int)rb.size() - 1;
    }
    const int R = (int)rb.size();
    if (R < 1 || R > dv->rows_cap) return -1;
    CK(hipMemcpyAsync(dv->prow_b, rb.data(), R * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(dv->ppos, pp.data(), R * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(dv->psrc, src.data(), R * 4, hipMemcpyHostToDevice, st));
    CKI(qtts_copy_rows(dv->px, d.H, dv->prefill, d.H, dv->psrc, R, d.H, st));
    const int QKV = dv->QKV(), AD = d.NH * d.HD, KVD = d.KV * d.HD;
    for (int l = 0; l < d.L; ++l) {
        Layer &ly = dv->tl[l];
        {
            GemvArgs a = gv(ly.wqkv, QKV, d.H, dv->px, d.H, dv->pqkv, QKV, 1, EPI_STORE);
            a.norm_w = ly.in; a.eps = d.eps; a.nt = 0;
            CKI(rows_proj(dv, a, R, true));
        }
        AttnArgs t;
        t.mode = 1; t.qkv = dv->pqkv; t.ld_qkv = QKV; t.qn_w = ly.qn; t.kn_w = ly.kn; t.eps = d.eps;
        t.rope_cos = dv->rope_cos; t.rope_sin = dv->rope_sin;
        t.kc = dv->kc + (size_t)l * dv->nb * dv->S * KVD; t.vc = dv->vc + (size_t)l * dv->nb * dv->S * KVD;
        t.S = dv->S; t.pos = dv->ppos; t.row_b = dv->prow_b; t.NH = d.NH; t.KV = d.KV; t.HD = d.HD;
        t.out = dv->patt; t.ld_out = AD; t.nrows = R;
        CKI(qtts_qk_prep(t, st));
        CKI(qtts_attention(t, st));
        {
            GemvArgs a = gv(ly.wo, d.H, AD, dv->patt, AD, dv->px, d.H, 1, EPI_RESID);
            a.nt = 0;
            CKI(rows_proj(dv, a, R, true));
            a = gv(ly.wgu, 2 * d.I, d.H, dv->px, d.H, dv->ph, d.I, 1, EPI_SWIGLU);
            a.norm_w = ly.post; a.eps = d.eps; a.nt = 0;
            CKI(rows_proj(dv, a, R, true));
            a = gv(ly.wdown, d.H, d.I, dv->ph, d.I, dv->px, d.H, 1, EPI_RESID);
            a.nt = 0;
            CKI(rows_proj(dv, a, R, true));
        }
    }
    return 0;
}

// talker prefill over all slots' prompt rows (T.c:254-472)
extern "C" int qtts_dev_prefill(qtts_dev_t *dv) {
    if (!dv || dv->nb < 1) return -1;
    hipSetDevice(dv->device);
    const qtts_dims_t &d = dv->d;
    hipStream_t st = dv->st;
    std::vector<int> slots(dv->nb), last;
    for (int b = 0; b < dv->nb; ++b) slots[b] = b;
    CKI(prefill_rows(dv, slots, dv->p_len_h, last));
    // last raw hidden of each slot -> x_tk; kv_len = prefill length
    CK(hipMemcpyAsync(dv->plast, last.data(), dv->nb * 4, hipMemcpyHostToDevice, st));
    CKI(qtts_copy_rows(dv->x_tk, d.H, dv->px, d.H, dv->plast, dv->nb, d.H, st));
    CK(hipMemcpyAsync(dv->kv_len, dv->p_len_h.data(), dv->nb * 4, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    return 0;
}

// Work queue: slot b of the live batch takes the utterance
// qtts_dev_prompt(b, ...) just assembled.  Its prompt rows but the last are
// prefilled (the KV cache positions 0 .. p_len - 2 of slot b); the last prompt
// row becomes the slot's talker input at kv_len = p_len - 1, so the next
// lock-step frame (the talker-first graph every running slot replays) runs
// that row through the talker at position p_len - 1 -- the same arithmetic the
// reference's prefill applies to it (T.c:254-472 vs T.c:478-533, the last
// row's hidden feeding codec_head, Q.c:1282-1295) -- then samples the
// utterance's frame 0.  The slot's counters start afresh (Q.c:1250-1270).
// Everything is ordered on the context stream after the frames already queued.
extern "C" int qtts_dev_refill(qtts_dev_t *dv, int b) {
    if (!dv || b < 0 || b >= dv->nb || dv->p_len_h[b] < 2) return -1;
    hipSetDevice(dv->device);
    const qtts_dims_t &d = dv->d;
    std::vector<int> last;
    CKI(prefill_rows(dv, std::vector<int>{b}, std::vector<int>{dv->p_len_h[b] - 1}, last));
    SlotResetArgs r;
    r.b = b; r.pos = dv->p_len_h[b] - 1; r.H = d.H; r.V = d.V;
    r.row = dv->prefill + ((size_t)b * dv->p_cap + r.pos) * d.H;
    r.x = dv->x_tk; r.kv_len = dv->kv_len; r.n_gen = dv->n_gen; r.cur_row = dv->cur_row; r.stopped = dv->stopped;
    r.stop_step = dv->stop_step; r.last_tok = dv->last_tok; r.counts = dv->counts;
    r.rng = dv->rng; r.st_rng = dv->st_rng; r.seed_bits = seed_bits(dv->par.seed);
    CKI(qtts_slot_reset(r, dv->st));
    CK(hipStreamSynchronize(dv->st));   // (the prefill's row lists are host vectors)
    // the host's stop mirror: no queued frame writes it for this slot (it was
    // stopped in all of them)
    if (dv->hstop && b < dv->hstop_cap) ((volatile int *)dv->hstop)[b] = 0;
    return 0;
}

// Work queue: stop slot b from the next queued frame on (its utterance reached
// max_new_tokens / the fixed length without EOS, Q.c:1282); stream-ordered.
extern "C" int qtts_dev_retire(qtts_dev_t *dv, int b) {
    if (!dv || b < 0 || b >= dv->nb) return -1;
    hipSetDevice(dv->device);
    CK(hipMemsetD32Async((hipDeviceptr_t)(dv->stopped + b), 1, 1, dv->st));
    return 0;
}

// Work queue, lagged as qtts_dev_frame_done: waits until frame `step` has
// finished and copies every slot's EOS mirror (1: drew EOS by then).
extern "C" int qtts_dev_frame_stops(qtts_dev_t *dv, int step, int *stopped) {
    if (!dv || !stopped || !dv->hstop) return -1;
    hipSetDevice(dv->device);
    if (dv->graph_key == 1) CK(hipEventSynchronize(dv->fev[step & 1]));
    else CK(hipStreamSynchronize(dv->st));
    for (int b = 0; b < dv->nrun; ++b) stopped[b] = ((volatile int *)dv->hstop)[b] != 0;
    return 0;
}

// Work queue, tail of a run (no utterance left to admit): slot `from`'s
// whole decode state moves to slot `to` (a freed slot below it), so that the
// running slots are the first ones and qtts_dev_set_rows can launch fewer
// rows.  Stream-ordered; the caller has synchronised (no frame in flight
// writes either slot).
extern "C" int qtts_dev_move_slot(qtts_dev_t *dv, int from, int to) {
    if (!dv || from < 0 || to < 0 || from >= dv->nb || to >= dv->nb || from == to) return -1;
    hipSetDevice(dv->device);
    const qtts_dims_t &d = dv->d;
    hipStream_t st = dv->st;
    int kv = 0;
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(&kv, dv->kv_len + from, 4, hipMemcpyDeviceToHost));
    if (kv < 0 || kv >= dv->S) return -1;
    const size_t KVD = (size_t)d.KV * d.HD, lstride = (size_t)dv->nb * dv->S * KVD * 4;
    const size_t w = (size_t)(kv + 1) * KVD * 4;   // positions 0 .. kv (the next step writes kv)
    for (float *c : {dv->kc, dv->vc})
        CK(hipMemcpy2DAsync((char *)c + (size_t)to * dv->S * KVD * 4, lstride,
                            (const char *)c + (size_t)from * dv->S * KVD * 4, lstride, w, d.L,
                            hipMemcpyDeviceToDevice, st));
    auto row = [&](void *base, size_t bytes) {
        return hipMemcpyAsync((char *)base + (size_t)to * bytes, (const char *)base + (size_t)from * bytes, bytes,
                              hipMemcpyDeviceToDevice, st);
    };
    CK(row(dv->x_tk, (size_t)d.H * 4));
    CK(row(dv->counts, (size_t)d.V * 4));
    CK(row(dv->codes, (size_t)(dv->max_frames + 1) * d.G * 4));
    CK(row(dv->trailing, (size_t)dv->tr_cap * d.H * 4));
    for (int *p : {dv->kv_len, dv->n_gen, dv->cur_row, dv->stopped, dv->stop_step, dv->last_tok, dv->n_trailing})
        CK(row(p, 4));
    CK(row(dv->rng, 4));
    CK(row(dv->st_rng, 4));
    CK(hipStreamSynchronize(st));
    dv->p_len_h[to] = dv->p_len_h[from];
    dv->n_tr_h[to] = dv->n_tr_h[from];
    if (dv->hstop && from < dv->hstop_cap && to < dv->hstop_cap)
        ((volatile int *)dv->hstop)[to] = ((volatile int *)dv->hstop)[from];
    return 0;
}

// Work queue: the next frames launch the first `rows` slots only (1 <= rows
// <= the slots of qtts_dev_begin; their own graph per row count).
extern "C" int qtts_dev_set_rows(qtts_dev_t *dv, int rows) {
    if (!dv || rows < 1 || rows > dv->nb || (rows < dv->nb && rows > QTTS_MAX_SLOTS)) return -1;
    dv->nrun = rows;
    return 0;
}

// sizes the per-slot trailing text rows for the longest utterance a run will
// see (a later qtts_dev_prompt never grows them, so the frame graphs stay)
extern "C" int qtts_dev_reserve(qtts_dev_t *dv, int max_trailing) {
    if (!dv || max_trailing < 0) return -1;
    hipSetDevice(dv->device);
    return ensure_trailing(dv, max_trailing);
}

extern "C" int qtts_dev_frame(qtts_dev_t *dv, int step) {
    if (!dv) return -1;
    hipSetDevice(dv->device);
    CKI(ensure_graphs(dv));
    if (dv->nrun < dv->nb && step == 0) return -1;   // (frame 0 runs every slot)
    if (dv->graph_key == 0) return record_frame(dv, step > 0);
    hipGraphExec_t g = step == 0 ? dv->g0 : dv->gN;
    if (dv->nrun < dv->nb) {
        hipGraphExec_t &gr = dv->gNr[dv->nrun];
        if (!gr) CKI(capture(dv, true, &gr));
        g = gr;
    }
    CK(hipGraphLaunch(g, dv->st));
    CK(hipEventRecord(dv->fev[step & 1], dv->st));
    return 0;
}

// EOS mode without a host round trip per frame: wait until frame `step` has
// finished (the caller has already queued frame step + 1) and report whether
// every running slot had drawn EOS by then.  At most one frame runs past the
// last stop, against up to poll_every - 1 with a synchronous poll (which also
// leaves the GPU idle until the next launch).
extern "C" int qtts_dev_frame_done(qtts_dev_t *dv, int step, int *all_stopped) {
    if (!dv || !all_stopped || !dv->hstop) return -1;
    hipSetDevice(dv->device);
    if (dv->graph_key == 1) CK(hipEventSynchronize(dv->fev[step & 1]));
    else CK(hipStreamSynchronize(dv->st));
    int all = 1;
    for (int b = 0; b < dv->nrun; ++b) all &= ((volatile int *)dv->hstop)[b] != 0;
    *all_stopped = all;
    return 0;
}

extern "C" int qtts_dev_poll(qtts_dev_t *dv, int *stopped, int *n_gen, int *stop_step) {
    if (!dv) return -1;
    hipSetDevice(dv->device);
    const size_t B = dv->nb;
    if (stopped) CK(hipMemcpyAsync(stopped, dv->stopped, B * 4, hipMemcpyDeviceToHost, dv->st));
    if (n_gen) CK(hipMemcpyAsync(n_gen, dv->n_gen, B * 4, hipMemcpyDeviceToHost, dv->st));
    if (stop_step) CK(hipMemcpyAsync(stop_step, dv->stop_step, B * 4, hipMemcpyDeviceToHost, dv->st));
    CK(hipStreamSynchronize(dv->st));
    return 0;
}

extern "C" int qtts_dev_get_codes(qtts_dev_t *dv, int b, int *host_codes, int max_frames) {
    if (!dv || b < 0 || b >= dv->nb) return -1;
    hipSetDevice(dv->device);
    int n = 0;
    CK(hipMemcpyAsync(&n, dv->n_gen + b, 4, hipMemcpyDeviceToHost, dv->st));
    CK(hipStreamSynchronize(dv->st));
    if (dv->te_ctl) {   // the persistent talker layer gave up waiting on a hand-off: its codes are garbage
        int ctl[2] = {0, 0};
        CK(hipMemcpy(ctl, dv->te_ctl, sizeof(ctl), hipMemcpyDeviceToHost));
        if (ctl[1]) {
            fprintf(stderr, "qtts: talker layer engine hand-off timed out (code %d, epoch %d)\n", ctl[1], ctl[0]);
            return -1;
        }
    }
    if (dv->gm_dbg && dv->te_g) {   // QTTS_HIP_GM_DBG + engine: k_tlayer phase stamps of two layers, last frame
        std::vector<unsigned long long> h(2 * 256 * 16);
        CK(hipMemcpy(h.data(), dv->gm_dbg, h.size() * 8, hipMemcpyDeviceToHost));
        static const char *ph[15] = {"start", "x staged", "qkv dot", "qkv put", "head got", "attn done", "att staged",
                                     "O dot", "x' got", "x' staged", "gu dot", "h staged", "down dot", "ld issued",
                                     "ld landed"};
        unsigned long long t00 = ~0ull;
        for (int i = 0; i < 256; ++i) if (h[i * 16] && h[i * 16] < t00) t00 = h[i * 16];
        for (int g = 0; g < 2; ++g) {
            const unsigned long long *b = h.data() + (size_t)g * 256 * 16;
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < 256; ++i) if (b[i * 16] && b[i * 16] < t0) t0 = b[i * 16];
            if (t0 == ~0ull) continue;
            fprintf(stderr, "[te_dbg] layer +%d starts %7.2f us after layer +0\n", g, (t0 - t00) * 0.01);
            for (int k = 0; k < 15; ++k) {
                std::vector<double> v;
                for (int i = 0; i < 256; ++i) if (b[i * 16 + k]) v.push_back((b[i * 16 + k] - t0) * 0.01);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                fprintf(stderr, "[te_dbg] +%d %-10s n %3zu  min %6.2f  med %6.2f  max %6.2f us\n", g, ph[k], v.size(), v[0],
                        v[v.size() / 2], v.back());
            }
        }
        hipMemsetAsync(dv->gm_dbg, 0, h.size() * 8, dv->st);
    } else if (dv->gm_dbg) {   // QTTS_HIP_GM_DBG: phase spans of the chosen talker layer's GEMVs, last frame
        std::vector<unsigned long long> h(4 * 2048 * 8);
        CK(hipMemcpy(h.data(), dv->gm_dbg, h.size() * 8, hipMemcpyDeviceToHost));
        static const char *op[4] = {"q|k|v", "O / -", "gate|up", "down"};
        // (k_gemvw: 3 epilogue, 4 after the prefetch sink, 5 weights issued,
        // 6 merged; k_gemvb: 2 = MFMAs done, 3 = after the final barrier,
        // 4 = after the epilogue stores, 5 = tiles summed, 6 = normalised)
        static const char *ph[7] = {"start", "x staged", "dot done", "epilogue", "pf landed", "w issued", "merged"};
        unsigned long long tq = 0;   // the first launch's first start: the launch offsets below
        for (int g = 0; g < 4; ++g) {
            const unsigned long long *b = h.data() + (size_t)g * 2048 * 8;
            unsigned long long t0 = ~0ull, tend = 0;
            for (int i = 0; i < 2048; ++i) if (b[i * 8] && b[i * 8] < t0) t0 = b[i * 8];
            for (int i = 0; i < 2048 * 8; ++i) if (b[i] > tend) tend = b[i];
            if (t0 != ~0ull) {
                if (!tq) tq = t0;
                fprintf(stderr, "[gm_dbg] %-8s launch at %7.2f us after the first, last stamp %6.2f us into it\n", op[g],
                        (t0 - tq) * 0.01, (tend - t0) * 0.01);
            }
            for (int k = 0; k < 7; ++k) {
                std::vector<double> v;
                for (int i = 0; i < 2048; ++i) if (b[i * 8 + k]) v.push_back((b[i * 8 + k] - t0) * 0.01);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                fprintf(stderr, "[gm_dbg] %-8s %-10s n %4zu  min %6.2f  med %6.2f  max %6.2f us\n", op[g], ph[k], v.size(),
                        v[0], v[v.size() / 2], v.back());
            }
        }
        hipMemsetAsync(dv->gm_dbg, 0, h.size() * 8, dv->st);
    }
    if (n > max_frames) n = max_frames;
    CK(hipMemcpyAsync(host_codes, dv->codes + (size_t)b * (dv->max_frames + 1) * dv->d.G, (size_t)n * dv->d.G * 4,
                      hipMemcpyDeviceToHost, dv->st));
    CK(hipStreamSynchronize(dv->st));
    return n;
}

extern "C" float *qtts_dev_codec_slot(qtts_dev_t *dv, int b, int T, int *out_samples) {
    if (out_samples) *out_samples = 0;
    if (!dv || b < 0 || b >= dv->nb || T < 1) return nullptr;
    hipSetDevice(dv->device);
    if (join_prime(dv)) return nullptr;   // the prime shares the codec scratch and split-K workspace
    return codec_decode(&dv->codec, dv->codes + (size_t)b * (dv->max_frames + 1) * dv->d.G, T, out_samples);
}

extern "C" int qtts_dev_codec_timing(qtts_dev_t *dv, int on) {
    if (!dv) return -1;
    dv->codec.timing = on != 0;
    return 0;
}

extern "C" int qtts_dev_codec_stage_ms(const qtts_dev_t *dv, float *ms) {
    if (!dv || !ms || !dv->codec.timed) return -1;
    for (int i = 0; i < 5; ++i) ms[i] = dv->codec.stage_ms[i];
    return 0;
}

// ----------------------------------------------------------------- streaming codec (exact, incremental)
// a pending prime (below) orders every later use of the stream state after it
static int join_prime(qtts_dev *dv) {
    if (!dv->prime_pending) return 0;
    dv->prime_pending = false;
    CK(hipStreamWaitEvent(dv->st, dv->cev, 0));
    return 0;
}

static int ensure_cst(qtts_dev *dv) {
    if (dv->cst) return 0;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&dv->cst, hipStreamNonBlocking, lo));   // lowest: the decode goes first
    CK(hipEventCreateWithFlags(&dv->cev, hipEventDisableTiming));
    return 0;
}

static int ensure_push_codes(qtts_dev *dv, size_t n) {
    if (n <= dv->push_cap) return 0;
    CK(hipDeviceSynchronize());
    if (dv->push_codes) CK(hipFree(dv->push_codes));
    dv->push_codes = nullptr;
    dv->push_cap = 0;
    const size_t cap = n < 4096 ? 4096 : n;
    CK(hipMalloc(&dv->push_codes, cap * 4));
    dv->push_cap = cap;
    return 0;
}

extern "C" int qtts_dev_codec_stream_begin(qtts_dev_t *dv, int max_frames) {
    return qtts_dev_codec_stream_begin_ex(dv, max_frames, 0);
}

extern "C" int qtts_dev_codec_stream_begin_ex(qtts_dev_t *dv, int max_frames, int chunk_frames) {
    if (!dv || max_frames < 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    CK(hipStreamSynchronize(dv->st));
    return codec_stream_begin(&dv->codec, max_frames, chunk_frames);
}

// Push T host frames through the stream on the second stream (cst) without
// waiting: their audio is dropped (device scratch), the carried state is what
// later pushes continue from.  The voice-clone reference frames go this way
// while the prefill runs on the context stream (SURVEY.md 8f N1 + N2).
extern "C" int qtts_dev_codec_stream_prime(qtts_dev_t *dv, const int *codes, int T) {
    if (!dv || !codes || T < 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    CKI(ensure_cst(dv));
    CKI(ensure_push_codes(dv, (size_t)T * dv->d.cq));
    const size_t need = (size_t)T * 1920;
    if (need > dv->pwav_cap) {
        CK(hipStreamSynchronize(dv->cst));
        if (dv->pwav) CK(hipFree(dv->pwav));
        dv->pwav = nullptr;
        dv->pwav_cap = 0;
        CK(hipMalloc(&dv->pwav, need * 4));
        dv->pwav_cap = need;
    }
    CK(hipEventRecord(dv->cev, dv->st));          // after the begin's resets on st
    CK(hipStreamWaitEvent(dv->cst, dv->cev, 0));
    CK(hipMemcpyAsync(dv->push_codes, codes, (size_t)T * dv->d.cq * 4, hipMemcpyHostToDevice, dv->cst));
    dv->codec.st = dv->cst;
    const int n = codec_stream_push_to(&dv->codec, dv->push_codes, dv->d.cq, T, dv->pwav, false);
    dv->codec.st = dv->st;
    if (n < 0) return -1;
    CK(hipEventRecord(dv->cev, dv->cst));
    dv->prime_pending = true;
    return 0;
}

extern "C" int qtts_dev_codec_stream_push_slot(qtts_dev_t *dv, int b, int frame0, int T, float *host_out) {
    if (!dv || b < 0 || b >= dv->nb || T < 1 || frame0 < 0 || frame0 + T > dv->max_frames + 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    const int *codes = dv->codes + (size_t)b * (dv->max_frames + 1) * dv->d.G + (size_t)frame0 * dv->d.G;
    return codec_stream_push(&dv->codec, codes, dv->d.G, T, host_out);
}

extern "C" int qtts_dev_codec_stream_push_host(qtts_dev_t *dv, const int *codes, int T, float *host_out) {
    if (!dv || !codes || T < 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    const size_t n = (size_t)T * dv->d.cq;
    CKI(ensure_push_codes(dv, n));   // persistent staging buffer: no allocation per push
    // ordered on the codec's stream before the push reads it; the synchronous
    // push waits for the stream before returning, so the host buffer may be reused
    CK(hipMemcpyAsync(dv->push_codes, codes, n * 4, hipMemcpyHostToDevice, dv->codec.st));
    return codec_stream_push(&dv->codec, dv->push_codes, dv->d.cq, T, host_out);
}

// ----------------------------------------------------------------- codec overlapped with the decode
// The exact streaming decode (codec_stream_*), run on a second stream while
// the frame graphs continue on the context stream: each push waits (event)
// for the frames already enqueued, decodes them into a device waveform, and
// nothing is waited for on the host until qtts_dev_codec_async_end.
extern "C" int qtts_dev_codec_async_begin(qtts_dev_t *dv, int max_frames) {
    if (!dv || max_frames < 1) return -1;
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    CKI(ensure_cst(dv));
    const size_t need = (size_t)max_frames * 1920;
    if (need > dv->cwav_cap) {
        CK(hipStreamSynchronize(dv->cst));
        if (dv->cwav) CK(hipFree(dv->cwav));
        dv->cwav = nullptr;
        CK(hipMalloc(&dv->cwav, need * 4));
        dv->cwav_cap = need;
    }
    CK(hipStreamSynchronize(dv->st));   // the stream state is shared with the synchronous paths
    dv->codec.st = dv->cst;
    const int rc = codec_stream_begin(&dv->codec, max_frames);
    dv->codec.st = dv->st;
    return rc;
}

extern "C" int qtts_dev_codec_async_push(qtts_dev_t *dv, int b, int frame0, int T) {
    if (!dv || !dv->cst || b < 0 || b >= dv->nb || T < 1 || frame0 < 0 || frame0 + T > dv->max_frames + 1 ||
        (size_t)(frame0 + T) * 1920 > dv->cwav_cap)
        return -1;
    hipSetDevice(dv->device);
    CK(hipEventRecord(dv->cev, dv->st));
    CK(hipStreamWaitEvent(dv->cst, dv->cev, 0));
    const int *codes = dv->codes + (size_t)b * (dv->max_frames + 1) * dv->d.G + (size_t)frame0 * dv->d.G;
    dv->codec.st = dv->cst;
    const int n = codec_stream_push_to(&dv->codec, codes, dv->d.G, T, dv->cwav + (size_t)frame0 * 1920, false);
    dv->codec.st = dv->st;
    return n;
}

extern "C" int qtts_dev_codec_async_end(qtts_dev_t *dv, float *host_out, int frames) {
    if (!dv || !dv->cst || frames < 0 || (size_t)frames * 1920 > dv->cwav_cap) return -1;
    hipSetDevice(dv->device);
    if (frames > 0)
        CK(hipMemcpyAsync(host_out, dv->cwav, (size_t)frames * 1920 * 4, hipMemcpyDeviceToHost, dv->cst));
    CK(hipStreamSynchronize(dv->cst));
    return frames * 1920;
}

// ----------------------------------------------------------------- host-pointer stage wrappers
static int ensure_slot0(qtts_dev *dv) {
    if (dv->nb >= 1) return 0;
    qtts_gen_params_t p{0.9f, 1.0f, 1.05f, 50, 0.9f, 1.0f, 50, 0, 42};
    return qtts_dev_begin(dv, 1, 4096, 256, &p);
}

extern "C" int qtts_dev_talker_prefill_host(qtts_dev_t *dv, const float *embeds, int n, float *hidden_out) {
    if (!dv) return -1;
    hipSetDevice(dv->device);
    CKI(ensure_slot0(dv));
    if (n > dv->p_cap) {
        qtts_gen_params_t p = dv->par;
        CKI(qtts_dev_begin(dv, dv->nb, dv->max_frames > 4096 ? dv->max_frames : 4096, n, &p));
    }
    const qtts_dims_t &d = dv->d;
    for (int b = 0; b < dv->nb; ++b) dv->p_len_h[b] = b == 0 ? n : 0;
    CK(hipMemcpy(dv->prefill, embeds, (size_t)n * d.H * 4, hipMemcpyHostToDevice));
    CKI(qtts_dev_prefill(dv));
    if (hidden_out) {
        GemvArgs a = gv(dv->head, d.V, d.H, dv->x_tk, d.H, dv->logits, d.V, 1, EPI_STORE);
        a.norm_w = dv->tk_norm; a.eps = d.eps; a.xcopy = dv->tk_hid; a.ldxc = d.H; a.xcopy_normed = 1;
        CKI(qtts_gemv(a, dv->st));
        CK(hipMemcpyAsync(hidden_out, dv->tk_hid, (size_t)d.H * 4, hipMemcpyDeviceToHost, dv->st));
        CK(hipStreamSynchronize(dv->st));
    }
    return 0;
}

extern "C" int qtts_dev_talker_forward_host(qtts_dev_t *dv, const float *embed, float *logits, float *hidden_out) {
    if (!dv) return -1;
    hipSetDevice(dv->device);
    CKI(ensure_slot0(dv));
    const qtts_dims_t &d = dv->d;
    dv->nrun = 1;  // slot 0 only
    int rc = 0;
    if (hipMemcpy(dv->x_tk, embed, (size_t)d.H * 4, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) rc = talker_layers(dv);
    if (!rc) rc = talker_tail(dv);
    dv->nrun = dv->nb;
    CKI(rc);
    int kl = 0;
    CK(hipMemcpyAsync(&kl, dv->kv_len, 4, hipMemcpyDeviceToHost, dv->st));
    CK(hipStreamSynchronize(dv->st));
    kl += 1;
    CK(hipMemcpy(dv->kv_len, &kl, 4, hipMemcpyHostToDevice));
    if (logits) CK(hipMemcpy(logits, dv->logits, (size_t)d.V * 4, hipMemcpyDeviceToHost));
    if (hidden_out) CK(hipMemcpy(hidden_out, dv->tk_hid, (size_t)d.H * 4, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int qtts_dev_subtalker_host(qtts_dev_t *dv, const float *hidden, int first_code, int *out_codes) {
    if (!dv) return -1;
    hipSetDevice(dv->device);
    CKI(ensure_slot0(dv));
    const qtts_dims_t &d = dv->d;
    CK(hipStreamSynchronize(dv->st));
    CK(hipMemcpy(dv->tk_hid, hidden, (size_t)d.H * 4, hipMemcpyHostToDevice));
    int zero = 0;
    uint32_t sb = seed_bits(dv->par.seed);
    CK(hipMemcpy(dv->cur_row, &zero, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv->stopped, &zero, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv->st_rng, &sb, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv->codes, &first_code, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv->last_tok, &first_code, 4, hipMemcpyHostToDevice));
    dv->nrun = 1;
    int rc = subtalker(dv);
    dv->nrun = dv->nb;
    CKI(rc);
    CK(hipMemcpyAsync(out_codes, dv->codes, (size_t)d.G * 4, hipMemcpyDeviceToHost, dv->st));
    CK(hipStreamSynchronize(dv->st));
    return 0;
}

extern "C" float *qtts_dev_codec_decode_host(qtts_dev_t *dv, const int *codes, int T, int *out_samples) {
    if (out_samples) *out_samples = 0;
    if (!dv || T < 1) return nullptr;
    hipSetDevice(dv->device);
    if (join_prime(dv)) return nullptr;
    int *dc = nullptr;
    if (hipMalloc(&dc, (size_t)T * dv->d.cq * 4) != hipSuccess) return nullptr;
    float *r = nullptr;
    if (hipMemcpy(dc, codes, (size_t)T * dv->d.cq * 4, hipMemcpyHostToDevice) == hipSuccess)
        r = codec_decode(&dv->codec, dc, T, out_samples);
    hipFree(dc);
    return r;
}

// Several utterances' codec passes at once (a batch's slots, run_batch): job
// i decodes host_codes[i] (T[i] frames, [T][cq] time-major) when given, else
// slot slot[i]'s first T[i] generated frames.  QTTS_HIP_CODEC_LANES (default
// 8, fewer when the extra lanes' scratch would pass 16 GB) passes run side by
// side (codec_decode_many); 1 decodes them one after another with
// codec_decode.  audio[i] is malloc'd host memory.  Measured (1.7B, 128
// frames, profiles/r05lm_ab_codec_lanes.txt): a batch of 8's codec 73.4 ->
// 60.7 ms, of 16 146.8 -> 120.0 ms (the passes are mostly conv throughput).
extern "C" int qtts_dev_codec_multi(qtts_dev_t *dv, int n, const int *const *host_codes, const int *slot, const int *T,
                                    float **audio, int *samples) {
    if (!dv || n < 1 || !T || !audio || !samples) return -1;
    for (int i = 0; i < n; ++i) {
        audio[i] = nullptr;
        samples[i] = 0;
        const bool host = host_codes && host_codes[i];
        if (T[i] < 1 || (!host && (!slot || slot[i] < 0 || slot[i] >= dv->nb || T[i] > dv->max_frames + 1)))
            return -1;
    }
    hipSetDevice(dv->device);
    CKI(join_prime(dv));
    const int cq = dv->d.cq;
    // host codes staged once for every job
    size_t nh = 0;
    for (int i = 0; i < n; ++i)
        if (host_codes && host_codes[i]) nh += (size_t)T[i] * cq;
    if (nh > dv->mcodes_cap) {
        CK(hipDeviceSynchronize());
        if (dv->mcodes) CK(hipFree(dv->mcodes));
        dv->mcodes = nullptr;
        dv->mcodes_cap = 0;
        CK(hipMalloc(&dv->mcodes, nh * 4));
        dv->mcodes_cap = nh;
    }
    std::vector<const int *> dcodes(n);
    size_t ho = 0;
    for (int i = 0; i < n; ++i) {
        if (host_codes && host_codes[i]) {
            CK(hipMemcpyAsync(dv->mcodes + ho, host_codes[i], (size_t)T[i] * cq * 4, hipMemcpyHostToDevice, dv->st));
            dcodes[i] = dv->mcodes + ho;
            ho += (size_t)T[i] * cq;
        } else {
            dcodes[i] = dv->codes + (size_t)slot[i] * (dv->max_frames + 1) * dv->d.G;
        }
    }
    const char *e = getenv("QTTS_HIP_CODEC_LANES");
    int nl = e ? atoi(e) : 8;
    if (nl < 1) nl = 1;
    if (nl > 16) nl = 16;
    if (nl > n) nl = n;
    // the extra lanes' scratch within 16 GB (a 128-frame decode state is ~0.4 GB,
    // a 4096-frame one ~12 GB: long EOS utterances decode on fewer lanes)
    int tmax = 1;
    for (int i = 0; i < n; ++i) tmax = T[i] > tmax ? T[i] : tmax;
    const size_t per_lane = codec_state_bytes(&dv->codec, tmax);
    while (nl > 1 && (size_t)(nl - 1) * per_lane > ((size_t)16 << 30)) --nl;
    auto fail = [&]() {
        for (int i = 0; i < n; ++i) {
            free(audio[i]);
            audio[i] = nullptr;
            samples[i] = 0;
        }
        return -1;
    };
    if (nl == 1) {
        for (int i = 0; i < n; ++i) {
            audio[i] = codec_decode(&dv->codec, dcodes[i], T[i], &samples[i]);
            if (!audio[i]) return fail();
        }
        return 0;
    }
    while ((int)dv->clanes.size() < nl - 1) {
        hipStream_t st = nullptr;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        dv->clane_st.push_back(st);
        dv->clanes.push_back(codec_lane_new(&dv->codec, st));
    }
    std::vector<CodecModel *> lanes(nl, nullptr);
    for (int k = 1; k < nl; ++k) lanes[k] = dv->clanes[k - 1];
    // one hop of samples per frame: the decoder's total upsampling (2 x 2 x 8 x
    // 5 x 4 x 3 = 1920 for the released codec), exactly codec_decode's L / T
    const size_t hop = (size_t)dv->d.ratios[0] * dv->d.ratios[1] * dv->d.rates[0] * dv->d.rates[1] *
                       dv->d.rates[2] * dv->d.rates[3];
    std::vector<size_t> off(n);
    size_t tot = 0;
    for (int i = 0; i < n; ++i) {
        off[i] = tot;
        tot += (size_t)T[i] * hop;
    }
    if (tot > dv->mwav_cap) {
        CK(hipDeviceSynchronize());
        if (dv->mwav) CK(hipFree(dv->mwav));
        dv->mwav = nullptr;
        dv->mwav_cap = 0;
        CK(hipMalloc(&dv->mwav, tot * 4));
        dv->mwav_cap = tot;
    }
    std::vector<int> ns(n, 0);
    if (codec_decode_many(&dv->codec, lanes.data(), nl, n, dcodes.data(), T, dv->mwav, off.data(), ns.data()))
        return fail();
    for (int i = 0; i < n; ++i) {
        if ((size_t)ns[i] != (size_t)T[i] * hop) return fail();
        audio[i] = (float *)malloc((size_t)ns[i] * sizeof(float));
        if (!audio[i] ||
            hipMemcpy(audio[i], dv->mwav + off[i], (size_t)ns[i] * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return fail();
        samples[i] = ns[i];
    }
    return 0;
}

// ----------------------------------------------------------------- kernel-level C-ABI
extern "C" int qtts_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int qtts_hip_sync(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : -1; }

// batch >= 2 goes to the matrix-core kernel (as prefill does), else the GEMV
static int matvec_any(const GemvArgs &a, hipStream_t st) {
    static float *inv = nullptr;   // per-row 1/rms scratch of this test-level entry
    if (a.nb >= 2) {
        if (!inv && hipMalloc(&inv, 64 * sizeof(float)) != hipSuccess) return -1;
        const int rc = qtts_mgemm(a, inv, st);
        if (rc != 1) return rc;
    }
    return qtts_gemv(a, st);
}

extern "C" int qtts_hip_matvec_bf16(float *out, const uint16_t *A, const float *x, int rows, int cols, int batch,
                                    void *stream) {
    GemvArgs a = gv(A, rows, cols, x, cols, out, rows, batch, EPI_STORE);
    return matvec_any(a, (hipStream_t)stream);
}

extern "C" int qtts_hip_rmsnorm_matvec_bf16(float *out, const uint16_t *A, const float *x, const float *w, float eps,
                                            int rows, int cols, int batch, void *stream) {
    GemvArgs a = gv(A, rows, cols, x, cols, out, rows, batch, EPI_STORE);
    a.norm_w = w; a.eps = eps;
    return matvec_any(a, (hipStream_t)stream);
}

// the decode dispatcher itself (qtts_gemv): batch 1 -> k_gemv1, 2..16 ->
// k_gemvm (matrix cores) where covered, else k_gemv
extern "C" int qtts_hip_decode_matvec_bf16(float *out, const uint16_t *A, const float *x, const float *w, float eps,
                                           int rows, int cols, int batch, void *stream) {
    GemvArgs a = gv(A, rows, cols, x, cols, out, rows, batch, EPI_STORE);
    a.norm_w = w; a.eps = eps;
    return qtts_gemv(a, (hipStream_t)stream);
}

extern "C" int qtts_hip_resident_matvec_bf16(float *out, const uint16_t *A, const float *x, const float *w, float eps,
                                             int rows, int cols, int epi, void *stream) {
    if (epi != EPI_STORE && epi != EPI_RESID && epi != EPI_SWIGLU) return -1;
    GemvArgs a = gv(A, rows, cols, x, cols, out, epi == EPI_SWIGLU ? rows / 2 : rows, 1, epi);
    a.norm_w = w; a.eps = eps; a.nt = 0;
    return qtts_gemv(a, (hipStream_t)stream);
}

extern "C" int qtts_hip_sample_top_k(int *out, const float *logits, int vocab, int top_k, float top_p, float temp,
                                     uint32_t *rng_bits, int batch, void *stream) {
    SampArgs s;
    s.logits = logits; s.ld = vocab; s.n = vocab; s.nb = batch; s.top_k = top_k; s.top_p = top_p; s.temp = temp;
    s.mode = 0; s.st_rng = rng_bits; s.out_tok = out;
    return qtts_sample(s, (hipStream_t)stream);
}

// One frame run eagerly with an event pair around every kernel launch on the
// context stream; returns the number of kernels, fills kind/bytes/ms.
extern "C" int qtts_dev_profile_frame(qtts_dev_t *dv, int step, int max, int *kind, double *bytes, float *ms,
                                      char *names) {
    if (!dv || dv->nb < 1) return -1;
    hipSetDevice(dv->device);
    CK(hipStreamSynchronize(dv->st));
    dv->prof.clear();
    dv->profiling = true;
    int rc = record_frame(dv, step > 0);
    dv->profiling = false;
    CK(hipStreamSynchronize(dv->st));
    int n = 0;
    for (auto &p : dv->prof) {
        float t = 0.f;
        hipEventElapsedTime(&t, p.a, p.b);
        if (n < max) {
            kind[n] = p.kind; bytes[n] = p.bytes; ms[n] = t;
            if (names) snprintf(names + (size_t)n * 64, 64, "%s", p.name ? p.name : "");
        }
        ++n;
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    dv->prof.clear();
    return rc ? -1 : n;
}
