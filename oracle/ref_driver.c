/*
 * ref_driver.c - test-only driver linked against the UNMODIFIED reference
 * sources (/root/reference/c/*.c) to produce oracle/_ref/libqtts_ref.so.
 *
 * TEST INFRASTRUCTURE ONLY: nothing in the product links or loads this.
 *
 * It adds two things the reference API does not expose:
 *   1. parameter setters for the public ctx fields main.c pokes
 *      (c/main.c:214-223), so Python (ctypes) need not mirror the struct;
 *   2. recording hooks, installed with `ld --wrap` (see oracle/Makefile) on
 *      the cross-object calls the reference makes:
 *        kernel_sample_top_k     (called from c/qwen_tts.c:1312,1318 and
 *                                 c/qwen_tts_talker.c:719,730)
 *        qwen_tts_subtalker_generate (c/qwen_tts.c:1336)
 *        qwen_tts_codec_decode   (c/qwen_tts.c:1421)
 *      Every sampler call (logits in, rng state in/out, id out), every
 *      sub-talker call (talker hidden, first code, 16 codes) and the codes
 *      handed to the codec are appended to in-memory logs the tests read.
 */
#include "qwen_tts.h"
#include "qwen_tts_kernels.h"
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

/* ---- recording state ---- */
typedef struct {
    int n, cap;
    int *vocab, *top_k, *result;
    float *top_p, *temp;
    uint32_t *rng_in, *rng_out;
    float *logits;          /* concatenated, variable length */
    size_t logit_n, logit_cap;
} samp_log_t;

static int g_record = 0;
static samp_log_t g_s;
static float *g_st_hidden = NULL; static int g_st_n = 0, g_st_cap = 0, g_st_dim = 0;
static int *g_st_codes = NULL;
static int *g_codec_codes = NULL; static int g_codec_T = 0, g_codec_Q = 0;

void ref_record(int on) {
    g_record = on;
    g_s.n = 0; g_s.logit_n = 0;
    g_st_n = 0;
    g_codec_T = 0;
}

static void grow_samp(void) {
    if (g_s.n < g_s.cap) return;
    int nc = g_s.cap ? g_s.cap * 2 : 256;
    g_s.vocab = realloc(g_s.vocab, nc * sizeof(int));
    g_s.top_k = realloc(g_s.top_k, nc * sizeof(int));
    g_s.result = realloc(g_s.result, nc * sizeof(int));
    g_s.top_p = realloc(g_s.top_p, nc * sizeof(float));
    g_s.temp = realloc(g_s.temp, nc * sizeof(float));
    g_s.rng_in = realloc(g_s.rng_in, nc * sizeof(uint32_t));
    g_s.rng_out = realloc(g_s.rng_out, nc * sizeof(uint32_t));
    g_s.cap = nc;
}

int __real_kernel_sample_top_k(const float *logits, int vocab_size, int top_k,
                               float top_p, float temperature, float *rng_state);
int __wrap_kernel_sample_top_k(const float *logits, int vocab_size, int top_k,
                               float top_p, float temperature, float *rng_state) {
    uint32_t rin; memcpy(&rin, rng_state, 4);
    int r = __real_kernel_sample_top_k(logits, vocab_size, top_k, top_p, temperature, rng_state);
    if (g_record) {
        grow_samp();
        int i = g_s.n++;
        g_s.vocab[i] = vocab_size; g_s.top_k[i] = top_k; g_s.result[i] = r;
        g_s.top_p[i] = top_p; g_s.temp[i] = temperature; g_s.rng_in[i] = rin;
        memcpy(&g_s.rng_out[i], rng_state, 4);
        if (g_s.logit_n + vocab_size > g_s.logit_cap) {
            size_t nc = g_s.logit_cap ? g_s.logit_cap * 2 : (1u << 20);
            while (nc < g_s.logit_n + vocab_size) nc *= 2;
            g_s.logits = realloc(g_s.logits, nc * sizeof(float));
            g_s.logit_cap = nc;
        }
        memcpy(g_s.logits + g_s.logit_n, logits, vocab_size * sizeof(float));
        g_s.logit_n += vocab_size;
    }
    return r;
}

void __real_qwen_tts_subtalker_generate(qwen_tts_ctx_t *ctx, const float *talker_hidden,
                                        int first_code, int *out_codes);
void __wrap_qwen_tts_subtalker_generate(qwen_tts_ctx_t *ctx, const float *talker_hidden,
                                        int first_code, int *out_codes) {
    __real_qwen_tts_subtalker_generate(ctx, talker_hidden, first_code, out_codes);
    if (g_record) {
        int H = ctx->config.talker_hidden, G = ctx->config.num_code_groups;
        if (g_st_n >= g_st_cap) {
            g_st_cap = g_st_cap ? g_st_cap * 2 : 256;
            g_st_hidden = realloc(g_st_hidden, (size_t)g_st_cap * H * sizeof(float));
            g_st_codes = realloc(g_st_codes, (size_t)g_st_cap * G * sizeof(int));
        }
        g_st_dim = H;
        memcpy(g_st_hidden + (size_t)g_st_n * H, talker_hidden, H * sizeof(float));
        memcpy(g_st_codes + (size_t)g_st_n * G, out_codes, G * sizeof(int));
        g_st_n++;
    }
}

float *__real_qwen_tts_codec_decode(qwen_tts_ctx_t *ctx, const int *codes, int T, int *n);
float *__wrap_qwen_tts_codec_decode(qwen_tts_ctx_t *ctx, const int *codes, int T, int *n) {
    if (g_record) {
        int Q = ctx->config.codec_num_quantizers;
        g_codec_codes = realloc(g_codec_codes, (size_t)T * Q * sizeof(int));
        memcpy(g_codec_codes, codes, (size_t)T * Q * sizeof(int));
        g_codec_T = T; g_codec_Q = Q;
    }
    return __real_qwen_tts_codec_decode(ctx, codes, T, n);
}

/* ---- log getters ---- */
int ref_samp_count(void) { return g_s.n; }
void ref_samp_get(int i, int *meta /*[vocab,top_k,result]*/, float *fmeta /*[top_p,temp]*/,
                  uint32_t *rng /*[in,out]*/, size_t *logit_off) {
    meta[0] = g_s.vocab[i]; meta[1] = g_s.top_k[i]; meta[2] = g_s.result[i];
    fmeta[0] = g_s.top_p[i]; fmeta[1] = g_s.temp[i];
    rng[0] = g_s.rng_in[i]; rng[1] = g_s.rng_out[i];
    size_t off = 0;
    for (int j = 0; j < i; j++) off += g_s.vocab[j];
    *logit_off = off;
}
const float *ref_samp_logits(void) { return g_s.logits; }
int ref_st_count(void) { return g_st_n; }
const float *ref_st_hidden(void) { return g_st_hidden; }
const int *ref_st_codes(void) { return g_st_codes; }
int ref_codec_T(void) { return g_codec_T; }
const int *ref_codec_codes(void) { return g_codec_codes; }

/* ---- ctx helpers ---- */
void ref_set_verbose(int v) { qwen_tts_verbose = v; }
void ref_set_params(qwen_tts_ctx_t *ctx, float temperature, int top_k, float top_p,
                    float rep, int max_tokens, int fixed, int seed,
                    float st_temp, int st_top_k, float st_top_p) {
    ctx->temperature = temperature; ctx->top_k = top_k; ctx->top_p = top_p;
    ctx->repetition_penalty = rep; ctx->max_new_tokens = max_tokens;
    ctx->fixed_codec_tokens = fixed; ctx->sample_seed = seed;
    ctx->subtalker_temperature = st_temp; ctx->subtalker_top_k = st_top_k;
    ctx->subtalker_top_p = st_top_p;
}
void ref_get_perf(qwen_tts_ctx_t *ctx, double *out /*[total,talker,codec,tokens]*/) {
    out[0] = ctx->perf_total_ms; out[1] = ctx->perf_talker_ms;
    out[2] = ctx->perf_codec_ms; out[3] = ctx->perf_codec_tokens;
}
int ref_kv_len(qwen_tts_ctx_t *ctx) { return ctx->talker_kv_len; }
void ref_set_kv_len(qwen_tts_ctx_t *ctx, int n) { ctx->talker_kv_len = n; }
const float *ref_tk_x(qwen_tts_ctx_t *ctx) { return ctx->tk_x; }
void ref_free(void *p) { free(p); }
