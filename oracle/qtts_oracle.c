/*
 * qtts_oracle.c - CPU RESTATEMENT of the reference hot path (TEST ORACLE).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (qwen3-tts-c_amd/) never links, loads or falls back to it.
 *
 * It restates, in my own structure, the arithmetic of the reference C CPU
 * path (the oracle named by BASELINE.json north_star).  Every function cites
 * the reference file:line it follows.  Floating-point operations are kept in
 * the reference's order (sequential fp32 sums, -ffp-contract=off) so that
 * this restatement reproduces the reference's scalar build BIT-EXACTLY; that
 * is how it is pinned (tests/test_oracle.py against the tests/golden fixtures made
 * from oracle/_ref by tests/golden/make_golden.py).
 *
 * Weights are handed in by the caller (Python reads the safetensors with the
 * safe loader and passes named pointers), so this file holds compute only.
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* model description                                                   */
/* ------------------------------------------------------------------ */
enum {  /* integer dims, order shared with tests/oracle_py.py */
    D_H, D_I, D_L, D_NH, D_KV, D_HD, D_TH, D_TV, D_V, D_G,
    D_HS, D_IS, D_LS, D_NHS, D_KVS, D_HDS, D_VS,
    D_MR0, D_MR1, D_MR2,
    D_CQ, D_CCB, D_CCBDIM, D_CHID, D_CLAT, D_CLAYERS, D_CHEADS, D_CKV, D_CINTER,
    D_CWIN, D_CDEC, D_UR0, D_UR1, D_UR2, D_UR3, D_UP0, D_UP1,
    D_PAD, D_BOS, D_EOS, D_THINK, D_NOTHINK, D_THINK_BOS, D_THINK_EOS,
    D_COUNT
};
enum { F_EPS, F_THETA, F_CEPS, F_COUNT };

#define MAXT 1024
typedef struct { char name[112]; const void *p; int bf16; long n; } tens_t;

typedef struct {
    int d[D_COUNT];
    float f[F_COUNT];
    tens_t t[MAXT];
    int nt;
    /* derived (owned) */
    float *cb_emb[32];                 /* codebooks = esum / max(usage,1e-5) */
    float *snake_a[64], *snake_b[64];  /* pre-exponentiated copies */
    int n_snake;
    /* talker state */
    float *kv_k, *kv_v; int kv_len, kv_max;
    float *tk_x;                       /* post-norm hidden of the last token */
    /* draw trace (tests/divergence.py): the sampler inputs of ONE draw of a
     * generation -- frame tr_f, group tr_g (0: the talker's code-0 draw) */
    int tr_f, tr_g, tr_done, tr_frame, tr_n, tr_xn, tr_result;
    float tr_rng;
    float *tr_logits, *tr_x;           /* the logits handed to the sampler, the head's input row */
} orc_t;

static float bf(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

static const tens_t *find(const orc_t *m, const char *name) {
    for (int i = 0; i < m->nt; i++) if (!strcmp(m->t[i].name, name)) return &m->t[i];
    return NULL;
}
static const tens_t *findf(const orc_t *m, const char *fmt, int a, int b) {
    char nm[160]; snprintf(nm, sizeof nm, fmt, a, b);
    return find(m, nm);
}
/* norms/biases are stored BF16 by HF checkpoints and read as f32 copies
 * (LOAD_F32, c/qwen_tts.c:364); element getter handles both */
static float el(const tens_t *t, long i) {
    return t->bf16 ? bf(((const uint16_t *)t->p)[i]) : ((const float *)t->p)[i];
}
static float *f32copy(const tens_t *t) {
    float *o = malloc(t->n * sizeof(float));
    for (long i = 0; i < t->n; i++) o[i] = el(t, i);
    return o;
}

API orc_t *orc_create(const int *dims, const float *fp) {
    orc_t *m = calloc(1, sizeof(orc_t));
    m->tr_f = -1;
    memcpy(m->d, dims, sizeof(m->d));
    memcpy(m->f, fp, sizeof(m->f));
    return m;
}
API int orc_set_tensor(orc_t *m, const char *name, const void *p, int is_bf16, long n) {
    if (m->nt >= MAXT) return -1;
    tens_t *t = &m->t[m->nt++];
    snprintf(t->name, sizeof t->name, "%s", name);
    t->p = p; t->bf16 = is_bf16; t->n = n;
    return 0;
}
API void orc_free(orc_t *m) {
    if (!m) return;
    for (int i = 0; i < 32; i++) free(m->cb_emb[i]);
    for (int i = 0; i < m->n_snake; i++) { free(m->snake_a[i]); free(m->snake_b[i]); }
    free(m->kv_k); free(m->kv_v); free(m->tk_x);
    free(m->tr_logits); free(m->tr_x);
    free(m);
}

/* ------------------------------------------------------------------ */
/* kernels (c/qwen_tts_kernels.c)                                      */
/* ------------------------------------------------------------------ */

/* K.c:27-39: inv = 1/sqrtf(mean(x^2)+eps); y = x*inv*w */
API void orc_rmsnorm(float *y, const float *x, const float *w, int n, float eps) {
    float ss = 0.0f;
    for (int i = 0; i < n; i++) ss += x[i] * x[i];
    float inv = 1.0f / sqrtf(ss / (float)n + eps);
    for (int i = 0; i < n; i++) y[i] = x[i] * inv * w[i];
}
static void rmsnorm_t(float *y, const float *x, const tens_t *w, int n, float eps) {
    float ss = 0.0f;
    for (int i = 0; i < n; i++) ss += x[i] * x[i];
    float inv = 1.0f / sqrtf(ss / (float)n + eps);
    for (int i = 0; i < n; i++) y[i] = x[i] * inv * el(w, i);
}

/* K.c:45-58 (two-pass mean/var) */
static void layernorm_t(float *y, const float *x, const tens_t *w, const tens_t *b, int n, float eps) {
    float mean = 0.0f;
    for (int i = 0; i < n; i++) mean += x[i];
    mean /= (float)n;
    float var = 0.0f;
    for (int i = 0; i < n; i++) { float d = x[i] - mean; var += d * d; }
    var /= (float)n;
    float inv = 1.0f / sqrtf(var + eps);
    for (int i = 0; i < n; i++) {
        float v = (x[i] - mean) * inv;
        v *= el(w, i);
        y[i] = v + el(b, i);
    }
}

/* K.c:139-148 (scalar path): out[r] = sum_c bf16(A[r,c]) * x[c], c ascending */
API void orc_matvec_bf16(float *out, const uint16_t *A, const float *x, int rows, int cols) {
#pragma omp parallel for schedule(static)
    for (int r = 0; r < rows; r++) {
        const uint16_t *a = A + (size_t)r * cols;
        float s = 0.0f;
        for (int c = 0; c < cols; c++) s += bf(a[c]) * x[c];
        out[r] = s;
    }
}
static void mv_t(float *out, const tens_t *A, const float *x, int rows, int cols) {
    if (A->bf16) { orc_matvec_bf16(out, A->p, x, rows, cols); return; }
    const float *a0 = A->p;
#pragma omp parallel for schedule(static)
    for (int r = 0; r < rows; r++) {
        const float *a = a0 + (size_t)r * cols;
        float s = 0.0f;
        for (int c = 0; c < cols; c++) s += a[c] * x[c];
        out[r] = s;
    }
}
/* K.c:168-207 (scalar): C[m,n] = sum_k A[m,k] * B[n,k] */
static void mm_t(float *C, const float *A, const tens_t *B, int M, int N, int K) {
    for (int i = 0; i < M; i++) mv_t(C + (size_t)i * N, B, A + (size_t)i * K, N, K);
}
static void add_bias_t(float *y, const tens_t *b, int n) {
    if (!b) return;
    for (int i = 0; i < n; i++) y[i] += el(b, i);
}
/* K.c:239-249 */
static float silu(float g) { return g / (1.0f + expf(-g)); }
static float gelu_tanh(float v) {
    return 0.5f * v * (1.0f + tanhf(0.7978845608028654f * (v + 0.044715f * v * v * v)));
}
/* K.c:371-378 */
API void orc_softmax(float *x, int n) {
    float mx = x[0];
    for (int i = 1; i < n; i++) if (x[i] > mx) mx = x[i];
    float s = 0.0f;
    for (int i = 0; i < n; i++) { x[i] = expf(x[i] - mx); s += x[i]; }
    float inv = 1.0f / s;
    for (int i = 0; i < n; i++) x[i] *= inv;
}

/* ---- sampling (K.c:384-558, Q.c:1302-1321) ---- */
/* xorshift32 over the bits of a float state (K.c:384-393) */
API float orc_rand_uniform(float *state) {
    uint32_t s; memcpy(&s, state, 4);
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    memcpy(state, &s, 4);
    return (float)(s & 0x7FFFFFFF) / (float)0x7FFFFFFF;
}
typedef struct { float v; int i; } vi_t;
/* descending value, ties: lower index first (== the reference's strict '>'
 * insertion, K.c:437-449) */
static int cmp_desc(const void *a, const void *b) {
    const vi_t *x = a, *y = b;
    if (x->v > y->v) return -1;
    if (x->v < y->v) return 1;
    return (x->i > y->i) - (x->i < y->i);
}
/* K.c:407-558 restated: fast top-k path via a full stable sort instead of
 * an insertion list (same selected set and order), slow path as written. */
API int orc_sample(const float *logits, int n, int top_k, float top_p, float temperature, float *rng) {
    if (temperature <= 0.0f) temperature = 1e-5f;
    if (top_p >= 1.0f && top_k > 0 && top_k < n) {
        vi_t *a = malloc((size_t)n * sizeof(vi_t));
        int m = 0;
        for (int i = 0; i < n; i++) {
            float v = logits[i] / temperature;
            if (!(v > -FLT_MAX)) continue;           /* never enters the list */
            a[m].v = v; a[m].i = i; m++;
        }
        qsort(a, m, sizeof(vi_t), cmp_desc);
        int k = top_k < m ? top_k : m;               /* unfilled slots keep idx -1, p = 0 */
        float mx = k > 0 ? a[0].v : 0.0f, sum = 0.0f;
        float *p = malloc((size_t)(k > 0 ? k : 1) * sizeof(float));
        for (int j = 0; j < k; j++) { p[j] = expf(a[j].v - mx); sum += p[j]; }
        int out = 0;
        if (sum > 0.0f) {
            float r = orc_rand_uniform(rng) * sum, c = 0.0f;
            for (int j = 0; j < k; j++) { c += p[j]; if (c >= r) { out = a[j].i; break; } }
        } else if (k > 0) {
            out = a[0].i;
        }
        free(p); free(a);
        return out;
    }
    /* full-softmax path */
    float *pr = malloc((size_t)n * sizeof(float));
    for (int i = 0; i < n; i++) pr[i] = logits[i] / temperature;
    orc_softmax(pr, n);
    if (top_k > 0 && top_k < n) {                    /* keep p >= k-th largest (K.c:494-511) */
        vi_t *a = malloc((size_t)n * sizeof(vi_t));
        for (int i = 0; i < n; i++) { a[i].v = pr[i]; a[i].i = i; }
        qsort(a, n, sizeof(vi_t), cmp_desc);
        float thr = a[top_k - 1].v;
        free(a);
        for (int i = 0; i < n; i++) if (pr[i] < thr) pr[i] = 0.0f;
    }
    if (top_p < 1.0f) {                              /* nucleus over a stable desc order (K.c:514-537) */
        vi_t *a = malloc((size_t)n * sizeof(vi_t));
        for (int i = 0; i < n; i++) { a[i].v = pr[i]; a[i].i = i; }
        qsort(a, n, sizeof(vi_t), cmp_desc);
        float c = 0.0f; int cut = n;
        for (int i = 0; i < n; i++) { c += a[i].v; if (c >= top_p) { cut = i + 1; break; } }
        for (int i = cut; i < n; i++) pr[a[i].i] = 0.0f;
        free(a);
    }
    float s = 0.0f;
    for (int i = 0; i < n; i++) s += pr[i];
    if (s > 0.0f) { float inv = 1.0f / s; for (int i = 0; i < n; i++) pr[i] *= inv; }
    float r = orc_rand_uniform(rng), c = 0.0f;
    int out = 0;
    for (int i = 0; i < n; i++) { c += pr[i]; if (c >= r) { out = i; break; } }
    free(pr);
    return out;
}

/* K.c:395-405: applied once per OCCURRENCE in the history */
API void orc_rep_penalty(float *logits, const int *hist, int n_hist, int vocab, float pen) {
    if (pen == 1.0f) return;
    for (int i = 0; i < n_hist; i++) {
        int t = hist[i];
        if (t < 0 || t >= vocab) continue;
        if (logits[t] > 0) logits[t] /= pen; else logits[t] *= pen;
    }
}

/* ---- RoPE (T.c:76-113, K.c:564-587) ---- */
static void rope_row(float *cs, float *sn, int pos, int hd, float theta) {
    int half = hd / 2;
    for (int i = 0; i < half; i++) {
        float freq = 1.0f / powf(theta, (float)(2 * i) / (float)hd);
        float ang = (float)pos * freq;
        cs[i] = cs[i + half] = cosf(ang);
        sn[i] = sn[i + half] = sinf(ang);
    }
}
/* rotate-half with a merged cos/sin row; for text all three M-RoPE streams
 * carry the same position, so the merge (T.c:158-171) selects identical
 * values and reduces to this. */
static void rope_heads(float *v, int nh, int hd, const float *cs, const float *sn) {
    int half = hd / 2;
    for (int h = 0; h < nh; h++) {
        float *q = v + h * hd;
        for (int i = 0; i < half; i++) {
            float a = q[i], b = q[i + half];
            q[i] = a * cs[i] - b * sn[i];
            q[i + half] = b * cs[i + half] + a * sn[i + half];
        }
    }
}
API void orc_rope_table(float *cs, float *sn, int npos, int hd, float theta) {
    for (int p = 0; p < npos; p++) rope_row(cs + (size_t)p * hd, sn + (size_t)p * hd, p, hd, theta);
}

/* ---- convolutions (K.c:659-972, scalar paths) ---- */
/* out[oc,t] = b + sum_{ic in group} sum_k w[oc,ic,k] * in[ic, t-(K-1)d+kd]  (left zero pad) */
API void orc_conv1d(float *out, const float *in, const float *w, const float *b,
                    int ci, int co, int K, int L, int d, int groups) {
    int cpg = ci / groups, opg = co / groups, pad = (K - 1) * d;
#pragma omp parallel for schedule(static)
    for (int oc = 0; oc < co; oc++) {
        int g = oc / opg;
        for (int t = 0; t < L; t++) {
            float acc = b ? b[oc] : 0.0f;
            for (int j = 0; j < cpg; j++) {
                const float *x = in + (size_t)(g * cpg + j) * L;
                const float *wk = w + ((size_t)oc * cpg + j) * K;
                for (int k = 0; k < K; k++) {
                    int ti = t - pad + k * d;
                    if (ti >= 0) acc += wk[k] * x[ti];
                }
            }
            out[(size_t)oc * L + t] = acc;
        }
    }
}
/* weight [ci, co, K]; output length L*s (right tail K-s dropped) */
API void orc_tconv1d(float *out, const float *in, const float *w, const float *b,
                     int ci, int co, int K, int s, int L) {
    int Lo = L * s;
#pragma omp parallel for schedule(static)
    for (int oc = 0; oc < co; oc++) {
        for (int ot = 0; ot < Lo; ot++) {
            float acc = b ? b[oc] : 0.0f;
            int t_hi = ot / s, t_lo = ot - (K - 1) < 0 ? 0 : (ot - (K - 1) + s - 1) / s;
            if (t_hi > L - 1) t_hi = L - 1;
            for (int ic = 0; ic < ci; ic++) {
                const float *x = in + (size_t)ic * L;
                const float *wr = w + ((size_t)ic * co + oc) * K;
                for (int t = t_lo; t <= t_hi; t++) acc += x[t] * wr[ot - t * s];
            }
            out[(size_t)oc * Lo + ot] = acc;
        }
    }
}
/* K.c:302-310 with pre-exponentiated a, inv_b (Q.c:596-602) */
API void orc_snake(float *y, const float *x, const float *a, const float *ib, int C, int L) {
#pragma omp parallel for schedule(static)
    for (int c = 0; c < C; c++)
        for (int t = 0; t < L; t++) {
            size_t i = (size_t)c * L + t;
            float s = sinf(x[i] * a[c]);
            y[i] = x[i] + ib[c] * s * s;
        }
}

/* ------------------------------------------------------------------ */
/* derived parameters (Q.c:577-602)                                    */
/* ------------------------------------------------------------------ */
static float *snake_a_of(orc_t *m, const tens_t *a, const tens_t *b, float **ib_out) {
    float *A = f32copy(a), *B = f32copy(b);
    for (long i = 0; i < a->n; i++) { A[i] = expf(A[i]); B[i] = 1.0f / (expf(B[i]) + 1e-9f); }
    m->snake_a[m->n_snake] = A; m->snake_b[m->n_snake] = B; m->n_snake++;
    *ib_out = B;
    return A;
}
static const float *codebook(orc_t *m, int q) {
    if (m->cb_emb[q]) return m->cb_emb[q];
    int CB = m->d[D_CCB], vq = m->d[D_CCBDIM] / 2;
    const tens_t *u, *e;
    if (q == 0) {
        u = find(m, "decoder.quantizer.rvq_first.vq.layers.0._codebook.cluster_usage");
        e = find(m, "decoder.quantizer.rvq_first.vq.layers.0._codebook.embedding_sum");
    } else {
        u = findf(m, "decoder.quantizer.rvq_rest.vq.layers.%d._codebook.cluster_usage", q - 1, 0);
        e = findf(m, "decoder.quantizer.rvq_rest.vq.layers.%d._codebook.embedding_sum", q - 1, 0);
    }
    float *o = malloc((size_t)CB * vq * sizeof(float));
    for (int c = 0; c < CB; c++) {
        float us = el(u, c);
        if (us < 1e-5f) us = 1e-5f;
        float inv = 1.0f / us;
        for (int k = 0; k < vq; k++) o[(size_t)c * vq + k] = el(e, (long)c * vq + k) * inv;
    }
    m->cb_emb[q] = o;
    return o;
}

/* ------------------------------------------------------------------ */
/* talker (c/qwen_tts_talker.c)                                        */
/* ------------------------------------------------------------------ */
typedef struct {
    const tens_t *wq, *wk, *wv, *wo, *qn, *kn, *in, *post, *gate, *up, *down;
} lw_t;
static void layer_w(const orc_t *m, lw_t *w, const char *pre, int i) {
    char b[160];
#define G(f, s) snprintf(b, sizeof b, "%s.layers.%d." s, pre, i); w->f = find(m, b);
    G(wq, "self_attn.q_proj.weight") G(wk, "self_attn.k_proj.weight")
    G(wv, "self_attn.v_proj.weight") G(wo, "self_attn.o_proj.weight")
    G(qn, "self_attn.q_norm.weight") G(kn, "self_attn.k_norm.weight")
    G(in, "input_layernorm.weight") G(post, "post_attention_layernorm.weight")
    G(gate, "mlp.gate_proj.weight") G(up, "mlp.up_proj.weight") G(down, "mlp.down_proj.weight")
#undef G
}

/* One decoder layer over `n` tokens at positions pos0.. with a KV cache of
 * row stride kvs (T.c:119-248 single token, T.c:320-454 prefill; the two are
 * the same arithmetic per token). */
static void dec_layer(const lw_t *w, float *x, int n, int pos0, int H, int NH, int KV, int HD, int I,
                      float eps, float theta, float *kk, float *vv, int mrope_full) {
    int qd = NH * HD, kd = KV * HD, gph = NH / KV;
    float *xn = malloc((size_t)n * H * sizeof(float));
    float *q = malloc((size_t)n * qd * sizeof(float));
    float *att = calloc((size_t)n * qd, sizeof(float));
    float *tmp = malloc((size_t)n * (H > I ? H : I) * sizeof(float));
    float *gt = malloc((size_t)n * I * sizeof(float)), *ut = malloc((size_t)n * I * sizeof(float));
    float *sc = malloc((size_t)(pos0 + n) * sizeof(float));
    float *cs = malloc(HD * sizeof(float)), *sn = malloc(HD * sizeof(float));
    (void)mrope_full;
    for (int t = 0; t < n; t++) rmsnorm_t(xn + (size_t)t * H, x + (size_t)t * H, w->in, H, eps);
    for (int t = 0; t < n; t++) {
        int p = pos0 + t;
        float *qt = q + (size_t)t * qd, *kt = kk + (size_t)p * kd, *vt = vv + (size_t)p * kd;
        mv_t(qt, w->wq, xn + (size_t)t * H, qd, H);
        mv_t(kt, w->wk, xn + (size_t)t * H, kd, H);
        mv_t(vt, w->wv, xn + (size_t)t * H, kd, H);
        for (int h = 0; h < NH; h++) rmsnorm_t(qt + h * HD, qt + h * HD, w->qn, HD, eps);
        for (int h = 0; h < KV; h++) rmsnorm_t(kt + h * HD, kt + h * HD, w->kn, HD, eps);
        rope_row(cs, sn, p, HD, theta);
        rope_heads(qt, NH, HD, cs, sn);
        rope_heads(kt, KV, HD, cs, sn);
    }
    float scale = 1.0f / sqrtf((float)HD);
    for (int t = 0; t < n; t++) {
        int p = pos0 + t;
        for (int h = 0; h < NH; h++) {
            const float *qh = q + (size_t)t * qd + h * HD;
            int kh = h / gph;
            for (int j = 0; j <= p; j++) {
                const float *kr = kk + (size_t)j * kd + kh * HD;
                float s = 0.0f;
                for (int e = 0; e < HD; e++) s += qh[e] * kr[e];
                sc[j] = s * scale;
            }
            orc_softmax(sc, p + 1);
            float *o = att + (size_t)t * qd + h * HD;
            for (int j = 0; j <= p; j++) {
                const float *vr = vv + (size_t)j * kd + kh * HD;
                for (int e = 0; e < HD; e++) o[e] += sc[j] * vr[e];
            }
        }
    }
    for (int t = 0; t < n; t++) {
        float *xt = x + (size_t)t * H;
        mv_t(tmp, w->wo, att + (size_t)t * qd, H, qd);
        for (int i = 0; i < H; i++) xt[i] += tmp[i];
        rmsnorm_t(xn + (size_t)t * H, xt, w->post, H, eps);
        mv_t(gt, w->gate, xn + (size_t)t * H, I, H);
        mv_t(ut, w->up, xn + (size_t)t * H, I, H);
        for (int i = 0; i < I; i++) gt[i] = silu(gt[i]) * ut[i];
        mv_t(tmp, w->down, gt, H, I);
        for (int i = 0; i < H; i++) xt[i] += tmp[i];
    }
    free(xn); free(q); free(att); free(tmp); free(gt); free(ut); free(sc); free(cs); free(sn);
}

static void ensure_kv(orc_t *m, int need) {
    int L = m->d[D_L], kd = m->d[D_KV] * m->d[D_HD];
    if (m->kv_max >= need) return;
    int nm = need + 512;
    float *nk = calloc((size_t)L * nm * kd, sizeof(float)), *nv = calloc((size_t)L * nm * kd, sizeof(float));
    for (int l = 0; l < L && m->kv_k; l++) {
        memcpy(nk + (size_t)l * nm * kd, m->kv_k + (size_t)l * m->kv_max * kd, (size_t)m->kv_len * kd * 4);
        memcpy(nv + (size_t)l * nm * kd, m->kv_v + (size_t)l * m->kv_max * kd, (size_t)m->kv_len * kd * 4);
    }
    free(m->kv_k); free(m->kv_v);
    m->kv_k = nk; m->kv_v = nv; m->kv_max = nm;
}

static void talker_run(orc_t *m, float *x, int n) {
    int H = m->d[D_H], L = m->d[D_L], kd = m->d[D_KV] * m->d[D_HD];
    ensure_kv(m, m->kv_len + n);
    for (int l = 0; l < L; l++) {
        lw_t w; layer_w(m, &w, "talker.model", l);
        dec_layer(&w, x, n, m->kv_len, H, m->d[D_NH], m->d[D_KV], m->d[D_HD], m->d[D_I],
                  m->f[F_EPS], m->f[F_THETA],
                  m->kv_k + (size_t)l * m->kv_max * kd, m->kv_v + (size_t)l * m->kv_max * kd, 1);
    }
    const tens_t *nw = find(m, "talker.model.norm.weight");
    for (int t = 0; t < n; t++) rmsnorm_t(x + (size_t)t * H, x + (size_t)t * H, nw, H, m->f[F_EPS]);
    if (!m->tk_x) m->tk_x = malloc(H * sizeof(float));
    memcpy(m->tk_x, x + (size_t)(n - 1) * H, H * sizeof(float));
    m->kv_len += n;
}

/* T.c:254-472: prefill from position 0; hidden_out = post-norm last hidden */
API void orc_talker_prefill(orc_t *m, const float *embeds, int n, float *hidden_out) {
    int H = m->d[D_H];
    float *x = malloc((size_t)n * H * sizeof(float));
    memcpy(x, embeds, (size_t)n * H * sizeof(float));
    m->kv_len = 0;
    talker_run(m, x, n);
    if (hidden_out) memcpy(hidden_out, m->tk_x, H * sizeof(float));
    free(x);
}
/* T.c:478-533 */
API void orc_talker_step(orc_t *m, const float *embed, float *logits, float *hidden_out) {
    int H = m->d[D_H];
    float *x = malloc(H * sizeof(float));
    memcpy(x, embed, H * sizeof(float));
    talker_run(m, x, 1);
    mv_t(logits, find(m, "talker.codec_head.weight"), m->tk_x, m->d[D_V], H);
    if (hidden_out) memcpy(hidden_out, m->tk_x, H * sizeof(float));
    free(x);
}
API void orc_talker_head(orc_t *m, const float *hidden, float *logits) {   /* Q.c:1295 */
    mv_t(logits, find(m, "talker.codec_head.weight"), hidden, m->d[D_V], m->d[D_H]);
}
API int orc_kv_len(orc_t *m) { return m->kv_len; }

/* draw trace: keep the sampler's inputs if (frame, group) is the armed draw */
static void trace_draw(orc_t *m, int g, const float *lg, int n, const float *x, int xn, float rng) {
    if (m->tr_f != m->tr_frame || m->tr_g != g || m->tr_done) return;
    m->tr_logits = realloc(m->tr_logits, (size_t)n * sizeof(float));
    m->tr_x = realloc(m->tr_x, (size_t)xn * sizeof(float));
    memcpy(m->tr_logits, lg, (size_t)n * sizeof(float));
    memcpy(m->tr_x, x, (size_t)xn * sizeof(float));
    m->tr_n = n; m->tr_xn = xn; m->tr_rng = rng; m->tr_done = 1;
}
static void trace_result(orc_t *m, int g, int tok) {
    if (m->tr_f == m->tr_frame && m->tr_g == g && m->tr_done == 1) { m->tr_result = tok; m->tr_done = 2; }
}
/* arm the trace for draw (frame, group) of the next generation */
API void orc_trace_arm(orc_t *m, int frame, int group) { m->tr_f = frame; m->tr_g = group; m->tr_done = 0; }
/* the traced draw: 1 if it happened; logits [n], x [xn] (caller-sized by
 * orc_trace_dims), rng state before the draw (float bits), the drawn id */
API int orc_trace_dims(orc_t *m, int *n, int *xn) { *n = m->tr_n; *xn = m->tr_xn; return m->tr_done == 2; }
API int orc_trace_get(orc_t *m, float *logits, float *x, float *rng, int *result) {
    if (m->tr_done != 2) return 0;
    memcpy(logits, m->tr_logits, (size_t)m->tr_n * sizeof(float));
    memcpy(x, m->tr_x, (size_t)m->tr_xn * sizeof(float));
    *rng = m->tr_rng; *result = m->tr_result;
    return 1;
}

/* T.c:539-736: sub-talker for one frame */
API void orc_subtalker(orc_t *m, const float *hidden, int code0, int top_k, float top_p,
                       float temp, int seed, int *codes) {
    int H = m->d[D_H], Hs = m->d[D_HS], Ls = m->d[D_LS], G = m->d[D_G], Vs = m->d[D_VS];
    int kd = m->d[D_KVS] * m->d[D_HDS], S = G + 2;
    float *kk = calloc((size_t)Ls * S * kd, sizeof(float)), *vv = calloc((size_t)Ls * S * kd, sizeof(float));
    float *x = malloc(Hs * sizeof(float)), *emb = malloc(H * sizeof(float)), *lg = malloc(Vs * sizeof(float));
    const tens_t *pw = find(m, "talker.code_predictor.small_to_mtp_projection.weight");
    const tens_t *pb = find(m, "talker.code_predictor.small_to_mtp_projection.bias");
    const tens_t *nw = find(m, "talker.code_predictor.model.norm.weight");
    lw_t lw[16];
    for (int l = 0; l < Ls; l++) layer_w(m, &lw[l], "talker.code_predictor.model", l);
    codes[0] = code0;
    float rng = (float)seed;                                 /* T.c:718: reset per frame */
    for (int g = 0; g < G; g++) {
        const float *src;
        if (g == 0) src = hidden;
        else {
            const tens_t *e = g == 1 ? find(m, "talker.model.codec_embedding.weight")
                                     : findf(m, "talker.code_predictor.model.codec_embedding.%d.weight", g - 2, 0);
            for (int i = 0; i < H; i++) emb[i] = el(e, (long)codes[g - 1] * H + i);
            src = emb;
        }
        if (pw) { mv_t(x, pw, src, Hs, H); add_bias_t(x, pb, Hs); }   /* T.c:693-702 */
        else { int c = H < Hs ? H : Hs; memcpy(x, src, c * sizeof(float)); for (int i = c; i < Hs; i++) x[i] = 0; }
        for (int l = 0; l < Ls; l++)
            dec_layer(&lw[l], x, 1, g, Hs, m->d[D_NHS], m->d[D_KVS], m->d[D_HDS], m->d[D_IS],
                      m->f[F_EPS], m->f[F_THETA], kk + (size_t)l * S * kd, vv + (size_t)l * S * kd, 0);
        rmsnorm_t(x, x, nw, Hs, m->f[F_EPS]);
        if (g >= 1) {            /* pass g samples code g from lm_head[g-1] (T.c:716-732) */
            const tens_t *hw = findf(m, "talker.code_predictor.lm_head.%d.weight", g - 1, 0);
            mv_t(lg, hw, x, Vs, Hs);
            trace_draw(m, g, lg, Vs, x, Hs, rng);
            codes[g] = orc_sample(lg, Vs, top_k, top_p, temp, &rng);
            trace_result(m, g, codes[g]);
        }
    }
    free(kk); free(vv); free(x); free(emb); free(lg);
}

/* ------------------------------------------------------------------ */
/* codec decoder (c/qwen_tts_codec.c)                                  */
/* ------------------------------------------------------------------ */
static void conv_t(float *out, const float *in, const char *wn, const char *bn,
                   const orc_t *m, int ci, int co, int K, int L, int d, int groups) {
    const tens_t *w = find(m, wn), *b = bn ? find(m, bn) : NULL;
    float *bb = b ? f32copy(b) : NULL;
    orc_conv1d(out, in, w->p, bb, ci, co, K, L, d, groups);
    free(bb);
}

API float *orc_codec_decode(orc_t *m, const int *codes, int T, int *n_out) {
    int Q = m->d[D_CQ], CB = m->d[D_CCB], vq = m->d[D_CCBDIM] / 2, lat = m->d[D_CLAT];
    int half = lat / 2, cbd = m->d[D_CCBDIM], hid = m->d[D_CHID];
    /* RVQ (Cd.c:127-261): per-branch gather-sum, then 1x1 output projections, summed */
    float *ss = calloc((size_t)vq * T, sizeof(float)), *as = calloc((size_t)vq * T, sizeof(float));
    for (int q = 0; q < Q; q++) {
        const float *e = codebook(m, q);
        float *dst = q == 0 ? ss : as;
        for (int t = 0; t < T; t++) {
            int c = codes[t * Q + q];
            if (c < 0 || c >= CB) c = 0;
            for (int k = 0; k < vq; k++) dst[(size_t)k * T + t] += e[(size_t)c * vq + k];
        }
    }
    float *h = malloc((size_t)half * T * sizeof(float));
    const float *ps = find(m, "decoder.quantizer.rvq_first.output_proj.weight")->p;
    const float *pa = find(m, "decoder.quantizer.rvq_rest.output_proj.weight")->p;
    for (int t = 0; t < T; t++)
        for (int o = 0; o < half; o++) {
            float s1 = 0, s2 = 0;
            for (int k = 0; k < vq; k++) s1 += ps[(size_t)o * vq + k] * ss[(size_t)k * T + t];
            for (int k = 0; k < vq; k++) s2 += pa[(size_t)o * vq + k] * as[(size_t)k * T + t];
            h[(size_t)o * T + t] = s1 + s2;
        }
    free(ss); free(as);
    /* pre-conv k=3 (Cd.c:616-621) */
    float *pc = malloc((size_t)lat * T * sizeof(float));
    conv_t(pc, h, "decoder.pre_conv.conv.weight", "decoder.pre_conv.conv.bias", m, cbd, lat, 3, T, 1, 1);
    free(h);
    /* transformer (Cd.c:267-461) on time-major [T, lat] */
    float *xs = malloc((size_t)T * lat * sizeof(float));
    for (int c = 0; c < lat; c++) for (int t = 0; t < T; t++) xs[(size_t)t * lat + c] = pc[(size_t)c * T + t];
    free(pc);
    {
        int nh = m->d[D_CHEADS], nkv = m->d[D_CKV], hd = hid / nh, kvd = nkv * hd, I = m->d[D_CINTER];
        int win = m->d[D_CWIN], gph = nh / nkv;
        float eps = m->f[F_CEPS];
        float *x = malloc((size_t)T * hid * sizeof(float)), *xn = malloc((size_t)T * hid * sizeof(float));
        float *q = malloc((size_t)T * nh * hd * sizeof(float)), *k = malloc((size_t)T * kvd * sizeof(float));
        float *v = malloc((size_t)T * kvd * sizeof(float)), *att = malloc((size_t)T * nh * hd * sizeof(float));
        float *g = malloc((size_t)T * I * sizeof(float)), *u = malloc((size_t)T * I * sizeof(float));
        float *sc = malloc((size_t)T * sizeof(float));
        float *cs = malloc((size_t)T * hd * sizeof(float)), *sn = malloc((size_t)T * hd * sizeof(float));
        orc_rope_table(cs, sn, T, hd, 10000.0f);                      /* Cd.c:309: theta fixed */
        mm_t(x, xs, find(m, "decoder.pre_transformer.input_proj.weight"), T, hid, lat);
        for (int t = 0; t < T; t++) add_bias_t(x + (size_t)t * hid, find(m, "decoder.pre_transformer.input_proj.bias"), hid);
        for (int l = 0; l < m->d[D_CLAYERS]; l++) {
            char p[96]; snprintf(p, sizeof p, "decoder.pre_transformer.layers.%d.", l);
            char b[160];
#define T_(s) (snprintf(b, sizeof b, "%s%s", p, s), find(m, b))
            for (int t = 0; t < T; t++) rmsnorm_t(xn + (size_t)t * hid, x + (size_t)t * hid, T_("input_layernorm.weight"), hid, eps);
            mm_t(q, xn, T_("self_attn.q_proj.weight"), T, nh * hd, hid);
            mm_t(k, xn, T_("self_attn.k_proj.weight"), T, kvd, hid);
            mm_t(v, xn, T_("self_attn.v_proj.weight"), T, kvd, hid);
            for (int t = 0; t < T; t++) {
                rope_heads(q + (size_t)t * nh * hd, nh, hd, cs + (size_t)t * hd, sn + (size_t)t * hd);
                rope_heads(k + (size_t)t * kvd, nkv, hd, cs + (size_t)t * hd, sn + (size_t)t * hd);
            }
            memset(att, 0, (size_t)T * nh * hd * sizeof(float));
            float scale = 1.0f / sqrtf((float)hd);
            for (int hh = 0; hh < nh; hh++) {
                int kh = hh / gph;
                for (int qi = 0; qi < T; qi++) {
                    int st = qi - win + 1; if (st < 0) st = 0;
                    int wl = qi - st + 1;
                    const float *qv = q + (size_t)qi * nh * hd + hh * hd;
                    for (int i = 0; i < wl; i++) {
                        const float *kr = k + (size_t)(st + i) * kvd + kh * hd;
                        float s = 0; for (int e = 0; e < hd; e++) s += qv[e] * kr[e];
                        sc[i] = s * scale;
                    }
                    orc_softmax(sc, wl);
                    float *o = att + (size_t)qi * nh * hd + hh * hd;
                    for (int i = 0; i < wl; i++) {
                        const float *vr = v + (size_t)(st + i) * kvd + kh * hd;
                        for (int e = 0; e < hd; e++) o[e] += sc[i] * vr[e];
                    }
                }
            }
            mm_t(xn, att, T_("self_attn.o_proj.weight"), T, hid, nh * hd);
            const tens_t *ls1 = T_("self_attn_layer_scale.scale");
            for (int t = 0; t < T; t++)
                for (int i = 0; i < hid; i++) {
                    float y = xn[(size_t)t * hid + i];
                    if (ls1) y *= el(ls1, i);
                    x[(size_t)t * hid + i] += y;
                }
            for (int t = 0; t < T; t++) rmsnorm_t(xn + (size_t)t * hid, x + (size_t)t * hid, T_("post_attention_layernorm.weight"), hid, eps);
            mm_t(g, xn, T_("mlp.gate_proj.weight"), T, I, hid);
            mm_t(u, xn, T_("mlp.up_proj.weight"), T, I, hid);
            for (size_t i = 0; i < (size_t)T * I; i++) g[i] = silu(g[i]) * u[i];
            mm_t(xn, g, T_("mlp.down_proj.weight"), T, hid, I);
            const tens_t *ls2 = T_("mlp_layer_scale.scale");
            for (int t = 0; t < T; t++)
                for (int i = 0; i < hid; i++) {
                    float y = xn[(size_t)t * hid + i];
                    if (ls2) y *= el(ls2, i);
                    x[(size_t)t * hid + i] += y;
                }
#undef T_
        }
        const tens_t *fn = find(m, "decoder.pre_transformer.norm.weight");
        if (fn) for (int t = 0; t < T; t++) rmsnorm_t(x + (size_t)t * hid, x + (size_t)t * hid, fn, hid, eps);
        mm_t(xs, x, find(m, "decoder.pre_transformer.output_proj.weight"), T, lat, hid);
        for (int t = 0; t < T; t++) add_bias_t(xs + (size_t)t * lat, find(m, "decoder.pre_transformer.output_proj.bias"), lat);
        free(x); free(xn); free(q); free(k); free(v); free(att); free(g); free(u); free(sc); free(cs); free(sn);
    }
    float *cur = malloc((size_t)lat * T * sizeof(float));
    for (int c = 0; c < lat; c++) for (int t = 0; t < T; t++) cur[(size_t)c * T + t] = xs[(size_t)t * lat + c];
    free(xs);
    int L = T;
    /* 2 x (transposed conv + ConvNeXt) (Cd.c:644-662, 467-522) */
    for (int s = 0; s < 2; s++) {
        int f = m->d[D_UP0 + s];
        char wn[96], bn[96];
        snprintf(wn, sizeof wn, "decoder.upsample.%d.0.conv.weight", s);
        snprintf(bn, sizeof bn, "decoder.upsample.%d.0.conv.bias", s);
        float *up = malloc((size_t)lat * L * f * sizeof(float));
        float *bb = f32copy(find(m, bn));
        orc_tconv1d(up, cur, find(m, wn)->p, bb, lat, lat, f, f, L);
        free(bb); free(cur); cur = up; L *= f;
        char p[64]; snprintf(p, sizeof p, "decoder.upsample.%d.1.", s);
        char b1[128], b2[128];
        snprintf(b1, sizeof b1, "%sdwconv.conv.weight", p); snprintf(b2, sizeof b2, "%sdwconv.conv.bias", p);
        float *dw = malloc((size_t)lat * L * sizeof(float));
        conv_t(dw, cur, b1, b2, m, lat, lat, 7, L, 1, lat);
        float *xl = malloc((size_t)L * lat * sizeof(float)), *h4 = malloc((size_t)4 * lat * sizeof(float));
        float *y = malloc(lat * sizeof(float));
        char nw[128], nb[128], w1[128], bb1[128], w2[128], bb2[128], gm[128];
        snprintf(nw, sizeof nw, "%snorm.weight", p); snprintf(nb, sizeof nb, "%snorm.bias", p);
        snprintf(w1, sizeof w1, "%spwconv1.weight", p); snprintf(bb1, sizeof bb1, "%spwconv1.bias", p);
        snprintf(w2, sizeof w2, "%spwconv2.weight", p); snprintf(bb2, sizeof bb2, "%spwconv2.bias", p);
        snprintf(gm, sizeof gm, "%sgamma", p);
        for (int c = 0; c < lat; c++) for (int t = 0; t < L; t++) xl[(size_t)t * lat + c] = dw[(size_t)c * L + t];
        for (int t = 0; t < L; t++) {
            float *r = xl + (size_t)t * lat;
            layernorm_t(r, r, find(m, nw), find(m, nb), lat, 1e-6f);
            mv_t(h4, find(m, w1), r, 4 * lat, lat);
            add_bias_t(h4, find(m, bb1), 4 * lat);
            for (int i = 0; i < 4 * lat; i++) h4[i] = gelu_tanh(h4[i]);
            mv_t(y, find(m, w2), h4, lat, 4 * lat);
            add_bias_t(y, find(m, bb2), lat);
            for (int i = 0; i < lat; i++) r[i] = y[i] * el(find(m, gm), i);
        }
        for (int c = 0; c < lat; c++)
            for (int t = 0; t < L; t++) cur[(size_t)c * L + t] = xl[(size_t)t * lat + c] + cur[(size_t)c * L + t];
        free(dw); free(xl); free(h4); free(y);
    }
    /* vocoder (Cd.c:665-735) */
    int dd = m->d[D_CDEC];
    float *voc = malloc((size_t)dd * L * sizeof(float));
    conv_t(voc, cur, "decoder.decoder.0.conv.weight", "decoder.decoder.0.conv.bias", m, lat, dd, 7, L, 1, 1);
    free(cur);
    int C = dd;
    for (int b = 0; b < 4; b++) {
        int r = m->d[D_UR0 + b], co = C / 2;
        char p[64]; snprintf(p, sizeof p, "decoder.decoder.%d.block.", b + 1);
        char an[128], bn2[128];
        snprintf(an, sizeof an, "%s0.alpha", p); snprintf(bn2, sizeof bn2, "%s0.beta", p);
        float *ib; float *a = snake_a_of(m, find(m, an), find(m, bn2), &ib);
        orc_snake(voc, voc, a, ib, C, L);
        char wn[128], wb[128];
        snprintf(wn, sizeof wn, "%s1.conv.weight", p); snprintf(wb, sizeof wb, "%s1.conv.bias", p);
        float *o = malloc((size_t)co * L * r * sizeof(float));
        float *bb = f32copy(find(m, wb));
        orc_tconv1d(o, voc, find(m, wn)->p, bb, C, co, 2 * r, r, L);
        free(bb); free(voc); voc = o; L *= r; C = co;
        static const int dil[3] = {1, 3, 9};
        float *res = malloc((size_t)C * L * sizeof(float)), *c1 = malloc((size_t)C * L * sizeof(float));
        for (int u = 0; u < 3; u++) {
            char q[96]; snprintf(q, sizeof q, "%s%d.", p, u + 2);
            char s1a[128], s1b[128], s2a[128], s2b[128], cw1[128], cb1[128], cw2[128], cb2[128];
            snprintf(s1a, sizeof s1a, "%sact1.alpha", q); snprintf(s1b, sizeof s1b, "%sact1.beta", q);
            snprintf(s2a, sizeof s2a, "%sact2.alpha", q); snprintf(s2b, sizeof s2b, "%sact2.beta", q);
            snprintf(cw1, sizeof cw1, "%sconv1.conv.weight", q); snprintf(cb1, sizeof cb1, "%sconv1.conv.bias", q);
            snprintf(cw2, sizeof cw2, "%sconv2.conv.weight", q); snprintf(cb2, sizeof cb2, "%sconv2.conv.bias", q);
            memcpy(res, voc, (size_t)C * L * sizeof(float));
            float *ib1; float *a1 = snake_a_of(m, find(m, s1a), find(m, s1b), &ib1);
            orc_snake(voc, voc, a1, ib1, C, L);
            conv_t(c1, voc, cw1, cb1, m, C, C, 7, L, dil[u], 1);
            float *ib2; float *a2 = snake_a_of(m, find(m, s2a), find(m, s2b), &ib2);
            orc_snake(c1, c1, a2, ib2, C, L);
            conv_t(voc, c1, cw2, cb2, m, C, C, 1, L, 1, 1);
            for (size_t i = 0; i < (size_t)C * L; i++) voc[i] += res[i];
        }
        free(res); free(c1);
    }
    float *ib; float *a = snake_a_of(m, find(m, "decoder.decoder.5.alpha"), find(m, "decoder.decoder.5.beta"), &ib);
    orc_snake(voc, voc, a, ib, C, L);
    float *wav = malloc((size_t)L * sizeof(float));
    conv_t(wav, voc, "decoder.decoder.6.conv.weight", "decoder.decoder.6.conv.bias", m, C, 1, 7, L, 1, 1);
    free(voc);
    for (int i = 0; i < L; i++) { if (wav[i] < -1.0f) wav[i] = -1.0f; if (wav[i] > 1.0f) wav[i] = 1.0f; }
    /* snake params are rebuilt per call; drop them */
    for (int i = 0; i < m->n_snake; i++) { free(m->snake_a[i]); free(m->snake_b[i]); }
    m->n_snake = 0;
    *n_out = L;
    return wav;
}

/* ------------------------------------------------------------------ */
/* prompt embedding + decode loop (c/qwen_tts.c:823-856, 1059-1443)    */
/* ------------------------------------------------------------------ */
/* Q.c:823-847: text_emb -> fc1 + b -> SiLU -> fc2 + b */
API void orc_embed_text(orc_t *m, int id, float *out) {
    int TH = m->d[D_TH], H = m->d[D_H];
    const tens_t *te = find(m, "talker.model.text_embedding.weight");
    float *e = malloc(TH * sizeof(float)), *h = malloc(TH * sizeof(float));
    for (int i = 0; i < TH; i++) e[i] = el(te, (long)id * TH + i);
    mv_t(h, find(m, "talker.text_projection.linear_fc1.weight"), e, TH, TH);
    add_bias_t(h, find(m, "talker.text_projection.linear_fc1.bias"), TH);
    for (int i = 0; i < TH; i++) h[i] = silu(h[i]);
    mv_t(out, find(m, "talker.text_projection.linear_fc2.weight"), h, H, TH);
    add_bias_t(out, find(m, "talker.text_projection.linear_fc2.bias"), H);
    free(e); free(h);
}
static void add_codec_emb(orc_t *m, int id, float *dst) {
    const tens_t *ce = find(m, "talker.model.codec_embedding.weight");
    int H = m->d[D_H];
    for (int i = 0; i < H; i++) dst[i] += el(ce, (long)id * H + i);
}

typedef struct {
    float temperature, top_p, rep, st_temperature, st_top_p;
    int top_k, max_tokens, fixed, seed, st_top_k;
} orc_params_t;

/* Builds the Q8 prompt layout; returns prefill length. spk/lang ids < 0 = absent */
API int orc_build_prompt(orc_t *m, const int *ids, int n, int spk, int lang,
                         float *prefill /*[16*H]*/, float *trailing /*[n*H]*/, int *n_trailing) {
    int H = m->d[D_H];
    int pre[8], np = 0;
    if (lang < 0) { pre[np++] = m->d[D_NOTHINK]; pre[np++] = m->d[D_THINK_BOS]; pre[np++] = m->d[D_THINK_EOS]; }
    else { pre[np++] = m->d[D_THINK]; pre[np++] = m->d[D_THINK_BOS]; pre[np++] = lang; pre[np++] = m->d[D_THINK_EOS]; }
    if (spk >= 0) pre[np++] = spk;
    pre[np++] = m->d[D_PAD];
    pre[np++] = m->d[D_BOS];
    int P = 3 + np;
    float *pad = malloc(H * sizeof(float)), *bos = malloc(H * sizeof(float)), *eos = malloc(H * sizeof(float));
    orc_embed_text(m, 151671, pad); orc_embed_text(m, 151672, bos); orc_embed_text(m, 151673, eos);
    for (int i = 0; i < 3; i++) orc_embed_text(m, ids[i], prefill + (size_t)i * H);
    for (int i = 0; i < np - 1; i++) {
        float *d = prefill + (size_t)(3 + i) * H;
        memcpy(d, i < np - 2 ? pad : bos, H * sizeof(float));
        add_codec_emb(m, pre[i], d);
    }
    float *d = prefill + (size_t)(P - 1) * H;
    orc_embed_text(m, ids[3], d);
    add_codec_emb(m, m->d[D_BOS], d);
    int nt = (n - 4 - 5) + 1; if (nt < 1) nt = 1;
    for (int i = 0; i < nt - 1; i++) orc_embed_text(m, ids[4 + i], trailing + (size_t)i * H);
    memcpy(trailing + (size_t)(nt - 1) * H, eos, H * sizeof(float));
    *n_trailing = nt;
    free(pad); free(bos); free(eos);
    return P;
}

/* Voice-clone (ICL) prompt: the Python reference's layout, which the c/
 * reference does not have (modeling_qwen3_tts.py:2104-2190 + generate_icl_prompt
 * :1967-2019).  PARITY UNPINNED: no C oracle and the Python package is not
 * importable here; this restates its published layout in the
 * fp32 arithmetic of the c/ path (embeddings bf16 -> f32, sums in f32).
 *   prefill = proj(ids[0:3]),
 *             (tts_pad x (nc-2), tts_bos) + [prefix codec ids.., spk_vec?, pad]
 *             then ICL rows, text_embed = proj(ref_ids[3:-2] ++ ids[3:-5]) ++ tts_eos,
 *                            codec_embed = codec_emb(bos) ++ sum_g emb_g(ref_codes[f][g])
 *     non_streaming: text_embed + codec_emb(pad) ; codec_embed + tts_pad ; trailing = [tts_pad]
 *     streaming:     text longer:  text_embed[:Lc] + codec_embed ; trailing = text_embed[Lc:]
 *                    else: (text_embed ++ tts_pad..) + codec_embed ; trailing = [tts_pad]
 * spk_vec (H floats, the speaker encoder's x-vector) or NULL; ref_codes may be
 * NULL / n_ref_frames 0 (x-vector-only mode: the plain layout with the vector
 * in the speaker slot).  Returns the prefill length; prefill must hold
 * 10 + n_ref_ids + n + n_ref_frames rows, trailing n + n_ref_ids + 1 rows. */
static void ref_frame_sum(orc_t *m, const int *fr, float *dst) {
    int H = m->d[D_H], G = m->d[D_G], Vs = m->d[D_VS], V = m->d[D_V];
    const tens_t *ce = find(m, "talker.model.codec_embedding.weight");
    for (int i = 0; i < H; i++) dst[i] = 0.0f;
    if (fr[0] >= 0 && fr[0] < V)
        for (int i = 0; i < H; i++) dst[i] += el(ce, (long)fr[0] * H + i);
    for (int g = 1; g < G; g++) {
        if (fr[g] < 0 || fr[g] >= Vs) continue;
        const tens_t *e = findf(m, "talker.code_predictor.model.codec_embedding.%d.weight", g - 1, 0);
        for (int i = 0; i < H; i++) dst[i] += el(e, (long)fr[g] * H + i);
    }
}
API int orc_build_icl_prompt(orc_t *m, const int *ids, int n, const int *ref_ids, int n_ref_ids,
                             const int *ref_codes, int n_ref_frames, const float *spk_vec, int lang,
                             int non_streaming, float *prefill, float *trailing, int *n_trailing) {
    int H = m->d[D_H];
    if (n < 8) return -1;
    int pre[8], np = 0;
    if (lang < 0) { pre[np++] = m->d[D_NOTHINK]; pre[np++] = m->d[D_THINK_BOS]; pre[np++] = m->d[D_THINK_EOS]; }
    else { pre[np++] = m->d[D_THINK]; pre[np++] = m->d[D_THINK_BOS]; pre[np++] = lang; pre[np++] = m->d[D_THINK_EOS]; }
    const int spk_slot = spk_vec ? np : -1;
    if (spk_vec) pre[np++] = -2;
    pre[np++] = m->d[D_PAD];
    pre[np++] = m->d[D_BOS];
    float *pad = malloc(H * sizeof(float)), *bos = malloc(H * sizeof(float)), *eos = malloc(H * sizeof(float));
    orc_embed_text(m, 151671, pad); orc_embed_text(m, 151672, bos); orc_embed_text(m, 151673, eos);
    int P = 0;
    for (int i = 0; i < 3; i++) orc_embed_text(m, ids[i], prefill + (size_t)P++ * H);
    for (int i = 0; i < np - 1; i++) {
        float *d = prefill + (size_t)P++ * H;
        memcpy(d, i < np - 2 ? pad : bos, H * sizeof(float));
        if (i == spk_slot) { for (int k = 0; k < H; k++) d[k] += spk_vec[k]; }
        else add_codec_emb(m, pre[i], d);
    }
    if ((!ref_codes || n_ref_frames <= 0) && non_streaming) {   /* M.py:2203-2226 */
        for (int i = 0; i < n - 8; i++) {
            float *d = prefill + (size_t)P++ * H;
            orc_embed_text(m, ids[3 + i], d);
            add_codec_emb(m, m->d[D_PAD], d);
        }
        float *d = prefill + (size_t)P++ * H;
        memcpy(d, eos, H * sizeof(float));
        add_codec_emb(m, m->d[D_PAD], d);
        d = prefill + (size_t)P++ * H;
        memcpy(d, pad, H * sizeof(float));
        add_codec_emb(m, m->d[D_BOS], d);
        memcpy(trailing, pad, H * sizeof(float));
        *n_trailing = 1;
        free(pad); free(bos); free(eos);
        return P;
    }
    if (!ref_codes || n_ref_frames <= 0) {      /* x-vector only: the plain tail (M.py:2191-2202, 2227-2232) */
        float *d = prefill + (size_t)P++ * H;
        orc_embed_text(m, ids[3], d);
        add_codec_emb(m, m->d[D_BOS], d);
        int nt = (n - 4 - 5) + 1; if (nt < 1) nt = 1;
        for (int i = 0; i < nt - 1; i++) orc_embed_text(m, ids[4 + i], trailing + (size_t)i * H);
        memcpy(trailing + (size_t)(nt - 1) * H, eos, H * sizeof(float));
        *n_trailing = nt;
        free(pad); free(bos); free(eos);
        return P;
    }
    const int nr = n_ref_ids - 5 > 0 ? n_ref_ids - 5 : 0, nx = n - 8 > 0 ? n - 8 : 0;
    const int Lt = nr + nx + 1, Lc = n_ref_frames + 1, G = m->d[D_G];
    float *te = malloc((size_t)Lt * H * sizeof(float)), *cemb = malloc((size_t)Lc * H * sizeof(float));
    for (int i = 0; i < nr; i++) orc_embed_text(m, ref_ids[3 + i], te + (size_t)i * H);
    for (int i = 0; i < nx; i++) orc_embed_text(m, ids[3 + i], te + (size_t)(nr + i) * H);
    memcpy(te + (size_t)(Lt - 1) * H, eos, H * sizeof(float));
    for (int k = 0; k < H; k++) cemb[k] = 0.0f;
    add_codec_emb(m, m->d[D_BOS], cemb);
    for (int f = 0; f < n_ref_frames; f++) ref_frame_sum(m, ref_codes + (size_t)f * G, cemb + (size_t)(f + 1) * H);
    if (non_streaming) {
        for (int i = 0; i < Lt; i++) {
            float *d = prefill + (size_t)P++ * H;
            memcpy(d, te + (size_t)i * H, H * sizeof(float));
            add_codec_emb(m, m->d[D_PAD], d);
        }
        for (int j = 0; j < Lc; j++) {
            float *d = prefill + (size_t)P++ * H;
            for (int k = 0; k < H; k++) d[k] = pad[k] + cemb[(size_t)j * H + k];
        }
        memcpy(trailing, pad, H * sizeof(float));
        *n_trailing = 1;
    } else {
        for (int j = 0; j < Lc; j++) {
            float *d = prefill + (size_t)P++ * H;
            const float *t = j < Lt ? te + (size_t)j * H : pad;
            for (int k = 0; k < H; k++) d[k] = t[k] + cemb[(size_t)j * H + k];
        }
        if (Lt > Lc) {
            memcpy(trailing, te + (size_t)Lc * H, (size_t)(Lt - Lc) * H * sizeof(float));
            *n_trailing = Lt - Lc;
        } else {
            memcpy(trailing, pad, H * sizeof(float));
            *n_trailing = 1;
        }
    }
    free(te); free(cemb); free(pad); free(bos); free(eos);
    return P;
}

/* Q.c:1282-1373 decode loop from an already-built prompt: returns the number
 * of generated frames; codes [frames,16]; *stop = 1 eos / 2 max_tokens. */
API int orc_generate_from_prompt(orc_t *m, const float *prefill, int P, const float *trail, int ntr,
                                 const orc_params_t *pp, int *codes, int max_frames, int *stop) {
    int H = m->d[D_H], V = m->d[D_V], G = m->d[D_G], eos = m->d[D_EOS];
    float *pad = malloc(H * sizeof(float));
    orc_embed_text(m, 151671, pad);
    orc_talker_prefill(m, prefill, P, NULL);
    int fixed = pp->fixed > 0 ? pp->fixed : 0;
    int maxt = fixed > 0 ? fixed : pp->max_tokens;
    if (maxt > max_frames) maxt = max_frames;
    int *hist = calloc(maxt + 1, sizeof(int)), ng = 0;
    float *lg = malloc(V * sizeof(float)), *nx = malloc(H * sizeof(float));
    float rng = (float)pp->seed;
    *stop = 2;
    const tens_t *ce = find(m, "talker.model.codec_embedding.weight");
    for (int step = 0; step < maxt; step++) {
        if (step == 0) orc_talker_head(m, m->tk_x, lg);
        else orc_talker_step(m, nx, lg, NULL);
        for (int i = V - 1024; i < V; i++) if (i != eos) lg[i] = -1e9f;     /* Q.c:1273-1305 */
        orc_rep_penalty(lg, hist, ng, V, pp->rep);
        m->tr_frame = ng;
        trace_draw(m, 0, lg, V, m->tk_x, H, rng);
        int tok = orc_sample(lg, V, pp->top_k, pp->top_p, pp->temperature, &rng);
        trace_result(m, 0, tok);
        if (fixed > 0 && tok == eos && ng < fixed) {                         /* Q.c:1315-1321 */
            float keep = lg[eos];
            lg[eos] = -1e9f;
            tok = orc_sample(lg, V, pp->top_k, pp->top_p, pp->temperature, &rng);
            lg[eos] = keep;
        }
        if (fixed == 0 && tok == eos) { *stop = 1; break; }
        hist[ng] = tok;
        int *cf = codes + (size_t)ng * G;
        orc_subtalker(m, m->tk_x, tok, pp->st_top_k, pp->st_top_p, pp->st_temperature, pp->seed, cf);
        ng++;
        /* Q.c:1345-1363: zero, + codec_emb(code0), + st_emb[g-1](code g), + trailing|pad */
        for (int i = 0; i < H; i++) nx[i] = 0.0f;
        for (int i = 0; i < H; i++) nx[i] += el(ce, (long)tok * H + i);
        for (int g = 1; g < G; g++) {
            const tens_t *e = findf(m, "talker.code_predictor.model.codec_embedding.%d.weight", g - 1, 0);
            for (int i = 0; i < H; i++) nx[i] += el(e, (long)cf[g] * H + i);
        }
        const float *tt = step < ntr ? trail + (size_t)step * H : pad;
        for (int i = 0; i < H; i++) nx[i] += tt[i];
    }
    free(pad); free(hist); free(lg); free(nx);
    return ng;
}

/* Q.c:1059-1443 minus I/O: returns the number of generated frames; codes
 * [frames,16]; *stop = 1 eos / 2 max_tokens; audio via orc_codec_decode. */
API int orc_generate_codes(orc_t *m, const int *ids, int n, int spk, int lang,
                           const orc_params_t *pp, int *codes, int max_frames, int *stop) {
    int H = m->d[D_H];
    if (n < 8) return -1;
    float *prefill = calloc((size_t)16 * H, sizeof(float)), *trail = calloc((size_t)n * H, sizeof(float));
    int ntr = 0;
    int P = orc_build_prompt(m, ids, n, spk, lang, prefill, trail, &ntr);
    int ng = orc_generate_from_prompt(m, prefill, P, trail, ntr, pp, codes, max_frames, stop);
    free(prefill); free(trail);
    return ng;
}
