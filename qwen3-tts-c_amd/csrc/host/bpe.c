/* bpe.c - Qwen2 byte-level BPE text tokenizer (host C11).
 *
 * The reference takes token ids only: c/qwen_tts.c:1071-1077 leaves "Add BPE
 * tokenizer for direct text input" as a TODO, and its browser front end calls
 * @huggingface/transformers' AutoTokenizer (web/wasm/app.js:241-267) on the
 * chat template  <|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n.
 * This file is that tokenizer in C over the model directory's own files:
 *   vocab.json          token (byte-level unicode string) -> id
 *   merges.txt          "a b" merge rules, rank = line order
 *   tokenizer_config.json  added_tokens_decoder: special tokens, matched first
 * Algorithm (transformers Qwen2Tokenizer): split on added tokens; pre-tokenize
 * every other span with the Qwen2 regex
 *   (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}
 *   | ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
 * (hand-compiled below; the \p{L} / \p{N} / \s tables are generated from the
 * Python `regex` module, tools/gen_unicode_tables.py); map each pre-token's
 * bytes through GPT-2's bytes_to_unicode; merge the lowest-ranked adjacent
 * pair (all its occurrences, left to right) until no rule applies; look the
 * symbols up in the vocabulary.  The input is taken as NFC (Qwen2Tokenizer
 * NFC-normalises first; NFC text is unchanged by that).
 */
#include "bpe.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qjson.h"
#include "unicode_tables.h"

/* ------------------------------------------------------------ hash map */
typedef struct {
    char **key;
    int *val;
    size_t cap, n;
} smap_t;

static uint64_t fnv1a(const char *s, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)s[i]) * 1099511628211ull;
    return h;
}

static int smap_init(smap_t *m, size_t n) {
    m->cap = 16;
    while (m->cap < 2 * n + 16) m->cap <<= 1;
    m->key = (char **)calloc(m->cap, sizeof(char *));
    m->val = (int *)calloc(m->cap, sizeof(int));
    m->n = 0;
    return m->key && m->val ? 0 : -1;
}

static void smap_free(smap_t *m) {
    if (m->key)
        for (size_t i = 0; i < m->cap; i++) free(m->key[i]);
    free(m->key);
    free(m->val);
    memset(m, 0, sizeof *m);
}

/* key of length n (not NUL-terminated); first insertion wins */
static int smap_put(smap_t *m, const char *k, size_t n, int v) {
    size_t i = fnv1a(k, n) & (m->cap - 1);
    while (m->key[i]) {
        if (strlen(m->key[i]) == n && memcmp(m->key[i], k, n) == 0) return 0;
        i = (i + 1) & (m->cap - 1);
    }
    char *c = (char *)malloc(n + 1);
    if (!c) return -1;
    memcpy(c, k, n);
    c[n] = 0;
    m->key[i] = c;
    m->val[i] = v;
    m->n++;
    return 0;
}

static int smap_get(const smap_t *m, const char *k, size_t n) {
    size_t i = fnv1a(k, n) & (m->cap - 1);
    while (m->key[i]) {
        if (strlen(m->key[i]) == n && memcmp(m->key[i], k, n) == 0) return m->val[i];
        i = (i + 1) & (m->cap - 1);
    }
    return -1;
}

/* ------------------------------------------------------------ tokenizer */
typedef struct {
    char *text;
    int len, id;
} special_t;

struct qtok {
    smap_t vocab, merges;
    char benc[256][3];       /* bytes_to_unicode: byte -> UTF-8 of its code point */
    unsigned char blen[256];
    special_t *sp;
    int nsp;
};

static void build_byte_encoder(qtok_t *t) {
    int bs[256], cs[256], n = 0, extra = 0;
    unsigned char in[256] = {0};
    for (int b = 33; b <= 126; b++) { bs[n] = b; cs[n] = b; in[b] = 1; n++; }
    for (int b = 161; b <= 172; b++) { bs[n] = b; cs[n] = b; in[b] = 1; n++; }
    for (int b = 174; b <= 255; b++) { bs[n] = b; cs[n] = b; in[b] = 1; n++; }
    for (int b = 0; b < 256; b++)
        if (!in[b]) { bs[n] = b; cs[n] = 256 + extra++; n++; }
    for (int i = 0; i < 256; i++) {
        const int cp = cs[i];
        char *o = t->benc[bs[i]];
        if (cp < 0x80) { o[0] = (char)cp; t->blen[bs[i]] = 1; }
        else { o[0] = (char)(0xC0 | (cp >> 6)); o[1] = (char)(0x80 | (cp & 0x3F)); t->blen[bs[i]] = 2; }
    }
}

static int add_special(qtok_t *t, const char *s, int id) {
    for (int i = 0; i < t->nsp; i++)
        if (strcmp(t->sp[i].text, s) == 0) return 0;
    special_t *n = (special_t *)realloc(t->sp, (size_t)(t->nsp + 1) * sizeof(special_t));
    if (!n) return -1;
    t->sp = n;
    t->sp[t->nsp].text = strdup(s);
    t->sp[t->nsp].len = (int)strlen(s);
    t->sp[t->nsp].id = id;
    t->nsp++;
    return 0;
}

qtok_t *qtok_load(const char *dir) {
    char path[4096];
    size_t len = 0;
    snprintf(path, sizeof path, "%s/vocab.json", dir);
    char *txt = qj_read_file(path, &len);
    if (!txt) {
        fprintf(stderr, "Error: tokenizer needs %s (and merges.txt) in the model directory\n", path);
        return NULL;
    }
    qj_t *v = qj_parse(txt, len);
    free(txt);
    if (!v || v->type != QJ_OBJ) {
        fprintf(stderr, "Error: cannot parse %s\n", path);
        qj_free(v);
        return NULL;
    }
    qtok_t *t = (qtok_t *)calloc(1, sizeof(qtok_t));
    if (!t || smap_init(&t->vocab, (size_t)v->n)) { qj_free(v); qtok_free(t); return NULL; }
    for (int i = 0; i < v->n; i++)
        if (v->items[i]->type == QJ_NUM && smap_put(&t->vocab, v->keys[i], strlen(v->keys[i]), (int)v->items[i]->num)) {
            qj_free(v);
            qtok_free(t);
            return NULL;
        }
    qj_free(v);
    snprintf(path, sizeof path, "%s/merges.txt", dir);
    txt = qj_read_file(path, &len);
    if (!txt) {
        fprintf(stderr, "Error: tokenizer needs %s\n", path);
        qtok_free(t);
        return NULL;
    }
    size_t nl = 0;
    for (size_t i = 0; i < len; i++) nl += txt[i] == '\n';
    if (smap_init(&t->merges, nl + 1)) { free(txt); qtok_free(t); return NULL; }
    int rank = 0;
    for (char *p = txt, *e = txt + len; p < e;) {
        char *q = memchr(p, '\n', (size_t)(e - p));
        if (!q) q = e;
        size_t n = (size_t)(q - p);
        if (n && p[n - 1] == '\r') n--;
        if (n && !(rank == 0 && n >= 8 && memcmp(p, "#version", 8) == 0) && memchr(p, ' ', n)) {
            if (smap_put(&t->merges, p, n, rank)) { free(txt); qtok_free(t); return NULL; }
            rank++;
        }
        p = q + 1;
    }
    free(txt);
    build_byte_encoder(t);
    /* added tokens: tokenizer_config.json added_tokens_decoder {"id": {"content": ...}} */
    snprintf(path, sizeof path, "%s/tokenizer_config.json", dir);
    txt = qj_read_file(path, &len);
    if (txt) {
        qj_t *c = qj_parse(txt, len);
        free(txt);
        const qj_t *ad = c ? qj_get(c, "added_tokens_decoder") : NULL;
        if (ad && ad->type == QJ_OBJ)
            for (int i = 0; i < ad->n; i++) {
                const qj_t *ct = qj_get(ad->items[i], "content");
                if (ct && ct->type == QJ_STR && ct->str[0]) add_special(t, ct->str, atoi(ad->keys[i]));
            }
        qj_free(c);
    }
    if (t->nsp == 0) {   /* the Qwen2 chat specials */
        add_special(t, "<|endoftext|>", 151643);
        add_special(t, "<|im_start|>", 151644);
        add_special(t, "<|im_end|>", 151645);
    }
    return t;
}

void qtok_free(qtok_t *t) {
    if (!t) return;
    smap_free(&t->vocab);
    smap_free(&t->merges);
    for (int i = 0; i < t->nsp; i++) free(t->sp[i].text);
    free(t->sp);
    free(t);
}

/* ------------------------------------------------------------ pre-tokenizer */
static int in_ranges(const uint32_t (*r)[2], int n, uint32_t c) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) / 2;
        if (c < r[mid][0]) hi = mid - 1;
        else if (c > r[mid][1]) lo = mid + 1;
        else return 1;
    }
    return 0;
}
static int isL(uint32_t c) { return c < 0x80 ? ((c | 32) >= 'a' && (c | 32) <= 'z') : in_ranges(qtok_L, QTOK_L_N, c); }
static int isN(uint32_t c) { return c < 0x80 ? (c >= '0' && c <= '9') : in_ranges(qtok_N, QTOK_N_N, c); }
static int isS(uint32_t c) { return in_ranges(qtok_S, QTOK_S_N, c); }
static int isNL(uint32_t c) { return c == '\r' || c == '\n'; }
static int isP(uint32_t c) { return !isS(c) && !isL(c) && !isN(c); }   /* [^\s\p{L}\p{N}] */

/* UTF-8 -> code points with byte offsets; an invalid byte stands for itself
 * (a single "other" character whose BPE input is that byte) */
static int decode_utf8(const unsigned char *s, int n, uint32_t *cp, int *off) {
    int k = 0;
    for (int i = 0; i < n;) {
        const unsigned char b = s[i];
        int len = 1;
        uint32_t c = b;
        if (b >= 0xC2 && b <= 0xDF) { len = 2; c = b & 0x1F; }
        else if (b >= 0xE0 && b <= 0xEF) { len = 3; c = b & 0x0F; }
        else if (b >= 0xF0 && b <= 0xF4) { len = 4; c = b & 0x07; }
        int ok = i + len <= n;
        for (int j = 1; ok && j < len; j++) {
            if ((s[i + j] & 0xC0) != 0x80) ok = 0;
            else c = (c << 6) | (s[i + j] & 0x3F);
        }
        if (!ok || (len > 1 && (c < 0x80 || (len == 3 && (c < 0x800 || (c >= 0xD800 && c <= 0xDFFF))) ||
                                (len == 4 && (c < 0x10000 || c > 0x10FFFF))))) {
            len = 1;
            c = 0xFFFD0000u | b;   /* invalid: not L / N / S, keeps its byte */
        }
        cp[k] = c;
        off[k] = i;
        k++;
        i += len;
    }
    off[k] = n;
    return k;
}

/* the end (code-point index) of the pre-token starting at i */
static int pretok_end(const uint32_t *c, int n, int i) {
    /* (?i:'s|'t|'re|'ve|'m|'ll|'d) */
    if (c[i] == '\'' && i + 1 < n) {
        const uint32_t a = c[i + 1] < 0x80 ? (c[i + 1] | 32) : c[i + 1];
        const uint32_t b = i + 2 < n ? (c[i + 2] < 0x80 ? (c[i + 2] | 32) : c[i + 2]) : 0;
        if (a == 's' || a == 0x17F || a == 't' || a == 'm' || a == 'd') return i + 2;
        if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return i + 3;
    }
    /* [^\r\n\p{L}\p{N}]?\p{L}+ */
    {
        int k = i;
        if (!isNL(c[k]) && !isL(c[k]) && !isN(c[k]) && k + 1 < n && isL(c[k + 1])) k++;
        if (isL(c[k])) {
            while (k < n && isL(c[k])) k++;
            return k;
        }
    }
    /* \p{N} */
    if (isN(c[i])) return i + 1;
    /*  ?[^\s\p{L}\p{N}]+[\r\n]* */
    {
        int k = i;
        if (c[k] == ' ' && k + 1 < n && isP(c[k + 1])) k++;
        if (isP(c[k])) {
            while (k < n && isP(c[k])) k++;
            while (k < n && isNL(c[k])) k++;
            return k;
        }
    }
    /* whitespace run [i, r) */
    int r = i;
    while (r < n && isS(c[r])) r++;
    if (r > i) {
        /* \s*[\r\n]+ : up to the run's last newline */
        for (int q = r - 1; q >= i; q--)
            if (isNL(c[q])) return q + 1;
        /* \s+(?!\S) */
        if (r == n) return r;
        if (r - i >= 2) return r - 1;
        /* \s+ */
        return r;
    }
    return i + 1;
}

/* ------------------------------------------------------------ BPE */
typedef struct {
    int *ids;
    int n, cap;
} ivec_t;

static int ipush(ivec_t *v, int x) {
    if (v->n == v->cap) {
        const int nc = v->cap ? 2 * v->cap : 64;
        int *p = (int *)realloc(v->ids, (size_t)nc * sizeof(int));
        if (!p) return -1;
        v->ids = p;
        v->cap = nc;
    }
    v->ids[v->n++] = x;
    return 0;
}

/* one pre-token (raw bytes) -> ids */
static int bpe_word(const qtok_t *t, const unsigned char *w, int nb, ivec_t *out) {
    /* symbols as byte-level strings: sym[i] = [st[i], st[i] + ln[i]) in buf */
    int nsym = nb;
    char *buf = (char *)malloc((size_t)nb * 2 + 1), *tmp = (char *)malloc((size_t)nb * 2 + 1);
    int *st = (int *)malloc(sizeof(int) * (size_t)nb * 2), *ln = st + nb;
    if (!buf || !tmp || !st) { free(buf); free(tmp); free(st); return -1; }
    int pos = 0;
    for (int i = 0; i < nb; i++) {
        memcpy(buf + pos, t->benc[w[i]], t->blen[w[i]]);
        st[i] = pos;
        ln[i] = t->blen[w[i]];
        pos += ln[i];
    }
    char key[1024];
    for (;;) {
        int best = -1, brank = 0;
        for (int i = 0; i + 1 < nsym; i++) {
            const int kl = ln[i] + 1 + ln[i + 1];
            if (kl > (int)sizeof key) continue;
            memcpy(key, buf + st[i], ln[i]);
            key[ln[i]] = ' ';
            memcpy(key + ln[i] + 1, buf + st[i + 1], ln[i + 1]);
            const int r = smap_get(&t->merges, key, kl);
            if (r >= 0 && (best < 0 || r < brank)) { best = i; brank = r; }
        }
        if (best < 0) break;
        /* merge every occurrence of the pair (a, b), left to right */
        const int la = ln[best], lb = ln[best + 1];
        char a[512], b[512];
        if (la >= (int)sizeof a || lb >= (int)sizeof b) break;
        memcpy(a, buf + st[best], la);
        memcpy(b, buf + st[best + 1], lb);
        int k = 0, p2 = 0;
        for (int i = 0; i < nsym;) {
            if (i + 1 < nsym && ln[i] == la && ln[i + 1] == lb && memcmp(buf + st[i], a, la) == 0 &&
                memcmp(buf + st[i + 1], b, lb) == 0) {
                memcpy(tmp + p2, a, la);
                memcpy(tmp + p2 + la, b, lb);
                st[k] = p2;
                ln[k] = la + lb;
                p2 += la + lb;
                i += 2;
            } else {
                memcpy(tmp + p2, buf + st[i], ln[i]);
                const int l0 = ln[i];
                st[k] = p2;
                ln[k] = l0;
                p2 += l0;
                i += 1;
            }
            k++;
        }
        nsym = k;
        char *sw = buf; buf = tmp; tmp = sw;
    }
    int rc = 0;
    for (int i = 0; i < nsym && rc == 0; i++) {
        const int id = smap_get(&t->vocab, buf + st[i], ln[i]);
        if (id < 0) {
            fprintf(stderr, "Error: tokenizer symbol '%.*s' not in vocab.json\n", ln[i], buf + st[i]);
            rc = -1;
        } else if (ipush(out, id)) {
            rc = -1;
        }
    }
    free(buf);
    free(tmp);
    free(st);
    return rc;
}

static int encode_span(const qtok_t *t, const unsigned char *s, int n, ivec_t *out) {
    if (n <= 0) return 0;
    uint32_t *cp = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n);
    int *off = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    if (!cp || !off) { free(cp); free(off); return -1; }
    const int nc = decode_utf8(s, n, cp, off);
    int rc = 0;
    for (int i = 0; i < nc && rc == 0;) {
        const int j = pretok_end(cp, nc, i);
        rc = bpe_word(t, s + off[i], off[j] - off[i], out);
        i = j;
    }
    free(cp);
    free(off);
    return rc;
}

int qtok_encode(const qtok_t *t, const char *text, int **ids_out) {
    *ids_out = NULL;
    if (!t || !text) return -1;
    ivec_t out = {0};
    const unsigned char *s = (const unsigned char *)text;
    const int n = (int)strlen(text);
    int i = 0, seg = 0, rc = 0;
    while (i < n && rc == 0) {
        int hit = -1;
        for (int k = 0; k < t->nsp; k++)   /* longest added token at i */
            if (t->sp[k].len <= n - i && memcmp(s + i, t->sp[k].text, t->sp[k].len) == 0 &&
                (hit < 0 || t->sp[k].len > t->sp[hit].len))
                hit = k;
        if (hit < 0) { i++; continue; }
        rc = encode_span(t, s + seg, i - seg, &out);
        if (rc == 0) rc = ipush(&out, t->sp[hit].id);
        i += t->sp[hit].len;
        seg = i;
    }
    if (rc == 0) rc = encode_span(t, s + seg, n - seg, &out);
    if (rc) { free(out.ids); return -1; }
    if (!out.ids) out.ids = (int *)malloc(sizeof(int));
    *ids_out = out.ids;
    return out.n;
}
