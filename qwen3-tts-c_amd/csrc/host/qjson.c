/* qjson.c - minimal recursive-descent JSON parser. */
#define _GNU_SOURCE
#include "qjson.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { const char *p, *end; } cur_t;

static void ws(cur_t *c) {
    while (c->p < c->end && (*c->p == ' ' || *c->p == '\n' || *c->p == '\r' || *c->p == '\t')) c->p++;
}

static qj_t *node(qj_type_t t) {
    qj_t *v = (qj_t *)calloc(1, sizeof(qj_t));
    if (v) v->type = t;
    return v;
}

static int push(qj_t *v, char *key, qj_t *item) {
    if (v->n == 0 || (v->n >= 4 && (v->n & (v->n - 1)) == 0)) {  /* capacity 4, 8, 16, ... */
        int cap = v->n ? v->n * 2 : 4;
        qj_t **ni = (qj_t **)realloc(v->items, cap * sizeof(qj_t *));
        if (!ni) return -1;
        v->items = ni;
        if (v->type == QJ_OBJ) {
            char **nk = (char **)realloc(v->keys, cap * sizeof(char *));
            if (!nk) return -1;
            v->keys = nk;
        }
    }
    if (v->type == QJ_OBJ) v->keys[v->n] = key;
    v->items[v->n++] = item;
    return 0;
}

static char *parse_str(cur_t *c) {
    if (c->p >= c->end || *c->p != '"') return NULL;
    c->p++;
    size_t cap = 16, n = 0;
    char *s = (char *)malloc(cap);
    while (c->p < c->end && *c->p != '"') {
        char ch = *c->p++;
        if (ch == '\\' && c->p < c->end) {
            char e = *c->p++;
            switch (e) {
                case 'n': ch = '\n'; break;
                case 't': ch = '\t'; break;
                case 'r': ch = '\r'; break;
                case 'b': ch = '\b'; break;
                case 'f': ch = '\f'; break;
                case 'u': ch = '?'; c->p += (c->end - c->p >= 4) ? 4 : (c->end - c->p); break;
                default: ch = e; break;
            }
        }
        if (n + 2 > cap) { cap *= 2; s = (char *)realloc(s, cap); }
        s[n++] = ch;
    }
    if (c->p >= c->end) { free(s); return NULL; }
    c->p++;
    s[n] = 0;
    return s;
}

static qj_t *parse_val(cur_t *c, int depth);

static qj_t *parse_val(cur_t *c, int depth) {
    if (depth > 64) return NULL;
    ws(c);
    if (c->p >= c->end) return NULL;
    char ch = *c->p;
    if (ch == '{') {
        qj_t *v = node(QJ_OBJ);
        c->p++;
        ws(c);
        if (c->p < c->end && *c->p == '}') { c->p++; return v; }
        for (;;) {
            ws(c);
            char *k = parse_str(c);
            if (!k) { qj_free(v); return NULL; }
            ws(c);
            if (c->p >= c->end || *c->p != ':') { free(k); qj_free(v); return NULL; }
            c->p++;
            qj_t *it = parse_val(c, depth + 1);
            if (!it || push(v, k, it)) { free(k); qj_free(it); qj_free(v); return NULL; }
            ws(c);
            if (c->p < c->end && *c->p == ',') { c->p++; continue; }
            if (c->p < c->end && *c->p == '}') { c->p++; return v; }
            qj_free(v);
            return NULL;
        }
    }
    if (ch == '[') {
        qj_t *v = node(QJ_ARR);
        c->p++;
        ws(c);
        if (c->p < c->end && *c->p == ']') { c->p++; return v; }
        for (;;) {
            qj_t *it = parse_val(c, depth + 1);
            if (!it || push(v, NULL, it)) { qj_free(it); qj_free(v); return NULL; }
            ws(c);
            if (c->p < c->end && *c->p == ',') { c->p++; continue; }
            if (c->p < c->end && *c->p == ']') { c->p++; return v; }
            qj_free(v);
            return NULL;
        }
    }
    if (ch == '"') {
        char *s = parse_str(c);
        if (!s) return NULL;
        qj_t *v = node(QJ_STR);
        v->str = s;
        return v;
    }
    if (!strncmp(c->p, "true", 4)) { c->p += 4; qj_t *v = node(QJ_BOOL); v->num = 1; return v; }
    if (!strncmp(c->p, "false", 5)) { c->p += 5; return node(QJ_BOOL); }
    if (!strncmp(c->p, "null", 4)) { c->p += 4; return node(QJ_NULL); }
    char buf[64];
    size_t n = 0;
    while (c->p < c->end && n < sizeof(buf) - 1 && strchr("+-0123456789.eE", *c->p)) buf[n++] = *c->p++;
    if (n == 0) return NULL;
    buf[n] = 0;
    qj_t *v = node(QJ_NUM);
    v->num = strtod(buf, NULL);
    v->str = strdup(buf);  /* keep the text: floats are read with strtof like c/qwen_tts.c:131 */
    return v;
}

qj_t *qj_parse(const char *text, size_t len) {
    cur_t c = {text, text + len};
    return parse_val(&c, 0);
}

void qj_free(qj_t *v) {
    if (!v) return;
    for (int i = 0; i < v->n; i++) {
        qj_free(v->items[i]);
        if (v->keys) free(v->keys[i]);
    }
    free(v->items);
    free(v->keys);
    free(v->str);
    free(v);
}

const qj_t *qj_get(const qj_t *o, const char *key) {
    if (!o || o->type != QJ_OBJ) return NULL;
    for (int i = 0; i < o->n; i++)
        if (!strcmp(o->keys[i], key)) return o->items[i];
    return NULL;
}

const qj_t *qj_path(const qj_t *root, const char *path) {
    char part[128];
    const qj_t *v = root;
    while (v && *path) {
        const char *dot = strchr(path, '.');
        size_t n = dot ? (size_t)(dot - path) : strlen(path);
        if (n >= sizeof(part)) return NULL;
        memcpy(part, path, n);
        part[n] = 0;
        v = qj_get(v, part);
        path += n + (dot ? 1 : 0);
    }
    return v;
}

int qj_int(const qj_t *root, const char *path, int def) {
    const qj_t *v = qj_path(root, path);
    return v && v->type == QJ_NUM ? (int)v->num : def;
}

float qj_float(const qj_t *root, const char *path, float def) {
    const qj_t *v = qj_path(root, path);
    return v && v->type == QJ_NUM ? strtof(v->str, NULL) : def;
}

int qj_ints(const qj_t *root, const char *path, int *out, int max) {
    const qj_t *v = qj_path(root, path);
    if (!v || v->type != QJ_ARR) return 0;
    int n = 0;
    for (int i = 0; i < v->n && n < max; i++)
        if (v->items[i]->type == QJ_NUM) out[n++] = (int)v->items[i]->num;
    return n;
}

char *qj_read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)n + 1);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) { free(buf); fclose(f); return NULL; }
    buf[n] = 0;
    fclose(f);
    if (len) *len = (size_t)n;
    return buf;
}
