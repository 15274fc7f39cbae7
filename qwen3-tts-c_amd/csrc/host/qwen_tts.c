/*
 * qwen_tts.c - C host for the MI355X hot path: config + checkpoint loading,
 * prompt layout, the per-frame decode loop and the public qwen_tts.h API.
 *
 * The arithmetic runs on the GPU through include/qtts_hip.h; this file owns
 * what the reference's c/qwen_tts.c owns on the host side:
 *   - config keys and defaults          (c/qwen_tts.c:235-355)
 *   - speaker / language lookup         (c/qwen_tts.c:1120-1145)
 *   - prompt layout (streaming layout)  (c/qwen_tts.c:1147-1243)
 *   - the generation loop, stop rules, progress callback, stderr lines and
 *     perf counters                     (c/qwen_tts.c:1258-1443)
 */
#define _GNU_SOURCE
#include "../../../include/qwen_tts.h"

#include <dirent.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../../include/qtts_hip.h"
#include "bpe.h"
#include "qjson.h"

int qwen_tts_verbose = 0;

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1000.0 + (double)ts.tv_nsec / 1e6;
}


/* ------------------------------------------------------------------ config */
static void read_map(const qj_t *root, const char *path, int *n, char ***names, int **ids) {
    const qj_t *m = qj_path(root, path);
    *n = 0;
    *names = NULL;
    *ids = NULL;
    if (!m || m->type != QJ_OBJ || m->n == 0) return;
    *names = (char **)calloc(m->n, sizeof(char *));
    *ids = (int *)calloc(m->n, sizeof(int));
    for (int i = 0; i < m->n; i++) {
        const qj_t *v = m->items[i];
        int id = -1;
        if (v->type == QJ_NUM) id = (int)v->num;
        else if (v->type == QJ_ARR && v->n > 0 && v->items[0]->type == QJ_NUM) id = (int)v->items[0]->num;
        (*names)[*n] = strdup(m->keys[i]);
        (*ids)[*n] = id;
        (*n)++;
    }
}

static int load_config(qwen_tts_ctx_t *ctx) {
    qwen_tts_config_t *c = &ctx->config;
    char path[1100];
    size_t len = 0;
    snprintf(path, sizeof path, "%s/config.json", ctx->model_dir);
    char *txt = qj_read_file(path, &len);
    if (!txt) { fprintf(stderr, "Error: cannot read %s\n", path); return -1; }
    qj_t *js = qj_parse(txt, len);
    free(txt);
    if (!js) { fprintf(stderr, "Error: cannot parse %s\n", path); return -1; }
#define TI(f, k, d) c->f = qj_int(js, "talker_config." k, d)
    TI(talker_vocab_size, "vocab_size", QWEN_TTS_TALKER_VOCAB);
    TI(talker_hidden, "hidden_size", QWEN_TTS_TALKER_HIDDEN);
    TI(talker_intermediate, "intermediate_size", QWEN_TTS_TALKER_INTERMEDIATE);
    TI(talker_layers, "num_hidden_layers", QWEN_TTS_TALKER_LAYERS);
    TI(talker_heads, "num_attention_heads", QWEN_TTS_TALKER_HEADS);
    TI(talker_kv_heads, "num_key_value_heads", QWEN_TTS_TALKER_KV_HEADS);
    TI(talker_head_dim, "head_dim", 0);
    if (c->talker_head_dim <= 0 && c->talker_heads > 0) c->talker_head_dim = c->talker_hidden / c->talker_heads;
    TI(talker_text_hidden, "text_hidden_size", QWEN_TTS_TALKER_TEXT_HIDDEN);
    TI(talker_text_vocab, "text_vocab_size", QWEN_TTS_TALKER_TEXT_VOCAB);
    TI(num_code_groups, "num_code_groups", QWEN_TTS_NUM_CODE_GROUPS);
    c->talker_rms_norm_eps = qj_float(js, "talker_config.rms_norm_eps", 1e-6f);
    c->talker_rope_theta = qj_float(js, "talker_config.rope_theta", 10000.0f);
    c->mrope_section[0] = 16; c->mrope_section[1] = 16; c->mrope_section[2] = 0;
    qj_ints(js, "talker_config.rope_scaling.mrope_section", c->mrope_section, 3);
    TI(subtalker_vocab_size, "code_predictor_config.vocab_size", QWEN_TTS_SUBTALKER_VOCAB);
    TI(subtalker_hidden, "code_predictor_config.hidden_size", QWEN_TTS_SUBTALKER_HIDDEN);
    TI(subtalker_intermediate, "code_predictor_config.intermediate_size", QWEN_TTS_SUBTALKER_INTERMEDIATE);
    TI(subtalker_layers, "code_predictor_config.num_hidden_layers", QWEN_TTS_SUBTALKER_LAYERS);
    TI(subtalker_heads, "code_predictor_config.num_attention_heads", QWEN_TTS_SUBTALKER_HEADS);
    TI(subtalker_kv_heads, "code_predictor_config.num_key_value_heads", QWEN_TTS_SUBTALKER_KV_HEADS);
    TI(subtalker_head_dim, "code_predictor_config.head_dim", QWEN_TTS_SUBTALKER_HEAD_DIM);
    TI(codec_pad_id, "codec_pad_id", QWEN_TTS_CODEC_PAD);
    TI(codec_bos_id, "codec_bos_id", QWEN_TTS_CODEC_BOS);
    TI(codec_eos_id, "codec_eos_token_id", QWEN_TTS_CODEC_EOS);
    TI(codec_nothink_id, "codec_nothink_id", QWEN_TTS_CODEC_NOTHINK);
    TI(codec_think_id, "codec_think_id", QWEN_TTS_CODEC_THINK);
    TI(codec_think_bos_id, "codec_think_bos_id", QWEN_TTS_CODEC_THINK_BOS);
    TI(codec_think_eos_id, "codec_think_eos_id", QWEN_TTS_CODEC_THINK_EOS);
#undef TI
    read_map(js, "talker_config.spk_id", &c->n_speakers, &c->speaker_names, &c->speaker_ids);
    read_map(js, "talker_config.codec_language_id", &c->n_languages, &c->language_names, &c->language_ids);
    qj_free(js);
    if (c->talker_heads <= 0 || c->talker_kv_heads <= 0 || c->talker_head_dim <= 0) {
        fprintf(stderr, "Error: invalid talker attention config (heads=%d kv_heads=%d head_dim=%d)\n",
                c->talker_heads, c->talker_kv_heads, c->talker_head_dim);
        return -1;
    }
    if (c->talker_heads % c->talker_kv_heads != 0) {
        fprintf(stderr, "Error: talker heads (%d) must be divisible by kv heads (%d)\n", c->talker_heads,
                c->talker_kv_heads);
        return -1;
    }
    if (c->talker_head_dim > 512 || c->subtalker_head_dim > 512) {
        fprintf(stderr, "Error: unsupported head_dim (talker=%d subtalker=%d, max=512)\n", c->talker_head_dim,
                c->subtalker_head_dim);
        return -1;
    }
    if (c->num_code_groups > QWEN_TTS_NUM_CODE_GROUPS) {
        fprintf(stderr, "Error: num_code_groups %d > %d\n", c->num_code_groups, QWEN_TTS_NUM_CODE_GROUPS);
        return -1;
    }

    snprintf(path, sizeof path, "%s/speech_tokenizer/config.json", ctx->model_dir);
    txt = qj_read_file(path, &len);
    if (!txt) { fprintf(stderr, "Error: cannot read %s\n", path); return -1; }
    js = qj_parse(txt, len);
    free(txt);
    if (!js) { fprintf(stderr, "Error: cannot parse %s\n", path); return -1; }
#define DI(f, k, d) c->f = qj_int(js, "decoder_config." k, d)
    DI(codec_num_quantizers, "num_quantizers", QWEN_TTS_CODEC_NUM_QUANTIZERS);
    DI(codec_codebook_size, "codebook_size", QWEN_TTS_CODEC_CODEBOOK_SIZE);
    DI(codec_codebook_dim, "codebook_dim", 128);
    DI(codec_hidden, "hidden_size", QWEN_TTS_CODEC_HIDDEN);
    DI(codec_latent, "latent_dim", QWEN_TTS_CODEC_LATENT);
    DI(codec_layers, "num_hidden_layers", QWEN_TTS_CODEC_LAYERS);
    DI(codec_heads, "num_attention_heads", QWEN_TTS_CODEC_HEADS);
    DI(codec_kv_heads, "num_key_value_heads", QWEN_TTS_CODEC_KV_HEADS);
    DI(codec_intermediate, "intermediate_size", QWEN_TTS_CODEC_INTERMEDIATE);
    DI(codec_sliding_window, "sliding_window", QWEN_TTS_CODEC_SLIDING_WINDOW);
    DI(codec_decoder_dim, "decoder_dim", QWEN_TTS_CODEC_DECODER_DIM);
#undef DI
    c->codec_rms_norm_eps = qj_float(js, "decoder_config.rms_norm_eps", 1e-5f);
    c->codec_layer_scale = qj_float(js, "decoder_config.layer_scale_initial_scale", 0.01f);
    int rates[4] = {8, 5, 4, 3}, ratios[2] = {2, 2};
    qj_ints(js, "decoder_config.upsample_rates", rates, 4);
    qj_ints(js, "decoder_config.upsampling_ratios", ratios, 2);
    memcpy(c->codec_upsample_rates, rates, sizeof rates);
    memcpy(c->codec_upsampling_ratios, ratios, sizeof ratios);
    qj_free(js);
    if (qwen_tts_verbose >= 1) {
        fprintf(stderr, "Config loaded:\n");
        fprintf(stderr, "  Talker: %d layers, hidden=%d, heads=%d/%d, head_dim=%d\n", c->talker_layers,
                c->talker_hidden, c->talker_heads, c->talker_kv_heads, c->talker_head_dim);
        fprintf(stderr, "  Sub-talker: %d layers, hidden=%d, heads=%d/%d, head_dim=%d\n", c->subtalker_layers,
                c->subtalker_hidden, c->subtalker_heads, c->subtalker_kv_heads, c->subtalker_head_dim);
        fprintf(stderr, "  Codec: %d layers, hidden=%d, codebook_dim=%d, decoder_dim=%d\n", c->codec_layers,
                c->codec_hidden, c->codec_codebook_dim, c->codec_decoder_dim);
        fprintf(stderr, "  Speakers: %d, Languages: %d\n", c->n_speakers, c->n_languages);
    }
    return 0;
}

/* ------------------------------------------------------------- checkpoint */
static int cmp_name(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

static int is_talker_attn_proj(const char *n) {
    if (strncmp(n, "talker.model.layers.", 20) != 0) return 0;
    const char *s = strstr(n, ".self_attn.");
    return s && s[11] && strchr("qkvo", s[11]) && !strcmp(s + 12, "_proj.weight");
}

/* mmap one .safetensors file and hand every tensor to the device */
static int upload_file(qtts_dev_t *dev, const char *path) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) { fprintf(stderr, "Error: cannot open %s\n", path); return -1; }
    struct stat st;
    if (fstat(fd, &st) < 0 || st.st_size < 8) { close(fd); return -1; }
    size_t size = (size_t)st.st_size;
    uint8_t *base = (uint8_t *)mmap(NULL, size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (base == MAP_FAILED) { fprintf(stderr, "Error: mmap failed for %s\n", path); return -1; }
    uint64_t hlen;
    memcpy(&hlen, base, 8);
    int rc = -1;
    qj_t *hdr = NULL;
    if (hlen + 8 > size || !(hdr = qj_parse((const char *)base + 8, (size_t)hlen)) || hdr->type != QJ_OBJ) {
        fprintf(stderr, "Error: bad safetensors header in %s\n", path);
        goto done;
    }
    const uint8_t *data = base + 8 + hlen;
    for (int i = 0; i < hdr->n; i++) {
        const char *name = hdr->keys[i];
        const qj_t *e = hdr->items[i];
        if (!strcmp(name, "__metadata__")) continue;
        const qj_t *dt = qj_get(e, "dtype"), *sh = qj_get(e, "shape"), *off = qj_get(e, "data_offsets");
        if (!dt || dt->type != QJ_STR || !sh || sh->type != QJ_ARR || !off || off->type != QJ_ARR || off->n != 2) {
            fprintf(stderr, "Error: malformed entry %s in %s\n", name, path);
            goto done;
        }
        int dtype = !strcmp(dt->str, "F32") ? 0 : !strcmp(dt->str, "BF16") ? 1 : !strcmp(dt->str, "F16") ? 2 : -1;
        if (is_talker_attn_proj(name) && dtype != 1) {  /* c/qwen_tts.c:389-393 */
            fprintf(stderr, "Error: tensor %s dtype mismatch: expected BF16, got %s\n", name, dt->str);
            goto done;
        }
        if (dtype < 0) continue;
        int64_t shape[8];
        int nd = sh->n < 8 ? sh->n : 8;
        size_t n = 1;
        for (int k = 0; k < nd; k++) { shape[k] = (int64_t)sh->items[k]->num; n *= (size_t)shape[k]; }
        size_t a = (size_t)off->items[0]->num, b = (size_t)off->items[1]->num;
        size_t esz = dtype == 0 ? 4 : 2;
        if (b < a || b - a != n * esz || 8 + hlen + b > size) {
            fprintf(stderr, "Error: tensor %s has inconsistent size in %s\n", name, path);
            goto done;
        }
        if (qtts_dev_put_tensor(dev, name, data + a, dtype, shape, nd) != 0) goto done;
    }
    rc = 0;
done:
    qj_free(hdr);
    munmap(base, size);
    return rc;
}

static int upload_dir(qtts_dev_t *dev, const char *dir) {
    DIR *d = opendir(dir);
    if (!d) { fprintf(stderr, "Error: cannot open directory %s\n", dir); return -1; }
    char **names = NULL;
    int n = 0, cap = 0;
    struct dirent *ent;
    while ((ent = readdir(d))) {
        const char *dot = strrchr(ent->d_name, '.');
        if (!dot || strcmp(dot, ".safetensors")) continue;
        if (n == cap) { cap = cap ? cap * 2 : 8; names = (char **)realloc(names, cap * sizeof(char *)); }
        names[n++] = strdup(ent->d_name);
    }
    closedir(d);
    if (n == 0) { fprintf(stderr, "Error: no .safetensors files in %s\n", dir); free(names); return -1; }
    qsort(names, n, sizeof(char *), cmp_name);
    int rc = 0;
    for (int i = 0; i < n; i++) {
        char p[1400];
        snprintf(p, sizeof p, "%s/%s", dir, names[i]);
        if (!rc && upload_file(dev, p)) rc = -1;
        free(names[i]);
    }
    free(names);
    return rc;
}

/* Voice-clone encoder config: config.json
 * `speaker_encoder_config` (defaults of Qwen3TTSSpeakerEncoderConfig,
 * configuration_qwen3_tts.py:47-57: enc_dim 1024; it must equal the talker
 * hidden the x-vector takes the place of, else the speaker encoder stays off) and speech_tokenizer/config.json `encoder_config`
 * (transformers MimiConfig defaults).  Returns 1 when either section exists. */
static int load_enc_config(const qwen_tts_ctx_t *ctx, qtts_enc_dims_t *e) {
    memset(e, 0, sizeof *e);
    char path[1100];
    size_t len = 0;
    int have = 0;
    snprintf(path, sizeof path, "%s/config.json", ctx->model_dir);
    char *txt = qj_read_file(path, &len);
    qj_t *js = txt ? qj_parse(txt, len) : NULL;
    free(txt);
    if (js && qj_path(js, "speaker_encoder_config")) have = 1;
#define SI(f, k, d) e->f = qj_int(js, "speaker_encoder_config." k, d)
    SI(mel_dim, "mel_dim", 128);
    SI(enc_dim, "enc_dim", 1024);   /* Qwen3TTSSpeakerEncoderConfig default */
    SI(att_ch, "enc_attention_channels", 128);
    SI(res2net_scale, "enc_res2net_scale", 8);
    SI(se_ch, "enc_se_channels", 128);
#undef SI
    static const int dch[5] = {512, 512, 512, 512, 1536}, dks[5] = {5, 3, 3, 3, 1}, ddl[5] = {1, 2, 3, 4, 1};
    memcpy(e->ch, dch, sizeof dch); memcpy(e->ks, dks, sizeof dks); memcpy(e->dil, ddl, sizeof ddl);
    e->n_ch = 5;
    if (js) {
        int n = qj_ints(js, "speaker_encoder_config.enc_channels", e->ch, 8);
        if (n > 0) e->n_ch = n;
        qj_ints(js, "speaker_encoder_config.enc_kernel_sizes", e->ks, 8);
        qj_ints(js, "speaker_encoder_config.enc_dilations", e->dil, 8);
    }
    qj_free(js);
    snprintf(path, sizeof path, "%s/speech_tokenizer/config.json", ctx->model_dir);
    txt = qj_read_file(path, &len);
    js = txt ? qj_parse(txt, len) : NULL;
    free(txt);
    if (js && qj_path(js, "encoder_config")) have = 1;
#define MI(f, k, d) e->f = qj_int(js, "encoder_config." k, d)
    MI(hidden, "hidden_size", 512);
    MI(n_filters, "num_filters", 64);
    MI(kernel, "kernel_size", 7);
    MI(last_kernel, "last_kernel_size", 3);
    MI(res_kernel, "residual_kernel_size", 3);
    MI(dil_growth, "dilation_growth_rate", 2);
    MI(n_res, "num_residual_layers", 1);
    MI(compress, "compress", 2);
    MI(layers, "num_hidden_layers", 8);
    MI(heads, "num_attention_heads", 8);
    MI(kv_heads, "num_key_value_heads", 8);
    MI(head_dim, "head_dim", 64);
    MI(inter, "intermediate_size", 2048);
    MI(window, "sliding_window", 250);
    MI(n_q, "num_quantizers", 32);
    MI(n_sem, "num_semantic_quantizers", 1);
    MI(cb_size, "codebook_size", 2048);
    MI(vq_dim, "vector_quantization_hidden_dimension", 256);
#undef MI
    e->n_valid = qj_int(js, "encoder_valid_num_quantizers", 16);
    e->norm_eps = qj_float(js, "encoder_config.norm_eps", 1e-5f);
    e->rope_theta = qj_float(js, "encoder_config.rope_theta", 0.f);
    if (e->rope_theta <= 0.f) e->rope_theta = qj_float(js, "encoder_config.rope_parameters.rope_theta", 10000.0f);
    int ratios[4] = {8, 6, 5, 4};
    if (js) qj_ints(js, "encoder_config.upsampling_ratios", ratios, 4);
    memcpy(e->ratios, ratios, sizeof ratios);
    qj_free(js);
    return have;
}

static void dims_of(const qwen_tts_config_t *c, qtts_dims_t *d) {
    memset(d, 0, sizeof *d);
    d->H = c->talker_hidden; d->I = c->talker_intermediate; d->L = c->talker_layers; d->NH = c->talker_heads;
    d->KV = c->talker_kv_heads; d->HD = c->talker_head_dim; d->TH = c->talker_text_hidden;
    d->TV = c->talker_text_vocab; d->V = c->talker_vocab_size; d->G = c->num_code_groups;
    d->Hs = c->subtalker_hidden; d->Is = c->subtalker_intermediate; d->Ls = c->subtalker_layers;
    d->NHs = c->subtalker_heads; d->KVs = c->subtalker_kv_heads; d->HDs = c->subtalker_head_dim;
    d->Vs = c->subtalker_vocab_size;
    d->eps = c->talker_rms_norm_eps; d->theta = c->talker_rope_theta;
    d->cq = c->codec_num_quantizers; d->ccb = c->codec_codebook_size; d->ccbdim = c->codec_codebook_dim;
    d->chid = c->codec_hidden; d->clat = c->codec_latent; d->clayers = c->codec_layers; d->cheads = c->codec_heads;
    d->ckv = c->codec_kv_heads; d->cinter = c->codec_intermediate; d->cwin = c->codec_sliding_window;
    d->cdec = c->codec_decoder_dim;
    memcpy(d->rates, c->codec_upsample_rates, sizeof d->rates);
    memcpy(d->ratios, c->codec_upsampling_ratios, sizeof d->ratios);
    d->ceps = c->codec_rms_norm_eps;
    d->pad_id = c->codec_pad_id; d->bos_id = c->codec_bos_id; d->eos_id = c->codec_eos_id;
}

qwen_tts_ctx_t *qwen_tts_load(const char *model_dir) { return qwen_tts_load_on(model_dir, -1); }

qwen_tts_ctx_t *qwen_tts_load_on(const char *model_dir, int device) {
    double t0 = now_ms();
    qwen_tts_ctx_t *ctx = (qwen_tts_ctx_t *)calloc(1, sizeof(qwen_tts_ctx_t));
    if (!ctx) return NULL;
    snprintf(ctx->model_dir, sizeof ctx->model_dir, "%s", model_dir);
    ctx->temperature = 0.9f;      /* c/qwen_tts.c:871-880 */
    ctx->subtalker_temperature = 0.9f;
    ctx->top_k = 50;
    ctx->subtalker_top_k = 50;
    ctx->top_p = 1.0f;
    ctx->subtalker_top_p = 1.0f;
    ctx->repetition_penalty = 1.05f;
    ctx->max_new_tokens = 4096;
    ctx->fixed_codec_tokens = 0;
    ctx->sample_seed = 42;
    if (load_config(ctx) != 0) { qwen_tts_free(ctx); return NULL; }
    int dev_id = device;
    if (dev_id < 0) {
        const char *e = getenv("QWEN_TTS_HIP_DEVICE");
        dev_id = e ? atoi(e) : 0;
    }
    if (qtts_hip_device_count() <= dev_id) {
        fprintf(stderr, "Error: no HIP device %d available (MI355X / gfx950 required)\n", dev_id);
        qwen_tts_free(ctx);
        return NULL;
    }
    ctx->hip_device = dev_id;
    qtts_dims_t dims;
    dims_of(&ctx->config, &dims);
    qtts_dev_t *dev = qtts_dev_create(&dims, dev_id);
    if (!dev) { qwen_tts_free(ctx); return NULL; }
    ctx->hip = dev;
    qtts_enc_dims_t ed;
    if (load_enc_config(ctx, &ed) && qtts_dev_enc_config(dev, &ed) != 0)   /* not fatal: encoders stay off */
        fprintf(stderr, "Warning: unsupported voice-clone encoder config: encoders disabled\n");
    char cdir[1100];
    snprintf(cdir, sizeof cdir, "%s/speech_tokenizer", model_dir);
    if (upload_dir(dev, model_dir) != 0 || upload_dir(dev, cdir) != 0 || qtts_dev_finalize(dev) != 0) {
        qwen_tts_free(ctx);
        return NULL;
    }
    ctx->tk_x = (float *)calloc(ctx->config.talker_hidden, sizeof(float));
    if (qwen_tts_verbose >= 1)
        fprintf(stderr, "Model loaded in %.1f ms (%.2f GB weights on HIP device %d)\n", now_ms() - t0,
                (double)qtts_dev_bytes(dev, 0) / 1e9, dev_id);
    return ctx;
}

/* the per-utterance results of the last qwen_tts_generate_queue */
static void queue_clear(qwen_tts_ctx_t *ctx) {
    if (ctx->queue_codes)
        for (int i = 0; i < ctx->queue_n; i++) free(ctx->queue_codes[i]);
    free(ctx->queue_codes);
    free(ctx->queue_frames);
    free(ctx->queue_stop_reason);
    free(ctx->queue_slot);
    ctx->queue_codes = NULL;
    ctx->queue_frames = ctx->queue_stop_reason = ctx->queue_slot = NULL;
    ctx->queue_n = 0;
    ctx->queue_frames_launched = 0;
    ctx->queue_slot_frames_used = 0;
    ctx->queue_rows_launched = 0;
    ctx->queue_refills = 0;
    ctx->queue_slots = 0;
}

void qwen_tts_free(qwen_tts_ctx_t *ctx) {
    if (!ctx) return;
    if (ctx->hip) qtts_dev_destroy((qtts_dev_t *)ctx->hip);
    for (int i = 0; i < ctx->config.n_speakers; i++) free(ctx->config.speaker_names[i]);
    free(ctx->config.speaker_names);
    free(ctx->config.speaker_ids);
    for (int i = 0; i < ctx->config.n_languages; i++) free(ctx->config.language_names[i]);
    free(ctx->config.language_names);
    free(ctx->config.language_ids);
    free(ctx->last_codes);
    free(ctx->tk_x);
    queue_clear(ctx);
    qtok_free((qtok_t *)ctx->tokenizer);
    free(ctx);
}

/* ------------------------------------------------------------------ text input (bpe.c) */
int *qwen_tts_tokenize(const char *model_dir, const char *text, int *n_ids) {
    if (n_ids) *n_ids = 0;
    if (!model_dir || !text || !n_ids) return NULL;
    qtok_t *t = qtok_load(model_dir);
    if (!t) return NULL;
    int *ids = NULL;
    const int n = qtok_encode(t, text, &ids);
    qtok_free(t);
    if (n < 0) return NULL;
    *n_ids = n;
    return ids;
}

char *qwen_tts_text_prompt(qwen_tts_ctx_t *ctx, const char *text) {
    if (!ctx || !text) return NULL;
    if (!ctx->tokenizer && !(ctx->tokenizer = qtok_load(ctx->model_dir))) return NULL;
    static const char pre[] = "<|im_start|>assistant\n", post[] = "<|im_end|>\n<|im_start|>assistant\n";
    const size_t lt = strlen(text);
    char *chat = (char *)malloc(sizeof pre + lt + sizeof post);
    if (!chat) return NULL;
    memcpy(chat, pre, sizeof pre - 1);
    memcpy(chat + sizeof pre - 1, text, lt);
    memcpy(chat + sizeof pre - 1 + lt, post, sizeof post);
    int *ids = NULL;
    const int n = qtok_encode((qtok_t *)ctx->tokenizer, chat, &ids);
    free(chat);
    if (n < 0) return NULL;
    char *csv = (char *)malloc((size_t)n * 12 + 1);
    if (!csv) { free(ids); return NULL; }
    size_t k = 0;
    for (int i = 0; i < n; i++) k += (size_t)sprintf(csv + k, i ? ",%d" : "%d", ids[i]);
    csv[k] = 0;
    free(ids);
    if (qwen_tts_verbose >= 1) fprintf(stderr, "Text: %d tokens (chat template)\n", n);
    return csv;
}

void qwen_tts_set_progress_callback(qwen_tts_ctx_t *ctx, qwen_tts_progress_cb cb, void *userdata) {
    ctx->progress_cb = cb;
    ctx->progress_cb_userdata = userdata;
}

/* ------------------------------------------------------------------ prompt */
static int parse_ids(const char *text, int **out) {
    *out = NULL;
    if (!text) return 0;
    int cap = 1;
    for (const char *p = text; *p; p++) cap += *p == ',';
    int *ids = (int *)malloc(cap * sizeof(int)), n = 0;
    const char *p = text;
    while (*p && n < cap) {
        while (*p == ' ' || *p == ',') p++;
        if (!*p) break;
        char *end = NULL;
        long v = strtol(p, &end, 10);
        if (end == p) {
            fprintf(stderr, "Error: invalid token ID near '%s'\n", p);
            free(ids);
            return -1;
        }
        ids[n++] = (int)v;
        p = end;
    }
    *out = ids;
    return n;
}

typedef struct {
    int *text;  /* text ids to project */
    int n_text;
    int *plan;  /* 5 ints per row */
    int nplan;
    int p_len, n_trailing, pad_row;
} prompt_t;

/* Streaming prompt layout of c/qwen_tts.c:1147-1243:
 *   prefill = proj(ids[0:3]),
 *             (tts_pad x (np-2), tts_bos) + codec_emb(prefix[0:np-1]),
 *             proj(ids[3]) + codec_emb(bos)
 *   trailing = proj(ids[4:-5]) ++ tts_eos; tts_pad once exhausted */
static int build_prompt(const qwen_tts_ctx_t *ctx, const int *ids, int n, int spk, int lang, int b, prompt_t *pr) {
    const qwen_tts_config_t *c = &ctx->config;
    int prefix[8], np = 0;
    if (lang < 0) {
        prefix[np++] = c->codec_nothink_id; prefix[np++] = c->codec_think_bos_id; prefix[np++] = c->codec_think_eos_id;
    } else {
        prefix[np++] = c->codec_think_id; prefix[np++] = c->codec_think_bos_id; prefix[np++] = lang;
        prefix[np++] = c->codec_think_eos_id;
    }
    if (spk >= 0) prefix[np++] = spk;
    prefix[np++] = c->codec_pad_id;
    prefix[np++] = c->codec_bos_id;
    int nt = (n - 4 - 5) + 1;
    if (nt < 1) nt = 1;
    pr->n_text = 7 + (nt - 1);
    pr->text = (int *)malloc(pr->n_text * sizeof(int));
    pr->plan = (int *)malloc((size_t)(3 + np + nt) * 5 * sizeof(int));
    int *t = pr->text;
    t[0] = ids[0]; t[1] = ids[1]; t[2] = ids[2];
    t[3] = QWEN_TTS_TOKEN_TTS_PAD; t[4] = QWEN_TTS_TOKEN_TTS_BOS; t[5] = QWEN_TTS_TOKEN_TTS_EOS; t[6] = ids[3];
    for (int i = 0; i < nt - 1; i++) t[7 + i] = ids[4 + i];
    int k = 0;
#define ROW(src, cid, kind, slot) do { int *r_ = pr->plan + 5 * k++; r_[0] = src; r_[1] = cid; r_[2] = kind; r_[3] = b; r_[4] = slot; } while (0)
    for (int i = 0; i < 3; i++) ROW(i, -1, 0, i);
    for (int i = 0; i < np - 1; i++) ROW(i < np - 2 ? 3 : 4, prefix[i], 0, 3 + i);
    ROW(6, c->codec_bos_id, 0, 3 + np - 1);
    for (int i = 0; i < nt - 1; i++) ROW(7 + i, -1, 1, i);
    ROW(5, -1, 1, nt - 1);
#undef ROW
    pr->nplan = k;
    pr->p_len = 3 + np;
    pr->n_trailing = nt;
    pr->pad_row = 3;
    return 0;
}

/* Voice clone (no c/ counterpart; the Python reference's layout,
 * modeling_qwen3_tts.py:2104-2232 + generate_icl_prompt :1967-2019; restated
 * by oracle/qtts_oracle.c orc_build_icl_prompt).  The speaker x-vector takes
 * the speaker-id slot (plan codec id -2); reference frames are plan codec ids
 * -3 - f (their 16 group embeddings summed on the device). */
typedef struct {
    const int *ref_ids;      /* ids of "<|im_start|>assistant\n{ref_text}<|im_end|>\n" (ICL) */
    int n_ref_ids;
    const int *ref_codes;    /* [n_ref][16] codes of the reference audio; NULL: x-vector only */
    int n_ref;
    const float *spk;        /* [hidden] speaker x-vector or NULL */
    int non_streaming;
} vclone_t;

static int build_icl_prompt(const qwen_tts_ctx_t *ctx, const int *ids, int n, const vclone_t *vc, int lang, int b,
                            prompt_t *pr) {
    const qwen_tts_config_t *c = &ctx->config;
    int prefix[8], np = 0;
    if (lang < 0) {
        prefix[np++] = c->codec_nothink_id; prefix[np++] = c->codec_think_bos_id; prefix[np++] = c->codec_think_eos_id;
    } else {
        prefix[np++] = c->codec_think_id; prefix[np++] = c->codec_think_bos_id; prefix[np++] = lang;
        prefix[np++] = c->codec_think_eos_id;
    }
    if (vc->spk) prefix[np++] = -2;
    prefix[np++] = c->codec_pad_id;
    prefix[np++] = c->codec_bos_id;
    const int icl = vc->ref_codes && vc->n_ref > 0;
    const int nr = icl && vc->n_ref_ids > 5 ? vc->n_ref_ids - 5 : 0, nx = n - 8 > 0 ? n - 8 : 0;
    /* text rows: 0-2 role, 3 pad, 4 bos, 5 eos, 6.. ref content ++ text content */
    /* (a plain-tail prompt of 8 ids still projects ids[3], as build_prompt does) */
    pr->n_text = 6 + nr + (!icl && nx == 0 ? 1 : nx);
    pr->text = (int *)malloc(pr->n_text * sizeof(int));
    int *t = pr->text;
    t[0] = ids[0]; t[1] = ids[1]; t[2] = ids[2];
    t[3] = QWEN_TTS_TOKEN_TTS_PAD; t[4] = QWEN_TTS_TOKEN_TTS_BOS; t[5] = QWEN_TTS_TOKEN_TTS_EOS;
    for (int i = 0; i < nr; i++) t[6 + i] = vc->ref_ids[3 + i];
    for (int i = 0; i < nx; i++) t[6 + nr + i] = ids[3 + i];
    if (!icl && nx == 0) t[6] = ids[3];
    const int Lt = nr + nx + 1, Lc = icl ? vc->n_ref + 1 : 0;
    pr->plan = (int *)malloc((size_t)(3 + np + 2 * (Lt + Lc) + 4) * 5 * sizeof(int));
    int k = 0, P = 0, nt = 0;
#define ROW(src, cid, kind, slot) do { int *r_ = pr->plan + 5 * k++; r_[0] = src; r_[1] = cid; r_[2] = kind; r_[3] = b; r_[4] = slot; } while (0)
#define TROW(j) ((j) < nr + nx ? 6 + (j) : 5)
#define CID(j) ((j) == 0 ? c->codec_bos_id : -3 - ((j) - 1))
    for (int i = 0; i < 3; i++) ROW(i, -1, 0, P++);
    for (int i = 0; i < np - 1; i++) ROW(i < np - 2 ? 3 : 4, prefix[i], 0, P++);
    if (!icl && !vc->non_streaming) {           /* x-vector only: the plain tail */
        ROW(6, c->codec_bos_id, 0, P++);        /* ids[3] = text row 6 */
        for (int j = 1; j < nx; j++) ROW(6 + j, -1, 1, nt++);
        ROW(5, -1, 1, nt++);
    } else if (!icl) {                          /* x-vector only, non-streaming (M.py:2203-2226) */
        for (int j = 0; j < Lt; j++) ROW(TROW(j), c->codec_pad_id, 0, P++);
        ROW(3, c->codec_bos_id, 0, P++);
        ROW(3, -1, 1, nt++);
    } else if (vc->non_streaming) {
        for (int j = 0; j < Lt; j++) ROW(TROW(j), c->codec_pad_id, 0, P++);
        for (int j = 0; j < Lc; j++) ROW(3, CID(j), 0, P++);
        ROW(3, -1, 1, nt++);
    } else {
        for (int j = 0; j < Lc; j++) ROW(j < Lt ? TROW(j) : 3, CID(j), 0, P++);
        if (Lt > Lc) for (int j = Lc; j < Lt; j++) ROW(TROW(j), -1, 1, nt++);
        else ROW(3, -1, 1, nt++);
    }
#undef CID
#undef TROW
#undef ROW
    pr->nplan = k;
    pr->p_len = P;
    pr->n_trailing = nt;
    pr->pad_row = 3;
    return 0;
}

static void lookup(const qwen_tts_ctx_t *ctx, const char *speaker, const char *language, int *spk, int *lang) {
    const qwen_tts_config_t *c = &ctx->config;
    *spk = -1;
    *lang = -1;
    if (speaker && strlen(speaker) > 0) {
        for (int i = 0; i < c->n_speakers; i++)
            if (strcasecmp(c->speaker_names[i], speaker) == 0) { *spk = c->speaker_ids[i]; break; }
        if (*spk < 0) fprintf(stderr, "Warning: speaker '%s' not found, using no speaker embedding\n", speaker);
    }
    if (language && strlen(language) > 0 && strcasecmp(language, "auto") != 0) {
        for (int i = 0; i < c->n_languages; i++)
            if (strcasecmp(c->language_names[i], language) == 0) { *lang = c->language_ids[i]; break; }
        if (*lang < 0) fprintf(stderr, "Warning: language '%s' not found\n", language);
    }
}

/* the reference codec's stderr lines around one full decode
 * (c/qwen_tts_codec.c:598-599 at -v, 740-746 at -v / -v -v) */
static void codec_log_begin(qwen_tts_ctx_t *ctx, int T) {
    qtts_dev_codec_timing((qtts_dev_t *)ctx->hip, qwen_tts_verbose >= 2);
    if (qwen_tts_verbose >= 1)
        fprintf(stderr, "Codec decode: %d timesteps, %d quantizers\n", T, ctx->config.codec_num_quantizers);
}

static void codec_log_end(qwen_tts_ctx_t *ctx, int samples) {
    if (qwen_tts_verbose < 1 || samples <= 0) return;
    fprintf(stderr, "Codec decode complete: %d samples (%.2f seconds)\n", samples,
            (float)samples / QWEN_TTS_SAMPLE_RATE);
    float ms[5];
    if (qwen_tts_verbose >= 2 && qtts_dev_codec_stage_ms((qtts_dev_t *)ctx->hip, ms) == 0)
        fprintf(stderr, "Codec stages (ms): rvq=%.1f preconv=%.1f transformer=%.1f upsample=%.1f vocoder=%.1f\n",
                ms[0], ms[1], ms[2], ms[3], ms[4]);
}

/* voice clone: keep the audio after the reference frames of a decode of
 * reference ++ generated codes (qwen3_tts_model.py:612-630, the same float
 * cut); takes ownership of w */
static void cut_reference(float *w, int nw, int n_ref, int tot, float **audio, int *samples) {
    const int cut = (int)((double)n_ref / (double)tot * (double)nw);
    *audio = NULL;
    *samples = 0;
    if (w && nw > cut) {
        memmove(w, w + cut, (size_t)(nw - cut) * sizeof(float));
        *audio = w;
        *samples = nw - cut;
    } else {
        free(w);
    }
}

static void params_of(const qwen_tts_ctx_t *ctx, qtts_gen_params_t *p) {
    p->temperature = ctx->temperature; p->top_p = ctx->top_p; p->repetition_penalty = ctx->repetition_penalty;
    p->top_k = ctx->top_k; p->st_temperature = ctx->subtalker_temperature; p->st_top_p = ctx->subtalker_top_p;
    p->st_top_k = ctx->subtalker_top_k; p->fixed_codec_tokens = ctx->fixed_codec_tokens; p->seed = ctx->sample_seed;
}

/* ------------------------------------------------------------- generation */
/* Runs nb utterances in lock-step frames.  Fills per-slot frame counts and
 * stop info; audio[i] decoded per slot.  Returns 0 on success. */
typedef struct {                 /* streaming output of run_batch (nb == 1) */
    qwen_tts_audio_cb cb;
    void *user;
    int chunk;
} stream_t;

static int run_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts, const char *const *speakers,
                     const char *const *languages, float **audio, int *samples, double t_start,
                     const stream_t *stream, const vclone_t *vcs /* [nb] or NULL */) {
    qtts_dev_t *dev = (qtts_dev_t *)ctx->hip;
    const qwen_tts_config_t *c = &ctx->config;
    const int G = c->num_code_groups;
    int rc = -1;
    prompt_t *pr = (prompt_t *)calloc(nb, sizeof(prompt_t));
    int max_p = 0;
    for (int b = 0; b < nb; b++) {
        int *ids = NULL;
        int n = parse_ids(texts[b], &ids);
        if (n < 8) {
            if (n >= 0) fprintf(stderr, "Error: need at least 8 text tokens (chat template format)\n");
            free(ids);
            goto out;
        }
        for (int i = 0; i < n; i++)
            if (ids[i] < 0 || ids[i] >= c->talker_text_vocab) {
                fprintf(stderr, "Error: text token id %d out of range\n", ids[i]);
                free(ids);
                goto out;
            }
        int spk, lang;
        lookup(ctx, speakers ? speakers[b] : NULL, languages ? languages[b] : NULL, &spk, &lang);
        if (vcs) build_icl_prompt(ctx, ids, n, &vcs[b], lang, b, &pr[b]);
        else build_prompt(ctx, ids, n, spk, lang, b, &pr[b]);
        free(ids);
        if (pr[b].p_len > max_p) max_p = pr[b].p_len;
    }
    const int fixed = ctx->fixed_codec_tokens > 0 ? ctx->fixed_codec_tokens : 0;
    const int max_tokens = fixed > 0 ? fixed : ctx->max_new_tokens;
    if (max_tokens < 1) goto out;
    qtts_gen_params_t gp;
    params_of(ctx, &gp);
    if (qtts_dev_begin(dev, nb, max_tokens, max_p, &gp) != 0) goto out;
    for (int b = 0; b < nb; b++)
        if ((vcs && qtts_dev_prompt_ref(dev, vcs[b].ref_codes, vcs[b].ref_codes ? vcs[b].n_ref : 0, vcs[b].spk) != 0) ||
            qtts_dev_prompt(dev, b, pr[b].text, pr[b].n_text, pr[b].plan, pr[b].nplan, pr[b].p_len,
                            pr[b].n_trailing, pr[b].pad_row) != 0)
            goto out;
    /* streaming voice clone: the reference frames go through the codec stream
     * first (their audio is dropped), so the carried codec state is that of
     * decoding reference ++ generated and the chunks start at the reference
     * boundary.  They run on a second HIP stream in one chunk while the
     * prefill runs (qtts_dev_codec_stream_prime); later pushes wait for them. */
    const int sref = stream && vcs && vcs[0].ref_codes && vcs[0].n_ref > 0 ? vcs[0].n_ref : 0;
    if (stream && (qtts_dev_codec_stream_begin_ex(dev, max_tokens + sref, sref) != 0 ||
                   (sref && qtts_dev_codec_stream_prime(dev, vcs[0].ref_codes, sref) != 0)))
        goto out;
    double t_prefill = now_ms();
    if (qtts_dev_prefill(dev) != 0) goto out;
    double t_prefill_done = now_ms();
    ctx->perf_prefill_ms = t_prefill_done - t_prefill;
    if (qwen_tts_verbose >= 1) {
        fprintf(stderr, "Talker prefill complete: %d tokens\n", pr[0].p_len);
        fprintf(stderr, "Prefill: %d tokens in %.1f ms\n", pr[0].p_len, t_prefill_done - t_prefill);
    }
    int *stopped = (int *)calloc(nb, sizeof(int)), *ngen = (int *)calloc(nb, sizeof(int));
    int *sstep = (int *)calloc(nb, sizeof(int));
    /* streaming: exact incremental codec decode of the frames produced so far */
    float *sbuf = NULL;
    int streamed = 0;
    double t_stream = 0;
    if (stream) {
        sbuf = (float *)malloc((size_t)max_tokens * 1920 * sizeof(float));
        if (!sbuf) { free(stopped); free(ngen); free(sstep); goto out; }
    }
    double t_gen = now_ms();
    const int poll_every = fixed > 0 ? 0 : 8;
    /* EOS mode without streaming: a lagged poll per frame (qtts_dev_frame_done)
     * instead of a synchronous one every 8 frames */
    const int lagged = fixed == 0 && !stream;
    int step = 0;
    for (; step < max_tokens; step++) {
        if (qtts_dev_frame(dev, step) != 0) { free(sbuf); free(stopped); free(ngen); free(sstep); goto out; }
        if (step == 0) {
            qtts_dev_poll(dev, NULL, NULL, NULL);
            ctx->perf_first_frame_ms = now_ms() - t_start;
        }
        if (ctx->progress_cb) ctx->progress_cb(step + 1, max_tokens, ctx->progress_cb_userdata);
        if (lagged) {   /* EOS mode: frame step is queued; stop once every slot had stopped by frame step - 1 */
            int done = 0;
            if (step >= 1 && qtts_dev_frame_done(dev, step - 1, &done) != 0) {
                free(sbuf); free(stopped); free(ngen); free(sstep); goto out;
            }
            if (qwen_tts_verbose >= 1 && step > 0 && step % 10 == 0)
                fprintf(stderr, "\r  Token %d (%.1f ms/token)...", step, (now_ms() - t_gen) / step);
            if (done) break;
            continue;
        }
        const int want_stream = stream && (step == 0 || step + 1 - streamed >= stream->chunk || step + 1 == max_tokens);
        if (want_stream || (poll_every && ((step + 1) % poll_every == 0 || step + 1 == max_tokens))) {
            qtts_dev_poll(dev, stopped, ngen, sstep);
            if (stream && ngen[0] > streamed) {
                const double t0 = now_ms();
                const int n = qtts_dev_codec_stream_push_slot(dev, 0, streamed, ngen[0] - streamed,
                                                              sbuf + (size_t)streamed * 1920);
                if (n < 0) { free(sbuf); free(stopped); free(ngen); free(sstep); goto out; }
                t_stream += now_ms() - t0;
                if (stream->cb) stream->cb(sbuf + (size_t)streamed * 1920, n, stream->user);
                if (streamed == 0) ctx->perf_first_packet_ms = now_ms() - t_start;
                streamed = ngen[0];
            }
            int all = 1;
            for (int b = 0; b < nb; b++) all &= stopped[b];
            if (qwen_tts_verbose >= 1 && ngen[0] > 0 && ngen[0] % 10 < poll_every)
                fprintf(stderr, "\r  Token %d (%.1f ms/token)...", ngen[0], (now_ms() - t_gen) / ngen[0]);
            if (all) break;
        }
    }
    qtts_dev_poll(dev, stopped, ngen, sstep);
    if (stream && ngen[0] > streamed) {
        const double t0 = now_ms();
        const int n = qtts_dev_codec_stream_push_slot(dev, 0, streamed, ngen[0] - streamed,
                                                      sbuf + (size_t)streamed * 1920);
        if (n < 0) { free(sbuf); free(stopped); free(ngen); free(sstep); goto out; }
        t_stream += now_ms() - t0;
        if (stream->cb) stream->cb(sbuf + (size_t)streamed * 1920, n, stream->user);
        if (streamed == 0) ctx->perf_first_packet_ms = now_ms() - t_start;
        streamed = ngen[0];
    }
    double t_gen_done = now_ms();
    ctx->perf_talker_ms = t_gen_done - t_gen - t_stream;
    ctx->perf_codec_tokens = ngen[0];
    ctx->last_stop_reason = stopped[0] ? 1 : 2;
    ctx->last_stop_step = stopped[0] ? sstep[0] : max_tokens;
    free(ctx->last_codes);
    ctx->last_codes = (int *)malloc((size_t)(ngen[0] > 0 ? ngen[0] : 1) * G * sizeof(int));
    ctx->last_frames = ngen[0] > 0 ? qtts_dev_get_codes(dev, 0, ctx->last_codes, ngen[0]) : 0;
    if (qwen_tts_verbose >= 1) {
        if (stopped[0]) fprintf(stderr, "EOS at step %d\n", sstep[0]);
        fprintf(stderr, "\r                                        \r");
        fprintf(stderr, "Generated %d codec tokens in %.1f ms (%.1f ms/token)\n", ngen[0], ctx->perf_talker_ms,
                ngen[0] > 0 ? ctx->perf_talker_ms / ngen[0] : 0);
        fprintf(stderr, "Stop: %s at step %d\n", stopped[0] ? "eos" : "max_tokens", ctx->last_stop_step);
        if (qwen_tts_verbose >= 2) {
            fprintf(stderr, "Token trace:");
            for (int i = 0; i < ctx->last_frames; i++)
                fprintf(stderr, "%s%d", i == 0 ? " " : ",", ctx->last_codes[(size_t)i * G]);
            fprintf(stderr, "\n");
        }
    }
    double t_codec = now_ms();
    rc = 0;
    if (stream) {   /* the streamed chunks already are the utterance */
        audio[0] = sbuf;
        samples[0] = streamed * 1920;
        if (streamed <= 0) { free(sbuf); audio[0] = NULL; rc = -1; }
        ctx->perf_codec_ms = t_stream;
    } else if (nb == 1) {
        audio[0] = NULL;
        samples[0] = 0;
        if (ngen[0] <= 0) {
            rc = -1;
        } else if (vcs && vcs[0].ref_codes && vcs[0].n_ref > 0) {
            /* voice clone: decode reference ++ generated codes, keep the part
             * after the reference (qwen3_tts_model.py:612-630, same float cut) */
            const vclone_t *vc = &vcs[0];
            const int tot = vc->n_ref + ngen[0];
            int *all = (int *)malloc((size_t)tot * G * sizeof(int)), nw = 0;
            if (all && qtts_dev_get_codes(dev, 0, all + (size_t)vc->n_ref * G, ngen[0]) == ngen[0]) {
                memcpy(all, vc->ref_codes, (size_t)vc->n_ref * G * sizeof(int));
                codec_log_begin(ctx, tot);
                float *w = qtts_dev_codec_decode_host(dev, all, tot, &nw);
                codec_log_end(ctx, w ? nw : 0);
                cut_reference(w, nw, vc->n_ref, tot, &audio[0], &samples[0]);
            }
            free(all);
            if (!audio[0]) rc = -1;
        } else {
            codec_log_begin(ctx, ngen[0]);
            audio[0] = qtts_dev_codec_slot(dev, 0, ngen[0], &samples[0]);
            codec_log_end(ctx, audio[0] ? samples[0] : 0);
            if (!audio[0] || samples[0] <= 0) rc = -1;
        }
    } else {
        /* a batch: every slot's codec pass in one call, several side by side
         * (qtts_dev_codec_multi); a voice-clone slot decodes its reference ++
         * generated codes and keeps the part after the reference */
        int **hc = (int **)calloc(nb, sizeof(int *));
        int *slot = (int *)calloc(nb, sizeof(int)), *tj = (int *)calloc(nb, sizeof(int));
        int *bj = (int *)calloc(nb, sizeof(int));
        float **aj = (float **)calloc(nb, sizeof(float *));
        int *sj = (int *)calloc(nb, sizeof(int));
        int nj = 0;
        for (int b = 0; b < nb; b++) {
            audio[b] = NULL;
            samples[b] = 0;
        }
        if (!hc || !slot || !tj || !bj || !aj || !sj) rc = -1;
        /* a slot without frames (or whose codes could not be read) gets no
         * audio and makes the call return -1; the other slots still decode */
        for (int b = 0; b < nb && hc && slot && tj && bj && aj && sj; b++) {
            if (ngen[b] <= 0) { rc = -1; continue; }
            const vclone_t *vc = vcs && vcs[b].ref_codes && vcs[b].n_ref > 0 ? &vcs[b] : NULL;
            slot[nj] = b;
            bj[nj] = b;
            tj[nj] = (vc ? vc->n_ref : 0) + ngen[b];
            if (vc) {
                hc[nj] = (int *)malloc((size_t)tj[nj] * G * sizeof(int));
                if (!hc[nj] || qtts_dev_get_codes(dev, b, hc[nj] + (size_t)vc->n_ref * G, ngen[b]) != ngen[b]) {
                    free(hc[nj]);
                    hc[nj] = NULL;
                    rc = -1;
                    continue;
                }
                memcpy(hc[nj], vc->ref_codes, (size_t)vc->n_ref * G * sizeof(int));
            }
            /* (-v lines per slot; the -v -v stage times are taken for a lone
             * decode only: the lanes of a batch run side by side) */
            if (qwen_tts_verbose >= 1)
                fprintf(stderr, "Codec decode: %d timesteps, %d quantizers\n", tj[nj], c->codec_num_quantizers);
            nj++;
        }
        if (nj > 0 && qtts_dev_codec_multi(dev, nj, (const int *const *)hc, slot, tj, aj, sj) != 0) rc = -1;
        for (int j = 0; j < nj; j++) {
            const int b = bj[j];
            if (qwen_tts_verbose >= 1 && aj[j] && sj[j] > 0)
                fprintf(stderr, "Codec decode complete: %d samples (%.2f seconds)\n", sj[j],
                        (float)sj[j] / QWEN_TTS_SAMPLE_RATE);
            if (hc[j]) {
                cut_reference(aj[j], sj[j], vcs[b].n_ref, tj[j], &audio[b], &samples[b]);
                aj[j] = NULL;
            } else {
                audio[b] = aj[j];
                samples[b] = sj[j];
                aj[j] = NULL;
            }
            if (!audio[b] || samples[b] <= 0) rc = -1;
        }
        for (int j = 0; j < nb; j++) {
            if (hc) free(hc[j]);
            if (aj) free(aj[j]);
        }
        free(hc); free(slot); free(tj); free(bj); free(aj); free(sj);
    }
    if (!stream) {
        ctx->perf_codec_ms = now_ms() - t_codec;
    }
    ctx->perf_total_ms = now_ms() - t_start;
    free(stopped); free(ngen); free(sstep);
out:
    for (int b = 0; b < nb; b++) { free(pr[b].text); free(pr[b].plan); }
    free(pr);
    return rc;
}

float *qwen_tts_generate(qwen_tts_ctx_t *ctx, const char *text, const char *speaker, const char *language,
                         int *out_samples) {
    if (!ctx || !out_samples) return NULL;
    *out_samples = 0;
    double t_start = now_ms();
    float *audio = NULL;
    int n = 0;
    const char *texts[1] = {text}, *spk[1] = {speaker}, *lang[1] = {language};
    int rc = run_batch(ctx, 1, texts, spk, lang, &audio, &n, t_start, NULL, NULL);
    if (rc != 0 || !audio || n <= 0) {
        free(audio);
        *out_samples = 0;
        return NULL;
    }
    if (qwen_tts_verbose >= 1) {
        fprintf(stderr, "Codec decode: %d samples in %.1f ms\n", n, ctx->perf_codec_ms);
        fprintf(stderr, "Total: %.1f ms (%.2f s audio, %.2fx realtime)\n", ctx->perf_total_ms,
                (float)n / QWEN_TTS_SAMPLE_RATE, ((float)n / QWEN_TTS_SAMPLE_RATE) / (ctx->perf_total_ms / 1000.0));
    }
    *out_samples = n;
    return audio;
}

int qwen_tts_generate_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts, const char *const *speakers,
                            const char *const *languages, float **out_audio, int *out_samples) {
    if (!ctx || nb < 1 || !texts || !out_audio || !out_samples) return -1;
    return run_batch(ctx, nb, texts, speakers, languages, out_audio, out_samples, now_ms(), NULL, NULL);
}

/* ------------------------------------------------------------- work queue */
/* EOS-mode utterances (Q.c:1282-1330: each stops at its own
 * EOS) on `nb` lock-step slots.  When a slot's utterance stops, its codes are
 * collected and the next queued utterance is prefilled into that slot inside
 * the live batch (qtts_dev_refill), so no slot rides along stopped while
 * others decode, except for the one frame the lagged stop poll costs.  The
 * frame loop is run_batch's: frame s + 1 is queued before the host waits for
 * frame s.  Every utterance decodes exactly as it would alone (its own KV
 * positions from 0, counters, repetition counts and RNG states from the seed);
 * the codec passes of all of them run at the end on the codec lanes
 * (qtts_dev_codec_multi). */
static int queue_pull(int nq, int *taken, int *next_seq, qwen_tts_queue_next_cb next, void *user) {
    if (next) {
        const int i = next(user);
        if (i < 0 || i >= nq || taken[i]) return -1;
        taken[i] = 1;
        return i;
    }
    while (*next_seq < nq && taken[*next_seq]) (*next_seq)++;
    if (*next_seq >= nq) return -1;
    taken[*next_seq] = 1;
    return (*next_seq)++;
}

static void queue_plan_slot(prompt_t *p, int b) {
    for (int k = 0; k < p->nplan; k++) p->plan[5 * k + 3] = b;
}

int qwen_tts_generate_queue(qwen_tts_ctx_t *ctx, int nq, const char *const *texts, const char *const *speakers,
                            const char *const *languages, int nb, qwen_tts_queue_next_cb next, void *user,
                            float **out_audio, int *out_samples) {
    if (!ctx || !ctx->hip || nq < 1 || nb < 1 || !texts || !out_audio || !out_samples) return -1;
    qtts_dev_t *dev = (qtts_dev_t *)ctx->hip;
    const qwen_tts_config_t *c = &ctx->config;
    const int G = c->num_code_groups;
    const double t_start = now_ms();
    int rc = -1;
    queue_clear(ctx);
    for (int i = 0; i < nq; i++) { out_audio[i] = NULL; out_samples[i] = 0; }
    prompt_t *pr = (prompt_t *)calloc(nq, sizeof(prompt_t));
    int *taken = (int *)calloc(nq, sizeof(int)), next_seq = 0;
    ctx->queue_codes = (int **)calloc(nq, sizeof(int *));
    ctx->queue_frames = (int *)malloc(nq * sizeof(int));
    ctx->queue_stop_reason = (int *)calloc(nq, sizeof(int));
    ctx->queue_slot = (int *)malloc(nq * sizeof(int));
    int *cur = (int *)malloc(nb * sizeof(int)), *first = (int *)calloc(nb, sizeof(int));
    int *retired = (int *)calloc(nb, sizeof(int)), *hst = (int *)calloc(nb, sizeof(int));
    int *cbuf = NULL;
    if (!pr || !taken || !ctx->queue_codes || !ctx->queue_frames || !ctx->queue_stop_reason || !ctx->queue_slot ||
        !cur || !first || !retired || !hst)
        goto out;
    ctx->queue_n = nq;
    for (int i = 0; i < nq; i++) { ctx->queue_frames[i] = -1; ctx->queue_slot[i] = -1; }
    /* every prompt up front (the prefill and trailing capacities cover all) */
    int max_p = 0, max_tr = 0;
    for (int i = 0; i < nq; i++) {
        int *ids = NULL;
        const int n = parse_ids(texts[i], &ids);
        if (n < 8) {
            if (n >= 0) fprintf(stderr, "Error: need at least 8 text tokens (chat template format)\n");
            free(ids);
            goto out;
        }
        for (int k = 0; k < n; k++)
            if (ids[k] < 0 || ids[k] >= c->talker_text_vocab) {
                fprintf(stderr, "Error: text token id %d out of range\n", ids[k]);
                free(ids);
                goto out;
            }
        int spk, lang;
        lookup(ctx, speakers ? speakers[i] : NULL, languages ? languages[i] : NULL, &spk, &lang);
        build_prompt(ctx, ids, n, spk, lang, 0, &pr[i]);
        free(ids);
        if (pr[i].p_len > max_p) max_p = pr[i].p_len;
        if (pr[i].n_trailing > max_tr) max_tr = pr[i].n_trailing;
    }
    const int fixed = ctx->fixed_codec_tokens > 0 ? ctx->fixed_codec_tokens : 0;
    const int max_tokens = fixed > 0 ? fixed : ctx->max_new_tokens;
    if (max_tokens < 1) goto out;
    /* the first nb utterances fill the slots */
    int ns = 0;
    while (ns < nb) {
        const int u = queue_pull(nq, taken, &next_seq, next, user);
        if (u < 0) break;
        cur[ns++] = u;
    }
    ctx->queue_slots = ns;
    if (ns == 0) { rc = 0; goto out; }   /* (another puller took everything) */
    qtts_gen_params_t gp;
    params_of(ctx, &gp);
    if (qtts_dev_begin(dev, ns, max_tokens, max_p, &gp) != 0 || qtts_dev_reserve(dev, max_tr) != 0) goto out;
    /* (a plan row's 4th int is the destination slot: set when the slot is known) */
#define PROMPT(b, u) (queue_plan_slot(&pr[u], (b)), \
                      qtts_dev_prompt(dev, (b), pr[u].text, pr[u].n_text, pr[u].plan, pr[u].nplan, pr[u].p_len, \
                                      pr[u].n_trailing, pr[u].pad_row))
    for (int b = 0; b < ns; b++)
        if (PROMPT(b, cur[b]) != 0) goto out;
    double t_prefill = now_ms();
    if (qtts_dev_prefill(dev) != 0) goto out;
    ctx->perf_prefill_ms = now_ms() - t_prefill;
    cbuf = (int *)malloc((size_t)(max_tokens + 1) * G * sizeof(int));
    if (!cbuf) goto out;
    int active = ns, done_n = 0, rows = ns, exhausted = 0;
    /* tail compaction (nothing left to admit): the running slots move to the
     * first rows and the frames launch those only (QTTS_QUEUE_COMPACT=0: off) */
    const char *ce = getenv("QTTS_QUEUE_COMPACT");
    const int compact = !(ce && !strcmp(ce, "0"));
    int step = 0;
    const double t_gen = now_ms();
    for (;; step++) {
        /* a slot whose utterance produced max_tokens frames by frame step - 1
         * stops before frame step (host count: no EOS draw marks it) */
        for (int b = 0; b < ns; b++)
            if (cur[b] >= 0 && !retired[b] && step - first[b] >= max_tokens) {
                if (qtts_dev_retire(dev, b) != 0) goto out;
                retired[b] = 1;
            }
        if (qtts_dev_frame(dev, step) != 0) goto out;
        ctx->queue_rows_launched += rows;
        if (step == 0) {
            qtts_dev_poll(dev, NULL, NULL, NULL);
            ctx->perf_first_frame_ms = now_ms() - t_start;
        }
        if (step < 1) continue;
        /* frame step is queued: which slots had stopped by frame step - 1 */
        if (qtts_dev_frame_stops(dev, step - 1, hst) != 0) goto out;
        for (int b = 0; b < ns; b++) {
            if (cur[b] < 0) continue;
            const int capped = step - first[b] >= max_tokens;
            if (!hst[b] && !capped) continue;
            /* utterance cur[b] is complete (slot b is a no-op in frame step) */
            const int u = cur[b];
            const int n = qtts_dev_get_codes(dev, b, cbuf, max_tokens);
            if (n < 0) goto out;
            ctx->queue_codes[u] = (int *)malloc((size_t)(n > 0 ? n : 1) * G * sizeof(int));
            if (!ctx->queue_codes[u]) goto out;
            memcpy(ctx->queue_codes[u], cbuf, (size_t)n * G * sizeof(int));
            ctx->queue_frames[u] = n;
            ctx->queue_stop_reason[u] = hst[b] ? 1 : 2;
            ctx->queue_slot[u] = b;
            ctx->queue_slot_frames_used += n;
            done_n++;
            if (qwen_tts_verbose >= 1)
                fprintf(stderr, "Queue: utterance %d on slot %d: %s at step %d (frame %d)\n", u, b,
                        hst[b] ? "eos" : "max_tokens", n, step - 1);
            cur[b] = -1;
            active--;
            const int u2 = exhausted ? -1 : queue_pull(nq, taken, &next_seq, next, user);
            if (u2 < 0) { exhausted = 1; continue; }
            if (PROMPT(b, u2) != 0 || qtts_dev_refill(dev, b) != 0) goto out;
            cur[b] = u2;
            first[b] = step + 1;   /* its frame 0 is the next frame launched */
            retired[b] = 0;
            hst[b] = 0;
            active++;
            ctx->queue_refills++;
        }
        if (active == 0) break;
        if (exhausted && compact && active < rows) {
            /* every freed slot below the last running one takes that one's state */
            for (int i = 0; i < rows; i++) {
                if (cur[i] >= 0) continue;
                int j = rows - 1;
                while (j > i && cur[j] < 0) j--;
                if (j <= i) break;
                if (qtts_dev_move_slot(dev, j, i) != 0) goto out;
                cur[i] = cur[j]; first[i] = first[j]; retired[i] = retired[j];
                cur[j] = -1;
            }
            rows = active;
            if (qtts_dev_set_rows(dev, rows) != 0) goto out;
        }
        if (ctx->progress_cb) ctx->progress_cb(done_n, nq, ctx->progress_cb_userdata);
    }
#undef PROMPT
    ctx->queue_frames_launched = step + 1;
    ctx->perf_talker_ms = now_ms() - t_gen;
    {
        /* every finished utterance's codec pass, several side by side */
        int nj = 0;
        int *uj = (int *)malloc(nq * sizeof(int)), *tj = (int *)malloc(nq * sizeof(int));
        int *sl = (int *)calloc(nq, sizeof(int)), *sj = (int *)calloc(nq, sizeof(int));
        const int **hc = (const int **)calloc(nq, sizeof(int *));
        float **aj = (float **)calloc(nq, sizeof(float *));
        if (!uj || !tj || !sl || !sj || !hc || !aj) {
            free(uj); free(tj); free(sl); free(sj); free(hc); free(aj);
            goto out;
        }
        rc = 0;
        for (int u = 0; u < nq; u++) {
            if (ctx->queue_frames[u] < 0) continue;   /* not taken by this ctx */
            if (ctx->queue_frames[u] == 0) { rc = -1; continue; }
            uj[nj] = u; tj[nj] = ctx->queue_frames[u]; hc[nj] = ctx->queue_codes[u];
            nj++;
        }
        const double t_codec = now_ms();
        if (nj > 0 && qtts_dev_codec_multi(dev, nj, hc, sl, tj, aj, sj) != 0) rc = -1;
        for (int j = 0; j < nj; j++) {
            out_audio[uj[j]] = aj[j];
            out_samples[uj[j]] = aj[j] ? sj[j] : 0;
            if (!aj[j] || sj[j] <= 0) rc = -1;
        }
        ctx->perf_codec_ms = now_ms() - t_codec;
        free(uj); free(tj); free(sl); free(sj); free(hc); free(aj);
    }
    ctx->perf_total_ms = now_ms() - t_start;
    if (qwen_tts_verbose >= 1)
        fprintf(stderr, "Queue: %d utterances on %d slots, %d frames (%lld slot rows), %d refills, occupancy %.3f\n",
                done_n, ns, ctx->queue_frames_launched, ctx->queue_rows_launched, ctx->queue_refills,
                (double)ctx->queue_slot_frames_used / (double)ctx->queue_rows_launched);
out:
    if (pr)
        for (int i = 0; i < nq; i++) { free(pr[i].text); free(pr[i].plan); }
    free(pr); free(taken); free(cur); free(first); free(retired); free(hst); free(cbuf);
    return rc;
}

int qwen_tts_queue_codes(qwen_tts_ctx_t *ctx, int i, int *codes, int max_frames) {
    if (!ctx || i < 0 || i >= ctx->queue_n || !ctx->queue_codes || !ctx->queue_codes[i] || max_frames < 0) return -1;
    const int n = ctx->queue_frames[i] < max_frames ? ctx->queue_frames[i] : max_frames;
    if (codes) memcpy(codes, ctx->queue_codes[i], (size_t)n * ctx->config.num_code_groups * sizeof(int));
    return n;
}

static int vclone_run(qwen_tts_ctx_t *ctx, int nb, const char *const *texts, const char *const *ref_texts,
                      const int *const *ref_codes, const int *n_ref_frames, const float *const *spk_embeds,
                      const char *const *languages, int non_streaming, float **out_audio, int *out_samples,
                      const stream_t *stream) {
    if (!ctx || nb < 1 || !texts || !out_audio || !out_samples || (stream && nb != 1)) return -1;
    for (int b = 0; b < nb; b++) { out_audio[b] = NULL; out_samples[b] = 0; }
    vclone_t *vcs = (vclone_t *)calloc(nb, sizeof(vclone_t));
    int rc = vcs ? 0 : -1;
    for (int b = 0; b < nb && rc == 0; b++) {
        vclone_t *vc = &vcs[b];
        const int *codes = ref_codes ? ref_codes[b] : NULL;
        const int nref = n_ref_frames ? n_ref_frames[b] : 0;
        vc->spk = spk_embeds ? spk_embeds[b] : NULL;
        vc->non_streaming = non_streaming;
        if (!(codes && nref > 0)) {
            if (!vc->spk) {
                fprintf(stderr, "Error: voice clone needs reference codes or a speaker embedding\n");
                rc = -1;
            }
            continue;
        }
        int *rid = NULL;
        vc->n_ref_ids = ref_texts && ref_texts[b] ? parse_ids(ref_texts[b], &rid) : 0;
        vc->ref_ids = rid;
        if (vc->n_ref_ids < 5) {
            fprintf(stderr, "Error: ICL voice clone needs the reference text ids (chat template, >= 5 ids)\n");
            rc = -1;
            continue;
        }
        for (int i = 0; i < vc->n_ref_ids; i++)
            if (rid[i] < 0 || rid[i] >= ctx->config.talker_text_vocab) {
                fprintf(stderr, "Error: text token id %d out of range\n", rid[i]);
                rc = -1;
                break;
            }
        vc->ref_codes = codes;
        vc->n_ref = nref;
    }
    if (rc == 0) rc = run_batch(ctx, nb, texts, NULL, languages, out_audio, out_samples, now_ms(), stream, vcs);
    if (vcs)
        for (int b = 0; b < nb; b++) free((void *)vcs[b].ref_ids);
    free(vcs);
    return rc;
}

int qwen_tts_generate_voice_clone_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts,
                                        const char *const *ref_texts, const int *const *ref_codes,
                                        const int *n_ref_frames, const float *const *spk_embeds,
                                        const char *const *languages, int non_streaming, float **out_audio,
                                        int *out_samples) {
    return vclone_run(ctx, nb, texts, ref_texts, ref_codes, n_ref_frames, spk_embeds, languages, non_streaming,
                      out_audio, out_samples, NULL);
}

float *qwen_tts_generate_voice_clone_stream(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                            const int *ref_codes, int n_ref_frames, const float *spk_embed,
                                            const char *language, int non_streaming, int chunk_frames,
                                            qwen_tts_audio_cb cb, void *userdata, int *out_samples) {
    if (!ctx || !out_samples) return NULL;
    *out_samples = 0;
    stream_t st = {cb, userdata, chunk_frames > 0 ? chunk_frames : 1};
    float *audio = NULL;
    int n = 0;
    const char *texts[1] = {text}, *rt[1] = {ref_text}, *lang[1] = {language};
    const int *rc1[1] = {ref_codes};
    const int nr1[1] = {n_ref_frames};
    const float *sv1[1] = {spk_embed};
    ctx->perf_first_packet_ms = 0;
    if (vclone_run(ctx, 1, texts, rt, rc1, nr1, sv1, lang, non_streaming, &audio, &n, &st) != 0 || !audio || n <= 0) {
        free(audio);
        return NULL;
    }
    *out_samples = n;
    return audio;
}

float *qwen_tts_generate_voice_clone(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                     const int *ref_codes, int n_ref_frames, const float *spk_embed,
                                     const char *language, int non_streaming, int *out_samples) {
    if (!ctx || !out_samples) return NULL;
    *out_samples = 0;
    float *audio = NULL;
    int n = 0;
    const char *texts[1] = {text}, *rt[1] = {ref_text}, *lang[1] = {language};
    const int *rc1[1] = {ref_codes};
    const int nr1[1] = {n_ref_frames};
    const float *sv1[1] = {spk_embed};
    if (qwen_tts_generate_voice_clone_batch(ctx, 1, texts, rt, rc1, nr1, sv1, lang, non_streaming, &audio, &n) != 0 ||
        !audio || n <= 0) {
        free(audio);
        return NULL;
    }
    *out_samples = n;
    return audio;
}

/* ------------------------------------------- voice clone from reference audio (N3) */
float *qwen_tts_speaker_embedding(qwen_tts_ctx_t *ctx, const float *wav, int n_samples, int *out_dim) {
    if (out_dim) *out_dim = 0;
    if (!ctx || !ctx->hip || !wav || n_samples <= 0) return NULL;
    const int dim = ctx->config.talker_hidden;
    float *out = (float *)malloc((size_t)dim * sizeof(float));
    if (!out) return NULL;
    const float *w[1] = {wav};
    const int n[1] = {n_samples};
    if (qtts_dev_speaker_embed((qtts_dev_t *)ctx->hip, 1, w, n, out, NULL) != 0) {
        free(out);
        return NULL;
    }
    if (out_dim) *out_dim = dim;
    return out;
}

int *qwen_tts_encode_audio(qwen_tts_ctx_t *ctx, const float *wav, int n_samples, int *out_frames) {
    if (out_frames) *out_frames = 0;
    if (!ctx || !ctx->hip || !wav || n_samples <= 0) return NULL;
    const int T = (n_samples + 1919) / 1920;
    int *codes = (int *)malloc((size_t)T * 16 * sizeof(int));
    if (!codes) return NULL;
    const float *w[1] = {wav};
    const int n[1] = {n_samples};
    int fr = 0;
    if (qtts_dev_encode_audio((qtts_dev_t *)ctx->hip, 1, w, n, codes, T, &fr, NULL) != 0) {
        free(codes);
        return NULL;
    }
    if (out_frames) *out_frames = fr;
    return codes;
}

/* create_voice_clone_prompt (qwen3_tts_model.py:356-458) + generate_voice_clone:
 * every reference audio is encoded in ONE padded batch (the tokenizer's batch
 * encode, :427), each x-vector on its own audio (:446), then the codes /
 * x-vector voice clone above.  x_vector_only[b] (NULL: all 0) drops the codes
 * of slot b (ref_code=None, :451). */
int qwen_tts_generate_voice_clone_audio_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts,
                                              const char *const *ref_texts, const float *const *ref_wavs,
                                              const int *n_ref_samples, const char *const *languages,
                                              const int *x_vector_only, int non_streaming, float **out_audio,
                                              int *out_samples) {
    if (!ctx || !ctx->hip || nb < 1 || nb > 16 || !texts || !ref_wavs || !n_ref_samples || !out_audio ||
        !out_samples) {
        fprintf(stderr, "Error: voice clone from audio needs 1..16 utterances with reference audio\n");
        return -1;
    }
    for (int b = 0; b < nb; b++) { out_audio[b] = NULL; out_samples[b] = 0; }
    qtts_dev_t *dev = (qtts_dev_t *)ctx->hip;
    if ((qtts_dev_enc_available(dev) & 3) != 3) {
        fprintf(stderr, "Error: the model directory has no speaker encoder / 12 Hz encoder weights\n");
        return -1;
    }
    for (int b = 0; b < nb; b++)
        if (!x_vector_only || !x_vector_only[b])
            if (!ref_texts || !ref_texts[b] || !ref_texts[b][0]) {
                fprintf(stderr, "Error: ref_text is required when x_vector_only_mode=False (ICL mode). Bad index=%d\n", b);
                return -1;
            }
    double t0 = now_ms();
    const int H = ctx->config.talker_hidden;
    int maxT = 0;
    for (int b = 0; b < nb; b++) {
        const int T = (n_ref_samples[b] + 1919) / 1920;
        if (T > maxT) maxT = T;
    }
    int *codes = (int *)malloc((size_t)nb * (maxT > 0 ? maxT : 1) * 16 * sizeof(int));
    float *xv = (float *)malloc((size_t)nb * H * sizeof(float));
    int frames[16];
    int rc = -1;
    if (codes && xv && qtts_dev_encode_audio(dev, nb, ref_wavs, n_ref_samples, codes, maxT, frames, NULL) == 0 &&
        qtts_dev_speaker_embed(dev, nb, ref_wavs, n_ref_samples, xv, NULL) == 0) {
        const int *rc_p[16];
        int nr[16];
        const float *sv[16];
        for (int b = 0; b < nb; b++) {
            const int xo = x_vector_only && x_vector_only[b];
            rc_p[b] = xo ? NULL : codes + (size_t)b * maxT * 16;
            nr[b] = xo ? 0 : frames[b];
            sv[b] = xv + (size_t)b * H;
        }
        if (qwen_tts_verbose >= 1) fprintf(stderr, "Reference audio encoded in %.1f ms\n", now_ms() - t0);
        const char *const *rt = ref_texts;
        const char *none[16] = {NULL};
        if (!rt) rt = none;
        rc = qwen_tts_generate_voice_clone_batch(ctx, nb, texts, rt, rc_p, nr, sv, languages, non_streaming, out_audio,
                                                 out_samples);
    }
    free(codes);
    free(xv);
    return rc;
}

/* streaming form of qwen_tts_generate_voice_clone_audio: the reference audio
 * is encoded first, then qwen_tts_generate_voice_clone_stream; the first
 * packet time (ctx->perf_first_packet_ms) counts from this call's entry */
float *qwen_tts_generate_voice_clone_audio_stream(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                                  const float *ref_wav, int n_ref_samples, const char *language,
                                                  int x_vector_only, int non_streaming, int chunk_frames,
                                                  qwen_tts_audio_cb cb, void *userdata, int *out_samples) {
    if (!out_samples) return NULL;
    *out_samples = 0;
    if (!ctx || !ctx->hip || !ref_wav || n_ref_samples <= 0) return NULL;
    qtts_dev_t *dev = (qtts_dev_t *)ctx->hip;
    if ((qtts_dev_enc_available(dev) & 3) != 3) {
        fprintf(stderr, "Error: the model directory has no speaker encoder / 12 Hz encoder weights\n");
        return NULL;
    }
    if (!x_vector_only && (!ref_text || !ref_text[0])) {
        fprintf(stderr, "Error: ref_text is required when x_vector_only_mode=False (ICL mode). Bad index=0\n");
        return NULL;
    }
    const double t0 = now_ms();
    const int T = (n_ref_samples + 1919) / 1920, H = ctx->config.talker_hidden;
    int *codes = (int *)malloc((size_t)T * 16 * sizeof(int));
    float *xv = (float *)malloc((size_t)H * sizeof(float));
    const float *w[1] = {ref_wav};
    const int n[1] = {n_ref_samples};
    int fr = 0;
    float *audio = NULL;
    if (codes && xv && qtts_dev_encode_audio(dev, 1, w, n, codes, T, &fr, NULL) == 0 &&
        qtts_dev_speaker_embed(dev, 1, w, n, xv, NULL) == 0) {
        const double enc_ms = now_ms() - t0;
        audio = qwen_tts_generate_voice_clone_stream(ctx, text, x_vector_only ? NULL : ref_text,
                                                     x_vector_only ? NULL : codes, x_vector_only ? 0 : fr, xv,
                                                     language, non_streaming, chunk_frames, cb, userdata, out_samples);
        if (audio && ctx->perf_first_packet_ms > 0) ctx->perf_first_packet_ms += enc_ms;
    }
    free(codes);
    free(xv);
    return audio;
}

float *qwen_tts_generate_voice_clone_audio(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                           const float *ref_wav, int n_ref_samples, const char *language,
                                           int x_vector_only, int non_streaming, int *out_samples) {
    if (!out_samples) return NULL;
    *out_samples = 0;
    float *audio = NULL;
    int n = 0;
    const char *texts[1] = {text}, *rt[1] = {ref_text}, *lang[1] = {language};
    const float *w[1] = {ref_wav};
    const int nn[1] = {n_ref_samples}, xo[1] = {x_vector_only};
    if (qwen_tts_generate_voice_clone_audio_batch(ctx, 1, texts, rt, w, nn, lang, xo, non_streaming, &audio, &n) != 0 ||
        !audio || n <= 0) {
        free(audio);
        return NULL;
    }
    *out_samples = n;
    return audio;
}

float *qwen_tts_generate_stream(qwen_tts_ctx_t *ctx, const char *text, const char *speaker, const char *language,
                                int chunk_frames, qwen_tts_audio_cb cb, void *userdata, int *out_samples) {
    if (!ctx || !out_samples) return NULL;
    *out_samples = 0;
    double t_start = now_ms();
    stream_t st = {cb, userdata, chunk_frames > 0 ? chunk_frames : 1};
    float *audio = NULL;
    int n = 0;
    const char *texts[1] = {text}, *spk[1] = {speaker}, *lang[1] = {language};
    ctx->perf_first_packet_ms = 0;
    int rc = run_batch(ctx, 1, texts, spk, lang, &audio, &n, t_start, &st, NULL);
    if (rc != 0 || !audio || n <= 0) {
        free(audio);
        return NULL;
    }
    if (qwen_tts_verbose >= 1) {
        fprintf(stderr, "First packet: %.1f ms\n", ctx->perf_first_packet_ms);
        fprintf(stderr, "Total: %.1f ms (%.2f s audio, %.2fx realtime)\n", ctx->perf_total_ms,
                (float)n / QWEN_TTS_SAMPLE_RATE, ((float)n / QWEN_TTS_SAMPLE_RATE) / (ctx->perf_total_ms / 1000.0));
    }
    *out_samples = n;
    return audio;
}

int qwen_tts_codec_stream_begin(qwen_tts_ctx_t *ctx, int max_frames) {
    if (!ctx || !ctx->hip) return -1;
    return qtts_dev_codec_stream_begin((qtts_dev_t *)ctx->hip, max_frames);
}

int qwen_tts_codec_stream_push(qwen_tts_ctx_t *ctx, const int *codes, int time_steps, float *out) {
    if (!ctx || !ctx->hip || !codes || !out || time_steps < 1) return -1;
    return qtts_dev_codec_stream_push_host((qtts_dev_t *)ctx->hip, codes, time_steps, out);
}

int qwen_tts_last_codes(qwen_tts_ctx_t *ctx, int *codes, int max_frames) {
    if (!ctx || !ctx->last_codes) return 0;
    int n = ctx->last_frames < max_frames ? ctx->last_frames : max_frames;
    memcpy(codes, ctx->last_codes, (size_t)n * ctx->config.num_code_groups * sizeof(int));
    return n;
}

int qwen_tts_last_codes_slot(qwen_tts_ctx_t *ctx, int slot, int *codes, int max_frames) {
    if (!ctx || !ctx->hip || slot < 0 || max_frames < 0) return -1;
    if (slot == 0) return qwen_tts_last_codes(ctx, codes, max_frames);
    return qtts_dev_get_codes((qtts_dev_t *)ctx->hip, slot, codes, max_frames);
}

/* -------------------------------------------------- stage functions (host) */
void qwen_tts_talker_prefill(qwen_tts_ctx_t *ctx, const float *input_embeds, int seq_len) {
    if (qtts_dev_talker_prefill_host((qtts_dev_t *)ctx->hip, input_embeds, seq_len, ctx->tk_x) != 0) {
        fprintf(stderr, "Error: talker prefill failed\n");
        return;
    }
    ctx->talker_kv_len = seq_len;
    if (qwen_tts_verbose >= 1) fprintf(stderr, "Talker prefill complete: %d tokens\n", seq_len);
}

void qwen_tts_talker_forward(qwen_tts_ctx_t *ctx, const float *input_embed, float *logits) {
    if (qtts_dev_talker_forward_host((qtts_dev_t *)ctx->hip, input_embed, logits, ctx->tk_x) != 0) {
        fprintf(stderr, "Error: talker forward failed\n");
        return;
    }
    ctx->talker_kv_len++;
}

void qwen_tts_subtalker_generate(qwen_tts_ctx_t *ctx, const float *talker_hidden, int first_code, int *out_codes) {
    qtts_gen_params_t gp;
    params_of(ctx, &gp);
    qtts_dev_t *dev = (qtts_dev_t *)ctx->hip;
    /* keep the device's sampling parameters in sync with the ctx fields */
    if (qtts_dev_begin(dev, 1, ctx->max_new_tokens > 0 ? ctx->max_new_tokens : 1, 16, &gp) != 0 ||
        qtts_dev_subtalker_host(dev, talker_hidden, first_code, out_codes) != 0)
        fprintf(stderr, "Error: sub-talker failed\n");
}

float *qwen_tts_codec_decode(qwen_tts_ctx_t *ctx, const int *codes, int time_steps, int *out_samples) {
    if (!ctx || !codes || !out_samples || time_steps <= 0) {
        if (out_samples) *out_samples = 0;
        return NULL;
    }
    codec_log_begin(ctx, time_steps);
    float *w = qtts_dev_codec_decode_host((qtts_dev_t *)ctx->hip, codes, time_steps, out_samples);
    codec_log_end(ctx, w ? *out_samples : 0);
    return w;
}

int qwen_tts_talker_hidden(qwen_tts_ctx_t *ctx, float *out) {
    if (!ctx || !ctx->tk_x) return -1;
    memcpy(out, ctx->tk_x, ctx->config.talker_hidden * sizeof(float));
    return 0;
}

/* ABI self-check for FFI bindings (tests/test_host.py compares this with the
 * ctypes mirror of qwen_tts_ctx_t) */
size_t qwen_tts_abi_sizeof_ctx(void) { return sizeof(qwen_tts_ctx_t); }
