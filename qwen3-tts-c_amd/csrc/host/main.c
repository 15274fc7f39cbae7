/*
 * main.c - `qwen-tts` CLI on the MI355X hot path.
 *
 * Flags, defaults and the stderr lines the reference harness parses are the
 * reference CLI's (c/main.c:25-69,126-173,266-271; regexes in
 * scripts/benchmark_py_vs_c.py:104-138, test/test_eos_regression.py:20-28):
 *   -d DIR -t IDS | -f FILE  -s SPK -l LANG -o OUT -v [-v]
 *   --temperature --top-k --top-p --repetition-penalty --max-tokens
 *   --fixed-codec-tokens --seed --subtalker-temperature --subtalker-top-k
 *   --subtalker-top-p --benchmark-runs --benchmark-warmup
 * Additions: --device N (HIP device), --batch N (N copies of the prompt in
 * one lock-step batch; the first one's audio is written), --stream N (exact
 * streaming decode: audio delivered after frame 0 and then every N frames;
 * prints "First packet: X ms").
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../../include/qwen_tts.h"

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1000.0 + (double)ts.tv_nsec / 1e6;
}

static void usage(const char *prog) {
    fprintf(stderr,
            "qwen-tts (MI355X / gfx950) - Qwen3-TTS talker + sub-talker decode and codec vocoder on the GPU\n\n"
            "usage: %s -d <model_dir> (-t <ids> | -f <file> | -T <text>) [options]\n\n"
            "  -d <dir>    model directory (config.json, *.safetensors, speech_tokenizer/)\n"
            "  -t <ids>    comma-separated token ids in the chat template\n"
            "  -f <file>   token ids from a file (comma- or newline-separated)\n"
            "  -T <text>   text, tokenized with the model dir's vocab.json / merges.txt (Qwen2 BPE)\n"
            "              inside the chat template; --print-ids prints the ids and exits\n"
            "  -s <name>   speaker (config.json spk_id)      -l <lang>  language or auto\n"
            "  -o <path>   output wav (default output.wav)   -v         verbose (repeatable)\n"
            "  --temperature F (0.9)   --top-k N (50)   --top-p F (1.0)   --repetition-penalty F (1.05)\n"
            "  --max-tokens N (4096)   --fixed-codec-tokens N   --seed N (42)\n"
            "  --subtalker-temperature F (0.9)   --subtalker-top-k N (50)   --subtalker-top-p F (1.0)\n"
            "  --benchmark-runs N (1)  --benchmark-warmup N (0)\n"
            "  --device N (HIP device, default 0)   --batch N (lock-step batch of N copies, default 1)\n"
            "  --stream N (streaming decode, audio chunks every N frames after the first)\n"
            "voice clone (include/qwen_tts.h qwen_tts_generate_voice_clone[_audio]):\n"
            "  --ref-audio <wav>   reference audio (mono/stereo PCM16 or float WAV; other rates are resampled\n"
            "                      to 24 kHz): encoded on the GPU (12 Hz codes + speaker x-vector)\n"
            "  --x-vector-only     with --ref-audio: x-vector only (no reference codes / ref text)\n"
            "  --ref-codes <file>  12 Hz codes of the reference audio, 16 ints per frame (any separators)\n"
            "  --ref-text <ids>    ids of \"<|im_start|>assistant\\n{ref text}<|im_end|>\\n\" (ICL mode)\n"
            "  --xvector <file>    speaker-encoder x-vector, talker-hidden floats (any separators)\n"
            "  --non-streaming     non-streaming text layout\n",
            prog);
}

static char *read_ids_file(const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) {
        fprintf(stderr, "Error: cannot open token file: %s\n", path);
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)n + 1);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) {
        free(buf);
        fclose(f);
        return NULL;
    }
    fclose(f);
    buf[n] = 0;
    for (long i = 0; i < n; i++)
        if (buf[i] == '\n' || buf[i] == '\r') buf[i] = ',';
    return buf;
}

/* whitespace / comma separated numbers of a text file (voice-clone inputs) */
static double *read_numbers(const char *path, int *n_out) {
    char *buf = read_ids_file(path);
    if (!buf) return NULL;
    int cap = 1024, n = 0;
    double *v = (double *)malloc(cap * sizeof(double));
    for (char *p = buf; *p;) {
        while (*p && (*p == ',' || *p == ' ' || *p == '\t')) p++;
        if (!*p) break;
        char *end = NULL;
        const double x = strtod(p, &end);
        if (end == p) { fprintf(stderr, "Error: bad number in %s near '%.16s'\n", path, p); free(v); free(buf); return NULL; }
        if (n == cap) v = (double *)realloc(v, (cap *= 2) * sizeof(double));
        v[n++] = x;
        p = end;
    }
    free(buf);
    *n_out = n;
    return v;
}

/* RIFF/WAVE reader for --ref-audio: PCM 16-bit or IEEE float 32-bit, any
 * channel count (averaged to mono, as qwen3_tts_tokenizer.py:152-153 does) */
static float *read_wav(const char *path, int *n_out, int *sr_out) {
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "Error: cannot open %s\n", path); return NULL; }
    unsigned char h[12];
    float *out = NULL;
    int fmt = 0, ch = 0, bits = 0, sr = 0;
    if (fread(h, 1, 12, f) != 12 || memcmp(h, "RIFF", 4) || memcmp(h + 8, "WAVE", 4)) {
        fprintf(stderr, "Error: %s is not a RIFF/WAVE file\n", path);
        fclose(f);
        return NULL;
    }
    for (;;) {
        unsigned char c[8];
        if (fread(c, 1, 8, f) != 8) break;
        const unsigned len = c[4] | c[5] << 8 | c[6] << 16 | (unsigned)c[7] << 24;
        if (!memcmp(c, "fmt ", 4)) {
            unsigned char b[40] = {0};
            if (len < 16 || fread(b, 1, len < 40 ? len : 40, f) != (len < 40 ? len : 40)) break;
            if (len > 40) fseek(f, len - 40, SEEK_CUR);
            fmt = b[0] | b[1] << 8;
            ch = b[2] | b[3] << 8;
            sr = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
            bits = b[14] | b[15] << 8;
            if (fmt == 0xFFFE && len >= 26) fmt = b[24] | b[25] << 8;   /* WAVE_FORMAT_EXTENSIBLE sub-format */
        } else if (!memcmp(c, "data", 4)) {
            const int bps = bits / 8;
            if (ch < 1 || !((fmt == 1 && bits == 16) || (fmt == 3 && bits == 32))) {
                fprintf(stderr, "Error: %s: only PCM16 or float32 WAV is supported\n", path);
                break;
            }
            const int n = (int)(len / (unsigned)(bps * ch));
            unsigned char *raw = (unsigned char *)malloc(len ? len : 1);
            out = (float *)malloc((size_t)(n > 0 ? n : 1) * sizeof(float));
            if (!raw || !out || fread(raw, 1, len, f) != len) { free(raw); free(out); out = NULL; break; }
            for (int i = 0; i < n; i++) {
                double acc = 0;
                for (int k = 0; k < ch; k++) {
                    const unsigned char *p = raw + ((size_t)i * ch + k) * bps;
                    if (fmt == 1) acc += (short)(p[0] | p[1] << 8) / 32768.0;
                    else { float v; memcpy(&v, p, 4); acc += v; }
                }
                out[i] = (float)(acc / ch);
            }
            free(raw);
            *n_out = n;
            *sr_out = sr;
            break;
        } else {
            fseek(f, len + (len & 1), SEEK_CUR);
        }
    }
    fclose(f);
    if (!out) fprintf(stderr, "Error: no audio data in %s\n", path);
    return out;
}

static void progress(int step, int total, void *u) {
    (void)total;
    (void)u;
    if (step % 50 == 0 || step < 5) {
        fprintf(stderr, "\rGenerating... step %d", step);
        fflush(stderr);
    }
}

int main(int argc, char **argv) {
    const char *dir = NULL, *ids = NULL, *ids_file = NULL, *spk = NULL, *lang = NULL, *out = "output.wav";
    int verbose = 0, runs = 1, warmup = 0, device = -1, batch = 1, stream_chunk = 0, non_streaming = 0;
    const char *ref_codes_file = NULL, *ref_text = NULL, *xvec_file = NULL, *text = NULL, *ref_audio = NULL;
    int print_ids = 0, xvec_only = 0;
    float temp = -1, st_temp = -1, top_p = -1, st_top_p = -1, rep = -1;
    int top_k = -1, st_top_k = -1, max_tokens = -1, fixed = -1, seed = -1;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        const int more = i + 1 < argc;
#define ARG(flag) (!strcmp(a, flag) && more)
        if (ARG("-d")) dir = argv[++i];
        else if (ARG("-t")) ids = argv[++i];
        else if (ARG("-f")) ids_file = argv[++i];
        else if (ARG("-T")) text = argv[++i];
        else if (!strcmp(a, "--print-ids")) print_ids = 1;
        else if (ARG("-s")) spk = argv[++i];
        else if (ARG("-l")) lang = argv[++i];
        else if (ARG("-o")) out = argv[++i];
        else if (!strcmp(a, "-v")) verbose++;
        else if (ARG("--temperature")) temp = strtof(argv[++i], NULL);
        else if (ARG("--top-k")) top_k = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--top-p")) top_p = strtof(argv[++i], NULL);
        else if (ARG("--repetition-penalty")) rep = strtof(argv[++i], NULL);
        else if (ARG("--max-tokens")) max_tokens = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--fixed-codec-tokens")) fixed = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--seed")) seed = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--subtalker-temperature")) st_temp = strtof(argv[++i], NULL);
        else if (ARG("--subtalker-top-k")) st_top_k = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--subtalker-top-p")) st_top_p = strtof(argv[++i], NULL);
        else if (ARG("--benchmark-runs")) runs = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--benchmark-warmup")) warmup = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--device")) device = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--batch")) batch = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--stream")) stream_chunk = (int)strtol(argv[++i], NULL, 10);
        else if (ARG("--ref-codes")) ref_codes_file = argv[++i];
        else if (ARG("--ref-text")) ref_text = argv[++i];
        else if (ARG("--xvector")) xvec_file = argv[++i];
        else if (ARG("--ref-audio")) ref_audio = argv[++i];
        else if (!strcmp(a, "--x-vector-only")) xvec_only = 1;
        else if (!strcmp(a, "--non-streaming")) non_streaming = 1;
        else if (!strcmp(a, "-h") || !strcmp(a, "--help")) { usage(argv[0]); return 0; }
        else {
            fprintf(stderr, "Unknown option: %s\n", a);
            usage(argv[0]);
            return 1;
        }
#undef ARG
    }
    if (!dir) { fprintf(stderr, "Error: model directory required (-d)\n\n"); usage(argv[0]); return 1; }
    if (!ids && !ids_file && !text) {
        fprintf(stderr, "Error: token IDs required (-t or -f) or text (-T)\n\n");
        usage(argv[0]);
        return 1;
    }
    if (text && print_ids) {   /* tokenizer only: no model load, no GPU */
        int n = 0;
        static const char pre[] = "<|im_start|>assistant\n", post[] = "<|im_end|>\n<|im_start|>assistant\n";
        char *chat = (char *)malloc(strlen(text) + sizeof pre + sizeof post);
        if (!chat) return 1;
        sprintf(chat, "%s%s%s", pre, text, post);
        int *tid = qwen_tts_tokenize(dir, chat, &n);
        free(chat);
        if (!tid) return 1;
        for (int k = 0; k < n; k++) printf(k ? ",%d" : "%d", tid[k]);
        printf("\n");
        free(tid);
        return 0;
    }
    if (runs < 1 || warmup < 0 || batch < 1) {
        fprintf(stderr, "Error: invalid benchmark settings (--benchmark-runs >= 1, --benchmark-warmup >= 0)\n");
        return 1;
    }
    char *file_ids = NULL;
    if (ids_file) {
        if (!(file_ids = read_ids_file(ids_file))) return 1;
        ids = file_ids;
    }
    /* voice clone inputs */
    int *ref_codes = NULL, n_ref = 0;
    float *xvec = NULL;
    int n_xvec = 0;
    const int clone = ref_codes_file || xvec_file || ref_audio;
    if (ref_audio && (ref_codes_file || xvec_file)) {
        fprintf(stderr, "Error: --ref-audio replaces --ref-codes / --xvector\n");
        free(file_ids);
        return 1;
    }
    float *ref_wav = NULL;
    int n_ref_wav = 0;
    if (ref_audio) {
        int sr = 0;
        if (!(ref_wav = read_wav(ref_audio, &n_ref_wav, &sr))) { free(file_ids); return 1; }
        if (sr != QWEN_TTS_SAMPLE_RATE) {   /* the reference resamples with librosa (qwen3_tts_model.py:441-444) */
            int n24 = 0;
            float *w24 = qwen_tts_resample(ref_wav, n_ref_wav, sr, QWEN_TTS_SAMPLE_RATE, &n24);
            free(ref_wav);
            if (!w24) { fprintf(stderr, "Error: cannot resample --ref-audio from %d Hz\n", sr); free(file_ids); return 1; }
            if (verbose >= 1)
                fprintf(stderr, "Reference audio resampled %d -> %d Hz (polyphase): %d -> %d samples\n", sr,
                        QWEN_TTS_SAMPLE_RATE, n_ref_wav, n24);
            ref_wav = w24;
            n_ref_wav = n24;
        }
        if (!xvec_only && !ref_text) {
            fprintf(stderr, "Error: ref_text is required when x_vector_only_mode=False (ICL mode): pass --ref-text or --x-vector-only\n");
            free(ref_wav); free(file_ids);
            return 1;
        }
    }
    if (clone && (batch != 1 || stream_chunk > 0)) {
        fprintf(stderr, "Error: voice clone runs at --batch 1 without --stream\n");
        free(file_ids);
        return 1;
    }
    if (ref_codes_file) {
        int n = 0;
        double *v = read_numbers(ref_codes_file, &n);
        if (!v || n < 16 || n % 16) {
            fprintf(stderr, "Error: --ref-codes needs 16 ints per frame (%d numbers read)\n", n);
            free(v); free(file_ids);
            return 1;
        }
        n_ref = n / 16;
        ref_codes = (int *)malloc((size_t)n * sizeof(int));
        for (int i = 0; i < n; i++) ref_codes[i] = (int)v[i];
        free(v);
    }
    if (xvec_file) {
        int n = 0;
        double *v = read_numbers(xvec_file, &n);
        if (!v || n < 1) { free(v); free(ref_codes); free(file_ids); return 1; }
        n_xvec = n;
        xvec = (float *)malloc((size_t)n * sizeof(float));
        for (int i = 0; i < n; i++) xvec[i] = (float)v[i];
        free(v);
        if (verbose >= 1) fprintf(stderr, "x-vector: %d floats\n", n);
    }
    qwen_tts_verbose = verbose;
    if (verbose >= 1) fprintf(stderr, "Loading model from %s...\n", dir);
    qwen_tts_ctx_t *ctx = qwen_tts_load_on(dir, device);
    if (!ctx) {
        fprintf(stderr, "Error: failed to load model\n");
        free(file_ids);
        return 1;
    }
    if (text && !ids) {   /* -T: the chat-template ids of the text (Qwen2 BPE, bpe.c) */
        if (!(file_ids = qwen_tts_text_prompt(ctx, text))) {
            fprintf(stderr, "Error: cannot tokenize the text\n");
            qwen_tts_free(ctx); free(ref_codes); free(xvec);
            return 1;
        }
        ids = file_ids;
    }
    if (xvec && n_xvec != ctx->config.talker_hidden) {
        fprintf(stderr, "Error: --xvector has %d floats, the talker hidden size is %d\n", n_xvec,
                ctx->config.talker_hidden);
        qwen_tts_free(ctx); free(ref_codes); free(xvec); free(file_ids);
        return 1;
    }
    if (temp >= 0) ctx->temperature = temp;
    if (st_temp >= 0) ctx->subtalker_temperature = st_temp;
    if (top_k >= 0) ctx->top_k = top_k;
    if (st_top_k >= 0) ctx->subtalker_top_k = st_top_k;
    if (top_p >= 0) ctx->top_p = top_p;
    if (st_top_p >= 0) ctx->subtalker_top_p = st_top_p;
    if (rep >= 0) ctx->repetition_penalty = rep;
    if (max_tokens >= 0) ctx->max_new_tokens = max_tokens;
    if (fixed >= 0) ctx->fixed_codec_tokens = fixed;
    if (seed >= 0) ctx->sample_seed = seed;
    if (verbose == 0) qwen_tts_set_progress_callback(ctx, progress, NULL);
    if (verbose >= 1) {
        fprintf(stderr, "Generation params: temp=%.2f top_k=%d top_p=%.2f rep_penalty=%.2f max_tokens=%d\n",
                ctx->temperature, ctx->top_k, ctx->top_p, ctx->repetition_penalty, ctx->max_new_tokens);
        if (ctx->fixed_codec_tokens > 0) fprintf(stderr, "Fixed codec tokens: %d\n", ctx->fixed_codec_tokens);
        fprintf(stderr, "Seed: %d\n", ctx->sample_seed);
        if (spk) fprintf(stderr, "Speaker: %s\n", spk);
        if (lang) fprintf(stderr, "Language: %s\n", lang);
    }
    float *audio = NULL;
    int n_samples = 0, rc = 0;
    for (int run = 0; run < warmup + runs; run++) {
        const double t0 = now_ms();
        float *ra = NULL;
        int rn = 0;
        long total_samples = 0;
        if (ref_wav) {
            ra = qwen_tts_generate_voice_clone_audio(ctx, ids, xvec_only ? NULL : ref_text, ref_wav, n_ref_wav, lang,
                                                     xvec_only, non_streaming, &rn);
            total_samples = rn;
        } else if (clone) {
            ra = qwen_tts_generate_voice_clone(ctx, ids, ref_text, ref_codes, n_ref, xvec, lang, non_streaming, &rn);
            total_samples = rn;
        } else if (batch == 1 && stream_chunk > 0) {
            ra = qwen_tts_generate_stream(ctx, ids, spk, lang, stream_chunk, NULL, NULL, &rn);
            total_samples = rn;
        } else if (batch == 1) {
            ra = qwen_tts_generate(ctx, ids, spk, lang, &rn);
            total_samples = rn;
        } else {
            const char **tx = (const char **)malloc(batch * sizeof(char *));
            const char **sp = (const char **)malloc(batch * sizeof(char *));
            const char **lg = (const char **)malloc(batch * sizeof(char *));
            float **au = (float **)calloc(batch, sizeof(float *));
            int *ns = (int *)calloc(batch, sizeof(int));
            for (int b = 0; b < batch; b++) { tx[b] = ids; sp[b] = spk; lg[b] = lang; }
            if (qwen_tts_generate_batch(ctx, batch, tx, sp, lg, au, ns) == 0) {
                ra = au[0];
                rn = ns[0];
                for (int b = 0; b < batch; b++) total_samples += ns[b];
            }
            for (int b = 1; b < batch; b++) free(au[b]);
            free(tx); free(sp); free(lg); free(au); free(ns);
        }
        const double el = now_ms() - t0;
        if (verbose == 0) fprintf(stderr, "\n");
        if (!ra || rn == 0) {
            fprintf(stderr, "Error: generation produced no audio\n");
            free(ra);
            rc = 1;
            break;
        }
        const int mi = run - warmup;
        if (mi >= 0 && runs > 1)
            fprintf(stderr,
                    "[persistent] run %d/%d: elapsed=%.1f ms, audio=%.2fs, talker=%.1f ms, codec=%.1f ms, "
                    "total=%.1f ms, tokens=%d\n",
                    mi + 1, runs, el, (float)total_samples / QWEN_TTS_SAMPLE_RATE, ctx->perf_talker_ms,
                    ctx->perf_codec_ms, ctx->perf_total_ms, ctx->perf_codec_tokens);
        free(audio);
        audio = ra;
        n_samples = rn;
    }
    if (rc == 0) {
        if (qwen_tts_write_wav(out, audio, n_samples, QWEN_TTS_SAMPLE_RATE) != 0) {
            fprintf(stderr, "Error: failed to write %s\n", out);
            rc = 1;
        } else {
            const float dur = (float)n_samples / QWEN_TTS_SAMPLE_RATE;
            fprintf(stderr, "Wrote %s: %.2f seconds (%d samples at %d Hz)\n", out, dur, n_samples,
                    QWEN_TTS_SAMPLE_RATE);
            if (verbose >= 1) {
                fprintf(stderr, "\nPerformance:\n");
                fprintf(stderr, "  Talker:  %.1f ms (%d tokens, %.1f ms/token)\n", ctx->perf_talker_ms,
                        ctx->perf_codec_tokens,
                        ctx->perf_codec_tokens > 0 ? ctx->perf_talker_ms / ctx->perf_codec_tokens : 0);
                fprintf(stderr, "  Codec:   %.1f ms\n", ctx->perf_codec_ms);
                fprintf(stderr, "  Total:   %.1f ms\n", ctx->perf_total_ms);
                fprintf(stderr, "  RTF:     %.2fx realtime\n", dur > 0 ? dur / (ctx->perf_total_ms / 1000.0) : 0);
                fprintf(stderr, "  First frame: %.1f ms\n", ctx->perf_first_frame_ms);
            }
        }
    }
    free(audio);
    qwen_tts_free(ctx);
    free(file_ids);
    free(ref_wav);
    free(ref_codes);
    free(xvec);
    return rc;
}
