/* wav.c - 16-bit PCM mono WAV writer (c/qwen_tts_audio.c semantics:
 * clamp to [-1, 1], (int16)(s * 32767) truncation, write to <path>.tmp then
 * rename so a reader never sees a partial file). */
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/qwen_tts.h"

static void le16(uint8_t *p, uint16_t v) { p[0] = v & 0xFF; p[1] = v >> 8; }
static void le32(uint8_t *p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (v >> (8 * i)) & 0xFF; }

int qwen_tts_write_wav(const char *path, const float *samples, int n_samples, int sample_rate) {
    char tmp[4096];
    int k = snprintf(tmp, sizeof tmp, "%s.tmp", path);
    if (k < 0 || k >= (int)sizeof tmp) {
        fprintf(stderr, "Error: output path too long: %s\n", path);
        return -1;
    }
    FILE *f = fopen(tmp, "wb");
    if (!f) {
        fprintf(stderr, "Error: cannot open %s for writing\n", tmp);
        return -1;
    }
    const uint32_t data_bytes = (uint32_t)n_samples * 2u;
    uint8_t h[44];
    memcpy(h, "RIFF", 4);
    le32(h + 4, 36 + data_bytes);
    memcpy(h + 8, "WAVEfmt ", 8);
    le32(h + 16, 16);
    le16(h + 20, 1);                       /* PCM */
    le16(h + 22, 1);                       /* mono */
    le32(h + 24, (uint32_t)sample_rate);
    le32(h + 28, (uint32_t)sample_rate * 2u);
    le16(h + 32, 2);
    le16(h + 34, 16);
    memcpy(h + 36, "data", 4);
    le32(h + 40, data_bytes);
    int ok = fwrite(h, 1, 44, f) == 44;
    int16_t *pcm = (int16_t *)malloc((size_t)(n_samples > 0 ? n_samples : 1) * 2);
    if (!pcm) ok = 0;
    for (int i = 0; ok && i < n_samples; i++) {
        float s = samples[i];
        if (s > 1.0f) s = 1.0f;
        if (s < -1.0f) s = -1.0f;
        pcm[i] = (int16_t)(s * 32767.0f);
    }
    if (ok && n_samples > 0 && fwrite(pcm, 2, (size_t)n_samples, f) != (size_t)n_samples) ok = 0;
    free(pcm);
    if (fclose(f) != 0) ok = 0;
    if (!ok) {
        fprintf(stderr, "Error: failed to write WAV data to %s\n", tmp);
        remove(tmp);
        return -1;
    }
    if (rename(tmp, path) != 0) {
        fprintf(stderr, "Error: failed to rename %s -> %s: %s\n", tmp, path, strerror(errno));
        remove(tmp);
        return -1;
    }
    return 0;
}

/* ------------------------------------------------------------------ resampling
 * Reference audio at another rate (the Python reference resamples it to 24 kHz
 * with librosa.resample, qwen_tts/inference/qwen3_tts_model.py:441-444).  This
 * is librosa's res_type="polyphase" path, i.e. scipy.signal.resample_poly
 * (up / down = sr_out / sr_in reduced by their gcd): the firwin low-pass of
 * 2 * 10 * max(up, down) + 1 taps, cutoff 1 / max(up, down), Kaiser window
 * beta 5, unit DC gain times up, zero padding, upfirdn with scipy's phase
 * alignment, ceil(n * up / down) samples out; computed in double precision.
 * (librosa's default res_type is soxr_hq, a different filter: parity with it
 * is unpinned; tests/test_resample.py pins this to scipy.) */
static double bessel_i0(double x) {
    double s = 1.0, t = 1.0;
    for (int k = 1; k < 200; k++) {
        t *= (x / (2.0 * k)) * (x / (2.0 * k));
        s += t;
        if (t < s * 1e-17) break;
    }
    return s;
}

static long gcd_l(long a, long b) {
    while (b) { long t = a % b; a = b; b = t; }
    return a;
}

float *qwen_tts_resample(const float *in, int n_in, int sr_in, int sr_out, int *n_out) {
    if (n_out) *n_out = 0;
    if (!in || n_in < 1 || sr_in < 1 || sr_out < 1 || !n_out) return NULL;
    const long g = gcd_l(sr_out, sr_in), up = sr_out / g, down = sr_in / g;
    const long no = (long)n_in * up / down + (((long)n_in * up) % down ? 1 : 0);
    float *out = (float *)malloc((size_t)(no > 0 ? no : 1) * sizeof(float));
    if (!out) return NULL;
    if (up == 1 && down == 1) {
        memcpy(out, in, (size_t)n_in * sizeof(float));
        *n_out = n_in;
        return out;
    }
    const long maxr = up > down ? up : down, half = 10 * maxr, taps = 2 * half + 1;
    /* firwin: cutoff * sinc(cutoff * m) x kaiser(taps, 5), scaled to unit DC gain, times up */
    const long pre = down - half % down;           /* scipy's n_pre_pad */
    const long L = pre + taps;                      /* (n_post_pad is never needed for n_out samples) */
    double *h = (double *)calloc((size_t)L, sizeof(double));
    if (!h) { free(out); return NULL; }
    const double fc = 1.0 / (double)maxr, beta = 5.0, i0b = bessel_i0(beta);
    double sum = 0.0;
    for (long j = 0; j < taps; j++) {
        const double m = (double)j - (double)(taps - 1) / 2.0;
        const double x = fc * m;
        const double sinc = x == 0.0 ? 1.0 : sin(M_PI * x) / (M_PI * x);
        const double r = 2.0 * (double)j / (double)(taps - 1) - 1.0;
        const double w = bessel_i0(beta * sqrt(1.0 - r * r > 0.0 ? 1.0 - r * r : 0.0)) / i0b;
        h[pre + j] = fc * sinc * w;
        sum += h[pre + j];
    }
    for (long j = 0; j < taps; j++) h[pre + j] = h[pre + j] / sum * (double)up;
    const long skip = (half + pre) / down;          /* scipy's n_pre_remove */
    for (long k = 0; k < no; k++) {
        /* upfirdn output index t = (k + skip) * down: z[t] = sum_i x[i] h[t - i * up] */
        const long t = (k + skip) * down;
        long i0 = t - (L - 1) <= 0 ? 0 : (t - (L - 1) + up - 1) / up;
        long i1 = t / up;
        if (i1 > n_in - 1) i1 = n_in - 1;
        double acc = 0.0;
        for (long i = i0; i <= i1; i++) acc += (double)in[i] * h[t - i * up];
        out[k] = (float)acc;
    }
    free(h);
    *n_out = (int)no;
    return out;
}
