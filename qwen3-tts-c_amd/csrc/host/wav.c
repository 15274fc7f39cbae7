/* wav.c - 16-bit PCM mono WAV writer (c/qwen_tts_audio.c semantics:
 * clamp to [-1, 1], (int16)(s * 32767) truncation, write to <path>.tmp then
 * rename so a reader never sees a partial file). */
#include <errno.h>
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
