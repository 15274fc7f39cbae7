/*
 * qwen_tts.h - public C API of the MI355X (gfx950) Qwen3-TTS hot path.
 *
 * Drop-in for the reference header c/qwen_tts.h: the same constants, the
 * same qwen_tts_config_t, the same public functions with the same
 * signatures, ownership and error behaviour (c/qwen_tts.h:448-502), and a
 * qwen_tts_ctx_t keeping every field name the reference CLI reads or writes
 * (config, generation parameters, progress callback, perf counters,
 * talker_kv_len; c/main.c:214-223,268-270,306-312).  Weights and all
 * generation state live on the GPU behind `hip` (include/qtts_hip.h); the
 * CPU-side weight/scratch fields of the reference struct are not present.
 *
 *   qwen_tts_load        NULL on failure, message on stderr
 *   qwen_tts_generate    malloc'd float32 PCM at 24 kHz, caller frees;
 *                        NULL and *out_samples = 0 on error
 *   qwen_tts_write_wav   0 / -1
 *
 * MI355X additions (not in the c/ reference): qwen_tts_load_on (device
 * choice per ctx; qwen_tts_load takes $QWEN_TTS_HIP_DEVICE or 0),
 * qwen_tts_generate_batch, qwen_tts_last_codes, streaming, text input, and
 * the Python reference's voice clone (codes / x-vector or reference audio).
 */
#ifndef QWEN_TTS_H
#define QWEN_TTS_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#define QWEN_TTS_SAMPLE_RATE      24000
#define QWEN_TTS_DECODE_UPSAMPLE  1920

/* defaults used when config.json omits a key (c/qwen_tts.h:25-78) */
#define QWEN_TTS_TALKER_VOCAB        3072
#define QWEN_TTS_TALKER_HIDDEN       1024
#define QWEN_TTS_TALKER_INTERMEDIATE 2048
#define QWEN_TTS_TALKER_LAYERS       20
#define QWEN_TTS_TALKER_HEADS        16
#define QWEN_TTS_TALKER_KV_HEADS     2
#define QWEN_TTS_TALKER_HEAD_DIM     64
#define QWEN_TTS_TALKER_TEXT_HIDDEN  2048
#define QWEN_TTS_TALKER_TEXT_VOCAB   151936
#define QWEN_TTS_NUM_CODE_GROUPS     32

#define QWEN_TTS_SUBTALKER_VOCAB        2048
#define QWEN_TTS_SUBTALKER_HIDDEN       1024
#define QWEN_TTS_SUBTALKER_INTERMEDIATE 3072
#define QWEN_TTS_SUBTALKER_LAYERS       5
#define QWEN_TTS_SUBTALKER_HEADS        16
#define QWEN_TTS_SUBTALKER_KV_HEADS     8
#define QWEN_TTS_SUBTALKER_HEAD_DIM     128

#define QWEN_TTS_CODEC_NUM_QUANTIZERS 16
#define QWEN_TTS_CODEC_CODEBOOK_SIZE  2048
#define QWEN_TTS_CODEC_HIDDEN         1024
#define QWEN_TTS_CODEC_LATENT         1024
#define QWEN_TTS_CODEC_LAYERS         8
#define QWEN_TTS_CODEC_HEADS          16
#define QWEN_TTS_CODEC_KV_HEADS       16
#define QWEN_TTS_CODEC_INTERMEDIATE   3072
#define QWEN_TTS_CODEC_SLIDING_WINDOW 72
#define QWEN_TTS_CODEC_DECODER_DIM    1536

#define QWEN_TTS_MAX_TALKER_LAYERS    32
#define QWEN_TTS_MAX_SUBTALKER_LAYERS 8
#define QWEN_TTS_MAX_CODEC_LAYERS     12

#define QWEN_TTS_TOKEN_IM_START  151644
#define QWEN_TTS_TOKEN_IM_END    151645
#define QWEN_TTS_TOKEN_ENDOFTEXT 151643
#define QWEN_TTS_TOKEN_TTS_PAD   151671
#define QWEN_TTS_TOKEN_TTS_BOS   151672
#define QWEN_TTS_TOKEN_TTS_EOS   151673

#define QWEN_TTS_CODEC_PAD       2148
#define QWEN_TTS_CODEC_BOS       2149
#define QWEN_TTS_CODEC_EOS       2150
#define QWEN_TTS_CODEC_THINK     2154
#define QWEN_TTS_CODEC_NOTHINK   2155
#define QWEN_TTS_CODEC_THINK_BOS 2156
#define QWEN_TTS_CODEC_THINK_EOS 2157

typedef struct {
    int talker_vocab_size;
    int talker_hidden;
    int talker_intermediate;
    int talker_layers;
    int talker_heads;
    int talker_kv_heads;
    int talker_head_dim;
    int talker_text_hidden;
    int talker_text_vocab;
    int num_code_groups;
    float talker_rms_norm_eps;
    float talker_rope_theta;
    int mrope_section[3];

    int subtalker_vocab_size;
    int subtalker_hidden;
    int subtalker_intermediate;
    int subtalker_layers;
    int subtalker_heads;
    int subtalker_kv_heads;
    int subtalker_head_dim;

    int codec_num_quantizers;
    int codec_codebook_size;
    int codec_codebook_dim;
    int codec_hidden;
    int codec_latent;
    int codec_layers;
    int codec_heads;
    int codec_kv_heads;
    int codec_intermediate;
    int codec_sliding_window;
    int codec_decoder_dim;
    float codec_rms_norm_eps;
    float codec_layer_scale;
    int codec_upsample_rates[4];
    int codec_upsampling_ratios[2];

    int n_speakers;
    char **speaker_names;
    int *speaker_ids;
    int n_languages;
    char **language_names;
    int *language_ids;

    int codec_pad_id;
    int codec_bos_id;
    int codec_eos_id;
    int codec_nothink_id;
    int codec_think_id;
    int codec_think_bos_id;
    int codec_think_eos_id;
} qwen_tts_config_t;

typedef void (*qwen_tts_progress_cb)(int step, int total, void *userdata);

typedef struct {
    qwen_tts_config_t config;
    char model_dir[512];

    /* device-resident model + generation state (include/qtts_hip.h) */
    void *hip;
    int hip_device;

    int talker_kv_len;          /* positions in the talker KV cache of slot 0 */
    float *tk_x;                /* host copy of the post-norm last talker hidden (stage API) */

    /* generation parameters (same names and defaults as the reference) */
    float temperature;
    float subtalker_temperature;
    int top_k;
    int subtalker_top_k;
    float top_p;
    float subtalker_top_p;
    float repetition_penalty;
    int max_new_tokens;
    int fixed_codec_tokens;
    int sample_seed;

    qwen_tts_progress_cb progress_cb;
    void *progress_cb_userdata;

    /* performance stats */
    double perf_total_ms;
    double perf_talker_ms;
    double perf_codec_ms;
    int perf_codec_tokens;

    /* MI355X additions */
    double perf_prefill_ms;
    double perf_first_frame_ms;  /* generate() entry -> first frame's codes on device */
    int *last_codes;             /* [last_frames][num_code_groups] of the last call (slot 0) */
    int last_frames;
    int last_stop_reason;        /* 1 eos, 2 max_tokens */
    int last_stop_step;
    double perf_first_packet_ms; /* qwen_tts_generate_stream(): entry -> first audio chunk delivered */
    void *tokenizer;             /* Qwen2 BPE of the model dir, loaded on first text input */
    /* the last qwen_tts_generate_queue, per utterance in input order */
    int queue_n;
    int **queue_codes;           /* [queue_n] [frames][num_code_groups] (NULL: not taken by this ctx) */
    int *queue_frames;           /* frames generated (-1: not taken) */
    int *queue_stop_reason;      /* 1 eos, 2 max_tokens */
    int *queue_slot;             /* the slot it decoded on */
    int queue_slots;             /* lock-step slots the run used */
    int queue_frames_launched;   /* lock-step frames launched */
    int queue_refills;           /* utterances admitted into a slot freed mid-run */
    long long queue_slot_frames_used; /* sum of frames generated */
    long long queue_rows_launched;    /* sum over launched frames of the slot rows they ran (the tail launches
                                         only the running slots): occupancy = frames_used / rows_launched */
} qwen_tts_ctx_t;

qwen_tts_ctx_t *qwen_tts_load(const char *model_dir);
void qwen_tts_free(qwen_tts_ctx_t *ctx);
void qwen_tts_set_progress_callback(qwen_tts_ctx_t *ctx, qwen_tts_progress_cb cb, void *userdata);
float *qwen_tts_generate(qwen_tts_ctx_t *ctx, const char *text, const char *speaker, const char *language,
                         int *out_samples);
int qwen_tts_write_wav(const char *path, const float *samples, int n_samples, int sample_rate);

static inline float bf16_to_f32(uint16_t bf16) {
    uint32_t f32_bits = ((uint32_t)bf16) << 16;
    float result;
    __builtin_memcpy(&result, &f32_bits, sizeof(float));
    return result;
}

/* stage functions (host pointers; c/qwen_tts.h:483-502) */
void qwen_tts_talker_prefill(qwen_tts_ctx_t *ctx, const float *input_embeds, int seq_len);
void qwen_tts_talker_forward(qwen_tts_ctx_t *ctx, const float *input_embed, float *logits);
void qwen_tts_subtalker_generate(qwen_tts_ctx_t *ctx, const float *talker_hidden, int first_code, int *out_codes);
float *qwen_tts_codec_decode(qwen_tts_ctx_t *ctx, const int *codes, int time_steps, int *out_samples);

/* post-final-norm hidden of the last talker token (the reference's ctx->tk_x) */
int qwen_tts_talker_hidden(qwen_tts_ctx_t *ctx, float *out);

/* ---- MI355X additions ---- */
/* qwen_tts_load on HIP device `device` (< 0: $QWEN_TTS_HIP_DEVICE or 0, which
 * is what qwen_tts_load uses).  No process-global state: one ctx per device
 * and host thread, each owning its device model, streams and graphs. */
qwen_tts_ctx_t *qwen_tts_load_on(const char *model_dir, int device);
/* nb utterances in lock-step frames on this ctx's GPU (weights read once per
 * frame for all of them).  out_audio[i] malloc'd (caller frees), out_samples[i]
 * set; returns 0 when every utterance produced audio. */
int qwen_tts_generate_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts, const char *const *speakers,
                            const char *const *languages, float **out_audio, int *out_samples);
/* Work queue (no c/ counterpart): nq utterances on at most nb
 * lock-step slots.  When a slot's utterance stops (EOS, or max_new_tokens /
 * fixed_codec_tokens frames), the next queued utterance is prefilled into that
 * slot inside the live batch, so a batch of EOS-variable lengths keeps its
 * slots busy instead of riding stopped rows to the longest one.  Each
 * utterance decodes as it would alone (own KV positions, counters, repetition
 * counts, RNG states from sample_seed).  `next` (optional) picks the utterance
 * to admit: it returns an index in [0, nq) not yet taken, or -1 when there is
 * none (e.g. a counter shared by the processes of several GPUs); NULL takes
 * them in order.  out_audio[i] / out_samples[i] (input order) are filled for
 * the utterances this ctx took (NULL / 0 for the others); codes and stop
 * reasons stay in ctx->queue_* until the next call.  Returns 0 when every
 * utterance taken produced audio. */
typedef int (*qwen_tts_queue_next_cb)(void *userdata);
int qwen_tts_generate_queue(qwen_tts_ctx_t *ctx, int nq, const char *const *texts, const char *const *speakers,
                            const char *const *languages, int nb, qwen_tts_queue_next_cb next, void *userdata,
                            float **out_audio, int *out_samples);
/* codes of utterance i of the last qwen_tts_generate_queue: copies up to
 * max_frames rows (codes may be NULL to query), returns the frame count, -1 if
 * this ctx did not decode it */
int qwen_tts_queue_codes(qwen_tts_ctx_t *ctx, int i, int *codes, int max_frames);
/* Voice clone (no c/ counterpart: the Python reference's generate_voice_clone,
 * qwen3_tts_model.py:506-630, modeling_qwen3_tts.py:1967-2232) from the 12 Hz
 * codes of the reference audio (ref_codes [n_ref_frames][16]) and/or the
 * speaker encoder's x-vector (spk_embed [talker hidden]); to start from the
 * reference AUDIO, use qwen_tts_generate_voice_clone_audio[_batch] below, which
 * run the encoders on the device first.
 *   ICL mode  : ref_codes + ref_text (ids CSV of
 *               "<|im_start|>assistant\n{ref}<|im_end|>\n"), spk_embed optional;
 *               the audio is decoded from reference ++ generated codes and the
 *               reference part cut off, as the Python reference does.
 *   x-vector  : ref_codes NULL / n_ref_frames 0, spk_embed set.
 * non_streaming selects the non-streaming text layout.  Returns malloc'd PCM
 * (caller frees); NULL on error. */
float *qwen_tts_generate_voice_clone(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                     const int *ref_codes, int n_ref_frames, const float *spk_embed,
                                     const char *language, int non_streaming, int *out_samples);
/* Streaming voice clone (as qwen_tts_generate_stream, after the type below):
 * the reference frames are pushed through the exact streaming codec first, so
 * chunks start at the reference boundary (sample n_ref_frames * 1920 of the
 * reference ++ generated decode).  The non-streamed call cuts at the Python
 * reference's float position int(ref / total * samples), which for ~5 % of
 * (ref, total) pairs is one sample earlier. */
/* nb voice-clone utterances in lock-step frames (BASELINE C5: batch 8 on one
 * GPU); per-slot arrays as above (ref_codes[b] / spk_embeds[b] may be NULL).
 * Returns 0 when every utterance produced audio. */
int qwen_tts_generate_voice_clone_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts,
                                        const char *const *ref_texts, const int *const *ref_codes,
                                        const int *n_ref_frames, const float *const *spk_embeds,
                                        const char *const *languages, int non_streaming, float **out_audio,
                                        int *out_samples);
/* Voice clone from reference AUDIO (the Python reference's
 * create_voice_clone_prompt, qwen3_tts_model.py:356-458, on the device).
 * Waveforms are mono float PCM at 24 kHz (the reference resamples other rates
 * with librosa first; here the caller resamples with qwen_tts_resample below,
 * as the CLI's --ref-audio does for other rates).  The model directory
 * must hold the speaker encoder (speaker_encoder.* + speaker_encoder_config)
 * and the 12 Hz tokenizer encoder (speech_tokenizer/ encoder.* +
 * encoder_config).
 * qwen_tts_speaker_embedding: the x-vector of extract_speaker_embedding
 *   (modeling_qwen3_tts.py:1941-1954: 128-bin log-mel, ECAPA-TDNN), malloc'd
 *   [talker hidden] floats, *out_dim set; NULL on error (> 384 samples needed).
 * qwen_tts_encode_audio: the 12 Hz codes of Qwen3TTSTokenizer.encode
 *   (modeling_qwen3_tts_tokenizer_v2.py:961-991: Mimi encoder, first 16
 *   codebooks), malloc'd [ceil(n / 1920)][16] ints, *out_frames set.
 * qwen_tts_generate_voice_clone_audio[_batch]: encode (all references in one
 *   zero-padded batch, as the tokenizer does) + qwen_tts_generate_voice_clone
 *   [_batch]; ICL mode needs ref_text, x_vector_only drops the codes.
 * All return NULL / -1 on error with a message on stderr; buffers are the
 * caller's to free(). */
float *qwen_tts_speaker_embedding(qwen_tts_ctx_t *ctx, const float *wav, int n_samples, int *out_dim);
int *qwen_tts_encode_audio(qwen_tts_ctx_t *ctx, const float *wav, int n_samples, int *out_frames);
float *qwen_tts_generate_voice_clone_audio(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                           const float *ref_wav, int n_ref_samples, const char *language,
                                           int x_vector_only, int non_streaming, int *out_samples);
int qwen_tts_generate_voice_clone_audio_batch(qwen_tts_ctx_t *ctx, int nb, const char *const *texts,
                                              const char *const *ref_texts, const float *const *ref_wavs,
                                              const int *n_ref_samples, const char *const *languages,
                                              const int *x_vector_only, int non_streaming, float **out_audio,
                                              int *out_samples);
/* audio chunk callback of the streaming calls (qwen_tts_generate_stream below) */
typedef void (*qwen_tts_audio_cb)(const float *pcm, int n_samples, void *userdata);
/* streaming form: encode, then qwen_tts_generate_voice_clone_stream; the
 * first-packet time counts from this call's entry (encode included) */
float *qwen_tts_generate_voice_clone_audio_stream(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                                  const float *ref_wav, int n_ref_samples, const char *language,
                                                  int x_vector_only, int non_streaming, int chunk_frames,
                                                  qwen_tts_audio_cb cb, void *userdata, int *out_samples);
/* Resample mono PCM from sr_in to sr_out Hz (reference audio at another rate;
 * the Python reference resamples to 24 kHz with librosa, qwen3_tts_model.py:
 * 441-444): librosa's "polyphase" method = scipy.signal.resample_poly (Kaiser
 * windowed-sinc FIR, ceil(n * sr_out / sr_in) samples).  malloc'd, *n_out set;
 * NULL on error. */
float *qwen_tts_resample(const float *in, int n_in, int sr_in, int sr_out, int *n_out);
/* codes of the last generate() (slot 0): copies up to max_frames rows of
 * num_code_groups ints, returns the frame count */
int qwen_tts_last_codes(qwen_tts_ctx_t *ctx, int *codes, int max_frames);
/* the same for slot `slot` of the last qwen_tts_generate_batch (slot 0 ==
 * qwen_tts_last_codes); -1 on a bad slot */
int qwen_tts_last_codes_slot(qwen_tts_ctx_t *ctx, int slot, int *codes, int max_frames);
/* Streaming generation (the reference has only a per-step
 * progress callback, c/qwen_tts.h:356): audio is decoded incrementally and
 * exactly (qtts_hip.h codec stream) and handed to `cb` as it is produced --
 * the first chunk after frame 0 (1920 samples, 80 ms), then every
 * `chunk_frames` frames, then the tail.  Returns the whole utterance like
 * qwen_tts_generate (malloc'd, caller frees); NULL on error. */
float *qwen_tts_generate_stream(qwen_tts_ctx_t *ctx, const char *text, const char *speaker, const char *language,
                                int chunk_frames, qwen_tts_audio_cb cb, void *userdata, int *out_samples);
float *qwen_tts_generate_voice_clone_stream(qwen_tts_ctx_t *ctx, const char *text, const char *ref_text,
                                            const int *ref_codes, int n_ref_frames, const float *spk_embed,
                                            const char *language, int non_streaming, int chunk_frames,
                                            qwen_tts_audio_cb cb, void *userdata, int *out_samples);
/* Incremental codec decode of host codes [time_steps][16]: begin, then push
 * any number of frames at a time; each push writes time_steps * 1920 samples
 * to `out` and returns that count (-1 on error).  The concatenation equals
 * qwen_tts_codec_decode of all frames at once. */
int qwen_tts_codec_stream_begin(qwen_tts_ctx_t *ctx, int max_frames);
int qwen_tts_codec_stream_push(qwen_tts_ctx_t *ctx, const int *codes, int time_steps, float *out);

/* Text input (the reference's TODO at c/qwen_tts.c:1071-1077,
 * its browser front end tokenizes with @huggingface/transformers,
 * web/wasm/app.js:241-267): Qwen2 byte-level BPE over the model directory's
 * vocab.json / merges.txt / tokenizer_config.json.
 * qwen_tts_tokenize: UTF-8 text (NFC) -> malloc'd ids (caller frees), NULL on
 * error with *n_ids = 0; needs no GPU.
 * qwen_tts_text_prompt: the comma-separated ids of the chat template
 * "<|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n" -- the
 * `text` argument of qwen_tts_generate* -- malloc'd, NULL on error. */
int *qwen_tts_tokenize(const char *model_dir, const char *text, int *n_ids);
char *qwen_tts_text_prompt(qwen_tts_ctx_t *ctx, const char *text);

/* sizeof(qwen_tts_ctx_t) as compiled into the library (FFI layout check) */
size_t qwen_tts_abi_sizeof_ctx(void);

extern int qwen_tts_verbose;

#endif /* QWEN_TTS_H */
