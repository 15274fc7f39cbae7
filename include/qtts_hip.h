/*
 * qtts_hip.h - thin C-ABI between the C host (qwen_tts.c, main.c) and the
 * MI355X (gfx950) HIP implementation of the Qwen3-TTS hot path.
 *
 * Plain C: opaque handles, plain pointers and sizes, int error codes
 * (0 = ok, <0 = error with a message on stderr).  No HIP or torch types.
 * "dev" pointers below are device (HBM) addresses; "host" pointers are
 * ordinary process memory.  `stream` arguments are hipStream_t passed as
 * void* (NULL = the default stream).
 *
 * Two layers:
 *   1. Model-level entry points used by the C host's decode loop
 *      (qwen_tts.c) - they replace the compute of
 *        qwen_tts_talker_prefill / qwen_tts_talker_forward   (c/qwen_tts.h:483-486,
 *                                                            c/qwen_tts_talker.c:254-533)
 *        qwen_tts_subtalker_generate                         (c/qwen_tts.h:489-494,
 *                                                            c/qwen_tts_talker.c:539-736)
 *        the per-frame loop body of qwen_tts_generate       (c/qwen_tts.c:1282-1373)
 *        qwen_tts_codec_decode                               (c/qwen_tts.h:497-502,
 *                                                            c/qwen_tts_codec.c:581-749)
 *   2. Kernel-level entry points on device buffers, one per kernel_* of
 *      c/qwen_tts_kernels.h the hot path uses, so each HIP kernel is parity
 *      tested against the CPU oracle in isolation.
 */
#ifndef QTTS_HIP_H
#define QTTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qtts_dev qtts_dev_t;

/* Model dimensions (same meaning as qwen_tts_config_t, c/qwen_tts.h:84-144). */
typedef struct {
    int H, I, L, NH, KV, HD, TH, TV, V, G;   /* talker */
    int Hs, Is, Ls, NHs, KVs, HDs, Vs;       /* sub-talker (code predictor) */
    float eps, theta;                        /* talker_rms_norm_eps / talker_rope_theta */
    int cq, ccb, ccbdim, chid, clat, clayers, cheads, ckv, cinter, cwin, cdec;  /* codec */
    int rates[4], ratios[2];
    float ceps;
    int pad_id, bos_id, eos_id;
} qtts_dims_t;

/* Voice-clone encoder dimensions: config.json
 * `speaker_encoder_config` (Qwen3TTSSpeakerEncoderConfig,
 * configuration_qwen3_tts.py:47-67) and speech_tokenizer/config.json
 * `encoder_config` (transformers MimiConfig) + `encoder_valid_num_quantizers`. */
typedef struct {
    /* speaker encoder (ECAPA-TDNN) */
    int mel_dim, enc_dim, n_ch;              /* n_ch = len(enc_channels), 3..8 */
    int ch[8], ks[8], dil[8];
    int att_ch, res2net_scale, se_ch;
    /* 12 Hz tokenizer encoder (Mimi) */
    int hidden, n_filters, ratios[4], kernel, last_kernel, res_kernel, dil_growth, n_res, compress;
    int layers, heads, kv_heads, head_dim, inter, window;
    int n_q, n_sem, cb_size, vq_dim, n_valid;
    float norm_eps, rope_theta;
} qtts_enc_dims_t;

/* Generation parameters (qwen_tts_ctx_t fields, c/qwen_tts.h:420-430). */
typedef struct {
    float temperature, top_p, repetition_penalty;
    int top_k;
    float st_temperature, st_top_p;
    int st_top_k;
    int fixed_codec_tokens;
    int seed;
} qtts_gen_params_t;

/* ---- device + model ---- */
int qtts_hip_device_count(void);
/* Creates the device model on HIP device `device` (selects it for the
 * calling thread).  Returns NULL on error. */
qtts_dev_t *qtts_dev_create(const qtts_dims_t *dims, int device);
void qtts_dev_destroy(qtts_dev_t *dev);
/* Hands one checkpoint tensor (by its safetensors name) to the device.
 * dtype: 0 = F32, 1 = BF16, 2 = F16.  Tensors the hot path does not use are
 * ignored.  Packing (fused [q;k;v], gate|up row quads), bf16 -> f32 of
 * norms/biases, codebook = embedding_sum / max(usage, 1e-5) and SnakeBeta
 * pre-exponentiation (c/qwen_tts.c:481-489, 577-602) happen here. */
int qtts_dev_put_tensor(qtts_dev_t *dev, const char *name, const void *host, int dtype,
                        const int64_t *shape, int ndim);
/* Validates that every required tensor arrived (reports the first missing
 * one like c/qwen_tts.c:381-427) and builds RoPE tables. */
int qtts_dev_finalize(qtts_dev_t *dev);
/* Device bytes currently allocated for weights / state. */
size_t qtts_dev_bytes(const qtts_dev_t *dev, int which /*0 weights, 1 state*/);

/* ---- generation (batch of nb utterances in lock-step frames) ---- */
/* Allocates state for nb slots, max_frames frames (KV capacity = max_prefill
 * + max_frames), resets counters / RNG, (re)captures the frame graphs. */
int qtts_dev_begin(qtts_dev_t *dev, int nb, int max_frames, int max_prefill, const qtts_gen_params_t *p);
/* Prompt for slot b (layout built by the host, c/qwen_tts.c:1147-1243):
 *   text_ids[n_text]  text tokens to embed+project (text_embedding -> fc1 ->
 *                     SiLU -> fc2, c/qwen_tts.c:823-847)
 *   plan[5*nplan]     per output row {text row, codec id or -1,
 *                     0 = prefill / 1 = trailing, b, slot}
 *   p_len, n_trailing prefill / trailing lengths; pad_row = text row of tts_pad */
int qtts_dev_prompt(qtts_dev_t *dev, int b, const int *text_ids, int n_text, const int *plan, int nplan,
                    int p_len, int n_trailing, int pad_row);
/* Voice-clone inputs consumed by the next qtts_dev_prompt (no c/ counterpart;
 * modeling_qwen3_tts.py:1967-2019, 2150-2190): reference codes
 * [n_ref][num_code_groups] that plan codec ids <= -3 address (-3 - frame: the
 * frame's 16 group embeddings summed), and the speaker x-vector [hidden] that
 * codec id -2 adds (NULL: none). */
int qtts_dev_prompt_ref(qtts_dev_t *dev, const int *ref_codes, int n_ref, const float *spk);
/* Talker prefill of all nb slots (leaves each slot's last raw hidden). */
int qtts_dev_prefill(qtts_dev_t *dev);
/* Enqueues frame `step` (step 0: codec_head on the prefill hidden; step > 0:
 * talker forward first): sample group 0 -> sub-talker 15 groups -> next
 * input embedding.  Asynchronous (one HIP graph launch). */
int qtts_dev_frame(qtts_dev_t *dev, int step);
/* Waits for the queued work; stopped[b] = 1 once slot b drew EOS
 * (non-fixed mode); n_gen[b] frames stored; stop_step[b] as in the
 * reference's "Stop: eos at step N". */
int qtts_dev_poll(qtts_dev_t *dev, int *stopped, int *n_gen, int *stop_step);
/* EOS mode, lagged: waits only until frame `step` has finished (launch frame
 * step + 1 first) and sets *all_stopped when every slot had drawn EOS by then
 * (the sampler mirrors the stops into pinned host memory). */
int qtts_dev_frame_done(qtts_dev_t *dev, int step, int *all_stopped);
/* ---- work queue (utterances of EOS-variable length on a
 * live lock-step batch; no c/ counterpart -- the reference decodes one
 * utterance per call, Q.c:1059-1443) ---- */
/* Sizes the per-slot trailing text rows for the longest utterance of the run
 * (call after qtts_dev_begin, before the first qtts_dev_prompt). */
int qtts_dev_reserve(qtts_dev_t *dev, int max_trailing);
/* Slot b takes the utterance the last qtts_dev_prompt(dev, b, ...) assembled,
 * inside the live batch: its prompt rows but the last are prefilled into slot
 * b's KV cache, the last row becomes the slot's talker input at position
 * p_len - 1 (the next frame's talker step runs it, then samples the
 * utterance's frame 0), and the slot's counters, repetition counts and RNG
 * states start afresh.  Stream-ordered after the frames already queued. */
int qtts_dev_refill(qtts_dev_t *dev, int b);
/* Stops slot b from the next queued frame on (max_new_tokens / fixed length
 * reached without EOS); stream-ordered. */
int qtts_dev_retire(qtts_dev_t *dev, int b);
/* Lagged like qtts_dev_frame_done: waits for frame `step`, then stopped[b] = 1
 * for every slot that had drawn EOS by then. */
int qtts_dev_frame_stops(qtts_dev_t *dev, int step, int *stopped);
/* Tail of a queue run (nothing left to admit): slot `from`'s whole decode
 * state (KV cache rows, input row, counters, codes, trailing rows, RNG)
 * moves to the freed slot `to`, so the running slots are the first ones;
 * set_rows then launches the first `rows` slots only (a graph per row count,
 * captured on first use).  Both need the stream idle (after frame_stops /
 * get_codes). */
int qtts_dev_move_slot(qtts_dev_t *dev, int from, int to);
int qtts_dev_set_rows(qtts_dev_t *dev, int rows);
/* Copies slot b's codes [n_gen][G] to host. */
int qtts_dev_get_codes(qtts_dev_t *dev, int b, int *host_codes, int max_frames);
/* Codec decode of slot b's generated codes (device-resident) into a malloc'd
 * host buffer of T*1920 samples (caller frees). */
float *qtts_dev_codec_slot(qtts_dev_t *dev, int b, int T, int *out_samples);
/* Per-stage timing of the full codec decodes (the reference's -v -v line
 * "Codec stages (ms): rvq= preconv= transformer= upsample= vocoder=",
 * c/qwen_tts_codec.c:743-746): on != 0 records HIP events between the stages
 * of every later qtts_dev_codec_slot / _decode_host; stage_ms fills ms[5] in
 * that order for the last one (-1 when it was not timed). */
int qtts_dev_codec_timing(qtts_dev_t *dev, int on);
int qtts_dev_codec_stage_ms(const qtts_dev_t *dev, float *ms);

/* Several utterances' full codec decodes (a batch's slots; the reference
 * decodes its one utterance after the loop, Q.c:1376-1383, Cd.c:581-749):
 * job i decodes host_codes[i] ([T[i]][16] host ints) when host_codes and
 * host_codes[i] are non-NULL, else slot slot[i]'s first T[i] generated frames.
 * Up to QTTS_HIP_CODEC_LANES (default 8; fewer when their scratch would pass
 * 16 GB) decodes run side by side on their own
 * streams and scratch, each the same kernels as a lone decode (bit-identical
 * audio).  audio[i] (malloc'd host floats, T[i] * 1920 samples) and samples[i]
 * are filled; returns 0, or -1 with every audio[i] NULL. */
int qtts_dev_codec_multi(qtts_dev_t *dev, int n, const int *const *host_codes, const int *slot, const int *T,
                         float **audio, int *samples);

/* Streaming codec decode, exact and incremental (every codec op is causal:
 * conv histories, transposed-conv tails and the window-72 transformer K/V are
 * carried between pushes).  begin resets the stream (max_frames bounds the
 * total frames); a push decodes T more frames into T * 1920 host samples and
 * returns the sample count (< 0 on error).  push_slot reads slot b's generated
 * codes [frame0, frame0 + T) on the device (no host round trip). */
int qtts_dev_codec_stream_begin(qtts_dev_t *dev, int max_frames);
/* the same with the internal chunk sized for pushes of up to chunk_frames
 * frames at once (<= 16: the default 16) */
int qtts_dev_codec_stream_begin_ex(qtts_dev_t *dev, int max_frames, int chunk_frames);
/* push T host frames [T][16] through the stream on a second HIP stream without
 * waiting, audio dropped; every later stream call is ordered after it (the
 * voice-clone reference frames, overlapped with the prefill) */
int qtts_dev_codec_stream_prime(qtts_dev_t *dev, const int *codes, int T);
int qtts_dev_codec_stream_push_slot(qtts_dev_t *dev, int b, int frame0, int T, float *host_out);
int qtts_dev_codec_stream_push_host(qtts_dev_t *dev, const int *codes, int T, float *host_out);

/* The same exact streaming decode overlapped with the decode loop: it runs on
 * a second (low-priority) HIP stream; push orders itself after the frames
 * already enqueued on the context stream (an event), decodes slot b's frames
 * [frame0, frame0 + T) into a device waveform and returns at once; end copies
 * `frames` * 1920 samples to host_out and waits.  Replaces the codec call
 * after the loop in qwen_tts_generate (Q.c:1376-1383) for one utterance. */
int qtts_dev_codec_async_begin(qtts_dev_t *dev, int max_frames);
int qtts_dev_codec_async_push(qtts_dev_t *dev, int b, int frame0, int T);
int qtts_dev_codec_async_end(qtts_dev_t *dev, float *host_out, int frames);

/* ---- voice-clone audio encoders (no c/ counterpart) ---- */
/* Encoder dimensions; call before the encoder tensors are put (speaker_encoder.*
 * of the model dir, encoder.* of speech_tokenizer/). */
int qtts_dev_enc_config(qtts_dev_t *dev, const qtts_enc_dims_t *dims);
/* bit 0: the speaker encoder is loaded, bit 1: the 12 Hz encoder is loaded */
int qtts_dev_enc_available(qtts_dev_t *dev);
/* Speaker x-vectors (extract_speaker_embedding, modeling_qwen3_tts.py:1941-1954)
 * of nb <= 16 host waveforms at 24 kHz (n[b] samples, > 384 each):
 * out[nb][enc_dim] host floats.  mel_out (optional) receives each utterance's
 * [128][T_b] log-mel back to back, T_b = (n[b] - 256) / 256 + 1. */
int qtts_dev_speaker_embed(qtts_dev_t *dev, int nb, const float *const *wav, const int *n, float *out,
                           float *mel_out);
/* 12 Hz reference codes (Qwen3TTSTokenizer.encode, qwen3_tts_tokenizer.py:208-257,
 * modeling_qwen3_tts_tokenizer_v2.py:961-991) of nb <= 16 host waveforms at
 * 24 kHz, zero-padded to the longest as the tokenizer's batch encode does:
 * codes[nb][max_frames][16] (host ints), frames[b] = ceil(n[b] / 1920).
 * latent (optional): [nb][hidden][max_frames] pre-quantizer embeddings. */
int qtts_dev_encode_audio(qtts_dev_t *dev, int nb, const float *const *wav, const int *n, int *codes,
                          int max_frames, int *frames, float *latent);

/* ---- host-pointer stage wrappers (oracle-level tests, c/qwen_tts.h:483-502) ---- */
int qtts_dev_talker_prefill_host(qtts_dev_t *dev, const float *embeds, int n, float *hidden_out);
int qtts_dev_talker_forward_host(qtts_dev_t *dev, const float *embed, float *logits, float *hidden_out);
int qtts_dev_subtalker_host(qtts_dev_t *dev, const float *hidden, int first_code, int *out_codes);
float *qtts_dev_codec_decode_host(qtts_dev_t *dev, const int *codes, int T, int *out_samples);

/* ---- kernel-level entry points (device buffers) ---- */
/* kernel_matvec_bf16 (c/qwen_tts_kernels.c:95): out[b*rows + r] = sum_c A[r,c] x[b*cols + c] */
int qtts_hip_matvec_bf16(float *out_dev, const uint16_t *A_dev, const float *x_dev, int rows, int cols,
                         int batch, void *stream);
/* kernel_rms_norm fused as a GEMV prologue; exported standalone for tests:
 * out = rmsnorm(x) @ A^T  (c/qwen_tts_kernels.c:27 + :95) */
int qtts_hip_rmsnorm_matvec_bf16(float *out_dev, const uint16_t *A_dev, const float *x_dev, const float *w_dev,
                                 float eps, int rows, int cols, int batch, void *stream);
/* the decode-loop GEMV dispatcher on `batch` lock-step rows (w_dev NULL: no norm):
 * batch 1 -> the batch-1 weight stream, 2..16 -> the matrix-core batch kernel
 * (c/qwen_tts_kernels.c:27 + :95 per row) */
int qtts_hip_decode_matvec_bf16(float *out_dev, const uint16_t *A_dev, const float *x_dev, const float *w_dev,
                                float eps, int rows, int cols, int batch, void *stream);
/* the batch-1 GEMV of the sub-talker chain (weights resident in the Infinity
 * Cache, default cache policy): w_dev NULL: no norm; epi 0 store, 3 residual
 * (out += A x), 4 SwiGLU over interleaved gate|up row quads (rows/2 outputs)
 * (c/qwen_tts_kernels.c:27 + :95 + :213) */
int qtts_hip_resident_matvec_bf16(float *out_dev, const uint16_t *A_dev, const float *x_dev, const float *w_dev,
                                  float eps, int rows, int cols, int epi, void *stream);
/* kernel_sample_top_k (c/qwen_tts_kernels.c:407) on `batch` logit rows; rng_bits
 * holds the float-bit xorshift state per row (updated in place). */
int qtts_hip_sample_top_k(int *out_dev, const float *logits_dev, int vocab, int top_k, float top_p,
                          float temperature, uint32_t *rng_bits_dev, int batch, void *stream);
/* kernel_causal_conv1d (c/qwen_tts_kernels.c:659): [ci, L] -> [co, L] */
int qtts_hip_causal_conv1d(float *out_dev, const float *in_dev, const float *w_dev, const float *b_dev, int ci,
                           int co, int k, int L, int dilation, int groups, void *stream);
/* kernel_transposed_conv1d (c/qwen_tts_kernels.c:873): [ci, L] -> [co, L*stride] */
int qtts_hip_transposed_conv1d(float *out_dev, const float *in_dev, const float *w_dev, const float *b_dev,
                               int ci, int co, int k, int stride, int L, void *stream);
/* kernel_snake_beta (c/qwen_tts_kernels.c:251), alpha/inv_beta pre-processed */
int qtts_hip_snake_beta(float *out_dev, const float *x_dev, const float *alpha_dev, const float *inv_beta_dev,
                        int channels, int length, void *stream);
/* glibc-exact expf replica used by the sampler (for the libm cross-check test) */
int qtts_hip_expf_glibc(float *out_dev, const float *in_dev, int n, void *stream);
int qtts_hip_sync(void);
/* Talker layers enqueued (or captured into a frame graph) on the persistent
 * one-launch layer (QTTS_HIP_TENGINE=1) since the library loaded. */
long long qtts_hip_tengine_layers(void);

/* Diagnostics: run ONE frame eagerly on the current generation state with an
 * event pair around every kernel launch on the context stream.  kind[i]:
 * 0 talker GEMV, 1 sub-talker GEMV, 2 attention, 3 sampler, 4 embed-sum;
 * bytes[i]: algorithmic bytes of GEMV launches; ms[i]: measured duration;
 * names (optional, max*64 chars): kernel instantiation of launch i as
 * rocprofv3 names it (e.g. "k_gemv1<8, 2, true>").
 * Returns the number of kernels (<0 on error).  Advances the state by one
 * frame, so call it after a generation, not in the middle of one. */
int qtts_dev_profile_frame(qtts_dev_t *dev, int step, int max, int *kind, double *bytes, float *ms, char *names);
/* Measurement: the current device's HBM stream bandwidth over two `bytes`-sized
 * buffers (>> the 256 MB Infinity Cache): a non-temporal float4 read stream and
 * a float4 copy (read + write bytes), `iters` timed launches each with HIP
 * events on their own stream, GB/s (the roofline against a
 * bandwidth measured on the box beside the 8 TB/s nominal). */
int qtts_hip_hbm_bw(size_t bytes, int iters, double *read_gbs, double *copy_gbs);

#ifdef __cplusplus
}
#endif
#endif /* QTTS_HIP_H */
