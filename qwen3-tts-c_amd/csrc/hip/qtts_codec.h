// qtts_codec.h - internal interface of the device codec decoder (C++ only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../../../include/qtts_hip.h"

// Exact streaming decode state (codec_stream_*): every codec op is causal, so
// decoding frames chunk by chunk with (a) the last (K-1)*dil input columns of
// every convolution, (b) the last input frame of every transposed conv with
// K = 2s and (c) the last window-1 K/V rows of every transformer layer
// carried across chunks equals the full decode (Cd.c:581-749) up to fp order.
struct CodecStream {
    bool active = false;
    int pos0 = 0;              // frames decoded so far (absolute transformer position)
    int tc = 0;                // max frames per internal chunk
    int hm = 64;               // left margin (columns) of every channel-major buffer
    std::vector<float *> hist; // history slots [C][H]
    std::vector<int> hist_c, hist_h;
    std::vector<float *> kc, vc;  // transformer layer caches [(win-1) + tc][kvd]
    float *kvtmp = nullptr;
    int hl = 0;                // valid history rows in the K/V caches
    float *bufA = nullptr, *bufB = nullptr, *bufC = nullptr, *bufD = nullptr;
    size_t buf_elems = 0;
    float *tx = nullptr, *txn = nullptr, *tq = nullptr, *tatt = nullptr, *tg = nullptr, *tu = nullptr;
    float *rvq_s = nullptr, *rvq_a = nullptr;
    float *rope_cos = nullptr, *rope_sin = nullptr;
    int rope_cap = 0;
    int *iota = nullptr;       // [0 .. win + tc)
    int *zeros = nullptr;
    std::vector<void *> allocs;
};

struct CodecModel {
    qtts_dims_t d{};
    hipStream_t st = nullptr;
    std::map<std::string, float *> w;                 // f32 device tensors by checkpoint name
    std::map<std::string, std::vector<int64_t>> shape;
    std::map<std::string, std::vector<float>> host_keep;  // usage / esum pending codebook build
    float *cb = nullptr;                              // [Q][CB][vq] codebooks
    size_t wbytes = 0;
    // scratch (grown on demand)
    std::vector<void *> scratch;
    size_t scratch_bytes = 0;
    float *bufA = nullptr, *bufB = nullptr, *bufC = nullptr, *bufD = nullptr;
    size_t buf_elems = 0;
    float *tq = nullptr, *tx = nullptr, *txn = nullptr, *tatt = nullptr, *tg = nullptr, *tu = nullptr;
    float *rope_cos = nullptr, *rope_sin = nullptr;
    int t_cap = 0, rope_cap = 0;
    int *codes_tmp = nullptr;
    float *wav = nullptr;
    std::map<std::string, float *> wt;         // conv weights re-laid [Kw][co][ci] for k_conv, by name
    float *xg_part = nullptr;                  // split-K workspace of the codec GEMMs
    size_t xg_part_elems = 0;
    CodecStream cs;
    // per-stage timing of codec_decode (the reference's -v -v "Codec stages
    // (ms)" line, c/qwen_tts_codec.c:743-746): events around rvq / preconv /
    // transformer / upsample / vocoder when `timing` is on
    bool timing = false, timed = false;
    hipEvent_t tev[6] = {};
    float stage_ms[5] = {};
};

void codec_init(CodecModel *m, const qtts_dims_t *d, hipStream_t st);
void codec_destroy(CodecModel *m);
void codec_free_state(CodecModel *m);
size_t codec_weight_bytes(const CodecModel *m);
int codec_put_tensor(CodecModel *m, const std::string &name, const void *host, int dtype, const int64_t *shape,
                     int ndim, size_t n);
int codec_finalize(CodecModel *m);
// codes: device int32 [T][cq] (time-major).  Returns malloc'd host audio.
float *codec_decode(CodecModel *m, const int *codes_dev, int T, int *out_samples);
// independent decodes side by side: job i (device codes[i], T[i] frames) on
// lane i % nl (lane 0 = m, lanes[k] from codec_lane_new for k >= 1), its
// waveform copied to dwav + dwav_off[i] (device), out_samples[i] samples;
// returns after every lane's stream has drained
size_t codec_state_bytes(const CodecModel *m, int T);   // one lane's scratch for T frames
CodecModel *codec_lane_new(CodecModel *m, hipStream_t st);
void codec_lane_delete(CodecModel *lane);
int codec_decode_many(CodecModel *m, CodecModel *const *lanes, int nl, int n, const int *const *codes, const int *T,
                      float *dwav, const size_t *dwav_off, int *out_samples);
// streaming decode: begin resets the state (max_frames bounds the absolute
// position; chunk > 16 sizes the internal chunk for long pushes); push decodes T more frames (device codes, rows of stride ldc
// ints) and writes T * 1920 samples to host_out.  Returns samples or -1.
int codec_stream_begin(CodecModel *m, int max_frames, int chunk = 0);
int codec_stream_push(CodecModel *m, const int *codes_dev, int ldc, int T, float *host_out);
// the same into `out` (host memory, synchronous; or device memory: enqueued on
// m->st only, nothing waited for)
int codec_stream_push_to(CodecModel *m, const int *codes_dev, int ldc, int T, float *out, bool host);
void codec_stream_free(CodecModel *m);

// ---- generic fp32 implicit GEMM (exported for the kernel-level C-ABI) ----
// C(m, n) = sum_k A(m, k) * B(k, n), fp32 products on v_mfma_f32_32x32x2_f32.
enum { XA_ROWS = 0, XA_TRANS = 1, XA_TCONV_W = 2 };
enum { XB_WT = 0, XB_CONV = 1, XB_TCONV = 2 };
enum {
    XE_STORE = 0,        // C[m][n]
    XE_BIAS_N,           // + bias[n]
    XE_BIAS_N_GELU,      // gelu_tanh(acc + bias[n])
    XE_SILU_MUL,         // silu(aux[m][n]) * acc
    XE_SCALE_RESID_N,    // C[m][n] += acc * vec[n]
    XE_BIAS_T,           // out[n][m] = acc + bias[n]
    XE_BIAS_GAMMA_RES_T, // out[n][m] = (acc + bias[n]) * vec[n] + res[n][m]
    XE_BIAS_M,           // conv: out[m][n] = acc + bias[m]
    XE_BIAS_M_RES,       // conv: out[m][n] = acc + bias[m] + res[m][n]
    XE_BIAS_M_SNAKE,     // conv: out[m][n] = snake(acc + bias[m]) with (alpha, inv_beta)[m]
};
struct XGemm {
    int M = 0, N = 0, K = 0;
    int amode = XA_ROWS, bmode = XB_WT, emode = XE_STORE;
    const float *A = nullptr;  int lda = 0;   // rows: A[m*lda+k]; trans: A[k*lda+m]; tconv w: [ci][co][Kw]
    const float *B = nullptr;  int ldb = 0;   // wt: B[n*ldb+k]; conv/tconv: x[ic*ldb + t]
    // conv geometry (XB_CONV: k = ic*Kw + tap; XB_TCONV: k = ic*2 + j)
    int Kw = 1, dil = 1, pad = 0, L = 0, stride = 1, phase = 0, co = 0;
    const float *sa = nullptr, *sb = nullptr;  // optional SnakeBeta on B's input channels
    float *C = nullptr; int ldc = 0;          // output (XE_*_T: out[n*ldc + m]); tconv: out[m*ldc + n*stride + phase]
    const float *bias = nullptr, *vec = nullptr, *aux = nullptr, *res = nullptr;
    int ldaux = 0, ldres = 0;
    const float *ea = nullptr, *eb = nullptr;  // epilogue snake params (XE_BIAS_M_SNAKE)
    float *part = nullptr;                     // split-K workspace (nullptr: no split)
    size_t part_elems = 0;
    int tmin = 0;                              // conv/tconv input columns t >= tmin are read (t < 0: the
                                               // streaming history kept in the buffer's left margin)
    const float *wt = nullptr;                 // XB_CONV: the weights as [Kw][M][K/Kw] (k_conv's layout)
    int kz = 0;                                // k_conv split over input channels (set by the launcher)
};
int qtts_xgemm(const XGemm &g, hipStream_t st);
