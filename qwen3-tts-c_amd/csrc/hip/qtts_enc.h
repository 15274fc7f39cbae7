// qtts_enc.h - internal interface of the device voice-clone encoders (C++ only).
//
// The two audio front ends of the Python reference's voice clone
// (qwen3_tts_model.py:356-458 create_voice_clone_prompt), which the c/
// reference does not have:
//   * speaker x-vector: mel_spectrogram + Qwen3TTSSpeakerEncoder (ECAPA-TDNN),
//     modeling_qwen3_tts.py:311-464, 1941-1954;
//   * 12 Hz reference codes: the tokenizer's MimiModel encoder,
//     modeling_qwen3_tts_tokenizer_v2.py:899-991.
// Every dense contraction (STFT, TDNN / SEANet convs, transformer linears,
// codebook distances aside) runs through k_econv: a batched implicit-GEMM
// conv1d on the bf16 matrix cores with exact 3-plane splits (fp32-equivalent
// products), any stride / dilation / padding mode, ELU or Res2Net-sum input
// prologues and bias / ReLU / tanh / GELU / LayerScale / residual epilogues.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../../../include/qtts_hip.h"

constexpr int ENC_MAXB = 16;   // utterances per encoder launch (BASELINE C5 uses 8)

struct EncW {                  // one conv / linear weight as three exact bf16 planes
    unsigned short *p = nullptr;   // [3][M][Kp]
    int M = 0, K = 0, Kp = 0, kw = 1;
};

struct EncModel {
    qtts_enc_dims_t d{};
    bool have_dims = false;
    hipStream_t st = nullptr;
    int device = 0;
    // host copies until enc_finalize builds the device layout
    std::map<std::string, std::vector<float>> host;
    std::map<std::string, std::vector<int64_t>> shape;
    bool got_spk = false, got_mimi = false;
    bool spk_ready = false, mimi_ready = false;
    // device weights
    std::map<std::string, EncW> cw;       // conv / linear planes by checkpoint name
    std::map<std::string, float *> fw;    // f32 vectors (biases, norms, scales, small GEMV matrices)
    EncW stft;                            // [2*513][1024] Hann-windowed DFT basis (cos rows, then -sin rows)
    float *melfb = nullptr;               // [128][513] slaney filterbank (librosa.filters.mel)
    float *cbk = nullptr;                 // [nvalid][CB][vq] Mimi codebooks (embed_sum / max(usage, 1e-5))
    float *rope_cos = nullptr, *rope_sin = nullptr;   // Mimi transformer [rope_cap][hd]
    int rope_cap = 0;
    std::vector<void *> wallocs;
    size_t wbytes = 0;
    // scratch (grown on demand)
    std::vector<void *> sallocs;
    size_t scap = 0;
    char *sbase = nullptr;
    float *part = nullptr;    // k_econv split-K partials (grown on demand)
    size_t part_cap = 0;
};

int enc_set_dims(EncModel *m, const qtts_enc_dims_t *d);
// returns 1 when the tensor belongs to an encoder (taken), 0 when not, <0 on error
int enc_put_tensor(EncModel *m, const std::string &name, const void *host, int dtype, const int64_t *shape, int ndim,
                   size_t n);
int enc_finalize(EncModel *m, int talker_hidden);
void enc_destroy(EncModel *m);
size_t enc_weight_bytes(const EncModel *m);
// x-vectors of nb waveforms (24 kHz, host) -> out[nb][enc_dim] (host); mel_out
// (optional) receives each utterance's [128][T_b] log-mel back to back
int enc_speaker(EncModel *m, int nb, const float *const *wav, const int *n, float *out, float *mel_out);
// 12 Hz codes of nb waveforms zero-padded to the longest (the tokenizer's
// batch encode) -> codes[nb][max_frames][16] (host), frames[b] =
// ceil(n[b] / 1920); latent (optional): [nb][hidden][max_frames] pre-quantizer
int enc_codes(EncModel *m, int nb, const float *const *wav, const int *n, int *codes, int max_frames, int *frames,
              float *latent);
