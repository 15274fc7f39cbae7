#!/usr/bin/env python3
"""Seeded synthetic Qwen3-TTS model directories (test/bench infrastructure).

No real checkpoint is available offline, so every test and benchmark runs on
random-init weights with the exact tensor names, shapes and dtypes the
reference loader binds (c/qwen_tts.c:433-769) and the config keys it parses
(c/qwen_tts.c:248-337).  Layout produced:

    <dir>/config.json                          talker_config.* (+ code_predictor_config)
    <dir>/model.safetensors                    talker.* tensors (BF16)
    <dir>/speech_tokenizer/config.json         decoder_config.*
    <dir>/speech_tokenizer/model.safetensors   decoder.* tensors (F32)

Presets with voice-clone encoders ("enc" below: tiny_vc, 0.6b, 1.7b) add
    <dir>/model-speaker.safetensors            speaker_encoder.* (BF16, the model dtype)
    <dir>/speech_tokenizer/model-encoder.safetensors   encoder.* (F32)
and the `speaker_encoder_config` / `encoder_config` keys (modeling_qwen3_tts.py
:311-393 ECAPA-TDNN, configuration_qwen3_tts.py:47-67; the 12 Hz tokenizer's
MimiModel encoder, configuration_qwen3_tts_tokenizer_v2.py:139-169).  They are
extra shards, so the tiny_vc talker/codec files are byte-identical to tiny's.

Shapes ("synth-0.6b", "synth-1.7b") follow SURVEY.md section 8 header; the
values marked there as not present in the reference (1.7B dims, I=3072 for
0.6B, mrope_section) are assumptions of this generator.

Weights are deterministic per tensor: each tensor gets its own PCG64 stream
seeded from (model seed, tensor name), so the files are reproducible
byte-for-byte and independent of write order.  Linear weights are uniform
with std gain/sqrt(fan_in); residual-branch outputs (o_proj, down_proj) are
scaled by 1/sqrt(2L); logit heads get a larger gain ("conditioned" heads) so
the sampled distributions are peaked.  Codec weights are scaled so the
waveform stays well inside [-1, 1].

Usage:  python tools/synth_model.py --preset tiny --out /tmp/qtts_tiny
"""
import argparse
import hashlib
import json
import os
import struct
import sys

import numpy as np

PRESETS = {
    # tiny: exercises every code path (input projection since H != Hs,
    # GQA, sliding window < T, all vocoder stages) at test-friendly sizes.
    "tiny": dict(
        H=128, I=256, L=2, NH=4, KV=2, HD=32, TH=64, TV=151936, V=3072, G=16,
        Hs=64, Is=128, Ls=2, NHs=4, KVs=2, HDs=16, Vs=2048,
        rope_theta=1000000.0, mrope=[8, 4, 4],
        c_hidden=64, c_latent=128, c_cbdim=64, c_layers=2, c_heads=4, c_kv=4,
        c_inter=128, c_window=72, c_dec=64, c_cb=2048, c_q=16,
        eos_gain=1.0,
    ),
    # tiny with H == Hs: no small_to_mtp_projection (0.6B-style sub-talker input)
    "tiny_eq": dict(
        H=64, I=128, L=2, NH=4, KV=2, HD=16, TH=64, TV=151936, V=3072, G=16,
        Hs=64, Is=128, Ls=2, NHs=4, KVs=2, HDs=16, Vs=2048,
        rope_theta=1000000.0, mrope=[4, 2, 2],
        c_hidden=64, c_latent=128, c_cbdim=64, c_layers=2, c_heads=4, c_kv=4,
        c_inter=128, c_window=72, c_dec=64, c_cb=2048, c_q=16,
        eos_gain=1.0,
    ),
    # tiny + voice-clone encoders (ECAPA-TDNN speaker encoder, Mimi encoder)
    "tiny_vc": dict(
        H=128, I=256, L=2, NH=4, KV=2, HD=32, TH=64, TV=151936, V=3072, G=16,
        Hs=64, Is=128, Ls=2, NHs=4, KVs=2, HDs=16, Vs=2048,
        rope_theta=1000000.0, mrope=[8, 4, 4],
        c_hidden=64, c_latent=128, c_cbdim=64, c_layers=2, c_heads=4, c_kv=4,
        c_inter=128, c_window=72, c_dec=64, c_cb=2048, c_q=16,
        eos_gain=1.0, enc="tiny",
    ),
    # the 0.6B talker's attention shape (NH 16 / KV 8 / HD 128, H 1024) in 2
    # narrow layers, tiny sub-talker and codec: cheap enough for the CPU
    # checkers to decode 600+ frames, so the talker's split-K attention runs
    # through 1, 2-8 and > 8 key splits (64 keys per split at HD 128)
    "hd128": dict(
        H=1024, I=1024, L=2, NH=16, KV=8, HD=128, TH=64, TV=151936, V=3072, G=16,
        Hs=64, Is=128, Ls=2, NHs=4, KVs=2, HDs=16, Vs=2048,
        rope_theta=1000000.0, mrope=[24, 20, 20],
        c_hidden=64, c_latent=128, c_cbdim=64, c_layers=2, c_heads=4, c_kv=4,
        c_inter=128, c_window=72, c_dec=64, c_cb=2048, c_q=16,
        eos_gain=1.0,
    ),
    "0.6b": dict(
        H=1024, I=3072, L=28, NH=16, KV=8, HD=128, TH=2048, TV=151936, V=3072, G=16,
        Hs=1024, Is=3072, Ls=5, NHs=16, KVs=8, HDs=128, Vs=2048,
        rope_theta=1000000.0, mrope=[24, 20, 20],
        c_hidden=1024, c_latent=1024, c_cbdim=512, c_layers=8, c_heads=16, c_kv=16,
        c_inter=3072, c_window=72, c_dec=1536, c_cb=2048, c_q=16,
        eos_gain=1.0, enc="full",
    ),
    "1.7b": dict(
        H=2048, I=6144, L=28, NH=16, KV=8, HD=128, TH=2048, TV=151936, V=3072, G=16,
        Hs=1024, Is=3072, Ls=5, NHs=16, KVs=8, HDs=128, Vs=2048,
        rope_theta=1000000.0, mrope=[24, 20, 20],
        c_hidden=1024, c_latent=1024, c_cbdim=512, c_layers=8, c_heads=16, c_kv=16,
        c_inter=3072, c_window=72, c_dec=1536, c_cb=2048, c_q=16,
        eos_gain=1.0, enc="full",
    ),
}

# Voice-clone encoders.  "full" = the reference defaults
# (Qwen3TTSSpeakerEncoderConfig, configuration_qwen3_tts.py:47-57, enc_dim =
# the talker hidden the x-vector is added to; MimiConfig defaults, which the
# 12 Hz tokenizer's 1920-sample frame implies: 8*6*5*4 * 2 = 1920).
ENC = {
    "tiny": dict(spk=dict(mel_dim=128, enc_channels=[32, 32, 32, 32, 96], enc_kernel_sizes=[5, 3, 3, 3, 1],
                          enc_dilations=[1, 2, 3, 4, 1], enc_attention_channels=16, enc_res2net_scale=8,
                          enc_se_channels=16),
                 mimi=dict(hidden_size=64, num_filters=8, num_hidden_layers=2, num_attention_heads=4,
                           num_key_value_heads=4, head_dim=16, intermediate_size=128, sliding_window=16,
                           num_quantizers=20, codebook_size=2048, codebook_dim=32,
                           vector_quantization_hidden_dimension=32)),
    "full": dict(spk=dict(mel_dim=128, enc_channels=[512, 512, 512, 512, 1536], enc_kernel_sizes=[5, 3, 3, 3, 1],
                          enc_dilations=[1, 2, 3, 4, 1], enc_attention_channels=128, enc_res2net_scale=8,
                          enc_se_channels=128),
                 mimi=dict(hidden_size=512, num_filters=64, num_hidden_layers=8, num_attention_heads=8,
                           num_key_value_heads=8, head_dim=64, intermediate_size=2048, sliding_window=250,
                           num_quantizers=32, codebook_size=2048, codebook_dim=256,
                           vector_quantization_hidden_dimension=256)),
}
MIMI_FIXED = dict(sampling_rate=24000, frame_rate=12.5, audio_channels=1, upsampling_ratios=[8, 6, 5, 4],
                  kernel_size=7, last_kernel_size=3, residual_kernel_size=3, dilation_growth_rate=2,
                  num_residual_layers=1, compress=2, use_causal_conv=True, pad_mode="constant",
                  trim_right_ratio=1.0, use_conv_shortcut=False, num_semantic_quantizers=1,
                  norm_eps=1e-5, rope_theta=10000.0, hidden_act="gelu", layer_scale_initial_scale=0.01,
                  max_position_embeddings=8000, upsample_groups=512, attention_bias=False)


def enc_configs(p):
    e = ENC[p["enc"]]
    spk = dict(e["spk"], enc_dim=p["H"], sample_rate=24000)
    mimi = dict(MIMI_FIXED, **e["mimi"])
    mimi["upsample_groups"] = min(mimi["upsample_groups"], mimi["hidden_size"])   # decoder half only
    return spk, mimi


def speaker_specs(p):
    """speaker_encoder.* (Qwen3TTSSpeakerEncoder, modeling_qwen3_tts.py:311-393)."""
    c, _ = enc_configs(p)
    ch, ks = c["enc_channels"], c["enc_kernel_sizes"]
    S = []

    def conv(name, co, ci, k, gain=1.4):
        S.append((name + ".weight", (co, ci, k), "conv", gain))
        S.append((name + ".bias", (co,), "bias", 0.02))

    P = "speaker_encoder."
    conv(P + "blocks.0.conv", ch[0], c["mel_dim"], ks[0], 0.5)
    sc = c["enc_res2net_scale"]
    for i in range(1, len(ch) - 1):
        b = f"{P}blocks.{i}."
        conv(b + "tdnn1.conv", ch[i], ch[i - 1], 1)
        for j in range(sc - 1):
            conv(f"{b}res2net_block.blocks.{j}.conv", ch[i] // sc, ch[i] // sc, ks[i])
        conv(b + "tdnn2.conv", ch[i], ch[i], 1)
        conv(b + "se_block.conv1", c["enc_se_channels"], ch[i], 1)
        conv(b + "se_block.conv2", ch[i], c["enc_se_channels"], 1)
    conv(P + "mfa.conv", ch[-1], ch[-1], ks[-1])
    conv(P + "asp.tdnn.conv", c["enc_attention_channels"], ch[-1] * 3, 1)
    conv(P + "asp.conv", ch[-1], c["enc_attention_channels"], 1, 2.0)
    conv(P + "fc", c["enc_dim"], ch[-1] * 2, 1, 1.0)
    return S


def mimi_encoder_specs(p):
    """encoder.* of the 12 Hz tokenizer (MimiModel without its decoder half,
    modeling_qwen3_tts_tokenizer_v2.py:899-908)."""
    _, m = enc_configs(p)
    S = []

    def conv(name, co, ci, k, gain=1.0, bias=True):
        S.append((name + ".weight", (co, ci, k), "conv", gain))
        if bias:
            S.append((name + ".bias", (co,), "bias", 0.02))

    P = "encoder.encoder.layers."
    nf = m["num_filters"]
    conv(P + "0.conv", nf, 1, m["kernel_size"], 1.0)
    li, scale = 1, 1
    for r in reversed(m["upsampling_ratios"]):
        d = scale * nf
        conv(f"{P}{li}.block.1.conv", d // m["compress"], d, m["residual_kernel_size"], 1.2)
        conv(f"{P}{li}.block.3.conv", d, d // m["compress"], 1, 0.6)
        li += 2
        conv(f"{P}{li}.conv", 2 * d, d, 2 * r, 1.2)
        li += 1
        scale *= 2
    li += 1
    conv(f"{P}{li}.conv", m["hidden_size"], scale * nf, m["last_kernel_size"], 1.2)
    hid, nh, nkv, hd, I = (m["hidden_size"], m["num_attention_heads"], m["num_key_value_heads"], m["head_dim"],
                           m["intermediate_size"])
    for l in range(m["num_hidden_layers"]):
        q = f"encoder.encoder_transformer.layers.{l}."
        S.append((q + "input_layernorm.weight", (hid,), "norm", 0.05))
        S.append((q + "input_layernorm.bias", (hid,), "bias", 0.02))
        S.append((q + "post_attention_layernorm.weight", (hid,), "norm", 0.05))
        S.append((q + "post_attention_layernorm.bias", (hid,), "bias", 0.02))
        S.append((q + "self_attn.q_proj.weight", (nh * hd, hid), "lin", 1.0))
        S.append((q + "self_attn.k_proj.weight", (nkv * hd, hid), "lin", 1.0))
        S.append((q + "self_attn.v_proj.weight", (nkv * hd, hid), "lin", 1.0))
        S.append((q + "self_attn.o_proj.weight", (hid, nh * hd), "lin", 1.0))
        S.append((q + "mlp.fc1.weight", (I, hid), "lin", 1.0))
        S.append((q + "mlp.fc2.weight", (hid, I), "lin", 1.0))
        S.append((q + "self_attn_layer_scale.scale", (hid,), "lscale", 0))
        S.append((q + "mlp_layer_scale.scale", (hid,), "lscale", 0))
    conv("encoder.downsample.conv", hid, hid, 4, 1.0, bias=False)
    vq, cb = m["vector_quantization_hidden_dimension"], m["codebook_size"]
    nsem = m["num_semantic_quantizers"]
    for kind, n in (("semantic", nsem), ("acoustic", m["num_quantizers"] - nsem)):
        q = f"encoder.quantizer.{kind}_residual_vector_quantizer."
        S.append((q + "input_proj.weight", (vq, hid, 1), "conv", 1.0))
        S.append((q + "output_proj.weight", (hid, vq, 1), "conv", 1.0))
        for i in range(n):
            S.append((f"{q}layers.{i}.codebook.initialized", (1,), "one", 0))
            S.append((f"{q}layers.{i}.codebook.cluster_usage", (cb,), "usage", 0))
            S.append((f"{q}layers.{i}.codebook.embed_sum", (cb, vq), "esum", 1.0 if i == 0 else 0.6))
    return S

SPEAKERS = {"aiden": 2900, "serena": 2901, "vivian": 2902}
LANGUAGES = {"english": 2050, "chinese": 2055, "japanese": 2058}
CODEC_IDS = dict(codec_pad_id=2148, codec_bos_id=2149, codec_eos_token_id=2150,
                 codec_think_id=2154, codec_nothink_id=2155,
                 codec_think_bos_id=2156, codec_think_eos_id=2157)


def _rng(seed, name):
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return np.random.Generator(np.random.PCG64(int.from_bytes(h[:8], "little")))


def _f32_to_bf16(a):
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u >> 16) & 1) + 0x7FFF
    return ((u + r) >> 16).astype(np.uint16)


class StWriter:
    """Streaming safetensors writer: header first (offsets precomputed), then
    each tensor's bytes, so a multi-GB model never sits in memory at once."""

    def __init__(self, path, specs):
        # specs: list of (name, dtype_str, shape)
        self.path = path
        self.specs = specs
        hdr = {}
        off = 0
        self.sizes = {}
        for name, dt, shape in specs:
            n = int(np.prod(shape)) * (2 if dt == "BF16" else 4)
            hdr[name] = {"dtype": dt, "shape": list(shape), "data_offsets": [off, off + n]}
            self.sizes[name] = n
            off += n
        hb = json.dumps(hdr, separators=(",", ":")).encode()
        hb += b" " * ((8 - len(hb) % 8) % 8)
        self.f = open(path, "wb")
        self.f.write(struct.pack("<Q", len(hb)))
        self.f.write(hb)
        self.expect = [s[0] for s in specs]
        self.i = 0

    def write(self, name, arr):
        assert self.expect[self.i] == name, (self.expect[self.i], name)
        dt = self.specs[self.i][1]
        if dt == "BF16":
            b = _f32_to_bf16(arr).tobytes() if arr.dtype != np.uint16 else arr.tobytes()
        else:
            b = np.ascontiguousarray(arr, dtype=np.float32).tobytes()
        assert len(b) == self.sizes[name], (name, len(b), self.sizes[name])
        self.f.write(b)
        self.i += 1

    def close(self):
        assert self.i == len(self.expect)
        self.f.close()


def _uniform(rng, shape, std):
    a = np.float32(std * np.sqrt(3.0))
    out = np.empty(shape, dtype=np.float32)
    flat = out.reshape(-1)
    step = 1 << 24
    for s in range(0, flat.size, step):
        n = min(step, flat.size - s)
        flat[s:s + n] = rng.random(n, dtype=np.float32)
    flat *= np.float32(2.0) * a
    flat -= a
    return out


def talker_specs(p):
    H, I, L, NH, KV, HD = p["H"], p["I"], p["L"], p["NH"], p["KV"], p["HD"]
    Hs, Is, Ls, NHs, KVs, HDs = p["Hs"], p["Is"], p["Ls"], p["NHs"], p["KVs"], p["HDs"]
    S = []
    S.append(("talker.model.codec_embedding.weight", (p["V"], H), "emb", 0.35))
    S.append(("talker.model.text_embedding.weight", (p["TV"], p["TH"]), "emb", 1.0))
    S.append(("talker.text_projection.linear_fc1.weight", (p["TH"], p["TH"]), "lin", 1.0))
    S.append(("talker.text_projection.linear_fc1.bias", (p["TH"],), "bias", 0.05))
    S.append(("talker.text_projection.linear_fc2.weight", (H, p["TH"]), "lin", 1.0))
    S.append(("talker.text_projection.linear_fc2.bias", (H,), "bias", 0.05))
    res = 1.0 / np.sqrt(2.0 * L)
    for i in range(L):
        pre = f"talker.model.layers.{i}."
        S.append((pre + "self_attn.q_proj.weight", (NH * HD, H), "lin", 1.0))
        S.append((pre + "self_attn.k_proj.weight", (KV * HD, H), "lin", 1.0))
        S.append((pre + "self_attn.v_proj.weight", (KV * HD, H), "lin", 1.0))
        S.append((pre + "self_attn.o_proj.weight", (H, NH * HD), "lin", res))
        S.append((pre + "self_attn.q_norm.weight", (HD,), "norm", 0.05))
        S.append((pre + "self_attn.k_norm.weight", (HD,), "norm", 0.05))
        S.append((pre + "input_layernorm.weight", (H,), "norm", 0.05))
        S.append((pre + "post_attention_layernorm.weight", (H,), "norm", 0.05))
        S.append((pre + "mlp.gate_proj.weight", (I, H), "lin", 1.0))
        S.append((pre + "mlp.up_proj.weight", (I, H), "lin", 1.0))
        S.append((pre + "mlp.down_proj.weight", (H, I), "lin", res))
    S.append(("talker.model.norm.weight", (H,), "norm", 0.05))
    S.append(("talker.codec_head.weight", (p["V"], H), "head", 3.0))
    for g in range(p["G"] - 1):
        S.append((f"talker.code_predictor.model.codec_embedding.{g}.weight", (p["Vs"], H), "emb", 0.35))
    if H != Hs:
        S.append(("talker.code_predictor.small_to_mtp_projection.weight", (Hs, H), "lin", 1.0))
        S.append(("talker.code_predictor.small_to_mtp_projection.bias", (Hs,), "bias", 0.05))
    sres = 1.0 / np.sqrt(2.0 * Ls)
    for i in range(Ls):
        pre = f"talker.code_predictor.model.layers.{i}."
        S.append((pre + "self_attn.q_proj.weight", (NHs * HDs, Hs), "lin", 1.0))
        S.append((pre + "self_attn.k_proj.weight", (KVs * HDs, Hs), "lin", 1.0))
        S.append((pre + "self_attn.v_proj.weight", (KVs * HDs, Hs), "lin", 1.0))
        S.append((pre + "self_attn.o_proj.weight", (Hs, NHs * HDs), "lin", sres))
        S.append((pre + "self_attn.q_norm.weight", (HDs,), "norm", 0.05))
        S.append((pre + "self_attn.k_norm.weight", (HDs,), "norm", 0.05))
        S.append((pre + "input_layernorm.weight", (Hs,), "norm", 0.05))
        S.append((pre + "post_attention_layernorm.weight", (Hs,), "norm", 0.05))
        S.append((pre + "mlp.gate_proj.weight", (Is, Hs), "lin", 1.0))
        S.append((pre + "mlp.up_proj.weight", (Is, Hs), "lin", 1.0))
        S.append((pre + "mlp.down_proj.weight", (Hs, Is), "lin", sres))
    S.append(("talker.code_predictor.model.norm.weight", (Hs,), "norm", 0.05))
    for g in range(p["G"] - 1):
        S.append((f"talker.code_predictor.lm_head.{g}.weight", (p["Vs"], Hs), "head", 3.0))
    return S


def codec_specs(p):
    CB, Q = p["c_cb"], p["c_q"]
    vq = p["c_cbdim"] // 2
    half = p["c_latent"] // 2
    lat, hid, inter = p["c_latent"], p["c_hidden"], p["c_inter"]
    S = []
    S.append(("decoder.quantizer.rvq_first.vq.layers.0._codebook.cluster_usage", (CB,), "usage", 0))
    S.append(("decoder.quantizer.rvq_first.vq.layers.0._codebook.embedding_sum", (CB, vq), "esum", 1.0))
    S.append(("decoder.quantizer.rvq_first.output_proj.weight", (half, vq, 1), "conv", 1.0))
    for q in range(Q - 1):
        S.append((f"decoder.quantizer.rvq_rest.vq.layers.{q}._codebook.cluster_usage", (CB,), "usage", 0))
        S.append((f"decoder.quantizer.rvq_rest.vq.layers.{q}._codebook.embedding_sum", (CB, vq), "esum", 0.3))
    S.append(("decoder.quantizer.rvq_rest.output_proj.weight", (half, vq, 1), "conv", 1.0))
    S.append(("decoder.pre_conv.conv.weight", (lat, p["c_cbdim"], 3), "conv", 1.0))
    S.append(("decoder.pre_conv.conv.bias", (lat,), "bias", 0.02))
    S.append(("decoder.pre_transformer.input_proj.weight", (hid, lat), "lin", 1.0))
    S.append(("decoder.pre_transformer.input_proj.bias", (hid,), "bias", 0.02))
    S.append(("decoder.pre_transformer.output_proj.weight", (lat, hid), "lin", 1.0))
    S.append(("decoder.pre_transformer.output_proj.bias", (lat,), "bias", 0.02))
    S.append(("decoder.pre_transformer.norm.weight", (hid,), "norm", 0.05))
    nh, nkv = p["c_heads"], p["c_kv"]
    hd = hid // nh
    for i in range(p["c_layers"]):
        pre = f"decoder.pre_transformer.layers.{i}."
        S.append((pre + "input_layernorm.weight", (hid,), "norm", 0.05))
        S.append((pre + "post_attention_layernorm.weight", (hid,), "norm", 0.05))
        S.append((pre + "self_attn_layer_scale.scale", (hid,), "lscale", 0))
        S.append((pre + "mlp_layer_scale.scale", (hid,), "lscale", 0))
        S.append((pre + "self_attn.q_proj.weight", (nh * hd, hid), "lin", 1.0))
        S.append((pre + "self_attn.k_proj.weight", (nkv * hd, hid), "lin", 1.0))
        S.append((pre + "self_attn.v_proj.weight", (nkv * hd, hid), "lin", 1.0))
        S.append((pre + "self_attn.o_proj.weight", (hid, nh * hd), "lin", 1.0))
        S.append((pre + "mlp.gate_proj.weight", (inter, hid), "lin", 1.0))
        S.append((pre + "mlp.up_proj.weight", (inter, hid), "lin", 1.0))
        S.append((pre + "mlp.down_proj.weight", (hid, inter), "lin", 1.0))
    for s in range(2):
        S.append((f"decoder.upsample.{s}.0.conv.weight", (lat, lat, 2), "tconv", 1.0))
        S.append((f"decoder.upsample.{s}.0.conv.bias", (lat,), "bias", 0.02))
        S.append((f"decoder.upsample.{s}.1.dwconv.conv.weight", (lat, 1, 7), "conv", 1.0))
        S.append((f"decoder.upsample.{s}.1.dwconv.conv.bias", (lat,), "bias", 0.02))
        S.append((f"decoder.upsample.{s}.1.norm.weight", (lat,), "norm", 0.05))
        S.append((f"decoder.upsample.{s}.1.norm.bias", (lat,), "bias", 0.02))
        S.append((f"decoder.upsample.{s}.1.pwconv1.weight", (4 * lat, lat), "lin", 1.0))
        S.append((f"decoder.upsample.{s}.1.pwconv1.bias", (4 * lat,), "bias", 0.02))
        S.append((f"decoder.upsample.{s}.1.pwconv2.weight", (lat, 4 * lat), "lin", 1.0))
        S.append((f"decoder.upsample.{s}.1.pwconv2.bias", (lat,), "bias", 0.02))
        S.append((f"decoder.upsample.{s}.1.gamma", (lat,), "gamma", 0))
    dd = p["c_dec"]
    S.append(("decoder.decoder.0.conv.weight", (dd, lat, 7), "conv", 1.0))
    S.append(("decoder.decoder.0.conv.bias", (dd,), "bias", 0.02))
    rates = [8, 5, 4, 3]
    for b in range(4):
        ci, co = dd >> b, dd >> (b + 1)
        pre = f"decoder.decoder.{b + 1}.block."
        S.append((pre + "0.alpha", (ci,), "snake", 0))
        S.append((pre + "0.beta", (ci,), "snake", 0))
        S.append((pre + "1.conv.weight", (ci, co, 2 * rates[b]), "tconv", 1.0))
        S.append((pre + "1.conv.bias", (co,), "bias", 0.02))
        for r in range(3):
            rp = pre + f"{r + 2}."
            S.append((rp + "act1.alpha", (co,), "snake", 0))
            S.append((rp + "act1.beta", (co,), "snake", 0))
            S.append((rp + "conv1.conv.weight", (co, co, 7), "conv", 1.0))
            S.append((rp + "conv1.conv.bias", (co,), "bias", 0.02))
            S.append((rp + "act2.alpha", (co,), "snake", 0))
            S.append((rp + "act2.beta", (co,), "snake", 0))
            S.append((rp + "conv2.conv.weight", (co, co, 1), "conv", 0.5))
            S.append((rp + "conv2.conv.bias", (co,), "bias", 0.02))
    S.append(("decoder.decoder.5.alpha", (dd // 16,), "snake", 0))
    S.append(("decoder.decoder.5.beta", (dd // 16,), "snake", 0))
    S.append(("decoder.decoder.6.conv.weight", (1, dd // 16, 7), "conv", 0.04))
    S.append(("decoder.decoder.6.conv.bias", (1,), "bias", 0.0))
    return S


def make_tensor(seed, name, shape, kind, gain, p):
    rng = _rng(seed, name)
    if kind in ("lin", "head"):
        t = _uniform(rng, shape, gain / np.sqrt(shape[-1]))
        if kind == "head" and name == "talker.codec_head.weight" and p.get("eos_gain", 1.0) != 1.0:
            t[CODEC_IDS["codec_eos_token_id"]] *= np.float32(p["eos_gain"])
        return t
    if kind == "emb":
        return _uniform(rng, shape, gain)
    if kind == "bias":
        return _uniform(rng, shape, gain)
    if kind == "norm":
        return np.float32(1.0) + _uniform(rng, shape, gain)
    if kind == "conv":  # [out, in, k]: fan_in = in*k
        return _uniform(rng, shape, gain / np.sqrt(shape[1] * shape[2]))
    if kind == "tconv":  # [in, out, k]: each output sums in*(k/stride)=2*in taps
        return _uniform(rng, shape, gain / np.sqrt(2.0 * shape[0]))
    if kind == "usage":
        u = (np.float32(0.5) + rng.random(shape, dtype=np.float32) * np.float32(1.5)).astype(np.float32)
        u[7] = np.float32(0.0)  # exercises the max(usage, 1e-5) clamp (qwen_tts.c:585-586)
        return u
    if kind == "esum":
        return _uniform(rng, shape, gain)
    if kind == "lscale":
        return np.float32(0.005) + rng.random(shape, dtype=np.float32) * np.float32(0.015)
    if kind == "gamma":
        return np.float32(0.05) + rng.random(shape, dtype=np.float32) * np.float32(0.1)
    if kind == "snake":
        return _uniform(rng, shape, 0.1)
    if kind == "one":
        return np.ones(shape, dtype=np.float32)
    raise ValueError(kind)


def write_model(out, preset="tiny", seed=0, overrides=None, quiet=False):
    p = dict(PRESETS[preset])
    if overrides:
        p.update(overrides)
    os.makedirs(os.path.join(out, "speech_tokenizer"), exist_ok=True)
    cfg = {
        "model_type": "qwen3_tts",
        "synthetic": {"preset": preset, "seed": seed, "generator": "tools/synth_model.py"},
        "talker_config": {
            "vocab_size": p["V"], "hidden_size": p["H"], "intermediate_size": p["I"],
            "num_hidden_layers": p["L"], "num_attention_heads": p["NH"],
            "num_key_value_heads": p["KV"], "head_dim": p["HD"],
            "text_hidden_size": p["TH"], "text_vocab_size": p["TV"],
            "num_code_groups": p["G"], "rms_norm_eps": 1e-6, "rope_theta": p["rope_theta"],
            "rope_scaling": {"mrope_section": p["mrope"], "interleaved": False},
            "code_predictor_config": {
                "vocab_size": p["Vs"], "hidden_size": p["Hs"], "intermediate_size": p["Is"],
                "num_hidden_layers": p["Ls"], "num_attention_heads": p["NHs"],
                "num_key_value_heads": p["KVs"], "head_dim": p["HDs"],
            },
            "spk_id": SPEAKERS,
            "codec_language_id": LANGUAGES,
            **CODEC_IDS,
        },
    }
    ccfg = {
        "decoder_config": {
            "num_quantizers": p["c_q"], "codebook_size": p["c_cb"], "codebook_dim": p["c_cbdim"],
            "hidden_size": p["c_hidden"], "latent_dim": p["c_latent"],
            "num_hidden_layers": p["c_layers"], "num_attention_heads": p["c_heads"],
            "num_key_value_heads": p["c_kv"], "intermediate_size": p["c_inter"],
            "sliding_window": p["c_window"], "decoder_dim": p["c_dec"],
            "rms_norm_eps": 1e-5, "layer_scale_initial_scale": 0.01,
            "upsample_rates": [8, 5, 4, 3], "upsampling_ratios": [2, 2],
        }
    }
    files = [(os.path.join(out, "model.safetensors"), talker_specs(p)),
             (os.path.join(out, "speech_tokenizer", "model.safetensors"), codec_specs(p))]
    if p.get("enc"):
        spk, mimi = enc_configs(p)
        cfg["speaker_encoder_config"] = spk
        ccfg.update({"encoder_config": mimi, "encoder_valid_num_quantizers": 16, "input_sample_rate": 24000,
                     "output_sample_rate": 24000, "encode_downsample_rate": 1920, "decode_upsample_rate": 1920})
        files += [(os.path.join(out, "model-speaker.safetensors"), speaker_specs(p)),
                  (os.path.join(out, "speech_tokenizer", "model-encoder.safetensors"), mimi_encoder_specs(p))]
    with open(os.path.join(out, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1)
    with open(os.path.join(out, "speech_tokenizer", "config.json"), "w") as f:
        json.dump(ccfg, f, indent=1)

    for path, specs in files:
        codec = "speech_tokenizer" in path
        sp = [(n, "F32" if (codec or k in ("usage", "one")) else "BF16", s) for n, s, k, g in specs]
        w = StWriter(path + ".tmp", sp)
        for n, s, k, g in specs:
            if not quiet and np.prod(s) > (1 << 24):
                print(f"  gen {n} {s}", file=sys.stderr)
            w.write(n, make_tensor(seed, n, s, k, g, p))
        w.close()
        os.replace(path + ".tmp", path)
    return out


def ensure_model(out, preset="tiny", seed=0, overrides=None):
    """Create the model dir unless an identical one (same preset/seed) exists."""
    stamp = os.path.join(out, ".synth_stamp")
    key = {"preset": preset, "seed": seed, "overrides": overrides or {}}
    if PRESETS[preset].get("enc"):
        key["encoders"] = 1
    want = json.dumps(key, sort_keys=True)
    if not (os.path.exists(stamp) and open(stamp).read() == want):
        write_model(out, preset, seed, overrides, quiet=True)
        with open(stamp, "w") as f:
            f.write(want)
    if not os.path.exists(os.path.join(out, "merges.txt")):   # text input (tools/synth_tokenizer.py)
        from synth_tokenizer import write as write_tokenizer
        write_tokenizer(out)
    return out


def ref_wave(seed, secs=5.0, sr=24000):
    """Seeded synthetic reference audio for voice clone (5 s
    of pink noise plus a tone, 24 kHz mono, peak < 1)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(round(secs * sr))
    f = np.fft.rfft(rng.standard_normal(n))
    f /= np.sqrt(np.maximum(np.arange(f.shape[0]), 1.0))
    w = np.fft.irfft(f, n)
    w /= np.abs(w).max()
    t = np.arange(n) / sr
    w = 0.5 * w + 0.3 * np.sin(2 * np.pi * (150 + 13 * (seed % 11)) * t)
    return np.clip(w, -0.95, 0.95).astype(np.float32)


def prompt_ids(kind="short", seed=1234):
    """Token-id prompts (chat template). 'short' = test/tokens_great_power.txt
    (SURVEY.md 4); 'p128' = 3 + 30 random content ids + 5."""
    if kind == "short":
        return [151644, 77091, 198, 2354, 2244, 2355, 4041, 2244, 11752, 13, 151645, 198, 151644, 77091, 198]
    rng = np.random.Generator(np.random.PCG64(seed))
    body = rng.integers(1000, 100000, size=30).tolist()
    return [151644, 77091, 198] + body + [151645, 198, 151644, 77091, 198]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="tiny", choices=sorted(PRESETS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--eos-gain", type=float, default=None)
    a = ap.parse_args()
    ov = {"eos_gain": a.eos_gain} if a.eos_gain is not None else None
    write_model(a.out, a.preset, a.seed, ov)
    print(a.out)
