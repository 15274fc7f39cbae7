"""Model-dir I/O shared by tests and bench (test infrastructure).

* `read_safetensors(path)`: safetensors reader on np.memmap (header JSON +
  raw bytes; executes nothing from the file).  BF16 tensors come back as
  uint16 arrays.
* `load_config(model_dir)`: the dims the reference derives from
  config.json / speech_tokenizer/config.json, with the reference's own
  defaults (c/qwen_tts.c:248-337, c/qwen_tts.h:26-78).
"""
import json
import os
import struct

import numpy as np

_DT = {"BF16": np.uint16, "F32": np.float32, "F16": np.float16, "I64": np.int64, "I32": np.int32}


def read_safetensors(path):
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        hdr = json.loads(f.read(n))
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    base = 8 + n
    out = {}
    for name, e in hdr.items():
        if name == "__metadata__":
            continue
        a, b = e["data_offsets"]
        arr = mm[base + a: base + b].view(_DT[e["dtype"]]).reshape(e["shape"])
        out[name] = (e["dtype"], arr)
    return out


def read_model_tensors(model_dir):
    t = {}
    for d in (model_dir, os.path.join(model_dir, "speech_tokenizer")):
        for fn in sorted(os.listdir(d)):
            if fn.endswith(".safetensors"):
                t.update(read_safetensors(os.path.join(d, fn)))
    return t


def _get(js, path, default):
    cur = js
    for k in path.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return default
        cur = cur[k]
    return cur


def load_config(model_dir):
    js = json.load(open(os.path.join(model_dir, "config.json")))
    cs = json.load(open(os.path.join(model_dir, "speech_tokenizer", "config.json")))
    tc = "talker_config."
    c = {}
    c["H"] = _get(js, tc + "hidden_size", 1024)
    c["I"] = _get(js, tc + "intermediate_size", 2048)
    c["L"] = _get(js, tc + "num_hidden_layers", 20)
    c["NH"] = _get(js, tc + "num_attention_heads", 16)
    c["KV"] = _get(js, tc + "num_key_value_heads", 2)
    c["HD"] = _get(js, tc + "head_dim", 0) or c["H"] // c["NH"]
    c["TH"] = _get(js, tc + "text_hidden_size", 2048)
    c["TV"] = _get(js, tc + "text_vocab_size", 151936)
    c["V"] = _get(js, tc + "vocab_size", 3072)
    c["G"] = _get(js, tc + "num_code_groups", 32)
    c["eps"] = float(_get(js, tc + "rms_norm_eps", 1e-6))
    c["theta"] = float(_get(js, tc + "rope_theta", 10000.0))
    c["mrope"] = list(_get(js, tc + "rope_scaling.mrope_section", [16, 16, 0]))
    cp = tc + "code_predictor_config."
    c["Vs"] = _get(js, cp + "vocab_size", 2048)
    c["Hs"] = _get(js, cp + "hidden_size", 1024)
    c["Is"] = _get(js, cp + "intermediate_size", 3072)
    c["Ls"] = _get(js, cp + "num_hidden_layers", 5)
    c["NHs"] = _get(js, cp + "num_attention_heads", 16)
    c["KVs"] = _get(js, cp + "num_key_value_heads", 8)
    c["HDs"] = _get(js, cp + "head_dim", 128)
    c["pad"] = _get(js, tc + "codec_pad_id", 2148)
    c["bos"] = _get(js, tc + "codec_bos_id", 2149)
    c["eos"] = _get(js, tc + "codec_eos_token_id", 2150)
    c["think"] = _get(js, tc + "codec_think_id", 2154)
    c["nothink"] = _get(js, tc + "codec_nothink_id", 2155)
    c["think_bos"] = _get(js, tc + "codec_think_bos_id", 2156)
    c["think_eos"] = _get(js, tc + "codec_think_eos_id", 2157)
    c["speakers"] = {k: (v[0] if isinstance(v, list) else v) for k, v in _get(js, tc + "spk_id", {}).items()}
    c["languages"] = {k: (v[0] if isinstance(v, list) else v)
                      for k, v in _get(js, tc + "codec_language_id", {}).items()}
    dc = "decoder_config."
    c["cq"] = _get(cs, dc + "num_quantizers", 16)
    c["ccb"] = _get(cs, dc + "codebook_size", 2048)
    c["ccbdim"] = _get(cs, dc + "codebook_dim", 128)
    c["chid"] = _get(cs, dc + "hidden_size", 1024)
    c["clat"] = _get(cs, dc + "latent_dim", 1024)
    c["clayers"] = _get(cs, dc + "num_hidden_layers", 8)
    c["cheads"] = _get(cs, dc + "num_attention_heads", 16)
    c["ckv"] = _get(cs, dc + "num_key_value_heads", 16)
    c["cinter"] = _get(cs, dc + "intermediate_size", 3072)
    c["cwin"] = _get(cs, dc + "sliding_window", 72)
    c["cdec"] = _get(cs, dc + "decoder_dim", 1536)
    c["ceps"] = float(_get(cs, dc + "rms_norm_eps", 1e-5))
    c["rates"] = list(_get(cs, dc + "upsample_rates", [8, 5, 4, 3]))
    c["ratios"] = list(_get(cs, dc + "upsampling_ratios", [2, 2]))
    return c


def lookup_ids(cfg, speaker, language):
    """strcasecmp lookups (c/qwen_tts.c:1120-1145); -1 = absent."""
    spk = -1
    if speaker:
        for k, v in cfg["speakers"].items():
            if k.lower() == speaker.lower():
                spk = v
                break
    lang = -1
    if language and language.lower() != "auto":
        for k, v in cfg["languages"].items():
            if k.lower() == language.lower():
                lang = v
                break
    return spk, lang


def bf16_to_f32(a):
    return (np.asarray(a, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(a):
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    return ((u + (((u >> 16) & 1) + 0x7FFF)) >> 16).astype(np.uint16)
