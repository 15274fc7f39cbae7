#!/usr/bin/env python3
"""Golden vectors for the voice-clone audio encoders --
TEST INFRASTRUCTURE.  Writes tests/golden/enc_tiny.npz.

The reference's own Python (qwen_tts/, modeling_qwen3_tts.py) is not
importable here (`from librosa.filters import mel` fails: librosa is not in
the image), and its encoders are third-party code anyway:

* the 12 Hz tokenizer's encoder IS `transformers.MimiModel`
  (modeling_qwen3_tts_tokenizer_v2.py:899-908, pinned 4.57.3 in the
  reference's pyproject.toml; 5.15.0 is installed here);
* the speaker encoder `Qwen3TTSSpeakerEncoder` (modeling_qwen3_tts.py:311-393)
  is module-for-module transformers' Qwen2.5-Omni `ECAPA_TimeDelayNet`
  (transformers/models/qwen2_5_omni/modeling_qwen2_5_omni.py), so that class
  runs it here;
* `mel_spectrogram` (modeling_qwen3_tts.py:399-464) is restated with torch.stft
  and transformers.audio_utils.mel_filter_bank(norm="slaney",
  mel_scale="slaney") standing in for librosa.filters.mel.

Inputs: the synthetic `tiny_vc` model (tools/synth_model.py: random encoder
weights of the reference's tensor names) and seeded waveforms.  Every module
runs in float64 except the Mimi codebook distances, which MimiEuclideanCodebook
computes in float32 (torch.cdist on .float(), modeling_mimi.py:985-990), as
the reference does.

    python tests/golden/make_golden_enc.py
"""
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from synth_model import ensure_model  # noqa: E402
import enc_oracle  # noqa: E402

# seeded test waveforms: (seed, seconds, kind)
WAVES = [(11, 2.0, "pink+tone"), (12, 1.2345, "pink+tone"), (13, 0.5, "noise")]


def make_wave(seed, secs, kind):
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(round(secs * 24000))
    w = rng.standard_normal(n)
    if kind == "pink+tone":
        f = np.fft.rfft(w)
        f /= np.sqrt(np.maximum(np.arange(f.shape[0]), 1.0))
        w = np.fft.irfft(f, n)
        w /= np.abs(w).max()
        t = np.arange(n) / 24000.0
        w = 0.5 * w + 0.3 * np.sin(2 * np.pi * (180 + 40 * seed % 7) * t)
    else:
        w *= 0.1
    return np.clip(w, -0.95, 0.95).astype(np.float32)


def mel_torch(y):
    from transformers.audio_utils import mel_filter_bank
    fb = mel_filter_bank(num_frequency_bins=513, num_mel_filters=128, min_frequency=0.0, max_frequency=12000.0,
                         sampling_rate=24000, norm="slaney", mel_scale="slaney").T          # [128, 513]
    basis = torch.from_numpy(fb.astype(np.float32)).double()
    y = torch.from_numpy(y).double()[None]
    p = (1024 - 256) // 2
    y = torch.nn.functional.pad(y[:, None], (p, p), mode="reflect")[:, 0]
    spec = torch.stft(y, 1024, hop_length=256, win_length=1024, window=torch.hann_window(1024).double(),
                      center=False, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    spec = torch.sqrt(torch.view_as_real(spec).pow(2).sum(-1) + 1e-9)
    mel = torch.matmul(basis, spec)
    return torch.log(torch.clamp(mel, min=1e-5))[0].numpy(), fb


def main():
    md = ensure_model("/tmp/qtts_golden_tiny_vc", "tiny_vc")
    W, scfg, M, mcfg = enc_oracle.load_encoder_weights(md)

    from transformers.models.qwen2_5_omni.modeling_qwen2_5_omni import ECAPA_TimeDelayNet
    ecapa = ECAPA_TimeDelayNet(types.SimpleNamespace(**scfg)).double().eval()
    sd = {k: torch.from_numpy(v) for k, v in W.items()}
    ecapa.load_state_dict(sd, strict=True)
    from transformers import MimiConfig, MimiModel
    mc = {k: v for k, v in mcfg.items() if k not in ("encoder_valid_num_quantizers", "rope_theta")}
    mimi = MimiModel(MimiConfig(**mc, rope_parameters={"rope_type": "default", "rope_theta": mcfg["rope_theta"]}))
    mimi = mimi.double().eval()
    res = mimi.load_state_dict({k: torch.from_numpy(v) for k, v in M.items()}, strict=False)
    bad = [k for k in res.missing_keys if not k.startswith(("decoder", "upsample", "quantizer"))]
    bad += [k for k in res.missing_keys if k.startswith("quantizer") and "output_proj" not in k]
    assert not bad and not res.unexpected_keys, (bad, res.unexpected_keys)

    out = {}
    fb_tf = None
    with torch.no_grad():
        for i, (seed, secs, kind) in enumerate(WAVES):
            w = make_wave(seed, secs, kind)
            out[f"wav{i}"] = w
            mel, fb_tf = mel_torch(w)
            out[f"mel{i}"] = mel.astype(np.float32)
            x = ecapa(torch.from_numpy(mel)[None].transpose(1, 2))[0]
            out[f"xvec{i}"] = x.numpy().astype(np.float32)
        out["mel_fb"] = fb_tf.astype(np.float32)                          # [128, 513]
        # Mimi: batch of waves 0 and 1 zero-padded to the longer (the feature
        # extractor's padding, qwen3_tts_tokenizer.py:243-256), then one alone
        wavs = [out["wav0"], out["wav1"]]
        n = max(w.shape[0] for w in wavs)
        xb = torch.zeros(len(wavs), 1, n, dtype=torch.float64)
        for b, w in enumerate(wavs):
            xb[b, 0, :w.shape[0]] = torch.from_numpy(w).double()
        for tag, inp, lens in (("b", xb, [w.shape[0] for w in wavs]),
                               ("s", torch.from_numpy(out["wav2"]).double()[None, None], [out["wav2"].shape[0]])):
            emb = mimi.encoder(inp)
            emb = mimi.encoder_transformer(emb.transpose(1, 2), return_dict=True)[0].transpose(1, 2)
            emb = mimi.downsample(emb)
            codes = mimi.quantizer.encode(emb, 16).transpose(0, 1)          # [B, 16, T12]
            full = mimi.encode(inp, return_dict=True).audio_codes[:, :16]
            assert torch.equal(full, codes), "MimiModel.encode path differs from the module chain"
            for b, L in enumerate(lens):
                keep = -(-L // 1920)
                out[f"codes_{tag}{b}"] = codes[b, :, :keep].T.numpy().astype(np.int32)   # [T12, 16]
                out[f"latent_{tag}{b}"] = emb[b, :, :keep].numpy().astype(np.float32)    # [hid, T12]
            out[f"lens_{tag}"] = np.array(lens, dtype=np.int32)
    np.savez_compressed(os.path.join(HERE, "enc_tiny.npz"), **out)
    man = {"generator": "tests/golden/make_golden_enc.py", "model": "tiny_vc (tools/synth_model.py, seed 0)",
           "waves": WAVES, "transformers": __import__("transformers").__version__, "torch": torch.__version__}
    with open(os.path.join(HERE, "enc_manifest.json"), "w") as f:
        json.dump(man, f, indent=1)
    print("wrote", os.path.join(HERE, "enc_tiny.npz"), sorted(out))


if __name__ == "__main__":
    main()
