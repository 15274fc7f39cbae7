"""Python (ctypes) binding of the MI355X drop-in library lib/libqwen_tts_amd.so.

This is the binding a maintainer of the reference would add next to its CLI
(see INTEGRATION.md): it mirrors `qwen_tts.h` (ctx struct + functions) and
`qtts_hip.h` (kernel-level entry points on device buffers).  Tests and
bench.py use it; device buffers for the kernel-level calls are torch tensors
(PyTorch is plumbing only: allocation, streams, torch.distributed).

The library is required: importing works without a GPU (symbols resolve),
but every compute call needs the HIP device and fails loudly without it.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# QTTS_LIB: another build of the same library (A/B measurements of two builds
# in one process tree); the default is the in-tree build
LIB_PATH = os.environ.get("QTTS_LIB") or os.path.join(HERE, "lib", "libqwen_tts_amd.so")
CLI_PATH = os.path.join(HERE, "bin", "qwen-tts")

_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int)

PROGRESS_CB = C.CFUNCTYPE(None, C.c_int, C.c_int, C.c_void_p)
QUEUE_NEXT_CB = C.CFUNCTYPE(C.c_int, C.c_void_p)
AUDIO_CB = C.CFUNCTYPE(None, C.POINTER(C.c_float), C.c_int, C.c_void_p)


class Config(C.Structure):  # qwen_tts_config_t (include/qwen_tts.h)
    _fields_ = [(n, C.c_int) for n in (
        "talker_vocab_size", "talker_hidden", "talker_intermediate", "talker_layers", "talker_heads",
        "talker_kv_heads", "talker_head_dim", "talker_text_hidden", "talker_text_vocab", "num_code_groups")] + [
        ("talker_rms_norm_eps", C.c_float), ("talker_rope_theta", C.c_float), ("mrope_section", C.c_int * 3)] + [
        (n, C.c_int) for n in (
            "subtalker_vocab_size", "subtalker_hidden", "subtalker_intermediate", "subtalker_layers",
            "subtalker_heads", "subtalker_kv_heads", "subtalker_head_dim",
            "codec_num_quantizers", "codec_codebook_size", "codec_codebook_dim", "codec_hidden", "codec_latent",
            "codec_layers", "codec_heads", "codec_kv_heads", "codec_intermediate", "codec_sliding_window",
            "codec_decoder_dim")] + [
        ("codec_rms_norm_eps", C.c_float), ("codec_layer_scale", C.c_float),
        ("codec_upsample_rates", C.c_int * 4), ("codec_upsampling_ratios", C.c_int * 2),
        ("n_speakers", C.c_int), ("speaker_names", C.POINTER(C.c_char_p)), ("speaker_ids", _ip),
        ("n_languages", C.c_int), ("language_names", C.POINTER(C.c_char_p)), ("language_ids", _ip)] + [
        (n, C.c_int) for n in ("codec_pad_id", "codec_bos_id", "codec_eos_id", "codec_nothink_id", "codec_think_id",
                               "codec_think_bos_id", "codec_think_eos_id")]


class Ctx(C.Structure):  # qwen_tts_ctx_t (include/qwen_tts.h)
    _fields_ = [
        ("config", Config), ("model_dir", C.c_char * 512), ("hip", C.c_void_p), ("hip_device", C.c_int),
        ("talker_kv_len", C.c_int), ("tk_x", _fp),
        ("temperature", C.c_float), ("subtalker_temperature", C.c_float), ("top_k", C.c_int),
        ("subtalker_top_k", C.c_int), ("top_p", C.c_float), ("subtalker_top_p", C.c_float),
        ("repetition_penalty", C.c_float), ("max_new_tokens", C.c_int), ("fixed_codec_tokens", C.c_int),
        ("sample_seed", C.c_int), ("progress_cb", C.c_void_p), ("progress_cb_userdata", C.c_void_p),
        ("perf_total_ms", C.c_double), ("perf_talker_ms", C.c_double), ("perf_codec_ms", C.c_double),
        ("perf_codec_tokens", C.c_int), ("perf_prefill_ms", C.c_double), ("perf_first_frame_ms", C.c_double),
        ("last_codes", _ip), ("last_frames", C.c_int), ("last_stop_reason", C.c_int), ("last_stop_step", C.c_int),
        ("perf_first_packet_ms", C.c_double),
        ("tokenizer", C.c_void_p),
        ("queue_n", C.c_int), ("queue_codes", C.POINTER(_ip)), ("queue_frames", _ip), ("queue_stop_reason", _ip),
        ("queue_slot", _ip), ("queue_slots", C.c_int), ("queue_frames_launched", C.c_int),
        ("queue_refills", C.c_int), ("queue_slot_frames_used", C.c_longlong), ("queue_rows_launched", C.c_longlong),
    ]


# Every symbol include/qwen_tts.h and include/qtts_hip.h declare (checked by tests/test_host.py)
EXPORTS = [
    "qwen_tts_load", "qwen_tts_free", "qwen_tts_set_progress_callback", "qwen_tts_generate", "qwen_tts_write_wav",
    "qwen_tts_talker_prefill", "qwen_tts_talker_forward", "qwen_tts_subtalker_generate", "qwen_tts_codec_decode",
    "qwen_tts_talker_hidden", "qwen_tts_load_on", "qwen_tts_generate_batch", "qwen_tts_last_codes", "qwen_tts_last_codes_slot",
    "qwen_tts_abi_sizeof_ctx", "qwen_tts_verbose", "qwen_tts_generate_stream", "qwen_tts_codec_stream_begin",
    "qwen_tts_codec_stream_push", "qwen_tts_generate_voice_clone",
    "qwen_tts_generate_voice_clone_batch", "qwen_tts_generate_voice_clone_stream", "qwen_tts_tokenize",
    "qwen_tts_text_prompt", "qwen_tts_speaker_embedding", "qwen_tts_encode_audio",
    "qwen_tts_generate_voice_clone_audio", "qwen_tts_generate_voice_clone_audio_batch",
    "qwen_tts_generate_voice_clone_audio_stream", "qtts_dev_codec_timing", "qtts_dev_codec_stage_ms", "qwen_tts_resample",
    "qtts_hip_device_count", "qtts_dev_create", "qtts_dev_destroy", "qtts_dev_put_tensor", "qtts_dev_finalize",
    "qtts_dev_bytes", "qtts_dev_begin", "qtts_dev_prompt", "qtts_dev_prompt_ref", "qtts_dev_prefill", "qtts_dev_frame", "qtts_dev_poll", "qtts_dev_frame_done",
    "qtts_dev_get_codes", "qtts_dev_codec_slot", "qtts_dev_talker_prefill_host", "qtts_dev_talker_forward_host",
    "qtts_dev_subtalker_host", "qtts_dev_codec_decode_host", "qtts_hip_matvec_bf16",
    "qtts_hip_rmsnorm_matvec_bf16", "qtts_hip_decode_matvec_bf16", "qtts_hip_resident_matvec_bf16", "qtts_hip_sample_top_k", "qtts_hip_causal_conv1d",
    "qtts_hip_transposed_conv1d", "qtts_hip_snake_beta", "qtts_hip_expf_glibc", "qtts_hip_sync",
    "qtts_dev_profile_frame", "qtts_hip_hbm_bw", "qtts_dev_codec_stream_begin", "qtts_dev_codec_stream_begin_ex",
    "qtts_dev_codec_stream_prime", "qtts_dev_codec_stream_push_slot",
    "qtts_dev_codec_stream_push_host", "qtts_dev_codec_async_begin", "qtts_dev_codec_async_push",
    "qtts_dev_codec_async_end", "qtts_dev_codec_multi", "qtts_dev_enc_config", "qtts_dev_enc_available", "qtts_dev_speaker_embed",
    "qtts_dev_encode_audio", "qwen_tts_generate_queue", "qwen_tts_queue_codes", "qtts_dev_reserve", "qtts_dev_refill",
    "qtts_dev_retire", "qtts_dev_frame_stops", "qtts_dev_move_slot", "qtts_dev_set_rows", "qtts_hip_tengine_layers",
]

_LIB = None


def tokenize(model_dir, text):
    """Qwen2 BPE ids of `text` (qwen_tts_tokenize: the model dir's vocab.json /
    merges.txt; no GPU needed).  None on error."""
    n = C.c_int(0)
    p = lib().qwen_tts_tokenize(model_dir.encode(), text.encode("utf-8"), C.byref(n))
    if not p:
        return None
    ids = np.ctypeslib.as_array(C.cast(p, _ip), shape=(n.value,)).tolist() if n.value else []
    _libc.free(C.c_void_p(p))
    return ids


def resample(wav, sr_in, sr_out=24000):
    """qwen_tts_resample (host C, no GPU needed): librosa's polyphase method =
    scipy.signal.resample_poly."""
    w = np.ascontiguousarray(wav, np.float32)
    n = C.c_int(0)
    p = lib().qwen_tts_resample(w.ctypes.data_as(_fp), w.shape[0], int(sr_in), int(sr_out), C.byref(n))
    if not p:
        return None
    out = np.ctypeslib.as_array(C.cast(p, _fp), shape=(n.value,)).copy()
    _libc.free(C.c_void_p(p))
    return out


def lib():
    """Load the in-tree library (raises if it was not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # torch bundles its own HIP runtime with the same soname (libamdhip64.so.7)
    # as /opt/rocm's.  Loading torch first makes this library bind to that one
    # runtime, so torch tensors, streams and our launches share it; loading
    # ours first would put two HIP runtimes in the process and break torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C qwen3-tts-c_amd` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.qwen_tts_load.restype = C.POINTER(Ctx)
    L.qwen_tts_load.argtypes = [C.c_char_p]
    L.qwen_tts_free.argtypes = [C.POINTER(Ctx)]
    L.qwen_tts_generate.restype = C.c_void_p
    L.qwen_tts_generate.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, C.c_char_p, _ip]
    L.qwen_tts_generate_batch.restype = C.c_int
    L.qwen_tts_generate_batch.argtypes = [C.POINTER(Ctx), C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                          C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), _ip]
    L.qwen_tts_last_codes.restype = C.c_int
    L.qwen_tts_last_codes.argtypes = [C.POINTER(Ctx), _ip, C.c_int]
    L.qwen_tts_last_codes_slot.restype = C.c_int
    L.qwen_tts_last_codes_slot.argtypes = [C.POINTER(Ctx), C.c_int, _ip, C.c_int]
    L.qwen_tts_generate_queue.restype = C.c_int
    L.qwen_tts_generate_queue.argtypes = [C.POINTER(Ctx), C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                          C.POINTER(C.c_char_p), C.c_int, QUEUE_NEXT_CB, C.c_void_p,
                                          C.POINTER(C.c_void_p), _ip]
    L.qwen_tts_queue_codes.restype = C.c_int
    L.qwen_tts_queue_codes.argtypes = [C.POINTER(Ctx), C.c_int, _ip, C.c_int]
    L.qwen_tts_talker_prefill.argtypes = [C.POINTER(Ctx), _fp, C.c_int]
    L.qwen_tts_talker_forward.argtypes = [C.POINTER(Ctx), _fp, _fp]
    L.qwen_tts_subtalker_generate.argtypes = [C.POINTER(Ctx), _fp, C.c_int, _ip]
    L.qwen_tts_codec_decode.restype = C.c_void_p
    L.qwen_tts_codec_decode.argtypes = [C.POINTER(Ctx), _ip, C.c_int, _ip]
    L.qwen_tts_talker_hidden.argtypes = [C.POINTER(Ctx), _fp]
    L.qwen_tts_load_on.restype = C.POINTER(Ctx)
    L.qwen_tts_load_on.argtypes = [C.c_char_p, C.c_int]
    L.qwen_tts_set_progress_callback.argtypes = [C.POINTER(Ctx), PROGRESS_CB, C.c_void_p]
    L.qwen_tts_write_wav.argtypes = [C.c_char_p, _fp, C.c_int, C.c_int]
    L.qwen_tts_abi_sizeof_ctx.restype = C.c_size_t
    L.qwen_tts_resample.restype = C.c_void_p
    L.qwen_tts_resample.argtypes = [_fp, C.c_int, C.c_int, C.c_int, _ip]
    L.qwen_tts_tokenize.restype = C.c_void_p
    L.qwen_tts_tokenize.argtypes = [C.c_char_p, C.c_char_p, _ip]
    L.qwen_tts_text_prompt.restype = C.c_void_p
    L.qwen_tts_text_prompt.argtypes = [C.POINTER(Ctx), C.c_char_p]
    L.qwen_tts_generate_stream.restype = C.c_void_p
    L.qwen_tts_generate_stream.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, AUDIO_CB,
                                           C.c_void_p, _ip]
    L.qwen_tts_generate_voice_clone_stream.restype = C.c_void_p
    L.qwen_tts_generate_voice_clone_stream.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, _ip, C.c_int, _fp,
                                                       C.c_char_p, C.c_int, C.c_int, AUDIO_CB, C.c_void_p, _ip]
    L.qwen_tts_generate_voice_clone.restype = C.c_void_p
    L.qwen_tts_generate_voice_clone.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, _ip, C.c_int, _fp,
                                                C.c_char_p, C.c_int, _ip]
    L.qwen_tts_generate_voice_clone_batch.restype = C.c_int
    L.qwen_tts_generate_voice_clone_batch.argtypes = [C.POINTER(Ctx), C.c_int, C.POINTER(C.c_char_p),
                                                      C.POINTER(C.c_char_p), C.POINTER(_ip), _ip, C.POINTER(_fp),
                                                      C.POINTER(C.c_char_p), C.c_int, C.POINTER(C.c_void_p), _ip]
    L.qwen_tts_codec_stream_begin.argtypes = [C.POINTER(Ctx), C.c_int]
    L.qwen_tts_codec_stream_push.argtypes = [C.POINTER(Ctx), _ip, C.c_int, _fp]
    L.qwen_tts_speaker_embedding.restype = C.c_void_p
    L.qwen_tts_speaker_embedding.argtypes = [C.POINTER(Ctx), _fp, C.c_int, _ip]
    L.qwen_tts_encode_audio.restype = C.c_void_p
    L.qwen_tts_encode_audio.argtypes = [C.POINTER(Ctx), _fp, C.c_int, _ip]
    L.qwen_tts_generate_voice_clone_audio.restype = C.c_void_p
    L.qwen_tts_generate_voice_clone_audio.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, _fp, C.c_int,
                                                      C.c_char_p, C.c_int, C.c_int, _ip]
    L.qwen_tts_generate_voice_clone_audio_batch.restype = C.c_int
    L.qwen_tts_generate_voice_clone_audio_batch.argtypes = [C.POINTER(Ctx), C.c_int, C.POINTER(C.c_char_p),
                                                            C.POINTER(C.c_char_p), C.POINTER(_fp), _ip,
                                                            C.POINTER(C.c_char_p), _ip, C.c_int,
                                                            C.POINTER(C.c_void_p), _ip]
    L.qwen_tts_generate_voice_clone_audio_stream.restype = C.c_void_p
    L.qwen_tts_generate_voice_clone_audio_stream.argtypes = [C.POINTER(Ctx), C.c_char_p, C.c_char_p, _fp, C.c_int,
                                                             C.c_char_p, C.c_int, C.c_int, C.c_int, AUDIO_CB,
                                                             C.c_void_p, _ip]
    L.qtts_dev_enc_available.restype = C.c_int
    L.qtts_dev_enc_available.argtypes = [C.c_void_p]
    L.qtts_dev_speaker_embed.restype = C.c_int
    L.qtts_dev_speaker_embed.argtypes = [C.c_void_p, C.c_int, C.POINTER(_fp), _ip, _fp, _fp]
    L.qtts_dev_encode_audio.restype = C.c_int
    L.qtts_dev_encode_audio.argtypes = [C.c_void_p, C.c_int, C.POINTER(_fp), _ip, _ip, C.c_int, _ip, _fp]
    L.qtts_hip_device_count.restype = C.c_int
    L.qtts_hip_tengine_layers.restype = C.c_longlong
    vp = C.c_void_p
    L.qtts_hip_matvec_bf16.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_rmsnorm_matvec_bf16.argtypes = [vp, vp, vp, vp, C.c_float, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_decode_matvec_bf16.argtypes = [vp, vp, vp, vp, C.c_float, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_resident_matvec_bf16.argtypes = [vp, vp, vp, vp, C.c_float, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_sample_top_k.argtypes = [vp, vp, C.c_int, C.c_int, C.c_float, C.c_float, vp, C.c_int, vp]
    L.qtts_hip_causal_conv1d.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_transposed_conv1d.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    L.qtts_hip_snake_beta.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, vp]
    L.qtts_hip_expf_glibc.argtypes = [vp, vp, C.c_int, vp]
    _LIB = L
    return L


_libc = C.CDLL("libc.so.6")
_libc.free.argtypes = [C.c_void_p]


def _take_audio(ptr, n):
    if not ptr or n <= 0:
        return None
    a = np.ctypeslib.as_array(C.cast(ptr, _fp), shape=(n,)).copy()
    _libc.free(ptr)
    return a


def set_verbose(v):
    C.c_int.in_dll(lib(), "qwen_tts_verbose").value = int(v)


class QwenTTS:
    """One model on one HIP device (the reference's qwen_tts_ctx_t)."""

    def __init__(self, model_dir, device=0):
        L = lib()
        self.ctx = L.qwen_tts_load_on(model_dir.encode(), int(device))
        if not self.ctx:
            raise RuntimeError(f"qwen_tts_load({model_dir}) failed")
        self.c = self.ctx.contents
        self.cfg = self.c.config
        self._last_nb = 1

    def close(self):
        if self.ctx:
            lib().qwen_tts_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, max_tokens=4096, fixed=0, seed=42, temperature=0.9, top_k=50, top_p=1.0, rep=1.05,
                   st_temperature=0.9, st_top_k=50, st_top_p=1.0):
        c = self.c
        c.temperature, c.top_k, c.top_p, c.repetition_penalty = temperature, top_k, top_p, rep
        c.subtalker_temperature, c.subtalker_top_k, c.subtalker_top_p = st_temperature, st_top_k, st_top_p
        c.max_new_tokens, c.fixed_codec_tokens, c.sample_seed = max_tokens, fixed, seed

    def generate(self, ids, speaker=None, language=None):
        csv = ",".join(str(int(i)) for i in ids).encode()
        n = C.c_int(0)
        p = lib().qwen_tts_generate(self.ctx, csv, speaker.encode() if speaker else None,
                                    language.encode() if language else None, C.byref(n))
        return _take_audio(p, n.value)

    def generate_voice_clone(self, ids, ref_ids=None, ref_codes=None, spk_embed=None, language=None,
                             non_streaming=False):
        """Voice clone from reference codes [T, 16] (+ the reference text ids)
        and / or a speaker x-vector (include/qwen_tts.h
        qwen_tts_generate_voice_clone; the Python reference's
        generate_voice_clone minus its audio encoders)."""
        csv = ",".join(str(int(i)) for i in ids).encode()
        rcsv = ",".join(str(int(i)) for i in ref_ids).encode() if ref_ids is not None else None
        rc = None if ref_codes is None else np.ascontiguousarray(ref_codes, np.int32)
        sv = None if spk_embed is None else np.ascontiguousarray(spk_embed, np.float32)
        n = C.c_int(0)
        p = lib().qwen_tts_generate_voice_clone(
            self.ctx, csv, rcsv, None if rc is None else rc.ctypes.data_as(_ip), 0 if rc is None else rc.shape[0],
            None if sv is None else sv.ctypes.data_as(_fp), language.encode() if language else None,
            int(non_streaming), C.byref(n))
        return _take_audio(p, n.value)

    def generate_voice_clone_batch(self, id_lists, ref_id_lists, ref_codes, spk_embeds=None, languages=None,
                                   non_streaming=False):
        """nb voice-clone utterances in lock step (BASELINE C5).  Returns (rc, [audio])."""
        nb = len(id_lists)
        enc = lambda ids: ",".join(str(int(i)) for i in ids).encode() if ids is not None else None
        tx = (C.c_char_p * nb)(*[enc(i) for i in id_lists])
        rt = (C.c_char_p * nb)(*[enc(i) for i in (ref_id_lists or [None] * nb)])
        keep = [None if c is None else np.ascontiguousarray(c, np.int32) for c in (ref_codes or [None] * nb)]
        rc = (_ip * nb)(*[None if c is None else c.ctypes.data_as(_ip) for c in keep])
        nr = (C.c_int * nb)(*[0 if c is None else c.shape[0] for c in keep])
        sk = [None if v is None else np.ascontiguousarray(v, np.float32) for v in (spk_embeds or [None] * nb)]
        sv = (_fp * nb)(*[None if v is None else v.ctypes.data_as(_fp) for v in sk])
        lg = (C.c_char_p * nb)(*[(s.encode() if s else None) for s in (languages or [None] * nb)])
        out = (C.c_void_p * nb)()
        ns = (C.c_int * nb)()
        r = lib().qwen_tts_generate_voice_clone_batch(self.ctx, nb, tx, rt, rc, nr, sv, lg, int(non_streaming), out,
                                                      ns)
        return r, [_take_audio(out[i], ns[i]) for i in range(nb)]

    # ---- voice-clone audio encoders (include/qtts_hip.h qtts_dev_speaker_embed / _encode_audio)
    def encoders_available(self):
        """bit 0: speaker encoder, bit 1: 12 Hz encoder."""
        return lib().qtts_dev_enc_available(C.c_void_p(self.c.hip))

    @staticmethod
    def _wav_args(wavs):
        ws = [np.ascontiguousarray(w, np.float32) for w in wavs]
        nb = len(ws)
        return ws, (_fp * nb)(*[w.ctypes.data_as(_fp) for w in ws]), (C.c_int * nb)(*[w.shape[0] for w in ws])

    def speaker_embed(self, wavs, mel=False):
        """x-vectors [nb, talker_hidden] of 24 kHz waveforms (one launch chain
        for the batch, each utterance at its own length); with mel=True also
        the list of [128, T_b] log-mels."""
        ws, wp, ns = self._wav_args(wavs)
        nb = len(ws)
        out = np.zeros((nb, self.cfg.talker_hidden), np.float32)
        T = [(w.shape[0] - 256) // 256 + 1 for w in ws]
        mbuf = np.zeros(sum(128 * t for t in T), np.float32) if mel else None
        rc = lib().qtts_dev_speaker_embed(C.c_void_p(self.c.hip), nb, wp, ns, out.ctypes.data_as(_fp),
                                          mbuf.ctypes.data_as(_fp) if mel else None)
        if rc != 0:
            raise RuntimeError(f"speaker encoder failed (rc={rc})")
        if not mel:
            return out
        mels, o = [], 0
        for t in T:
            mels.append(mbuf[o:o + 128 * t].reshape(128, t).copy())
            o += 128 * t
        return out, mels

    def encode_audio(self, wavs, latent=False):
        """12 Hz codes of 24 kHz waveforms, batch-encoded zero-padded to the
        longest: list of [ceil(n / 1920), 16] int arrays (+ pre-quantizer
        latents [hidden, frames] with latent=True)."""
        ws, wp, ns = self._wav_args(wavs)
        nb = len(ws)
        maxT = max(-(-w.shape[0] // 1920) for w in ws)
        codes = np.zeros((nb, maxT, 16), np.int32)
        frames = (C.c_int * nb)()
        hid = None
        lat = None
        if latent:
            import json
            with open(os.path.join(self.c.model_dir.decode(), "speech_tokenizer", "config.json")) as f:
                hid = json.load(f).get("encoder_config", {}).get("hidden_size", 512)
            lat = np.zeros((nb, hid, maxT), np.float32)
        rc = lib().qtts_dev_encode_audio(C.c_void_p(self.c.hip), nb, wp, ns, codes.ctypes.data_as(_ip), maxT, frames,
                                         lat.ctypes.data_as(_fp) if latent else None)
        if rc != 0:
            raise RuntimeError(f"audio encoder failed (rc={rc})")
        cl = [codes[b, :frames[b]].copy() for b in range(nb)]
        if not latent:
            return cl
        return cl, [lat[b, :, :frames[b]].copy() for b in range(nb)]

    def speaker_embedding_api(self, wav):
        """qwen_tts_speaker_embedding (the public C API)."""
        w = np.ascontiguousarray(wav, np.float32)
        n = C.c_int(0)
        p = lib().qwen_tts_speaker_embedding(self.ctx, w.ctypes.data_as(_fp), w.shape[0], C.byref(n))
        return _take_audio(p, n.value)

    def encode_audio_api(self, wav):
        """qwen_tts_encode_audio (the public C API): [frames, 16] or None."""
        w = np.ascontiguousarray(wav, np.float32)
        n = C.c_int(0)
        p = lib().qwen_tts_encode_audio(self.ctx, w.ctypes.data_as(_fp), w.shape[0], C.byref(n))
        if not p:
            return None
        a = np.ctypeslib.as_array(C.cast(p, _ip), shape=(n.value * 16,)).reshape(n.value, 16).copy()
        _libc.free(C.c_void_p(p))
        return a

    def generate_voice_clone_audio(self, ids, ref_wav, ref_ids=None, language=None, x_vector_only=False,
                                   non_streaming=False):
        """Voice clone from reference audio (qwen_tts_generate_voice_clone_audio)."""
        csv = ",".join(str(int(i)) for i in ids).encode()
        rcsv = ",".join(str(int(i)) for i in ref_ids).encode() if ref_ids is not None else None
        w = np.ascontiguousarray(ref_wav, np.float32)
        n = C.c_int(0)
        p = lib().qwen_tts_generate_voice_clone_audio(self.ctx, csv, rcsv, w.ctypes.data_as(_fp), w.shape[0],
                                                      language.encode() if language else None, int(x_vector_only),
                                                      int(non_streaming), C.byref(n))
        return _take_audio(p, n.value)

    def generate_voice_clone_audio_stream(self, ids, ref_wav, ref_ids=None, language=None, x_vector_only=False,
                                          non_streaming=False, chunk_frames=4, on_chunk=None):
        """Streaming voice clone from reference audio; first packet counts the encode."""
        csv = ",".join(str(int(i)) for i in ids).encode()
        rcsv = ",".join(str(int(i)) for i in ref_ids).encode() if ref_ids is not None else None
        w = np.ascontiguousarray(ref_wav, np.float32)
        n = C.c_int(0)

        def _cb(p, k, u):
            if on_chunk is not None:
                on_chunk(np.ctypeslib.as_array(p, shape=(k,)).copy())
        cb = AUDIO_CB(_cb)
        p = lib().qwen_tts_generate_voice_clone_audio_stream(
            self.ctx, csv, rcsv, w.ctypes.data_as(_fp), w.shape[0], language.encode() if language else None,
            int(x_vector_only), int(non_streaming), int(chunk_frames), cb, None, C.byref(n))
        return _take_audio(p, n.value)

    def generate_voice_clone_audio_batch(self, id_lists, ref_wavs, ref_id_lists=None, languages=None,
                                         x_vector_only=None, non_streaming=False):
        """nb voice clones from reference audio in lock step (BASELINE C5 as
        stated: ref-audio encode + decode + codec).  Returns (rc, [audio])."""
        nb = len(id_lists)
        enc = lambda ids: ",".join(str(int(i)) for i in ids).encode() if ids is not None else None
        tx = (C.c_char_p * nb)(*[enc(i) for i in id_lists])
        rt = (C.c_char_p * nb)(*[enc(i) for i in (ref_id_lists or [None] * nb)])
        ws, wp, ns = self._wav_args(ref_wavs)
        lg = (C.c_char_p * nb)(*[(s.encode() if s else None) for s in (languages or [None] * nb)])
        xo = (C.c_int * nb)(*[int(bool(v)) for v in (x_vector_only or [False] * nb)])
        out = (C.c_void_p * nb)()
        on = (C.c_int * nb)()
        r = lib().qwen_tts_generate_voice_clone_audio_batch(self.ctx, nb, tx, rt, wp, ns, lg, xo, int(non_streaming),
                                                            out, on)
        return r, [_take_audio(out[i], on[i]) for i in range(nb)]

    def generate_batch(self, id_lists, speakers=None, languages=None):
        nb = len(id_lists)
        tx = (C.c_char_p * nb)(*[",".join(str(int(i)) for i in ids).encode() for ids in id_lists])
        sp = (C.c_char_p * nb)(*[(s.encode() if s else None) for s in (speakers or [None] * nb)])
        lg = (C.c_char_p * nb)(*[(s.encode() if s else None) for s in (languages or [None] * nb)])
        out = (C.c_void_p * nb)()
        ns = (C.c_int * nb)()
        rc = lib().qwen_tts_generate_batch(self.ctx, nb, tx, sp, lg, out, ns)
        self._last_nb = nb
        audio = [_take_audio(out[i], ns[i]) for i in range(nb)]
        return rc, audio

    def generate_queue(self, id_lists, speakers=None, languages=None, slots=8, next_fn=None):
        """Work queue (qwen_tts_generate_queue): the utterances on at most
        `slots` lock-step slots, each freed slot refilled with the next
        utterance inside the live batch.  next_fn() (optional) returns the index
        of the next utterance to admit or -1 (e.g. a counter shared by several
        GPUs' processes); default: in order.  Returns (rc, [audio or None])."""
        nq = len(id_lists)
        tx = (C.c_char_p * nq)(*[",".join(str(int(i)) for i in ids).encode() for ids in id_lists])
        sp = (C.c_char_p * nq)(*[(s.encode() if s else None) for s in (speakers or [None] * nq)])
        lg = (C.c_char_p * nq)(*[(s.encode() if s else None) for s in (languages or [None] * nq)])
        out = (C.c_void_p * nq)()
        ns = (C.c_int * nq)()
        cb = QUEUE_NEXT_CB(lambda u: int(next_fn())) if next_fn is not None else QUEUE_NEXT_CB()
        rc = lib().qwen_tts_generate_queue(self.ctx, nq, tx, sp, lg, int(slots), cb, None, out, ns)
        return rc, [_take_audio(out[i], ns[i]) for i in range(nq)]

    def queue_codes(self, i):
        """codes [frames, groups] of utterance i of the last generate_queue (None: not decoded here)"""
        n = lib().qwen_tts_queue_codes(self.ctx, int(i), None, 1 << 30)
        if n < 0:
            return None
        buf = np.zeros((max(n, 1), self.cfg.num_code_groups), np.int32)
        lib().qwen_tts_queue_codes(self.ctx, int(i), buf.ctypes.data_as(_ip), n)
        return buf[:n].copy()

    def queue_stats(self):
        """{slots, frames, refills, used, occupancy, stop_reason[], frames_per_utt[]} of the last generate_queue"""
        c = self.c
        n = c.queue_n
        launched = c.queue_frames_launched
        rl = int(c.queue_rows_launched)
        return {"slots": c.queue_slots, "frames": launched, "refills": c.queue_refills,
                "used": int(c.queue_slot_frames_used), "rows_launched": rl,
                "occupancy": (c.queue_slot_frames_used / rl) if rl else 0.0,
                "occupancy_full_width": (c.queue_slot_frames_used / (c.queue_slots * launched))
                if launched and c.queue_slots else 0.0,
                "stop_reason": [c.queue_stop_reason[i] for i in range(n)] if n else [],
                "frames_per_utt": [c.queue_frames[i] for i in range(n)] if n else [],
                "slot": [c.queue_slot[i] for i in range(n)] if n else []}

    def generate_stream(self, ids, speaker=None, language=None, chunk_frames=4, on_chunk=None):
        """Streaming generation; on_chunk(np.ndarray) gets each audio chunk as
        it is decoded.  Returns the whole utterance."""
        csv = ",".join(str(int(i)) for i in ids).encode()
        n = C.c_int(0)

        def _cb(p, k, u):
            if on_chunk is not None:
                on_chunk(np.ctypeslib.as_array(p, shape=(k,)).copy())
        cb = AUDIO_CB(_cb)
        p = lib().qwen_tts_generate_stream(self.ctx, csv, speaker.encode() if speaker else None,
                                           language.encode() if language else None, int(chunk_frames), cb, None,
                                           C.byref(n))
        return _take_audio(p, n.value)

    def generate_voice_clone_stream(self, ids, ref_ids=None, ref_codes=None, spk_embed=None, language=None,
                                    non_streaming=False, chunk_frames=4, on_chunk=None):
        """Streaming voice clone; chunks start at the reference boundary."""
        csv = ",".join(str(int(i)) for i in ids).encode()
        rcsv = ",".join(str(int(i)) for i in ref_ids).encode() if ref_ids is not None else None
        rc = None if ref_codes is None else np.ascontiguousarray(ref_codes, np.int32)
        sv = None if spk_embed is None else np.ascontiguousarray(spk_embed, np.float32)
        n = C.c_int(0)

        def _cb(p, k, u):
            if on_chunk is not None:
                on_chunk(np.ctypeslib.as_array(p, shape=(k,)).copy())
        cb = AUDIO_CB(_cb)
        p = lib().qwen_tts_generate_voice_clone_stream(
            self.ctx, csv, rcsv, None if rc is None else rc.ctypes.data_as(_ip), 0 if rc is None else rc.shape[0],
            None if sv is None else sv.ctypes.data_as(_fp), language.encode() if language else None,
            int(non_streaming), int(chunk_frames), cb, None, C.byref(n))
        return _take_audio(p, n.value)

    def codec_stream(self, chunks, max_frames=4096):
        """Exact incremental codec decode of a list of [t, 16] code arrays."""
        L = lib()
        if L.qwen_tts_codec_stream_begin(self.ctx, int(max_frames)) != 0:
            raise RuntimeError("codec stream begin failed")
        outs = []
        for c in chunks:
            c = np.ascontiguousarray(c, np.int32)
            o = np.zeros(c.shape[0] * 1920, np.float32)
            k = L.qwen_tts_codec_stream_push(self.ctx, c.ctypes.data_as(_ip), c.shape[0], o.ctypes.data_as(_fp))
            if k != len(o):
                raise RuntimeError(f"codec stream push failed ({k})")
            outs.append(o)
        return outs

    def last_codes(self):
        G = self.cfg.num_code_groups
        n = self.c.last_frames
        buf = np.zeros((max(n, 1), G), np.int32)
        k = lib().qwen_tts_last_codes(self.ctx, buf.ctypes.data_as(_ip), n)
        return buf[:k].copy()

    def last_codes_slot(self, slot, max_frames=4096):
        """codes of batch slot `slot` of the last generate_batch (frames x groups)"""
        buf = np.zeros((max_frames, self.cfg.num_code_groups), np.int32)
        k = lib().qwen_tts_last_codes_slot(self.ctx, int(slot), buf.ctypes.data_as(_ip), max_frames)
        if k < 0:
            raise ValueError(f"no batch slot {slot}")
        return buf[:k].copy()

    def last_codes_batch(self, nb=None, max_frames=4096):
        return [self.last_codes_slot(b, max_frames) for b in range(nb if nb is not None else self._last_nb)]

    # stage functions (host pointers)
    def prefill(self, embeds):
        e = np.ascontiguousarray(embeds, np.float32)
        lib().qwen_tts_talker_prefill(self.ctx, e.ctypes.data_as(_fp), e.shape[0])
        return self.hidden()

    def hidden(self):
        h = np.zeros(self.cfg.talker_hidden, np.float32)
        lib().qwen_tts_talker_hidden(self.ctx, h.ctypes.data_as(_fp))
        return h

    def step(self, embed):
        e = np.ascontiguousarray(embed, np.float32)
        lg = np.zeros(self.cfg.talker_vocab_size, np.float32)
        lib().qwen_tts_talker_forward(self.ctx, e.ctypes.data_as(_fp), lg.ctypes.data_as(_fp))
        return lg, self.hidden()

    def subtalker(self, hidden, code0):
        out = np.zeros(self.cfg.num_code_groups, np.int32)
        h = np.ascontiguousarray(hidden, np.float32)
        lib().qwen_tts_subtalker_generate(self.ctx, h.ctypes.data_as(_fp), int(code0), out.ctypes.data_as(_ip))
        return out

    def codec_decode(self, codes):
        c = np.ascontiguousarray(codes, np.int32)
        n = C.c_int(0)
        p = lib().qwen_tts_codec_decode(self.ctx, c.ctypes.data_as(_ip), c.shape[0], C.byref(n))
        return _take_audio(p, n.value)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    import torch
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


class Kernels:
    """Kernel-level entry points of qtts_hip.h on torch device tensors."""

    @staticmethod
    def matvec_bf16(out, A_u16, x, rows, cols, batch=1):
        _ok(lib().qtts_hip_matvec_bf16(_ptr(out), _ptr(A_u16), _ptr(x), rows, cols, batch, _stream()), "matvec")

    @staticmethod
    def rmsnorm_matvec_bf16(out, A_u16, x, w, eps, rows, cols, batch=1):
        _ok(lib().qtts_hip_rmsnorm_matvec_bf16(_ptr(out), _ptr(A_u16), _ptr(x), _ptr(w), eps, rows, cols, batch,
                                               _stream()), "rmsnorm_matvec")

    @staticmethod
    def decode_matvec_bf16(out, A_u16, x, w, eps, rows, cols, batch=1):
        _ok(lib().qtts_hip_decode_matvec_bf16(_ptr(out), _ptr(A_u16), _ptr(x), _ptr(w) if w is not None else None,
                                              eps, rows, cols, batch, _stream()), "decode_matvec")

    @staticmethod
    def resident_matvec_bf16(out, A_u16, x, w, eps, rows, cols, epi=0):
        _ok(lib().qtts_hip_resident_matvec_bf16(_ptr(out), _ptr(A_u16), _ptr(x), _ptr(w) if w is not None else None,
                                                eps, rows, cols, epi, _stream()), "resident_matvec")

    @staticmethod
    def sample_top_k(out_i32, logits, vocab, top_k, top_p, temperature, rng_u32, batch=1):
        _ok(lib().qtts_hip_sample_top_k(_ptr(out_i32), _ptr(logits), vocab, top_k, top_p, temperature,
                                        _ptr(rng_u32), batch, _stream()), "sample")

    @staticmethod
    def causal_conv1d(out, x, w, b, ci, co, k, L, dil=1, groups=1):
        _ok(lib().qtts_hip_causal_conv1d(_ptr(out), _ptr(x), _ptr(w), _ptr(b), ci, co, k, L, dil, groups,
                                         _stream()), "conv1d")

    @staticmethod
    def transposed_conv1d(out, x, w, b, ci, co, k, stride, L):
        _ok(lib().qtts_hip_transposed_conv1d(_ptr(out), _ptr(x), _ptr(w), _ptr(b), ci, co, k, stride, L,
                                             _stream()), "tconv1d")

    @staticmethod
    def snake_beta(out, x, alpha, inv_beta, C_, L):
        _ok(lib().qtts_hip_snake_beta(_ptr(out), _ptr(x), _ptr(alpha), _ptr(inv_beta), C_, L, _stream()), "snake")

    @staticmethod
    def expf_glibc(out, x, n):
        _ok(lib().qtts_hip_expf_glibc(_ptr(out), _ptr(x), n, _stream()), "expf")
