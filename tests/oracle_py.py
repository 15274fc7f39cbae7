"""ctypes bindings for the two CPU checkers (TEST INFRASTRUCTURE ONLY).

* `Oracle`    -> oracle/_port/liboracle.so   (CPU restatement, oracle/qtts_oracle.c)
* `RefLib`    -> oracle/_ref/libqtts_ref.so  (the reference c/ sources compiled
                 unmodified + oracle/ref_driver.c hooks; present only where it
                 was built, it travels to the GPU box as a prebuilt .so)

Neither is ever used by the product path.
"""
import ctypes as C
import os

import numpy as np

from qtts_io import load_config, read_model_tensors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_port", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libqtts_ref.so")

_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int)


def fptr(a):
    return a.ctypes.data_as(_fp)


def iptr(a):
    return a.ctypes.data_as(_ip)


class OrcParams(C.Structure):
    _fields_ = [("temperature", C.c_float), ("top_p", C.c_float), ("rep", C.c_float),
                ("st_temperature", C.c_float), ("st_top_p", C.c_float),
                ("top_k", C.c_int), ("max_tokens", C.c_int), ("fixed", C.c_int),
                ("seed", C.c_int), ("st_top_k", C.c_int)]


GREEDY = dict(temperature=1.0, top_k=1, top_p=1.0, rep=1.0, st_temperature=1.0, st_top_k=1, st_top_p=1.0)
DEFAULT = dict(temperature=0.9, top_k=50, top_p=1.0, rep=1.05, st_temperature=0.9, st_top_k=50, st_top_p=1.0)


def make_params(max_tokens=4096, fixed=0, seed=42, **kw):
    p = dict(DEFAULT)
    p.update(kw)
    return OrcParams(p["temperature"], p["top_p"], p["rep"], p["st_temperature"], p["st_top_p"],
                     p["top_k"], max_tokens, fixed, seed, p["st_top_k"])


def _lib_oracle():
    lib = C.CDLL(ORACLE_SO)
    lib.orc_create.restype = C.c_void_p
    lib.orc_create.argtypes = [_ip, _fp]
    lib.orc_set_tensor.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int, C.c_long]
    lib.orc_free.argtypes = [C.c_void_p]
    lib.orc_matvec_bf16.argtypes = [_fp, C.c_void_p, _fp, C.c_int, C.c_int]
    lib.orc_rmsnorm.argtypes = [_fp, _fp, _fp, C.c_int, C.c_float]
    lib.orc_softmax.argtypes = [_fp, C.c_int]
    lib.orc_sample.restype = C.c_int
    lib.orc_sample.argtypes = [_fp, C.c_int, C.c_int, C.c_float, C.c_float, _fp]
    lib.orc_rand_uniform.restype = C.c_float
    lib.orc_rand_uniform.argtypes = [_fp]
    lib.orc_rep_penalty.argtypes = [_fp, _ip, C.c_int, C.c_int, C.c_float]
    lib.orc_rope_table.argtypes = [_fp, _fp, C.c_int, C.c_int, C.c_float]
    lib.orc_conv1d.argtypes = [_fp, _fp, _fp, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.orc_tconv1d.argtypes = [_fp, _fp, _fp, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.orc_snake.argtypes = [_fp, _fp, _fp, _fp, C.c_int, C.c_int]
    lib.orc_talker_prefill.argtypes = [C.c_void_p, _fp, C.c_int, _fp]
    lib.orc_talker_step.argtypes = [C.c_void_p, _fp, _fp, _fp]
    lib.orc_talker_head.argtypes = [C.c_void_p, _fp, _fp]
    lib.orc_kv_len.restype = C.c_int
    lib.orc_kv_len.argtypes = [C.c_void_p]
    lib.orc_subtalker.argtypes = [C.c_void_p, _fp, C.c_int, C.c_int, C.c_float, C.c_float, C.c_int, _ip]
    lib.orc_codec_decode.restype = C.c_void_p
    lib.orc_codec_decode.argtypes = [C.c_void_p, _ip, C.c_int, _ip]
    lib.orc_embed_text.argtypes = [C.c_void_p, C.c_int, _fp]
    lib.orc_build_prompt.restype = C.c_int
    lib.orc_build_prompt.argtypes = [C.c_void_p, _ip, C.c_int, C.c_int, C.c_int, _fp, _fp, _ip]
    lib.orc_generate_codes.restype = C.c_int
    lib.orc_generate_codes.argtypes = [C.c_void_p, _ip, C.c_int, C.c_int, C.c_int, C.POINTER(OrcParams),
                                       _ip, C.c_int, _ip]
    lib.orc_build_icl_prompt.restype = C.c_int
    lib.orc_build_icl_prompt.argtypes = [C.c_void_p, _ip, C.c_int, _ip, C.c_int, _ip, C.c_int, _fp, C.c_int,
                                         C.c_int, _fp, _fp, _ip]
    lib.orc_trace_arm.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.orc_trace_dims.restype = C.c_int
    lib.orc_trace_dims.argtypes = [C.c_void_p, _ip, _ip]
    lib.orc_trace_get.restype = C.c_int
    lib.orc_trace_get.argtypes = [C.c_void_p, _fp, _fp, _fp, _ip]
    lib.orc_generate_from_prompt.restype = C.c_int
    lib.orc_generate_from_prompt.argtypes = [C.c_void_p, _fp, C.c_int, _fp, C.c_int, C.POINTER(OrcParams),
                                             _ip, C.c_int, _ip]
    return lib


_LIBC = C.CDLL("libc.so.6")
_LIBC.free.argtypes = [C.c_void_p]


class Oracle:
    """CPU restatement bound to one synthetic model dir."""

    def __init__(self, model_dir):
        self.lib = _lib_oracle()
        self.cfg = c = load_config(model_dir)
        self.tensors = read_model_tensors(model_dir)   # keep memmaps alive
        dims = [c["H"], c["I"], c["L"], c["NH"], c["KV"], c["HD"], c["TH"], c["TV"], c["V"], c["G"],
                c["Hs"], c["Is"], c["Ls"], c["NHs"], c["KVs"], c["HDs"], c["Vs"],
                c["mrope"][0], c["mrope"][1], c["mrope"][2],
                c["cq"], c["ccb"], c["ccbdim"], c["chid"], c["clat"], c["clayers"], c["cheads"], c["ckv"],
                c["cinter"], c["cwin"], c["cdec"], *c["rates"], *c["ratios"],
                c["pad"], c["bos"], c["eos"], c["think"], c["nothink"], c["think_bos"], c["think_eos"]]
        self._dims = np.array(dims, dtype=np.int32)
        self._fp = np.array([c["eps"], c["theta"], c["ceps"]], dtype=np.float32)
        self.h = self.lib.orc_create(iptr(self._dims), fptr(self._fp))
        self._keep = []
        for name, (dt, arr) in self.tensors.items():
            a = np.ascontiguousarray(arr)
            self._keep.append(a)
            self.lib.orc_set_tensor(self.h, name.encode(), a.ctypes.data, 1 if dt == "BF16" else 0, a.size)

    def close(self):
        if self.h:
            self.lib.orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # stages
    def prefill(self, embeds):
        e = np.ascontiguousarray(embeds, dtype=np.float32)
        hid = np.zeros(self.cfg["H"], np.float32)
        self.lib.orc_talker_prefill(self.h, fptr(e), e.shape[0], fptr(hid))
        return hid

    def step(self, embed):
        e = np.ascontiguousarray(embed, dtype=np.float32)
        lg = np.zeros(self.cfg["V"], np.float32)
        hid = np.zeros(self.cfg["H"], np.float32)
        self.lib.orc_talker_step(self.h, fptr(e), fptr(lg), fptr(hid))
        return lg, hid

    def head(self, hidden):
        lg = np.zeros(self.cfg["V"], np.float32)
        self.lib.orc_talker_head(self.h, fptr(np.ascontiguousarray(hidden, np.float32)), fptr(lg))
        return lg

    def subtalker(self, hidden, code0, top_k=50, top_p=1.0, temp=0.9, seed=42):
        out = np.zeros(self.cfg["G"], np.int32)
        self.lib.orc_subtalker(self.h, fptr(np.ascontiguousarray(hidden, np.float32)), int(code0),
                               top_k, top_p, temp, seed, iptr(out))
        return out

    def codec_decode(self, codes):
        c = np.ascontiguousarray(codes, dtype=np.int32)
        n = C.c_int(0)
        p = self.lib.orc_codec_decode(self.h, iptr(c), c.shape[0], C.byref(n))
        out = np.ctypeslib.as_array(C.cast(p, _fp), shape=(n.value,)).copy()
        _LIBC.free(p)
        return out

    def embed_text(self, tid):
        o = np.zeros(self.cfg["H"], np.float32)
        self.lib.orc_embed_text(self.h, int(tid), fptr(o))
        return o

    def build_prompt(self, ids, spk=-1, lang=-1):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        H = self.cfg["H"]
        pre = np.zeros((16, H), np.float32)
        tr = np.zeros((max(len(ids), 2), H), np.float32)
        ntr = C.c_int(0)
        P = self.lib.orc_build_prompt(self.h, iptr(ids), len(ids), spk, lang, fptr(pre), fptr(tr), C.byref(ntr))
        return pre[:P].copy(), tr[:ntr.value].copy()

    def build_icl_prompt(self, ids, ref_ids=None, ref_codes=None, spk_vec=None, lang=-1, non_streaming=False):
        """Voice-clone prompt (oracle/qtts_oracle.c orc_build_icl_prompt; parity unpinned)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        rid = np.ascontiguousarray(ref_ids if ref_ids is not None else [], dtype=np.int32)
        rc = None if ref_codes is None else np.ascontiguousarray(ref_codes, dtype=np.int32)
        nrf = 0 if rc is None else rc.shape[0]
        H = self.cfg["H"]
        pre = np.zeros((12 + len(rid) + len(ids) + nrf, H), np.float32)
        tr = np.zeros((len(ids) + len(rid) + 2, H), np.float32)
        ntr = C.c_int(0)
        sv = None if spk_vec is None else np.ascontiguousarray(spk_vec, dtype=np.float32)
        P = self.lib.orc_build_icl_prompt(self.h, iptr(ids), len(ids), iptr(rid), len(rid),
                                          None if rc is None else iptr(rc), nrf, None if sv is None else fptr(sv),
                                          lang, int(non_streaming), fptr(pre), fptr(tr), C.byref(ntr))
        assert P > 0
        return pre[:P].copy(), tr[:ntr.value].copy()

    def generate_from_prompt(self, prefill, trailing, max_frames=4096, **params):
        p = make_params(**params)
        cap = min(max_frames, p.fixed if p.fixed > 0 else p.max_tokens)
        codes = np.zeros((max(cap, 1), self.cfg["G"]), np.int32)
        stop = C.c_int(0)
        pre = np.ascontiguousarray(prefill, np.float32)
        tr = np.ascontiguousarray(trailing, np.float32)
        n = self.lib.orc_generate_from_prompt(self.h, fptr(pre), pre.shape[0], fptr(tr), tr.shape[0], C.byref(p),
                                              iptr(codes), cap, C.byref(stop))
        return codes[:n].copy(), stop.value

    def trace_draw(self, ids, spk, lang, frame, group, **params):
        """The sampler's inputs at draw (frame, group) of this utterance's
        generation (group 0: the talker's code-0 draw; 1..15 the sub-talker's):
        dict(logits, x = the logit head's input row, rng_bits, result), or
        None if the generation stopped before it."""
        self.lib.orc_trace_arm(self.h, int(frame), int(group))
        self.generate_codes(ids, spk, lang, max_frames=int(frame) + 1, **params)
        n, xn = C.c_int(0), C.c_int(0)
        ok = self.lib.orc_trace_dims(self.h, C.byref(n), C.byref(xn))
        if not ok:
            self.lib.orc_trace_arm(self.h, -1, -1)
            return None
        lg = np.zeros(n.value, np.float32)
        x = np.zeros(xn.value, np.float32)
        rng = np.zeros(1, np.float32)
        res = C.c_int(0)
        got = self.lib.orc_trace_get(self.h, fptr(lg), fptr(x), fptr(rng), C.byref(res))
        self.lib.orc_trace_arm(self.h, -1, -1)
        assert got == 1
        return {"logits": lg, "x": x, "rng_bits": int(rng.view(np.uint32)[0]), "result": res.value}

    def generate_codes(self, ids, spk=-1, lang=-1, max_frames=4096, **params):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        p = make_params(**params)
        cap = min(max_frames, p.fixed if p.fixed > 0 else p.max_tokens)
        codes = np.zeros((max(cap, 1), self.cfg["G"]), np.int32)
        stop = C.c_int(0)
        n = self.lib.orc_generate_codes(self.h, iptr(ids), len(ids), spk, lang, C.byref(p),
                                        iptr(codes), cap, C.byref(stop))
        return codes[:n].copy(), stop.value


# ---------------------------------------------------------------- reference
class RefLib:
    """The reference c/ build (oracle/_ref/libqtts_ref.so) via ctypes."""

    def __init__(self, model_dir, verbose=0):
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(REF_SO)
        lib = self.lib = C.CDLL(REF_SO)
        lib.qwen_tts_load.restype = C.c_void_p
        lib.qwen_tts_load.argtypes = [C.c_char_p]
        lib.qwen_tts_free.argtypes = [C.c_void_p]
        lib.qwen_tts_generate.restype = C.c_void_p
        lib.qwen_tts_generate.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, _ip]
        lib.qwen_tts_talker_prefill.argtypes = [C.c_void_p, _fp, C.c_int]
        lib.qwen_tts_talker_forward.argtypes = [C.c_void_p, _fp, _fp]
        lib.qwen_tts_subtalker_generate.argtypes = [C.c_void_p, _fp, C.c_int, _ip]
        lib.qwen_tts_codec_decode.restype = C.c_void_p
        lib.qwen_tts_codec_decode.argtypes = [C.c_void_p, _ip, C.c_int, _ip]
        lib.ref_set_params.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int,
                                       C.c_int, C.c_float, C.c_int, C.c_float]
        lib.ref_get_perf.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        lib.ref_kv_len.restype = C.c_int
        lib.ref_kv_len.argtypes = [C.c_void_p]
        lib.ref_set_kv_len.argtypes = [C.c_void_p, C.c_int]
        lib.ref_tk_x.restype = C.c_void_p
        lib.ref_tk_x.argtypes = [C.c_void_p]
        lib.ref_samp_get.argtypes = [C.c_int, _ip, _fp, C.POINTER(C.c_uint32), C.POINTER(C.c_size_t)]
        lib.ref_samp_logits.restype = C.c_void_p
        lib.ref_st_hidden.restype = C.c_void_p
        lib.ref_st_codes.restype = C.c_void_p
        lib.ref_codec_codes.restype = C.c_void_p
        lib.ref_free.argtypes = [C.c_void_p]
        lib.kernel_sample_top_k.restype = C.c_int
        lib.kernel_sample_top_k.argtypes = [_fp, C.c_int, C.c_int, C.c_float, C.c_float, _fp]
        lib.kernel_matvec_bf16.argtypes = [_fp, C.c_void_p, _fp, C.c_int, C.c_int]
        lib.kernel_causal_conv1d.argtypes = [_fp, _fp, _fp, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int]
        lib.kernel_transposed_conv1d.argtypes = [_fp, _fp, _fp, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, _ip]
        lib.kernel_snake_beta.argtypes = [_fp, _fp, _fp, _fp, C.c_int, C.c_int]
        lib.ref_set_verbose(verbose)
        self.cfg = load_config(model_dir)
        self.ctx = lib.qwen_tts_load(model_dir.encode())
        if not self.ctx:
            raise RuntimeError("reference qwen_tts_load failed")

    def close(self):
        if self.ctx:
            self.lib.qwen_tts_free(self.ctx)
            self.ctx = None

    def set_params(self, max_tokens=4096, fixed=0, seed=42, **kw):
        p = dict(DEFAULT)
        p.update(kw)
        self.lib.ref_set_params(self.ctx, p["temperature"], p["top_k"], p["top_p"], p["rep"], max_tokens, fixed,
                                seed, p["st_temperature"], p["st_top_k"], p["st_top_p"])

    def generate(self, ids, speaker=None, language=None, record=True):
        csv = ",".join(str(int(i)) for i in ids).encode()
        n = C.c_int(0)
        self.lib.ref_record(1 if record else 0)
        p = self.lib.qwen_tts_generate(self.ctx, csv, speaker.encode() if speaker else None,
                                       language.encode() if language else None, C.byref(n))
        audio = None
        if p:
            audio = np.ctypeslib.as_array(C.cast(p, _fp), shape=(n.value,)).copy()
            self.lib.ref_free(p)
        return audio

    def perf(self):
        o = (C.c_double * 4)()
        self.lib.ref_get_perf(self.ctx, o)
        return dict(total_ms=o[0], talker_ms=o[1], codec_ms=o[2], tokens=int(o[3]))

    def recorded_codes(self):
        T = self.lib.ref_codec_T()
        if T <= 0:
            return np.zeros((0, self.cfg["cq"]), np.int32)
        p = self.lib.ref_codec_codes()
        return np.ctypeslib.as_array(C.cast(p, _ip), shape=(T, self.cfg["cq"])).copy()

    def recorded_subtalker(self):
        n = self.lib.ref_st_count()
        H, G = self.cfg["H"], self.cfg["G"]
        if n == 0:
            return np.zeros((0, H), np.float32), np.zeros((0, G), np.int32)
        hid = np.ctypeslib.as_array(C.cast(self.lib.ref_st_hidden(), _fp), shape=(n, H)).copy()
        cod = np.ctypeslib.as_array(C.cast(self.lib.ref_st_codes(), _ip), shape=(n, G)).copy()
        return hid, cod

    def recorded_samples(self):
        n = self.lib.ref_samp_count()
        out = []
        lp = self.lib.ref_samp_logits()
        for i in range(n):
            meta = (C.c_int * 3)()
            fm = (C.c_float * 2)()
            rng = (C.c_uint32 * 2)()
            off = C.c_size_t(0)
            self.lib.ref_samp_get(i, meta, fm, rng, C.byref(off))
            V = meta[0]
            lg = np.ctypeslib.as_array(C.cast(lp + off.value * 4, _fp), shape=(V,)).copy()
            out.append(dict(vocab=V, top_k=meta[1], result=meta[2], top_p=fm[0], temp=fm[1],
                            rng_in=rng[0], rng_out=rng[1], logits=lg))
        return out

    def prefill(self, embeds):
        e = np.ascontiguousarray(embeds, np.float32)
        self.lib.ref_set_kv_len(self.ctx, 0)
        self.lib.qwen_tts_talker_prefill(self.ctx, fptr(e), e.shape[0])
        return np.ctypeslib.as_array(C.cast(self.lib.ref_tk_x(self.ctx), _fp), shape=(self.cfg["H"],)).copy()

    def step(self, embed):
        lg = np.zeros(self.cfg["V"], np.float32)
        self.lib.qwen_tts_talker_forward(self.ctx, fptr(np.ascontiguousarray(embed, np.float32)), fptr(lg))
        hid = np.ctypeslib.as_array(C.cast(self.lib.ref_tk_x(self.ctx), _fp), shape=(self.cfg["H"],)).copy()
        return lg, hid

    def subtalker(self, hidden, code0):
        out = np.zeros(self.cfg["G"], np.int32)
        self.lib.qwen_tts_subtalker_generate(self.ctx, fptr(np.ascontiguousarray(hidden, np.float32)), int(code0),
                                             iptr(out))
        return out

    def codec_decode(self, codes):
        c = np.ascontiguousarray(codes, np.int32)
        n = C.c_int(0)
        p = self.lib.qwen_tts_codec_decode(self.ctx, iptr(c), c.shape[0], C.byref(n))
        out = np.ctypeslib.as_array(C.cast(p, _fp), shape=(n.value,)).copy()
        self.lib.ref_free(p)
        return out
