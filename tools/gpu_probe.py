#!/usr/bin/env python3
"""Quick end-to-end probe of the HIP path against the CPU oracle on the tiny
synthetic model (development tool; the real checks live in tests/)."""
import os
import sys
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "qwen3-tts-c_amd")]

import torch  # noqa: E402
import qtts  # noqa: E402
from oracle_py import Oracle, GREEDY, DEFAULT  # noqa: E402
from qtts_io import lookup_ids, f32_to_bf16  # noqa: E402
from synth_model import ensure_model, prompt_ids  # noqa: E402


def step(name, fn):
    t = time.time()
    try:
        r = fn()
        print(f"[ok]   {name} ({time.time() - t:.2f}s) {r if r is not None else ''}", flush=True)
    except Exception as e:  # keep probing the other layers
        print(f"[FAIL] {name}: {e}", flush=True)
        traceback.print_exc()


def main():
    md = ensure_model("/tmp/qtts_probe_tiny", "tiny")
    o = Oracle(md)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)

    def k_matvec():
        for R, Cc, B in [(256, 128, 1), (3072, 128, 1), (512, 256, 3), (1000, 192, 16)]:
            A = rng.standard_normal((R, Cc)).astype(np.float32)
            Ab = f32_to_bf16(A)
            x = rng.standard_normal((B, Cc)).astype(np.float32)
            ref = np.stack([(Ab.astype(np.uint32) << 16).view(np.float32) @ x[b] for b in range(B)])
            out = torch.zeros(B * R, device=dev)
            qtts.Kernels.matvec_bf16(out, torch.from_numpy(Ab.view(np.int16)).to(dev), torch.from_numpy(x).to(dev),
                                     R, Cc, B)
            torch.cuda.synchronize()
            err = np.abs(out.cpu().numpy().reshape(B, R) - ref).max()
            assert err < 1e-3, (R, Cc, B, err)
        return "max err ok"

    def k_sample():
        bad = 0
        for i in range(200):
            V = 3072 if i % 2 else 2048
            lg = (rng.standard_normal(V) * 3).astype(np.float32)
            if i % 7 == 0:
                lg[rng.integers(0, V, 20)] = lg.max()  # ties
            k = [1, 50, 5, 300][i % 4]
            tp = 1.0 if i % 5 else 0.8
            temp = 0.9
            st = np.array([np.float32(42 + i)], np.float32)
            st_ref = st.copy()
            exp = o.lib.orc_sample(lg.ctypes.data_as(qtts._fp), V, k, tp, temp, st_ref.ctypes.data_as(qtts._fp))
            out = torch.zeros(1, dtype=torch.int32, device=dev)
            rs = torch.from_numpy(st.view(np.int32).copy()).to(dev)
            qtts.Kernels.sample_top_k(out, torch.from_numpy(lg).to(dev), V, k, tp, temp, rs)
            torch.cuda.synchronize()
            got = int(out.item())
            if got != exp or int(rs.item()) != int(st_ref.view(np.int32)[0]):
                bad += 1
        assert bad == 0, f"{bad} mismatches"
        return "200 draws identical"

    def stages():
        m = qtts.QwenTTS(md)
        spk, lang = lookup_ids(o.cfg, "aiden", "english")
        pre, tr = o.build_prompt(prompt_ids("short"), spk, lang)
        h_o = o.prefill(pre)
        h_g = m.prefill(pre)
        e1 = np.abs(h_o - h_g).max()
        lg_o, hh_o = o.step(tr[0])
        lg_g, hh_g = m.step(tr[0])
        e2 = np.abs(lg_o - lg_g).max()
        codes_o = o.subtalker(hh_o, 5, top_k=1, temp=1.0)
        m.set_params(st_top_k=1, st_temperature=1.0)
        codes_g = m.subtalker(hh_o, 5)
        m.close()
        return f"prefill hid err {e1:.2e}, step logits err {e2:.2e}, subtalker codes equal {bool((codes_o == codes_g).all())}"

    def e2e():
        m = qtts.QwenTTS(md)
        ids = prompt_ids("short")
        spk, lang = lookup_ids(o.cfg, "aiden", "english")
        res = []
        for name, pp, fixed in [("greedy", GREEDY, 40), ("sampled", DEFAULT, 40), ("eos", DEFAULT, 0)]:
            m.set_params(max_tokens=60, fixed=fixed, seed=42, **pp)
            t = time.time()
            a = m.generate(ids, "aiden", "english")
            dt = time.time() - t
            cg = m.last_codes()
            co, _ = o.generate_codes(ids, spk, lang, max_tokens=60, fixed=fixed, seed=42, **pp)
            same = cg.shape == co.shape and bool((cg == co).all())
            ao = o.codec_decode(co)
            mse = float(np.mean((ao - a) ** 2)) if a is not None and a.shape == ao.shape else None
            first = None
            if not same and cg.shape[0] and co.shape[0]:
                n = min(len(cg), len(co))
                d = np.nonzero((cg[:n] != co[:n]).any(1))[0]
                first = int(d[0]) if len(d) else n
            res.append(f"{name}: codes equal={same} (first diff frame {first}) audio mse={mse} {dt:.2f}s")
        m.close()
        return "; ".join(res)

    def codec_only():
        m = qtts.QwenTTS(md)
        codes = rng.integers(0, 2048, size=(80, 16)).astype(np.int32)
        a_g = m.codec_decode(codes)
        a_o = o.codec_decode(codes)
        m.close()
        return f"len {len(a_g)} vs {len(a_o)}, mse {float(np.mean((a_g - a_o) ** 2)):.3e}, max {np.abs(a_g - a_o).max():.3e}"

    step("matvec_bf16", k_matvec)
    step("sampler vs oracle", k_sample)
    step("codec decode vs oracle", codec_only)
    step("stage functions vs oracle", stages)
    step("e2e vs oracle", e2e)


if __name__ == "__main__":
    main()
