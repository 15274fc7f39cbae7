#!/usr/bin/env python3
"""C5 bench-shape voice-clone fixture (TEST INFRASTRUCTURE), from the ORACLE
port: the reference c/ has no voice clone, so its pin is the oracle's
restatement of the Python reference's ICL layout (orc_build_icl_prompt,
modeling_qwen3_tts.py:1967-2019 / 2104-2232) -- parity against the Python
reference itself is unpinned (not importable here).

Exactly the 8 utterances `bench.py --voice-clone --vc-codes --batch 8` rank 0
decodes: p128 seeds 1234-1241 (rank_prompt_seeds(0, 8)), 63 seeded reference
frames, a 20-id reference text and an x-vector per slot (seed + 7), seed 42,
default sampling -- here 32 generated frames per slot.  Each slot is one
oracle run (slots in parallel processes):

  python tests/golden/make_golden_vc.py            # -> tests/golden/vc_c5_b8.npz
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools"), ROOT]

FRAMES = 32
REF_FRAMES = 63
AUDIO_STRIDE = 16


def bench_inputs(G=16, H=2048):
    """bench.py's voice-clone inputs for rank 0, batch 8 (bench.py main())"""
    import bench
    from synth_model import prompt_ids
    out = []
    for sd in bench.rank_prompt_seeds(0, 8):
        r = np.random.default_rng(sd + 7)
        codes = r.integers(0, 2048, size=(REF_FRAMES, G)).astype(np.int32)
        rids = [151644, 77091, 198] + r.integers(1000, 100000, size=20).tolist() + [151645, 198]
        spk = (r.standard_normal(H) * 0.05).astype(np.float32)
        out.append((prompt_ids("p128", seed=sd), rids, codes, spk))
    return out


def one_slot(b):
    from conftest import model_dir
    from oracle_py import DEFAULT, Oracle
    from qtts_io import lookup_ids
    o = Oracle(model_dir("1.7b"))
    ids, rids, refs, spk = bench_inputs(o.cfg["G"], o.cfg["H"])[b]
    _, lang = lookup_ids(o.cfg, "aiden", "english")
    pre, tr = o.build_icl_prompt(ids, rids, refs, spk, lang, 0)
    codes, _ = o.generate_from_prompt(pre, tr, max_tokens=4096, fixed=FRAMES, seed=42, **DEFAULT)
    full = o.codec_decode(np.concatenate([refs, codes]))
    T = refs.shape[0]
    cut = int(T / (T + len(codes)) * full.shape[0])
    a = full[cut:]
    o.close()
    print(f"slot {b}: {len(codes)} frames, prefill rows {pre.shape[0]}", file=sys.stderr, flush=True)
    return codes, a[::AUDIO_STRIDE].copy(), a[-1920:].copy(), len(a), pre.shape[0]


def main():
    with ProcessPoolExecutor(8) as ex:
        res = list(ex.map(one_slot, range(8)))
    np.savez_compressed(os.path.join(HERE, "vc_c5_b8.npz"),
                        codes=np.stack([r[0] for r in res]), audio_sub=np.stack([r[1] for r in res]),
                        audio_last=np.stack([r[2] for r in res]), audio_len=np.array([r[3] for r in res]),
                        prefill_rows=np.array([r[4] for r in res]), frames=np.array(FRAMES),
                        ref_frames=np.array(REF_FRAMES), audio_stride=np.array(AUDIO_STRIDE))


if __name__ == "__main__":
    main()
