#!/usr/bin/env python3
"""Classify one divergence from a reference fixture (tests/divergence.py):
fp near-tie or bug.  Runs the oracle port (CPU) up to the divergent frame.

  python tools/classify_divergence.py --fixture long_eos17 --utt 1 --frame 69 --group 2 [--got ID]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden")]
from conftest import model_dir  # noqa: E402
from divergence import classify, describe  # noqa: E402
from oracle_py import DEFAULT, Oracle  # noqa: E402
from qtts_io import lookup_ids  # noqa: E402

KEYS = {"long_eos17": ("eos17", "1.7b"), "long_eos17q": ("eos17q", "1.7b"), "long_17b_b8": ("b8", "1.7b"),
        "long_17b_b8bench": ("b8bench", "1.7b"), "long_hd128_max": ("hd128max", "hd128"),
        "long_17b_1100": ("k1100", "1.7b")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", required=True, choices=sorted(KEYS))
    ap.add_argument("--utt", type=int, required=True)
    ap.add_argument("--frame", type=int, required=True)
    ap.add_argument("--group", type=int, required=True)
    ap.add_argument("--got", type=int, default=None)
    a = ap.parse_args()
    key, preset = KEYS[a.fixture]
    g = np.load(os.path.join(ROOT, "tests", "golden", a.fixture + ".npz"))
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "long_manifest.json")))[key]
    single = g["prompt_ids"].ndim == 1   # one-utterance fixtures (codes [frames][groups])
    ids = g["prompt_ids"] if single else g["prompt_ids"][a.utt, :int(g["prompt_len"][a.utt])]
    ovr = {"eos_gain": man["eos_gain"]} if "eos_gain" in man else {}
    md = model_dir(preset, **ovr)
    o = Oracle(md)
    spk = man["speaker"] if single else man["speakers"][a.utt]
    s, l = lookup_ids(o.cfg, spk, man.get("language", "english"))
    fixed = 0 if "eos_gain" in man else man["frames"]
    params = dict(max_tokens=4096, fixed=fixed, seed=man["seed"], **DEFAULT)
    c = classify(o, ids, s, l, a.frame, a.group, params, got=a.got)
    want = int(g["codes"][a.frame, a.group] if single else g["codes"][a.utt, a.frame, a.group])
    c["fixture_code"] = want
    print(json.dumps({k: (float(v) if isinstance(v, (np.floating,)) else v) for k, v in c.items()}))
    print(describe(c))
    assert c.get("reference") in (None, want), ("the oracle's draw is not the fixture's", c.get("reference"), want)


if __name__ == "__main__":
    main()
