#!/usr/bin/env python3
"""Synthetic Qwen2-style byte-level BPE files for a model directory:
vocab.json, merges.txt, tokenizer_config.json (development / test data).

The real Qwen3-TTS vocabulary (151k tokens) is not in the reference and
cannot be downloaded here, so the C tokenizer (qwen3-tts-c_amd/csrc/host/bpe.c)
is checked on these files:
  * the 256 byte tokens take ids 0..255 in GPT-2 bytes_to_unicode order, as in
    Qwen2's vocabulary ("." = 13, "\\n" = 198, " " = 220);
  * merge chains placed first (lowest ranks) build the words of the
    reference's only tokenizer fixture, test/tokens_great_power.txt, with its
    ids: "With great power comes great responsibility." in the chat template
    -> 151644,77091,198,2354,2244,2355,4041,2244,11752,13,151645,198,151644,77091,198;
  * then a small BPE trained on a seeded mixed-script corpus (Latin, accented
    Latin, Greek, Cyrillic, CJK, kana, digits, punctuation) so random texts
    exercise real merge competition;
  * added tokens (<|endoftext|>, <|im_start|>, <|im_end|> and the TTS text
    specials) in tokenizer_config.json's added_tokens_decoder.
Anything beyond the fixture is PARITY UNPINNED against the real vocabulary;
tests/test_tokenizer.py compares the C tokenizer with transformers'
Qwen2Tokenizer on these same files.
"""
import collections
import json
import os

import numpy as np
import regex

PRETOK = regex.compile(r"""(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+""")

FIXTURE_WORDS = {"With": 2354, "Ġgreat": 2244, "Ġpower": 2355, "Ġcomes": 4041, "Ġresponsibility": 11752,
                 "assistant": 77091}
SPECIALS = {151643: "<|endoftext|>", 151644: "<|im_start|>", 151645: "<|im_end|>", 151671: "<|tts_pad|>",
            151672: "<|tts_text_bos|>", 151673: "<|tts_text_eod|>"}


def bytes_to_unicode():
    bs = list(range(33, 127)) + list(range(161, 173)) + list(range(174, 256))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs])), bs


def corpus(seed=7, n_words=6000):
    rng = np.random.default_rng(seed)
    alpha = {
        "latin": "etaoinshrdlcumwfgypbvkjxqz",
        "accent": "éèêàâçôûüöäßñ",
        "greek": "αβγδεζηθικλμνξοπρστυφχψω",
        "cyr": "абвгдежзийклмнопрстуфхцчшщыэюя",
        "cjk": "的一是不了人我在有他这中大来上国个到说们为子和你地出道也时年",
        "kana": "あいうえおかきくけこさしすせそアイウエオカキクケコ",
    }
    words = []
    keys = list(alpha)
    for _ in range(n_words):
        k = keys[rng.integers(0, len(keys))] if rng.random() < 0.4 else "latin"
        a = alpha[k]
        L = int(rng.integers(1, 9))
        w = "".join(a[min(int(rng.exponential(len(a) / 4)), len(a) - 1)] for _ in range(L))
        if rng.random() < 0.15:
            w = w.capitalize()
        words.append(w)
    text = []
    for w in words:
        r = rng.random()
        sep = " " if r < 0.8 else (", " if r < 0.88 else (". " if r < 0.94 else ("\n" if r < 0.97 else " 12 ")))
        text.append(w + sep)
    return "".join(text) + "I'm here, it's 2024! They'll say \"ok\"... don't; we've 3.14 and 100%.\n\n"


def build(n_merges=2000, seed=7):
    enc, order = bytes_to_unicode()
    vocab = {enc[b]: i for i, b in enumerate(order)}     # ids 0..255
    used = set(vocab.values()) | set(FIXTURE_WORDS.values()) | set(SPECIALS)
    next_id = [256]

    def fresh():
        while next_id[0] in used:
            next_id[0] += 1
        used.add(next_id[0])
        return next_id[0]

    merges = []
    for word, wid in FIXTURE_WORDS.items():   # prefix chains, lowest ranks
        cur = word[0]
        for i in range(1, len(word)):
            nxt = cur + word[i]
            merges.append((cur, word[i]))
            if nxt not in vocab:
                vocab[nxt] = wid if i == len(word) - 1 else fresh()
            cur = nxt
    # BPE training over the corpus's pre-tokens (byte-level symbols)
    words = collections.Counter()
    for m in PRETOK.finditer(corpus(seed)):
        words[tuple(enc[b] for b in m.group(0).encode("utf-8"))] += 1
    have = set(merges)
    for _ in range(n_merges):
        pairs = collections.Counter()
        for w, c in words.items():
            for a, b in zip(w, w[1:]):
                pairs[(a, b)] += c
        pairs = [(c, p) for p, c in pairs.items() if p not in have]
        if not pairs:
            break
        c, best = max(pairs, key=lambda x: (x[0], x[1]))
        if c < 2:
            break
        have.add(best)
        merges.append(best)
        tok = best[0] + best[1]
        if tok not in vocab:
            vocab[tok] = fresh()
        nw = collections.Counter()
        for w, cnt in words.items():
            out, i = [], 0
            while i < len(w):
                if i + 1 < len(w) and (w[i], w[i + 1]) == best:
                    out.append(tok)
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            nw[tuple(out)] += cnt
        words = nw
    return vocab, merges


def build_cached(n_merges=2000):
    """build() is deterministic and takes ~20 s; keep one copy per machine."""
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"qtts_synth_tokenizer_{n_merges}_v1.json")
    if os.path.exists(path):
        with open(path, encoding="utf-8") as f:
            d = json.load(f)
        return d["vocab"], [tuple(m) for m in d["merges"]]
    vocab, merges = build(n_merges)
    tmp = path + f".{os.getpid()}"
    with open(tmp, "w", encoding="utf-8") as f:
        json.dump({"vocab": vocab, "merges": merges}, f, ensure_ascii=False)
    os.replace(tmp, path)
    return vocab, merges


def write(model_dir, n_merges=2000):
    vocab, merges = build_cached(n_merges)
    with open(os.path.join(model_dir, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    with open(os.path.join(model_dir, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n")
        for a, b in merges:
            f.write(f"{a} {b}\n")
    cfg = {"tokenizer_class": "Qwen2Tokenizer", "model_max_length": 131072,
           "added_tokens_decoder": {str(i): {"content": t, "special": True, "lstrip": False, "rstrip": False,
                                             "normalized": False, "single_word": False}
                                    for i, t in sorted(SPECIALS.items())}}
    with open(os.path.join(model_dir, "tokenizer_config.json"), "w", encoding="utf-8") as f:
        json.dump(cfg, f, ensure_ascii=False, indent=1)


if __name__ == "__main__":
    import sys
    write(sys.argv[1])
