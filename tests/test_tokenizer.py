"""Text input: the Qwen2 byte-level BPE of csrc/host/bpe.c (SURVEY.md §8f N4;
the reference leaves it as a TODO at c/qwen_tts.c:1071-1077 and tokenizes in
the browser with @huggingface/transformers, web/wasm/app.js:241-267).

Pins, CPU only (the tokenizer needs no GPU):
  * the reference's only tokenizer fixture, test/tokens_great_power.txt, from
    "With great power comes great responsibility." in the chat template, on
    the synthetic vocabulary that carries those ids (tools/synth_tokenizer.py);
  * every other text against transformers' Qwen2Tokenizer (the tokenizers
    backend: NFC + the Qwen2 split regex + byte-level BPE) built from the SAME
    vocab.json / merges.txt.  Against the real 151k-token Qwen3-TTS vocabulary
    parity is UNPINNED: it is not in the reference and cannot be fetched.
"""
import json
import os
import subprocess
import unicodedata

import numpy as np
import pytest

import qtts

FIXTURE = [151644, 77091, 198, 2354, 2244, 2355, 4041, 2244, 11752, 13, 151645, 198, 151644, 77091, 198]
QUOTE = "With great power comes great responsibility."


def chat(text):
    return f"<|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n"


@pytest.fixture(scope="module")
def hf_tok(tiny_dir):
    from transformers import Qwen2Tokenizer
    with open(os.path.join(tiny_dir, "vocab.json"), encoding="utf-8") as f:
        v = json.load(f)
    with open(os.path.join(tiny_dir, "merges.txt"), encoding="utf-8") as f:
        m = [tuple(l.rstrip("\n").split(" ")) for l in f if not l.startswith("#version")]
    return Qwen2Tokenizer(vocab=v, merges=m)


def test_fixture_tokens_great_power(tiny_dir):
    assert qtts.tokenize(tiny_dir, chat(QUOTE)) == FIXTURE


def test_cli_text_flag_prints_fixture(tiny_dir):
    r = subprocess.run([qtts.CLI_PATH, "-d", tiny_dir, "-T", QUOTE, "--print-ids"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert [int(x) for x in r.stdout.strip().split(",")] == FIXTURE


def _random_texts(n, seed=0):
    rng = np.random.default_rng(seed)
    pieces = ["the", "The", "power", "great", "responsibility", "ALL", "I", "'m", "'S", "'Re", "'ll", "'D", "'ve",
              "'t", "don't", "it's", "O'Neil", "12", "3.14", "2024", "100%", "Ⅻ", "٣", "½", "wörld", "Ærø", "façade",
              "naïve", "αβγ", "Ωμέγα", "привет", "мир", "的一是", "不了人", "あいう", "カタカナ", "한국어", "עברית",
              "العربية", "🙂", "🚀🚀", "...", "!!", "?", ",", ";", ":", "--", "(x)", "[y]", "{z}", "\"q\"", "$5",
              "#tag", "@me", "a_b", "e-mail", " ", "　", " ", "ſ", "ǅ", "ﬁ", "x\ty"]
    seps = [" ", "  ", "   ", "\n", "\n\n", " \n", "\n ", "\r\n", "\t", "", " \t ", "\n\n\n  ", "  \n\n"]
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 14))
        s = ""
        for _ in range(k):
            s += pieces[int(rng.integers(0, len(pieces)))] + seps[int(rng.integers(0, len(seps)))]
        if rng.random() < 0.3:
            s = seps[int(rng.integers(0, len(seps)))] + s
        out.append(s)
    return out


def test_random_texts_match_transformers(tiny_dir, hf_tok):
    bad = []
    for t in _random_texts(400) + ["", " ", "\n", "  \n  \n x", "a  b", "a \n\n b", "x  ", "'s'S'", "1234567",
                                   "Hello, World!", "ünïcödé ünïcödé"]:
        t = unicodedata.normalize("NFC", t)
        got = qtts.tokenize(tiny_dir, t)
        want = hf_tok(t, add_special_tokens=False)["input_ids"]
        if got != want:
            bad.append((t, got, want))
    assert not bad, bad[:3]


def test_added_tokens_split_first(tiny_dir, hf_tok):
    """Added tokens are matched before the regex, anywhere in the text."""
    t = "a<|im_end|>b <|tts_pad|>\n<|endoftext|>"
    got = qtts.tokenize(tiny_dir, t)
    plain = lambda s: hf_tok(s, add_special_tokens=False)["input_ids"]
    assert got == plain("a") + [151645] + plain("b ") + [151671] + plain("\n") + [151643]


def test_missing_vocab_fails_loudly(tmp_path):
    assert qtts.tokenize(str(tmp_path), "hello") is None
