"""BPE pre-tokenizers (koboldcpp_amd/csrc/tokenizer.h, through the host-only C-ABI probe kcpp_pretokenize) vs the
reference's split regexes (llm_tokenizer_bpe's regex_exprs, src/llama-vocab.cpp:597-712) run by the Python
`regex` module on random Unicode text: letters and digits of many scripts (\\p{N} includes Nl / No: superscripts,
Roman numerals, fullwidth and Arabic-Indic digits), marks, symbols, emoji, every White_Space code point,
contractions in both cases.  The reference executes these regexes with hand-written matchers
(unicode_regex_split_custom_llama3 / _gpt2, src/unicode.cpp) whose semantics are the regexes' leftmost-first
alternation; the C++ restates those matchers over the Unicode classes generated from the same `regex` tables
(tools/gen_unicode_ranges.py).  The words must tile the text and equal the regex's matches one for one."""
import ctypes

import numpy as np
import pytest
import regex

LLAMA3 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
          r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
QWEN2 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}|"
         r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
# the reference's gpt2 expression ends at \s+(?!\S); its matcher keeps the remaining whitespace as a word, i.e. \s+
GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"

POOLS = [
    "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ",
    "0123456789",
    "'''sStTmMdDreREveVEllLL",
    " " * 12 + "\t\n\r\n\x0b\x0c",
    "!\"#$%&()*+,-./:;<=>?@[\\]^_`{|}~",
    "éèàüößçñøåÆŒĳǅ",                       # Latin letters incl. titlecase / ligatures
    "абвгдЖЗИЙ",                              # Cyrillic
    "中文字符日本語カタカナひらがな한국어",     # CJK / kana / Hangul (Lo)
    "مرحبا",                                   # Arabic letters
    "٠١٢٣٤٥٦٧٨٩０１２３²³¹½ⅫⅣ",              # Nd / No / Nl numbers
    "ً́̈‍‌",          # combining marks, ZWJ / ZWNJ (neither L, N nor \s)
    "€£¥©®™°±×÷§¶•…—–",                        # symbols and punctuation
    "😀🚀👍🏽\U0001F9D1",                       # emoji (astral)
    "         　\u0085",   # non-ASCII White_Space
    "\U0001D400\U0001D7CE\U00010400",          # astral letters / digits
]


@pytest.fixture(scope="module")
def lib():
    import koboldcpp_amd.lib as K
    return K.raw()


def pretok(lib, pre, text):
    b = text.encode("utf-8")
    cap = len(b) + 1
    ends = (ctypes.c_int64 * cap)()
    n = lib.kcpp_pretokenize(pre.encode(), b, ends, cap)
    assert n >= 0
    words, s = [], 0
    for e in ends[:n]:
        words.append(b[s:e].decode("utf-8"))
        s = e
    assert s == len(b), "words do not tile the text"
    return words


def random_texts(seed, count):
    rng = np.random.default_rng(seed)
    for _ in range(count):
        n = int(rng.integers(0, 48))
        out = []
        for _ in range(n):
            pool = POOLS[int(rng.integers(0, len(POOLS)))]
            out.append(pool[int(rng.integers(0, len(pool)))])
        yield "".join(out)


FIXED = ["Hello world", "I'm here, you're there; they'LL see", "  leading and trailing  ", "a\n\n  b\r\n\tc  \n",
         "12345678 ٣٤٥٦ ²³ Ⅻ", "naïve café — 中文 😀!!", "x y　z", "don't\nDON'T", "'s's", "   ", "\n", "",
         "tab\tsep\x0bvt", "́abc", "áb", "$$$ %%%\n\n", " ' ", "'"]


@pytest.mark.parametrize("pre,rx", [("llama-bpe", LLAMA3), ("qwen2", QWEN2), ("gpt-2", GPT2)])
def test_pretokenizer_matches_reference_regex(lib, pre, rx):
    pat = regex.compile(rx)
    bad = []
    for text in FIXED + list(random_texts(len(pre), 3000)):
        want = pat.findall(text)
        assert "".join(want) == text
        got = pretok(lib, pre, text)
        if got != want:
            bad.append((text, got, want))
    assert not bad, bad[:3]


def test_pre_type_mapping(lib):
    """llama3 family vs gpt2 family on a text where they differ (number grouping, case-insensitive contraction)"""
    t = "It'S 123456"
    assert pretok(lib, "llama3", t) == ["It", "'S", " ", "123", "456"]
    assert pretok(lib, "smaug-bpe", t) == pretok(lib, "llama-bpe", t)
    assert pretok(lib, "gpt-2", t) == ["It", "'", "S", " 123456"]
    assert pretok(lib, "qwen2", t) == ["It", "'S", " ", "1", "2", "3", "4", "5", "6"]


# ---------------------------------------------------------------- byte-level BPE end to end vs HF tokenizers
LLAMA3_ORIG = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|"
               r"\s*[\r\n]+|\s+(?!\S)|\s+")
SPECIALS = ["<|begin_of_text|>", "<|eot_id|>", "<|start_header_id|>"]


def _train_bpe(corpus):
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE(ignore_merges=True))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_ORIG), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tr = trainers.BpeTrainer(vocab_size=700, special_tokens=SPECIALS, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus, tr)
    return tok


def test_bpe_encode_matches_hf_tokenizers(lib, tmp_path):
    """a Llama-3-style byte-level BPE (ignore_merges, llama3 split, special tokens) trained with HF `tokenizers`,
    written as a GGUF vocabulary (tokens, merges, token types, pre "llama-bpe"), then tokenized by the runtime's
    tokenizer (kcpp_tokenize_probe) and by `tokenizers` on random text with special tokens inside: equal ids"""
    import json
    import gguf_writer as GW
    corpus = list(random_texts(7, 400)) + FIXED * 20 + ["the quick brown fox jumps over the lazy dog " * 5] * 50
    tok = _train_bpe(corpus)
    m = json.loads(tok.to_str())["model"]
    vocab = sorted(m["vocab"].items(), key=lambda kv: kv[1])
    assert [i for _, i in vocab] == list(range(len(vocab)))
    merges = [" ".join(x) if isinstance(x, list) else x for x in m["merges"]]
    ttype = [3 if t in SPECIALS else 1 for t, _ in vocab]
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": "llama-bpe",
          "tokenizer.ggml.tokens": (GW.STR, [t for t, _ in vocab]), "tokenizer.ggml.token_type": (GW.I32, ttype),
          "tokenizer.ggml.merges": (GW.STR, merges), "tokenizer.ggml.bos_token_id": 0,
          "tokenizer.ggml.add_bos_token": True}
    path = str(tmp_path / "bpe.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(vocab)], np.zeros((len(vocab), 8), np.float32))])
    rng = np.random.default_rng(11)
    bad = []
    for text in FIXED + list(random_texts(13, 600)):
        if rng.random() < 0.3:                     # special tokens inside the text
            k = int(rng.integers(0, len(text) + 1))
            text = text[:k] + SPECIALS[int(rng.integers(0, len(SPECIALS)))] + text[k:]
        want = tok.encode(text, add_special_tokens=False).ids
        b = text.encode("utf-8")
        out = (ctypes.c_int32 * (len(b) + 8))()
        n = lib.kcpp_tokenize_probe(path.encode(), b, 0, out, len(b) + 8)
        assert n >= 0
        if list(out[:n]) != want:
            bad.append((text, list(out[:n]), want))
    assert not bad, bad[:3]
    # BOS per the vocabulary
    out = (ctypes.c_int32 * 8)()
    assert lib.kcpp_tokenize_probe(path.encode(), b"hi", 1, out, 8) >= 1 and out[0] == 0


@pytest.mark.parametrize("case", ["kv", "text", "none"])
def test_special_ids_eot(lib, tmp_path, case):
    """EOT as llm_load_vocab finds it (src/llama.cpp:6606, 6642-6661): the tokenizer.ggml.eot_token_id key, else a
    token whose text is a known end-of-turn marker, else none (-1); generate() suppresses and stops on it like EOS"""
    import gguf_writer as GW
    toks = ["<unk>", "<s>", "</s>", "a", "b", "<|eot_id|>", "c"]
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "llama",
          "tokenizer.ggml.tokens": (GW.STR, toks if case != "none" else toks[:5] + ["x", "c"]),
          "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2}
    if case == "kv":
        kv["tokenizer.ggml.eot_token_id"] = 6
    path = str(tmp_path / "v.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(toks)], np.zeros((len(toks), 8), np.float32))])
    out = (ctypes.c_int32 * 3)()
    assert lib.kcpp_tokenizer_special_ids(path.encode(), out) == 0
    assert list(out) == [1, 2, {"kv": 6, "text": 5, "none": -1}[case]]
