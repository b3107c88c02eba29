"""The runtime tokenizer (koboldcpp_amd/csrc/tokenizer.h, through the host-only probe kcpp_tokenize_probe) pinned to
the REFERENCE tokenizer itself: src/llama-vocab.cpp + src/unicode.cpp compiled from /root/reference into
oracle/_ref/ref_vocab (oracle/ref_vocab.cpp fills llama_vocab as llm_load_vocab does and calls
llama_tokenize_internal).  Both tokenize the same random Unicode texts with the same vocabulary (byte-level BPE
trained with HF `tokenizers`, under every pre-tokenizer name llm_load_vocab accepts; a SentencePiece-style SPM
vocabulary with byte fallback): the token ids must be equal; and every vocabulary id's streamed piece
(llama_token_to_piece_impl, special = false) must be equal byte for byte.  Runs where the reference sources are (the build
container); skipped elsewhere."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_VOCAB = os.path.join(ROOT, "oracle", "_ref", "ref_vocab")

from test_tokenizer_unicode import FIXED, random_texts  # noqa: E402


@pytest.fixture(scope="module")
def ref_bin():
    if not os.path.exists(REF_VOCAB):
        if not os.path.isdir("/root/reference/src"):
            pytest.skip("reference sources not present (oracle/_ref/ref_vocab cannot be built here)")
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref_vocab"])
    return REF_VOCAB


@pytest.fixture(scope="module")
def lib():
    import koboldcpp_amd.lib as K
    return K.raw()


def _hex(s):
    b = s.encode("utf-8") if isinstance(s, str) else s
    return b.hex() if b else "-"


def ref_tokenize(*args, **kw):
    return ref_run(*args, **kw)[0]


def ref_run(ref_bin, tmp, kind, tokens, scores, ttypes, merges, texts, bos=-1, eos=-1, unk=-1, add_bos=-1):
    """the reference's ids for each text and its piece (special = false) for each vocabulary id"""
    vp, tp, op = (os.path.join(tmp, n) for n in ("v.txt", "t.txt", "o.txt"))
    with open(vp, "w") as f:
        f.write(kind + "\n%d\n" % len(tokens))
        for t, s, y in zip(tokens, scores, ttypes):
            f.write("%s %r %d\n" % (_hex(t), float(s), y))
        f.write("%d\n" % len(merges))
        for a, b in merges:
            f.write("%s %s\n" % (_hex(a), _hex(b)))
        f.write("%d %d %d %d\n" % (bos, eos, unk, add_bos))
    with open(tp, "w") as f:
        f.write("%d\n" % len(texts))
        for t in texts:
            f.write(_hex(t) + "\n")
    subprocess.check_call([ref_bin, vp, tp, op])
    with open(op) as f:
        lines = f.read().split("\n")
    ids = [[int(x) for x in line.split()] for line in lines[:len(texts)]]
    pieces = [b"" if h == "-" else bytes.fromhex(h) for h in lines[len(texts):len(texts) + len(tokens)]]
    assert len(pieces) == len(tokens)
    return ids, pieces


def ours_pieces(lib, path, n):
    cap = 1 << 20
    buf = ctypes.create_string_buffer(cap)
    ends = (ctypes.c_int64 * n)()
    assert lib.kcpp_pieces_probe(path.encode(), buf, cap, ends, n) == n and ends[n - 1] <= cap
    raw, out, s = buf.raw, [], 0
    for e in ends:
        out.append(raw[s:e])
        s = e
    return out


def ours_tokenize(lib, path, texts):
    out = []
    for text in texts:
        b = text.encode("utf-8")
        buf = (ctypes.c_int32 * (len(b) + 8))()
        n = lib.kcpp_tokenize_probe(path.encode(), b, 0, buf, len(b) + 8)
        assert n >= 0
        out.append(list(buf[:n]))
    return out


SPECIALS = ["<|begin_of_text|>", "<|eot_id|>", "<|im_start|>"]


def _bpe_vocab():
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tr = trainers.BpeTrainer(vocab_size=900, special_tokens=SPECIALS, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    corpus = list(random_texts(17, 500)) + FIXED * 20 + ["the quick brown fox jumps over the lazy dog 1234567 " * 4] * 60
    tok.train_from_iterator(corpus, tr)
    m = json.loads(tok.to_str())["model"]
    vocab = sorted(m["vocab"].items(), key=lambda kv: kv[1])
    merges = [tuple(x) if isinstance(x, list) else tuple(x.split(" ")) for x in m["merges"]]
    return [t for t, _ in vocab], merges


@pytest.fixture(scope="module")
def bpe_vocab():
    return _bpe_vocab()


def _texts(seed, count):
    rng = np.random.default_rng(seed)
    out = []
    for text in FIXED + list(random_texts(seed, count)):
        if rng.random() < 0.2:
            k = int(rng.integers(0, len(text) + 1))
            text = text[:k] + SPECIALS[int(rng.integers(0, len(SPECIALS)))] + text[k:]
        out.append(text)
    return out


PRE_TYPES = ["llama-bpe", "llama3", "dbrx", "smaug-bpe", "qwen2", "stablelm2", "gpt-2", "phi-2", "jina-v2-code", "mpt",
             "olmo", "jais", "starcoder", "refact", "command-r", "smollm", "codeshell", "exaone", "deepseek-llm",
             "deepseek-coder", "falcon", "bloom", "gpt3-finnish", "poro-chat", "viking", "chatglm-bpe", "tekken",
             "chameleon", "default"]


@pytest.mark.parametrize("pre", PRE_TYPES)
def test_bpe_matches_reference_tokenizer(ref_bin, lib, bpe_vocab, tmp_path, pre):
    import gguf_writer as GW
    tokens, merges = bpe_vocab
    ttype = [3 if t in SPECIALS else 1 for t in tokens]
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": pre,
          "tokenizer.ggml.tokens": (GW.STR, tokens), "tokenizer.ggml.token_type": (GW.I32, ttype),
          "tokenizer.ggml.merges": (GW.STR, [a + " " + b for a, b in merges])}
    path = str(tmp_path / "bpe.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(tokens)], np.zeros((len(tokens), 8), np.float32))])
    texts = _texts(23, 400)
    want = ref_tokenize(ref_bin, str(tmp_path), "bpe " + pre, tokens, [0.0] * len(tokens), ttype, merges, texts)
    assert sum(len(w) for w in want) > 4 * len(texts)
    got = ours_tokenize(lib, path, texts)
    bad = [(t, g, w) for t, g, w in zip(texts, got, want) if g != w]
    assert not bad, (len(bad), bad[:2])


def _spm_vocab():
    """a SentencePiece-style vocabulary: <unk> <s> </s>, the 256 <0xXX> byte tokens, then "▁"-joined words and
    their prefixes / substrings from a corpus with descending scores (frequency order), plus two user-defined tokens"""
    from collections import Counter
    corpus = list(random_texts(31, 400)) + FIXED * 10 + ["the quick brown fox jumps over the lazy dog"] * 30
    cnt = Counter()
    for t in corpus:
        s = "▁" + t.replace(" ", "▁")
        for i in range(len(s)):
            for L in (1, 2, 3, 4, 6):
                if i + L <= len(s):
                    cnt[s[i:i + L]] += 1
    pieces = [p for p, _ in cnt.most_common(1500)]
    tokens = ["<unk>", "<s>", "</s>"] + ["<0x%02X>" % b for b in range(256)] + ["<|im_start|>", "<|im_end|>"]
    ttype = [2, 3, 3] + [6] * 256 + [4, 4]
    seen = set(tokens)
    for p in pieces:
        if p not in seen:
            tokens.append(p)
            ttype.append(1)
            seen.add(p)
    scores = [0.0] * (259 + 2) + [-float(i) for i in range(len(tokens) - 261)]
    return tokens, scores, ttype


def test_spm_matches_reference_tokenizer(ref_bin, lib, tmp_path):
    import gguf_writer as GW
    tokens, scores, ttype = _spm_vocab()
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "llama",
          "tokenizer.ggml.tokens": (GW.STR, tokens), "tokenizer.ggml.scores": (GW.F32, scores),
          "tokenizer.ggml.token_type": (GW.I32, ttype), "tokenizer.ggml.bos_token_id": 1,
          "tokenizer.ggml.eos_token_id": 2, "tokenizer.ggml.unknown_token_id": 0}
    path = str(tmp_path / "spm.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(tokens)], np.zeros((len(tokens), 8), np.float32))])
    rng = np.random.default_rng(41)
    texts = []
    for text in FIXED + list(random_texts(43, 400)):
        if rng.random() < 0.2:
            k = int(rng.integers(0, len(text) + 1))
            text = text[:k] + ["<|im_start|>", "<|im_end|>"][int(rng.integers(0, 2))] + text[k:]
        texts.append(text)
    want = ref_tokenize(ref_bin, str(tmp_path), "spm", tokens, scores, ttype, [], texts, bos=1, eos=2, unk=0)
    assert sum(len(w) for w in want) > 4 * len(texts) and any(259 <= i < 261 for w in want for i in w)
    got = ours_tokenize(lib, path, texts)
    bad = [(t, g, w) for t, g, w in zip(texts, got, want) if g != w]
    assert not bad, (len(bad), bad[:2])


# token types as GGUF stores them (llama_token_type): 0 undefined, 1 normal, 2 unknown, 3 control, 4 user-defined,
# 5 unused, 6 byte -- every one in both vocabularies, plus normal BPE tokens outside the byte map ("[UNK_BYTE_0x..]")
EXTRA = [("中文", 1), ("a中b", 1), ("<user>", 4), ("<unused0>", 5), ("<undef>", 0), ("<bpe_byte>", 6),
         ("<unk_t>", 2), ("▁x▁y", 1)]


def test_pieces_match_reference(ref_bin, lib, bpe_vocab, tmp_path):
    """detokenization pinned to the reference: every vocabulary id's streamed text (what generate() appends per
    token: llama_token_to_piece_impl with special = false, src/llama-vocab.cpp:2007-2077) equal, byte for byte,
    for a byte-level BPE and an SPM vocabulary holding every token type"""
    import gguf_writer as GW
    tokens, merges = bpe_vocab
    tokens = tokens + [t for t, _ in EXTRA]
    ttype = [3 if t in SPECIALS else 1 for t in bpe_vocab[0]] + [y for _, y in EXTRA]
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "gpt2", "tokenizer.ggml.pre": "llama-bpe",
          "tokenizer.ggml.tokens": (GW.STR, tokens), "tokenizer.ggml.token_type": (GW.I32, ttype),
          "tokenizer.ggml.merges": (GW.STR, [a + " " + b for a, b in merges])}
    path = str(tmp_path / "bpe.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(tokens)], np.zeros((len(tokens), 8), np.float32))])
    _, want = ref_run(ref_bin, str(tmp_path), "bpe llama-bpe", tokens, [0.0] * len(tokens), ttype, merges, [])
    assert any(w.startswith(b"[UNK_BYTE_0x") for w in want) and want[tokens.index("<user>")] == b"<user>"
    got = ours_pieces(lib, path, len(tokens))
    bad = [(i, tokens[i], g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:4])

    tokens, scores, ttype = _spm_vocab()
    tokens = tokens + [t for t, _ in EXTRA]
    ttype = ttype + [y for _, y in EXTRA]
    scores = scores + [-1e4] * len(EXTRA)
    kv = {"general.architecture": "llama", "tokenizer.ggml.model": "llama",
          "tokenizer.ggml.tokens": (GW.STR, tokens), "tokenizer.ggml.scores": (GW.F32, scores),
          "tokenizer.ggml.token_type": (GW.I32, ttype), "tokenizer.ggml.bos_token_id": 1,
          "tokenizer.ggml.eos_token_id": 2, "tokenizer.ggml.unknown_token_id": 0}
    path = str(tmp_path / "spm.gguf")
    GW.write(path, kv, [("token_embd.weight", 0, [8, len(tokens)], np.zeros((len(tokens), 8), np.float32))])
    _, want = ref_run(ref_bin, str(tmp_path), "spm", tokens, scores, ttype, [], [], bos=1, eos=2, unk=0)
    assert want[3 + 0x41] == b"A" and want[tokens.index("\u2581x\u2581y")] == b" x y"
    got = ours_pieces(lib, path, len(tokens))
    bad = [(i, tokens[i], g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[:4])
