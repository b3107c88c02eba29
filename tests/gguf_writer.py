"""Minimal GGUF v3 writer for test models (own implementation of the published layout: header, typed
key/values, tensor directory, 32-byte aligned data).  Used to build small synthetic Llama files whose
weights equal the runtime's synthetic weights (refharness.synth), so a model loaded through the
koboldcpp ABI can be checked against the same model built in-process."""
import struct

import numpy as np

U32, I32, F32, BOOL, STR, ARR, U64 = 4, 5, 6, 7, 8, 9, 10

# SentencePiece merges only through pieces that exist: every word has its whole prefix chain
WORDS = ["▁h", "▁he", "▁hel", "▁hell", "▁hello", "▁w", "▁wo", "▁wor", "▁worl", "▁world", "▁t", "▁th", "▁the",
         "a", "b", "ab", "▁a", "▁b", "▁of", "▁to"]


def _s(x):
    b = x.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _val(v):
    if isinstance(v, bool):
        return struct.pack("<I", BOOL) + struct.pack("<B", int(v))
    if isinstance(v, int):
        return struct.pack("<I", U32) + struct.pack("<I", v)
    if isinstance(v, float):
        return struct.pack("<I", F32) + struct.pack("<f", v)
    if isinstance(v, str):
        return struct.pack("<I", STR) + _s(v)
    if isinstance(v, tuple):                       # (elem_type, list)
        et, items = v
        out = [struct.pack("<I", ARR) + struct.pack("<IQ", et, len(items))]
        if et == STR:
            out += [_s(it) for it in items]
        elif et == F32:
            out.append(struct.pack("<%df" % len(items), *items))
        elif et == I32:
            out.append(struct.pack("<%di" % len(items), *items))
        else:
            raise ValueError(et)
        return b"".join(out)
    raise ValueError(type(v))


def _len(data):
    return data if isinstance(data, int) else memoryview(data).nbytes


def write(path, kv, tensors, align=32):
    """kv: dict key -> value (int -> u32, float -> f32, str, bool, (type, list));
    tensors: list of (name, ggml_type, ne list, bytes -- or an int: that many zero bytes, left as a hole of a sparse
    file, so a full-size model costs no disk and no write time)"""
    parts = [b"GGUF" + struct.pack("<IQQ", 3, len(tensors), len(kv))]
    for k, v in kv.items():
        parts.append(_s(k) + _val(v))
    off = 0
    offs = []
    for name, t, ne, data in tensors:
        offs.append(off)
        off += (_len(data) + align - 1) // align * align
    for (name, t, ne, data), o in zip(tensors, offs):
        parts.append(_s(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", n) for n in ne))
        parts.append(struct.pack("<IQ", t, o))
    head = b"".join(parts)
    pad = (-len(head)) % align
    with open(path, "wb") as f:
        f.write(head + b"\0" * pad)
        base = f.tell()
        for (name, t, ne, data), o in zip(tensors, offs):
            if isinstance(data, int):
                f.seek(base + o + (data + align - 1) // align * align)
            else:
                f.seek(base + o)
                f.write(bytes(data))
                f.write(b"\0" * ((-_len(data)) % align))
        f.truncate(base + off)


def spm_vocab(n_vocab, words):
    """<unk>, <s>, </s>, 256 byte tokens, then the given pieces (scored by order), padded with
    unused tokens up to n_vocab.  Returns (tokens, scores, types)."""
    toks = ["<unk>", "<s>", "</s>"] + ["<0x%02X>" % b for b in range(256)]
    types = [2, 3, 3] + [6] * 256
    scores = [0.0, 0.0, 0.0] + [0.0] * 256
    for i, w in enumerate(words):
        toks.append(w)
        types.append(1)
        scores.append(-float(i))
    while len(toks) < n_vocab:
        toks.append("<unused%d>" % len(toks))
        types.append(5)
        scores.append(-1e9)
    return toks[:n_vocab], scores[:n_vocab], types[:n_vocab]


LAYER_NAMES = ["attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "ffn_norm", "ffn_gate", "ffn_up", "ffn_down"]


def llama_gguf(path, hp, types, seed, words, split_experts=False, kv_extra=None, rope_freqs=None, sparse=False):
    """Llama GGUF with the runtime's synthetic weights.  MoE (hp["n_expert"]): gate/up/down as 3-D
    blk.N.ffn_*_exps tensors [k, n, n_expert] plus blk.N.ffn_gate_inp, or with split_experts the older
    per-expert blk.N.ffn_gate.E tensors (both accepted by llm_load_tensors, src/llama.cpp:7176-7215).
    sparse: every tensor's data left as zeros in a sparse file (bench.py's full-size generate() leg: the weights are
    then synthesized on the device, kcpp_expose_synth_weights)."""
    import refharness as R
    toks, scores, ttypes = spm_vocab(hp["n_vocab"], words)
    kv = {
        "general.architecture": "llama",
        "general.alignment": 32,
        "llama.context_length": int(hp["n_ctx"]),
        "llama.embedding_length": int(hp["n_embd"]),
        "llama.block_count": int(hp["n_layer"]),
        "llama.feed_forward_length": int(hp["n_ff"]),
        "llama.attention.head_count": int(hp["n_head"]),
        "llama.attention.head_count_kv": int(hp["n_head_kv"]),
        "llama.attention.layer_norm_rms_epsilon": float(hp["eps"]),
        "llama.rope.freq_base": float(hp["rope_base"]),
        "tokenizer.ggml.model": "llama",
        "tokenizer.ggml.tokens": (STR, toks),
        "tokenizer.ggml.scores": (F32, scores),
        "tokenizer.ggml.token_type": (I32, ttypes),
        "tokenizer.ggml.bos_token_id": 1,
        "tokenizer.ggml.eos_token_id": 2,
    }
    if kv_extra:
        kv.update(kv_extra)
    ne_ = int(hp.get("n_expert", 0))
    if ne_:
        kv["llama.expert_count"] = ne_
        kv["llama.expert_used_count"] = int(hp["n_expert_used"])
    names = ["token_embd.weight", "output_norm.weight", "output.weight"]
    for il in range(hp["n_layer"]):
        if ne_:
            names += ["blk.%d.%s.weight" % (il, n) for n in LAYER_NAMES[:6]]
            names += ["blk.%d.%s_exps.weight" % (il, n) for n in LAYER_NAMES[6:]]
            names += ["blk.%d.ffn_gate_inp.weight" % il]
        else:
            names += ["blk.%d.%s.weight" % (il, n) for n in LAYER_NAMES]
    tensors = []
    for idx, ((k, n), t) in enumerate(zip(R.weight_shapes(hp), types)):
        ns = R.n_slices(hp, idx)
        if sparse:
            ne = [k] if n == 1 else ([k, n] if ns == 1 else [k, n, ns])
            tensors.append((names[idx], t, ne, R.row_bytes(t, k) * n * ns))
            continue
        if ns == 1:
            data = R.synth(t, seed, idx, k, n)
            ne = [k] if n == 1 else [k, n]
            tensors.append((names[idx], t, ne, np.ascontiguousarray(data).tobytes()))
        elif split_experts:
            base = names[idx].replace("_exps.weight", "")
            for e in range(ns):
                data = R.synth(t, seed, idx * 256 + e, k, n)
                tensors.append(("%s.%d.weight" % (base, e), t, [k, n], np.ascontiguousarray(data).tobytes()))
        else:
            data = R.synth_tensor(hp, t, seed, idx)
            tensors.append((names[idx], t, [k, n, ns], np.ascontiguousarray(data).tobytes()))
    if rope_freqs is not None:      # rope_freqs.weight (Llama-3.1 / 3.2), F32 [head_dim / 2]
        rf = np.ascontiguousarray(rope_freqs, dtype=np.float32)
        tensors.append(("rope_freqs.weight", R.F32, [len(rf)], rf.tobytes()))
    write(path, kv, tensors)
    return toks
