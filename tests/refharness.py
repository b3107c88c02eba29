"""TEST INFRASTRUCTURE: ctypes access to the C restatement (oracle/liboracle.so) and a
driver for the reference-ggml harness (oracle/_ref/ref_llama).  Only tests/, smoke() and
bench.py's cpu_baseline leg use this module."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_llama")
REF_BIN_SCALAR = os.path.join(ROOT, "oracle", "_ref", "scalar", "ref_llama")   # no-SIMD build (make ref_scalar)

# ggml_type ids (ggml/include/ggml.h:364-399)
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1, Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 2, 3, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15
IQ4_NL, IQ4_XS = 20, 23
IQ2_XXS, IQ2_XS, IQ3_XXS, IQ1_S, IQ3_S, IQ2_S, IQ1_M = 16, 17, 18, 19, 21, 22, 29
BLOCK = {F32: (1, 4), F16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22), Q5_1: (32, 24), Q8_0: (32, 34), Q8_1: (32, 36), Q2_K: (256, 84), Q3_K: (256, 110), Q4_K: (256, 144),
         Q5_K: (256, 176), Q6_K: (256, 210), Q8_K: (256, 292), IQ4_NL: (32, 18), IQ4_XS: (256, 136),
         IQ2_XXS: (256, 66), IQ2_XS: (256, 74), IQ2_S: (256, 82), IQ3_XXS: (256, 98), IQ3_S: (256, 110),
         IQ1_S: (256, 50), IQ1_M: (256, 56)}
# the grid types (ggml-common.h:340-405): name -> type id
IQ_GRID = {"iq2_xxs": IQ2_XXS, "iq2_xs": IQ2_XS, "iq2_s": IQ2_S, "iq3_xxs": IQ3_XXS, "iq3_s": IQ3_S,
           "iq1_s": IQ1_S, "iq1_m": IQ1_M}


def row_bytes(t, k):
    e, b = BLOCK[t]
    return k // e * b


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "all"])
        L = ctypes.CDLL(ORACLE_SO)
        P, I, I64, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
        L.orc_dequantize_row.argtypes = [I, P, P, I64]
        L.orc_quantize_row.argtypes = [I, P, P, I64]
        L.orc_vec_dot.argtypes = [I, I, P, P]
        L.orc_vec_dot.restype = F
        L.orc_vec_dot_type.argtypes = [I]
        L.orc_mul_mat.argtypes = [I, P, I64, I64, P, I64, P, I]
        L.orc_rms_norm.argtypes = [P, P, P, I64, I64, F]
        L.orc_rope.argtypes = [P, P, I64, I64, I64, P, I, F, F, P, F, F, F, F, I]
        L.orc_flash_attn_ext.argtypes = [P, P, P, I64, P, P, I, I, I, I, I, F, I]
        L.orc_synth_fill.argtypes = [I, ctypes.c_uint64, ctypes.c_uint64, I64, P]
        L.orc_llama_create.argtypes = [P, P, P, I]
        L.orc_llama_create.restype = P
        L.orc_llama_free.argtypes = [P]
        L.orc_llama_eval.argtypes = [P, P, I, I, P]
        L.orc_llama_last_hidden.argtypes = [P, P]
        L.orc_llama_set_kv_types.argtypes = [P, I, I]
        L.orc_flash_attn_ext_q.argtypes = [P, P, P, I64, I64, I, I, P, P, I, I, I, I, I, F, I]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def synth(t, seed, tid, k, n):
    """Synthetic tensor bytes [n rows x k elems] of ggml type t (include/kcpp_synth.h)."""
    e, b = BLOCK[t]
    nbl = (k // e) * n
    out = np.empty(nbl * b, dtype=np.uint8)
    lib().orc_synth_fill(t, seed, tid, nbl, ptr(out))
    return out


def dequant(t, data, k):
    y = np.empty(k, dtype=np.float32)
    lib().orc_dequantize_row(t, ptr(np.ascontiguousarray(data)), ptr(y), k)
    return y


def quantize(vt, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(row_bytes(vt, x.size), dtype=np.uint8)
    lib().orc_quantize_row(vt, ptr(x), ptr(out), x.size)
    return out


def mul_mat(t, w, K, N, X, nthreads=0):
    X = np.ascontiguousarray(X, dtype=np.float32).reshape(-1, K)
    M = X.shape[0]
    dst = np.empty((M, N), dtype=np.float32)
    lib().orc_mul_mat(t, ptr(np.ascontiguousarray(w)), K, N, ptr(X), M, ptr(dst), nthreads)
    return dst


def rms_norm(x, w, eps):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    n = x.shape[-1]
    lib().orc_rms_norm(ptr(x), ptr(np.ascontiguousarray(w, dtype=np.float32)) if w is not None else None,
                       ptr(y), n, x.size // n, eps)
    return y


def rope(x, pos, base, freq_scale=1.0):
    """x [T][H][D] f32, NORM mode (adjacent pairs)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    T, H, D = x.shape
    y = np.empty_like(x)
    pos = np.ascontiguousarray(pos, dtype=np.int32)
    lib().orc_rope(ptr(x), ptr(y), D, H, T, ptr(pos), D, base, freq_scale, None, 0.0, 1.0, 32.0, 1.0, 4096)
    return y


def flash_attn(q, k, v, mask, nthreads=0):
    """q [T][H][D] f32; k,v [n_kv][HKV][D] f16 (uint16 view ok); mask [T][n_kv] f16 or None."""
    q = np.ascontiguousarray(q, dtype=np.float32)
    T, H, D = q.shape
    k = np.ascontiguousarray(k).view(np.uint16)
    v = np.ascontiguousarray(v).view(np.uint16)
    n_kv, HKV, _ = k.shape
    out = np.empty_like(q)
    m = ptr(np.ascontiguousarray(mask).view(np.uint16)) if mask is not None else None
    lib().orc_flash_attn_ext(ptr(q), ptr(k), ptr(v), HKV * D, m, ptr(out), D, T, H, n_kv, HKV,
                             1.0 / np.sqrt(D), nthreads)
    return out


class HParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n_vocab", "n_embd", "n_head", "n_head_kv", "n_layer", "n_ff", "n_ctx")] + \
               [(n, ctypes.c_float) for n in ("eps", "rope_base", "rope_freq_scale")] + \
               [(n, ctypes.c_int) for n in ("n_expert", "n_expert_used")]


def per_layer(hp):
    return 10 if hp.get("n_expert", 0) else 9


def weight_shapes(hp):
    """(K, N) per canonical weight index: tok_embd, output_norm, output, then 9 per layer (10 with MoE:
    + ffn_gate_inp [n_embd, n_expert]; the expert tensors' (K, N) is per expert slice)."""
    E, F, V = hp["n_embd"], hp["n_ff"], hp["n_vocab"]
    EKV = hp["n_head_kv"] * (E // hp["n_head"])
    s = [(E, V), (E, 1), (E, V)]
    for _ in range(hp["n_layer"]):
        s += [(E, 1), (E, E), (E, EKV), (E, EKV), (E, E), (E, 1), (E, F), (E, F), (F, E)]
        if hp.get("n_expert", 0):
            s += [(E, hp["n_expert"])]
    return s


def n_slices(hp, idx):
    """experts per tensor index (1 for dense tensors)"""
    if idx < 3 or not hp.get("n_expert", 0):
        return 1
    return hp["n_expert"] if (idx - 3) % 10 in (6, 7, 8) else 1


def synth_tensor(hp, t, seed, idx):
    """bytes of canonical tensor idx; expert e of an _exps tensor uses tid idx * 256 + e"""
    k, n = weight_shapes(hp)[idx]
    ns = n_slices(hp, idx)
    if ns == 1:
        return synth(t, seed, idx, k, n)
    return np.concatenate([synth(t, seed, idx * 256 + e, k, n) for e in range(ns)])


def flash_attn_q(q, k, v, ktype, vtype, mask, nthreads=0):
    """q [T][H][D] f32; k / v: uint8 [n_kv][row bytes] ggml block rows (Q8_0 / Q4_0) of HKV*D elements;
    mask [T][n_kv] f16 or None"""
    q = np.ascontiguousarray(q, dtype=np.float32)
    T, H, D = q.shape
    k, v = np.ascontiguousarray(k, dtype=np.uint8), np.ascontiguousarray(v, dtype=np.uint8)
    n_kv = k.shape[0]
    HKV = k.shape[1] // row_bytes(ktype, D)
    out = np.empty_like(q)
    m = ptr(np.ascontiguousarray(mask).view(np.uint16)) if mask is not None else None
    lib().orc_flash_attn_ext_q(ptr(q), ptr(k), ptr(v), k.shape[1], v.shape[1], ktype, vtype, m, ptr(out), D, T, H,
                               n_kv, HKV, np.float32(1) / np.sqrt(np.float32(D)), nthreads)
    return out


class OracleLlama:
    def __init__(self, hp, types, seed, nthreads=0, kv_types=None):
        self.hp = hp
        self.bufs = [synth_tensor(hp, t, seed, i) for i, t in enumerate(types)]
        arr = (ctypes.c_void_p * len(self.bufs))(*[b.ctypes.data for b in self.bufs])
        tarr = (ctypes.c_int * len(types))(*types)
        h = HParams(*[hp[n] for n in ("n_vocab", "n_embd", "n_head", "n_head_kv", "n_layer", "n_ff", "n_ctx")],
                    hp["eps"], hp["rope_base"], hp.get("rope_freq_scale", 1.0), hp.get("n_expert", 0),
                    hp.get("n_expert_used", 0))
        self._arr, self._tarr, self._h = arr, tarr, h
        self.m = lib().orc_llama_create(ctypes.byref(h), arr, tarr, nthreads)
        if kv_types is not None:
            assert lib().orc_llama_set_kv_types(self.m, *kv_types) == 0

    def eval(self, tokens, n_past):
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        logits = np.empty(self.hp["n_vocab"], dtype=np.float32)
        rc = lib().orc_llama_eval(self.m, ptr(tok), len(tok), n_past, ptr(logits))
        assert rc == 0
        return logits

    def __del__(self):
        if getattr(self, "m", None):
            lib().orc_llama_free(self.m)
            self.m = None


def ref_available():
    return os.path.exists(REF_BIN)


def run_ref_llama(hp, types, seed, prompt, n_gen, nthreads=4, ubatch=512, timeout=600, forced=None, hidden=False,
                  binary=None, skip_prefix=0, kshift=None, rope_freqs=None):
    """Run the reference ggml graph; returns (logits [1+n_gen, V], info dict).
    forced: decode these tokens (teacher forcing) instead of the greedy argmax.
    hidden: also return info["hidden"] = residual stream after layers 0..n_layer-2 of the prefill,
            [n_layer-1][n_prompt][n_embd] (single-ubatch prompts); MoE: info["router"] = those layers' router
            logits [n_layer-1][n_prompt][n_expert].
    binary: ref_llama build to run (default: the AVX2 build; REF_BIN_SCALAR for the scalar one).
    skip_prefix: the first skip_prefix prompt positions are taken as cached (zeroed K/V), not computed (timing only).
    kshift: (p0, diff) -- context shift after the prompt (the reference's seq_rm / seq_add + build_k_shift), the
            decode then continues at n_prompt - diff.
    rope_freqs: head_dim / 2 frequency factors (the model's rope_freqs.weight) fed to every rope and the K-shift."""
    import json
    with tempfile.TemporaryDirectory() as td:
        cfg = os.path.join(td, "cfg.txt")
        out = os.path.join(td, "logits.bin")
        hout = os.path.join(td, "hidden.bin")
        with open(cfg, "w") as f:
            f.write(" ".join(str(hp[n]) for n in ("n_vocab", "n_embd", "n_head", "n_head_kv", "n_layer", "n_ff", "n_ctx")))
            f.write(" %r %r %r %d %d %d\n" % (float(hp["eps"]), float(hp["rope_base"]), float(hp.get("rope_freq_scale", 1.0)),
                                             seed, hp.get("n_expert", 0), hp.get("n_expert_used", 0)))
            f.write(" ".join(map(str, types)) + "\n")
            f.write("%d %d %d %d\n" % (nthreads, len(prompt), n_gen, ubatch))
            f.write(" ".join(map(str, prompt)) + "\n" + out + "\n")
            fl = [int(t) for t in (forced if forced is not None else [])]
            f.write("%d %s\n" % (len(fl), " ".join(map(str, fl))))
            if hidden:
                f.write(hout + "\n")
        rff = ""
        if rope_freqs is not None:
            rff = os.path.join(td, "rope_freqs.bin")
            np.ascontiguousarray(rope_freqs, dtype=np.float32).tofile(rff)
        r = subprocess.run([binary or REF_BIN, "llama", cfg], capture_output=True, text=True, timeout=timeout,
                           env=dict(os.environ, OMP_NUM_THREADS=str(nthreads), REF_SKIP_PREFIX=str(skip_prefix),
                                    REF_KSHIFT="%d %d" % tuple(kshift) if kshift else "", REF_ROPE_FREQS=rff))
        if r.returncode != 0:
            raise RuntimeError("ref_llama failed: %s %s" % (r.returncode, r.stderr))
        info = json.loads(r.stdout.strip().splitlines()[-1])
        logits = np.fromfile(out, dtype=np.float32).reshape(-1, hp["n_vocab"])
        if hidden:
            info["hidden"] = np.fromfile(hout, dtype=np.float32).reshape(hp["n_layer"] - 1, len(prompt), hp["n_embd"])
            if hp.get("n_expert", 0):      # MoE: the router logits of the same layers
                info["router"] = np.fromfile(hout + ".router", dtype=np.float32).reshape(
                    hp["n_layer"] - 1, len(prompt), hp["n_expert"])
        return logits, info


def run_ref_op(op, inp_bytes, out_count, args, nthreads=4, dtype=np.float32):
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(inp_bytes)
        r = subprocess.run([REF_BIN, "op", op, fi, fo] + [str(a) for a in args], capture_output=True, text=True,
                           env=dict(os.environ, REF_THREADS=str(nthreads)))
        if r.returncode != 0:
            raise RuntimeError("ref op %s failed rc=%s %s" % (op, r.returncode, r.stderr))
        return np.fromfile(fo, dtype=dtype)[:out_count]


TINY = dict(n_vocab=512, n_embd=512, n_head=4, n_head_kv=1, n_layer=2, n_ff=1024, n_ctx=256,
            eps=1e-5, rope_base=500000.0)


def llama31_rope_freqs(base, dim, factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0, old_context_len=8192):
    """rope_freqs.weight as the reference's converter writes it for rope_type "llama3" (Llama-3.1 / 3.2;
    convert_hf_to_gguf.py:1622-1650, generate_extra_tensors)"""
    import math
    freqs = 1.0 / (np.float32(base) ** (np.arange(0, dim, 2, dtype=np.float32) / np.float32(dim)))
    low_wl, high_wl = old_context_len / low_freq_factor, old_context_len / high_freq_factor
    out = []
    for f in freqs.astype(np.float64):
        wl = 2 * math.pi / f
        if wl < high_wl:
            out.append(1.0)
        elif wl > low_wl:
            out.append(factor)
        else:
            smooth = (old_context_len / wl - low_freq_factor) / (high_freq_factor - low_freq_factor)
            out.append(1 / ((1 - smooth) / factor + smooth))
    return np.array(out, np.float32)


# Mixtral-style tiny MoE (4 experts, top-2): BASELINE config 5's structure at test size
TINY_MOE = dict(TINY, n_expert=4, n_expert_used=2)


def moe_types(n_layer, t=Q5_K, router=F16):
    """Q5_K_M-like MoE mix: Q5_K everywhere, Q6_K ffn_down_exps on the 'more bits' layers, F16 router"""
    ty = [Q4_K, F32, Q6_K]
    for il in range(n_layer):
        more = il < n_layer // 8 or il >= 7 * n_layer // 8 or (il - n_layer // 8) % 3 == 2
        ty += [F32, t, t, t, t, F32, t, t, Q6_K if more else t, router]
    return ty


def mixtral_q5_k_m_types(n_layer):
    """Q5_K_M policy for an 8-expert model (src/llama.cpp:17986-18157): Q5_K default (token_embd too),
    Q8_0 attn_k / attn_v (n_expert == 8), Q6_K ffn_down_exps on the 'more bits' layers, Q6_K output,
    F32 router (ffn_gate_inp is never quantized)"""
    ty = [Q5_K, F32, Q6_K]
    for il in range(n_layer):
        more = il < n_layer // 8 or il >= 7 * n_layer // 8 or (il - n_layer // 8) % 3 == 2
        ty += [F32, Q5_K, Q8_0, Q8_0, Q5_K, F32, Q5_K, Q5_K, Q6_K if more else Q5_K, F32]
    return ty


def q2_k_types(n_layer):
    """Q2_K-like per-tensor policy (llama_tensor_get_type for LLAMA_FTYPE_MOSTLY_Q2_K, src/llama.cpp:17979-18208):
    Q2_K by default (token_embd too), output Q6_K, attn_v / attn_output / ffn_down Q3_K"""
    types = [Q2_K, F32, Q6_K]
    for _ in range(n_layer):
        types += [F32, Q2_K, Q2_K, Q3_K, Q3_K, F32, Q2_K, Q2_K, Q3_K]
    return types


def q5_0_types(n_layer):
    """LLAMA_FTYPE_MOSTLY_Q5_0 (llama_tensor_get_type, src/llama.cpp:17979-18208): Q5_0 everywhere (token_embd too),
    output Q6_K"""
    return uniform_types(n_layer, Q5_0, Q6_K)


def q4_1_types(n_layer):
    """LLAMA_FTYPE_MOSTLY_Q4_1: Q4_1 everywhere, output Q6_K"""
    return uniform_types(n_layer, Q4_1, Q6_K)


def iq4_nl_types(n_layer):
    """LLAMA_FTYPE_MOSTLY_IQ4_NL (src/llama.cpp llama_model_quantize_internal): IQ4_NL everywhere, output Q6_K"""
    return uniform_types(n_layer, IQ4_NL, Q6_K)


def iq4_xs_types(n_layer):
    """LLAMA_FTYPE_MOSTLY_IQ4_XS: IQ4_XS everywhere, output Q6_K"""
    return uniform_types(n_layer, IQ4_XS, Q6_K)


def iq_grid_types(n_layer, t):
    """a grid-type file (LLAMA_FTYPE_MOSTLY_IQ2_XXS .. IQ1_M): the type everywhere, output Q6_K"""
    return uniform_types(n_layer, t, Q6_K)


def q5_1_types(n_layer):
    """LLAMA_FTYPE_MOSTLY_Q5_1: Q5_1 everywhere, output Q6_K"""
    return uniform_types(n_layer, Q5_1, Q6_K)


def q3_k_m_types(n_layer):
    """Q3_K_M per-tensor policy (llama_tensor_get_type, src/llama.cpp:17979-18208): Q3_K by default (token_embd
    too), output Q6_K, attn_v Q5_K on the first two layers else Q4_K, attn_output Q4_K, ffn_down Q5_K below
    n_layer / 16, Q4_K on the 'more bits' layers, else Q3_K"""
    types = [Q3_K, F32, Q6_K]
    for i in range(n_layer):
        more = i < n_layer // 8 or i >= 7 * n_layer // 8 or (i - n_layer // 8) % 3 == 2
        v = Q5_K if i < 2 else Q4_K
        down = Q5_K if i < n_layer // 16 else (Q4_K if more else Q3_K)
        types += [F32, Q3_K, Q3_K, v, Q4_K, F32, Q3_K, Q3_K, down]
    return types


def q4_k_m_types(n_layer, tok=Q4_K, out=Q6_K):
    """Q4_K_M per-tensor policy (src/llama.cpp:17986-18157): Q6_K for attn_v/ffn_down on 'more bits'
    layers (i<L/8, i>=7L/8, (i-L/8)%3==2), output Q6_K, everything else Q4_K."""
    types = [tok, F32, out]
    for i in range(n_layer):
        more = i < n_layer // 8 or i >= 7 * n_layer // 8 or (i - n_layer // 8) % 3 == 2
        v = Q6_K if more else Q4_K
        types += [F32, Q4_K, Q4_K, v, Q4_K, F32, Q4_K, Q4_K, v]
    return types


def uniform_types(n_layer, t, out=None):
    types = [t, F32, out if out is not None else t]
    for _ in range(n_layer):
        types += [F32, t, t, t, t, F32, t, t, t]
    return types
