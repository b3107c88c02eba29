"""ctypes binding of koboldcpp_hipblas.so (include/kcpp_mi355x.h).

Host-side mirror of the reference's operator interface for this path: the same ggml type ids,
the same op semantics (mul_mat / rms_norm / rope_ext / flash_attn_ext) and the same error
behaviour (a non-zero return is raised as KcppError instead of aborting the process).
Fails loudly when the native library is absent -- there is no Python/CPU fallback.
"""
import ctypes
import os

from . import LIB_PATH

F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1, Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 2, 3, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15
IQ4_NL, IQ4_XS = 20, 23
# device-internal row-major decode layouts of Q4_K / Q6_K (include/kcpp_synth.h; never ggml ids)
Q4_K_RS, Q5_K_RS, Q6_K_RS = 112, 113, 114
# device-internal Q8_0 tile layout and its activation layout (kcpp_common.h, csrc/gemm_q80t.hip)
Q8_0_T, Q8_0_TA = 115, 116
BLOCK = {F32: (1, 4), F16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22), Q5_1: (32, 24), Q8_0: (32, 34), Q8_1: (32, 36), Q2_K: (256, 84), Q3_K: (256, 110), Q4_K: (256, 144),
         Q5_K: (256, 176), Q6_K: (256, 210), Q8_K: (256, 292), Q4_K_RS: (256, 144), Q5_K_RS: (256, 176), Q6_K_RS: (256, 210),
         IQ4_NL: (32, 18), IQ4_XS: (256, 136), Q8_0_T: (32, 34)}
# the lattice-grid types (ggml-common.h:340-405), kept in the ggml layout on the device (csrc/iq_grid.h)
IQ2_XXS, IQ2_XS, IQ3_XXS, IQ1_S, IQ3_S, IQ2_S, IQ1_M = 16, 17, 18, 19, 21, 22, 29
BLOCK.update({IQ2_XXS: (256, 66), IQ2_XS: (256, 74), IQ2_S: (256, 82), IQ3_XXS: (256, 98), IQ3_S: (256, 110),
              IQ1_S: (256, 50), IQ1_M: (256, 56)})


class KcppError(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError("native library missing: %s (run __graft_entry__.build())" % LIB_PATH)

_L = ctypes.CDLL(LIB_PATH)
P, I, I64, U64, Fl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float

_SIGS = {
    "kcpp_weight_repack": [I, P, P, I64, I64, I, P],
    "kcpp_weight_synth": [I, U64, U64, P, I64, I64, P],
    "kcpp_dequantize": [I, P, P, I64, I64, P],
    "kcpp_get_rows": [I, P, I64, I64, P, I64, P, I64, P],
    "kcpp_quantize_act": [I, P, I64, P, I64, I64, P],
    "kcpp_quantize_act_glu": [P, I64, I64, P, I64, I64, P],
    "kcpp_gemv": [I, P, P, I64, I64, P, I64, P, I64, P, I64, I, P],
    "kcpp_gemm": [I, P, P, I64, I64, P, I64, P, I64, P, I64, I, P, P],
    "kcpp_q6p_image_bytes": [I64, I64],
    "kcpp_gemm_rms_norm": [I, P, I64, I64, P, I64, P, I64, P, I64, P, P, P, Fl, P],
    "kcpp_gemm_q6p_rms_norm": [P, P, I64, I64, P, I64, P, I64, P, I64, P, P, P, Fl, P],
    "kcpp_reduce_rms_norm": [P, I, I64, P, I64, P, I64, P, P, I64, I64, Fl, P],
    "kcpp_q6p_build": [P, I64, I64, P, P],
    "kcpp_gemm_q6p": [P, P, P, P, I64, I64, P, I64, P, I64, P, I64, I, P, P],
    "kcpp_rms_norm": [P, I64, P, P, I64, P, I64, I64, Fl, P],
    "kcpp_rms_norm_q80": [P, I64, P, P, I64, I64, Fl, P],
    "kcpp_gemm_q80_glu_q80": [P, P, I64, I64, P, I64, P, P, P],
    "kcpp_rope_table": [P, I, I, Fl, Fl, P, Fl, Fl, Fl, Fl, I],
    "kcpp_rope_row": [P, I, I, Fl, Fl, Fl, Fl, Fl, Fl, I],
    "kcpp_kv_shift_rows": [P, P, P, P, I64, I, P, P],
    "kcpp_moe_route_norm": [P, I64, P, Fl, P, I, I64, I, I, P, P, I, P],
    "kcpp_model_kv_shift": [P, I, I, I],
    "kcpp_rope_kv": [P, I64, P, P, P, P, I, I, I, I, I, P, P, P],
    "kcpp_flash_attn": [P, P, P, P, P, P, I, I, I, I, I, P, I, Fl, I, P],
    "kcpp_flash_attn_prefill_mfma": [P, P, P, P, I, I, I, I, I, Fl, P],
    "kcpp_flash_attn_prefill_mfma_ex": [P, P, P, P, P, P, I, I, I, I, I, Fl, P],
    "kcpp_fa_split_ws_bytes": [I],
    "kcpp_flash_attn_dec_ta": [P, P, P, P, P, P, I, I, I, I, P, I, Fl, P],
    "kcpp_fa_decode_ex": [P, P, P, I64, I64, P, P, P, I, I, I, P, I, Fl, I, P],
    "kcpp_fa_set_stamps": [P],
    "kcpp_gguf_check": [ctypes.c_char_p, ctypes.c_char_p, I],
    "kcpp_pretokenize": [ctypes.c_char_p, ctypes.c_char_p, P, I],
    "kcpp_tokenize_probe": [ctypes.c_char_p, ctypes.c_char_p, I, P, I],
    "kcpp_pieces_probe": [ctypes.c_char_p, P, I64, P, I],
    "kcpp_tokenizer_special_ids": [ctypes.c_char_p, P],
    "kcpp_engine_bench": [P, P, I, I, P, U64, I, I, I, I, P],
    "kcpp_expose_synth_weights": [U64],
    "kcpp_gemm_q80t": [P, P, I, P, I64, P, I64, P, I64, P, I64, I, P, P, P],
    "kcpp_gemm_q80t_qkv_rope": [P, P, I64, P, I64, P, I, P, I, P, P, P, P, P],
    "kcpp_rms_norm_q80t": [P, I64, P, P, I64, I64, Fl, P],
    "kcpp_q80t_ws_bytes": [I64, I64, I64],
    "kcpp_pipeline_trace": [I, I, I, I, I, ctypes.c_char_p, I],
    "kcpp_split_layers": [I, I, P, P],
    "kcpp_model_argmax_async": [P],
    "kcpp_model_step_dev": [P, I],
    "kcpp_add": [P, P, P, I64, P],
    "kcpp_silu_mul": [P, P, P, I64, P],
    "kcpp_moe_route": [P, I64, P, I, I64, I, I, P, P, I, P],
    "kcpp_moe_gather": [P, I64, P, I, I64, P, P],
    "kcpp_moe_scatter": [P, I64, P, P, P, I, I64, P],
    "kcpp_moe_combine": [P, P, I64, I, I64, P],
    "kcpp_ggml_binary": [I, P, P, P, P, P, P, P],
    "kcpp_ggml_unary": [I, P, P, P, P, Fl, P],
    "kcpp_ggml_cpy": [I, P, P, I, P, P, P],
    "kcpp_ggml_rms_norm": [P, P, P, P, Fl, P],
    "kcpp_ggml_rms_norm_mul": [P, P, P, P, P, P, P, P, Fl, P],
    "kcpp_ggml_rope": [P, P, P, P, P, P, I, I, I, Fl, Fl, Fl, Fl, Fl, Fl, P],
    "kcpp_ggml_rope_f16": [P, P, P, P, P, P, P, I, I, I, Fl, Fl, Fl, Fl, Fl, Fl, P],
    "kcpp_ggml_soft_max": [P, P, P, I, I64, I64, P, P, Fl, P],
    "kcpp_ggml_argsort": [P, P, P, I64, I, P],
    "kcpp_ggml_sum_rows": [P, P, P, P, P],
    "kcpp_ggml_get_rows": [I, P, P, P, P, P, P, P],
    "kcpp_ggml_mul_mat_f": [I, P, P, P, P, P, P, P],
    "kcpp_flash_attn_ext": [P, I64, I64, P, P, P, I64, P, P, I, I, I, I, I, Fl, P],
    "kcpp_model_create": [P, P, I, I, I, I, I, I],
    "kcpp_model_synth_weights": [P, U64],
    "kcpp_model_set_tensor": [P, I, P, I64],
    "kcpp_model_free": [P],
    "kcpp_model_decode": [P, P, I, I, P],
    "kcpp_model_decode_async": [P, P, I, I],
    "kcpp_model_device": [P],
    "kcpp_model_hidden": [P],
    "kcpp_model_read_hidden": [P, P, I64, I64],
    "kcpp_model_stream": [P],
    "kcpp_model_hidden_io": [P, P, I64, I64, I],
    "kcpp_model_sync": [P],
    "kcpp_model_read_logits": [P, P],
    "kcpp_model_forward_hidden": [P, I, I],
    "kcpp_model_argmax": [P, P],
    "kcpp_model_decode_greedy": [P, I, P],
    "kcpp_model_decode_greedy_lagged": [P, I, P],
    "kcpp_model_greedy_drain": [P, P],
    "kcpp_model_set_graphs": [P, I],
    "kcpp_model_set_fused_decode": [P, I],
    "kcpp_model_set_row_split": [P, I, P, P],
    "kcpp_row_split_range": [I64, I, P, I, P, P],
    "kcpp_model_set_fa_exact": [P, I],
    "kcpp_model_set_rope_freqs": [P, P, I],
    "kcpp_gradient_ai_rope_base": [Fl, I, I, I],
    "kcpp_model_moe_ids": [P, P, I],
    "kcpp_model_moe_trace": [P, I],
    "kcpp_model_moe_trace_read": [P, P, I],
    "kcpp_model_set_fused_route": [P, I],
    "kcpp_model_fused_route_count": [P],
    "kcpp_model_set_moe_grouped": [P, I],
    "kcpp_model_moe_grouped_count": [P],
    "kcpp_gemm_grouped": [I, P, P, I64, I64, I64, P, I64, P, P, I, P, P, I, P, P],
    "kcpp_gemm_grouped_ws_bytes": [I, I64, I64, I],
    "kcpp_flash_attn_exact": [P, P, P, P, I, I, I, I, I, P, Fl, P],
    "kcpp_model_weight_bytes": [P],
    "kcpp_model_set_kv_types": [P, I, I],
    "kcpp_rope_qk_inplace": [P, I64, I, I, I, I, I, P, P, P],
    "kcpp_kv_store_q": [I, I, P, I64, I64, I64, I, I64, P, P, I64, I, P, P],
    "kcpp_flash_attn_q": [I, I, P, I64, P, P, P, I, I, I, I, I64, I, P, Fl, P],
}
_RES = {"kcpp_gradient_ai_rope_base": Fl, "kcpp_q6p_image_bytes": I64, "kcpp_model_fused_route_count": I64, "kcpp_model_moe_grouped_count": I64, "kcpp_gemm_grouped_ws_bytes": I64, "kcpp_fa_split_ws_bytes": I64, "kcpp_q80t_ws_bytes": I64, "kcpp_act_bytes": I64, "kcpp_fa_ext_workspace_bytes": I64, "kcpp_fa_workspace_bytes": I64, "kcpp_gemm_workspace_bytes": I64,
        "kcpp_model_create": P, "kcpp_model_hidden": P, "kcpp_model_stream": P, "kcpp_model_weight_bytes": I64,
        "kcpp_last_error": ctypes.c_char_p, "kcpp_model_free": None, "kcpp_fa_set_stamps": None}
_L.kcpp_act_bytes.argtypes = [I, I64, I64]
_L.kcpp_kv_cache_bytes.argtypes = [I, I64, I64]
_L.kcpp_kv_cache_bytes.restype = I64
_L.kcpp_fa_workspace_bytes.argtypes = [I, I, I]
_L.kcpp_fa_ext_workspace_bytes.argtypes = [I, I, I, I]
_L.kcpp_gemm_workspace_bytes.argtypes = [I, I64, I64, I64]
_L.kcpp_vec_dot_type.argtypes = [I]
_L.kcpp_gemv_dec.argtypes = [I, P, I, I, I, P]
_L.kcpp_gemv_dec_args_size.restype = I64
_L.kcpp_gemv_stream.argtypes = [I, P, I, I, P]
_L.kcpp_gemv_q4k.argtypes = [P, I, I, P]
_L.kcpp_gemv_rs.argtypes = [I, P, I, I, P]
_L.kcpp_rs_supported.argtypes = [I, I64]
for _n, _a in _SIGS.items():
    getattr(_L, _n).argtypes = _a
for _n, _r in _RES.items():
    getattr(_L, _n).restype = _r


def exported_symbols():
    return sorted(set(_SIGS) | set(_RES) | {"kcpp_vec_dot_type", "kcpp_gemv_dec", "kcpp_gemv_dec_args_size",
                                             "kcpp_gemv_stream", "kcpp_gemv_q4k",
                                             "kcpp_gemv_rs", "kcpp_rs_supported"})


def raw():
    return _L


def _chk(rc, name):
    if rc != 0:
        raise KcppError("%s failed rc=%d: %s" % (name, rc, (_L.kcpp_last_error() or b"").decode()))


def call(name, *args):
    _chk(getattr(_L, name)(*args), name)


def row_bytes(t, k):
    e, b = BLOCK[t]
    return k // e * b


def act_bytes(wtype, K, M):
    return int(_L.kcpp_act_bytes(wtype, K, M))


def vec_dot_type(wtype):
    return int(_L.kcpp_vec_dot_type(wtype))


def fa_workspace_bytes(T, H, n_kv):
    return int(_L.kcpp_fa_workspace_bytes(T, H, n_kv))


class TDesc(ctypes.Structure):
    """struct kcpp_tdesc: ggml shape ne[4] and byte strides nb[4] (innermost first)"""
    _fields_ = [("ne", I64 * 4), ("nb", I64 * 4)]


def tdesc(t):
    """kcpp_tdesc of a torch tensor (any strides): ne/nb are the reversed shape/strides, in bytes"""
    shape, strides = list(t.shape)[::-1], [s * t.element_size() for s in t.stride()][::-1]
    while len(shape) < 4:
        shape.append(1)
        strides.append(strides[-1] * shape[-2] if strides else t.element_size())
    d = TDesc()
    for i in range(4):
        d.ne[i], d.nb[i] = int(shape[i]), int(strides[i])
    return d


def fa_ext_workspace_bytes(T, H, n_kv, D=128):
    return int(_L.kcpp_fa_ext_workspace_bytes(T, H, n_kv, D))


class DecArgs(ctypes.Structure):
    """mirror of struct DecArgs (koboldcpp_amd/csrc/kcpp_internal.h), checked against
    kcpp_gemv_dec_args_size() at import"""
    _fields_ = [("W", P * 3), ("Y", P * 3), ("N", I64 * 3), ("role", I * 3), ("nseg", I), ("W2", P), ("K", I64),
                ("act", P), ("x", P), ("nw", P), ("eps", Fl), ("res", P), ("q16", P), ("kc", P), ("vc", P),
                ("ekv", I64), ("D", I), ("pos", P), ("rope_tab", P), ("eid", P), ("ebytes", I64), ("escale", P),
                ("act_mtot", I64), ("act_col", I64), ("n_exp", I64), ("pre", P), ("eid1", P),
                ("route_w", P), ("route_wt", I), ("route_ne", I), ("route_ids", P), ("route_wts", P)]


if ctypes.sizeof(DecArgs) != _L.kcpp_gemv_dec_args_size():
    raise ImportError("DecArgs layout mismatch: %d vs %d" % (ctypes.sizeof(DecArgs), _L.kcpp_gemv_dec_args_size()))


def gemv_dec(wtype, args, mode, pro, rows_per_wave, stream):
    """fused single-token mat-vec; returns the native rc (-8 = K too large for the fused kernel)"""
    return int(_L.kcpp_gemv_dec(wtype, ctypes.byref(args), mode, pro, rows_per_wave, stream))


class HParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n_vocab", "n_embd", "n_head", "n_head_kv", "n_layer", "n_ff", "n_ctx")] + \
               [(n, ctypes.c_float) for n in ("eps", "rope_base", "rope_freq_scale")] + \
               [(n, ctypes.c_int) for n in ("n_expert", "n_expert_used")]


def hparams(hp):
    return HParams(*[int(hp[n]) for n in ("n_vocab", "n_embd", "n_head", "n_head_kv", "n_layer", "n_ff", "n_ctx")],
                   float(hp["eps"]), float(hp["rope_base"]), float(hp.get("rope_freq_scale", 1.0)),
                   int(hp.get("n_expert", 0)), int(hp.get("n_expert_used", 0)))


def engine_bench(hp, types, n_dev, n_prompt, ubatch, n_warm, n_steps, seed=1234, tensor_split=None):
    """the drop-in engine (load_model's layer-split stages over n_dev GPUs, RCCL / copy hand-off, greedy tokens moved
    home on device) on synthetic weights: {prefill_s, decode_s, n_past, rccl}"""
    h = hparams(hp)
    t = (ctypes.c_int * len(types))(*types)
    ts = (ctypes.c_float * 16)(*((tensor_split or [1.0] * n_dev) + [0.0] * (16 - n_dev)))
    out = (ctypes.c_double * 4)()
    _chk(_L.kcpp_engine_bench(ctypes.byref(h), t, len(types), n_dev, ts, seed, n_prompt, ubatch, n_warm, n_steps, out),
         "engine_bench")
    return {"prefill_s": out[0], "decode_s": out[1], "n_past": int(out[2]), "rccl": bool(out[3])}


class Model:
    """One pipeline stage of a Llama model on one GPU (kcpp_model_*)."""

    def __init__(self, hp, types, device=0, il0=0, il1=None, has_embed=True, has_output=True, max_ubatch=512):
        self.hp = dict(hp)
        self._h = hparams(hp)
        self._t = (ctypes.c_int * len(types))(*types)
        il1 = hp["n_layer"] if il1 is None else il1
        self.m = _L.kcpp_model_create(ctypes.byref(self._h), self._t, device, il0, il1, int(has_embed),
                                      int(has_output), max_ubatch)
        if not self.m:
            raise KcppError("kcpp_model_create failed: %s" % (_L.kcpp_last_error() or b"").decode())

    def kv_shift(self, p0, diff, n_past):
        """context shift: cache rows [p0+diff, n_past) -> [p0, n_past-diff), K re-rotated by -diff"""
        _chk(_L.kcpp_model_kv_shift(self.m, p0, diff, n_past), "kv_shift")

    def synth(self, seed):
        _chk(_L.kcpp_model_synth_weights(self.m, seed), "synth")

    def set_tensor(self, idx, arr):
        _chk(_L.kcpp_model_set_tensor(self.m, idx, arr.ctypes.data_as(P), arr.nbytes), "set_tensor")

    def decode(self, tokens, n_past, want_logits=True, n_tokens=None):
        """llama_decode of len(tokens) tokens at n_past.  A stage without the embedding takes
        tokens=None and n_tokens=T: its input is the residual stream placed with hidden_io."""
        import numpy as np
        if tokens is None:
            tok, T = None, int(n_tokens)
        else:
            tok = np.ascontiguousarray(tokens, dtype=np.int32)
            T = len(tok)
        logits = np.empty(self.hp["n_vocab"], np.float32) if want_logits else None
        _chk(_L.kcpp_model_decode(self.m, tok.ctypes.data_as(P) if tok is not None else None, T, n_past,
                                  logits.ctypes.data_as(P) if want_logits else None), "decode")
        return logits

    def decode_async(self, tokens, n_past, n_tokens=None):
        """enqueue the decode on the stage stream without a host sync (prefill ubatches of a pipeline); the
        token array is copied before this returns"""
        import numpy as np
        if tokens is None:
            tok, T = None, int(n_tokens)
        else:
            tok = np.ascontiguousarray(tokens, dtype=np.int32)
            T = len(tok)
        _chk(_L.kcpp_model_decode_async(self.m, tok.ctypes.data_as(P) if tok is not None else None, T, n_past),
             "decode_async")

    def argmax(self):
        v = ctypes.c_int32(0)
        _chk(_L.kcpp_model_argmax(self.m, ctypes.byref(v)), "argmax")
        return v.value

    def decode_greedy(self, n_past):
        """one greedy step on the device-resident previous argmax; returns this step's token"""
        v = ctypes.c_int32(0)
        _chk(_L.kcpp_model_decode_greedy(self.m, n_past, ctypes.byref(v)), "decode_greedy")
        return v.value

    def decode_greedy_lagged(self, n_past):
        """one greedy step, the host one token behind: returns the previous step's token (-1 after a drain)"""
        v = ctypes.c_int32(0)
        _chk(_L.kcpp_model_decode_greedy_lagged(self.m, n_past, ctypes.byref(v)), "decode_greedy_lagged")
        return v.value

    def greedy_drain(self):
        """the last lagged step's token; resets the readback ring"""
        v = ctypes.c_int32(0)
        _chk(_L.kcpp_model_greedy_drain(self.m, ctypes.byref(v)), "greedy_drain")
        return v.value

    def forward_hidden(self, T, n_past):
        _chk(_L.kcpp_model_forward_hidden(self.m, T, n_past), "forward_hidden")

    def read_hidden(self, n, offset=0):
        import numpy as np
        out = np.empty(n, np.float32)
        _chk(_L.kcpp_model_read_hidden(self.m, out.ctypes.data_as(P), n, offset), "read_hidden")
        return out

    def hidden_io(self, ptr, n, offset=0, to_buf=False):
        """stream-ordered copy between the residual stream and ptr (device or host address)"""
        _chk(_L.kcpp_model_hidden_io(self.m, ptr, n, offset, int(to_buf)), "hidden_io")

    def sync(self):
        _chk(_L.kcpp_model_sync(self.m), "sync")

    def hidden_ptr(self):
        return _L.kcpp_model_hidden(self.m)

    def stream(self):
        return _L.kcpp_model_stream(self.m)

    def set_fused_decode(self, on):
        _L.kcpp_model_set_fused_decode(self.m, int(on))

    def set_rope_freqs(self, ff):
        """rope frequency factors (rope_freqs.weight: head_dim / 2 float32)"""
        import numpy as np
        a = np.ascontiguousarray(ff, dtype=np.float32)
        _chk(_L.kcpp_model_set_rope_freqs(self.m, a.ctypes.data_as(P), len(a)), "set_rope_freqs")

    def set_fa_exact(self, on):
        """strict-parity attention (reference order, f16 accumulation); see kcpp_flash_attn_exact"""
        _chk(_L.kcpp_model_set_fa_exact(self.m, int(on)), "set_fa_exact")

    def set_kv_types(self, type_k, type_v):
        """K / V cache types: F16 (default) or Q8_0 / Q4_0 for both (koboldcpp --quantkv); clears the caches"""
        _chk(_L.kcpp_model_set_kv_types(self.m, int(type_k), int(type_v)), "set_kv_types")

    def moe_ids(self, T, k):
        import numpy as np
        out = np.zeros((T, k), np.int32)
        _chk(_L.kcpp_model_moe_ids(self.m, out.ctypes.data, T * k), "moe_ids")
        return out

    def moe_trace(self, on):
        _chk(_L.kcpp_model_moe_trace(self.m, int(on)), "moe_trace")

    def set_fused_route(self, on, pair_down=None):
        """MoE decode fusions (default on): the router inside the two-slot gate|up launch, and (pair_down, default =
        on) both slots' down projections in one launch; off = the separate router launch / two chained launches"""
        pd = on if pair_down is None else pair_down
        _chk(_L.kcpp_model_set_fused_route(self.m, int(bool(on)) | (2 * int(bool(pd)))), "set_fused_route")

    def fused_route_count(self):
        """(routed gate|up launches, two-slot down launches) enqueued so far"""
        v = int(_L.kcpp_model_fused_route_count(self.m))
        return v & 0xFFFFFFFF, v >> 32

    def set_moe_grouped(self, on):
        """MoE prefill: grouped expert GEMMs (default) or the per-expert loop; returns the previous setting"""
        return bool(_L.kcpp_model_set_moe_grouped(self.m, int(bool(on))))

    def moe_grouped_count(self):
        """grouped MoE prefill layers run so far"""
        return int(_L.kcpp_model_moe_grouped_count(self.m))

    def moe_trace_read(self, n_layer, k):
        import numpy as np
        out = np.zeros((n_layer, k), np.int32)
        _chk(_L.kcpp_model_moe_trace_read(self.m, out.ctypes.data, n_layer * k), "moe_trace_read")
        return out

    def set_graphs(self, on):
        _L.kcpp_model_set_graphs(self.m, int(on))

    def set_row_split(self, devices, tensor_split):
        """LLAMA_SPLIT_MODE_ROW over `devices` (lanes may repeat a GPU); before synth / set_tensor"""
        n = len(devices)
        d = (ctypes.c_int * n)(*devices)
        ts = (ctypes.c_float * n)(*tensor_split)
        _chk(_L.kcpp_model_set_row_split(self.m, n, d, ts), "set_row_split")


    def weight_bytes(self):
        return int(_L.kcpp_model_weight_bytes(self.m))

    def close(self):
        if getattr(self, "m", None):
            _L.kcpp_model_free(self.m)
            self.m = None

    def __del__(self):
        self.close()


def row_split_range(nrows, tensor_split, i):
    """(lo, hi) of device i's rows (kcpp_row_split_range)"""
    n = len(tensor_split)
    ts = (ctypes.c_float * n)(*tensor_split)
    lo, hi = ctypes.c_int64(0), ctypes.c_int64(0)
    _chk(_L.kcpp_row_split_range(int(nrows), n, ts, int(i), ctypes.byref(lo), ctypes.byref(hi)), "row_split_range")
    return lo.value, hi.value


def pipeline_trace(n_stages, ubatch, T, n_past, steps):
    """the pipeline schedule's enqueue order (expose.cpp forward / greedy_step over the trace backend): host only"""
    buf = ctypes.create_string_buffer(1 << 16)
    n = _L.kcpp_pipeline_trace(n_stages, ubatch, T, n_past, steps, buf, len(buf))
    if n < 0:
        raise KcppError("kcpp_pipeline_trace failed")
    return buf.value.decode().split()


def split_layers(n_layer, n_dev, tensor_split=None):
    """load_model's layer placement: (device per layer, output head's device)"""
    ts = (ctypes.c_float * 16)(*((list(tensor_split) if tensor_split else [1.0] * n_dev) + [0.0] * (16 - n_dev)))
    out = (ctypes.c_int * (n_layer + 1))()
    if _L.kcpp_split_layers(n_layer, n_dev, ts, out) != 0:
        raise KcppError("kcpp_split_layers failed")
    return list(out[:n_layer]), out[n_layer]
