"""Generate tests/golden/*.npz from the REFERENCE ggml (oracle/_ref, built from /root/reference
sources by `make -C oracle ref`).  Run in the build container only; the fixtures are committed
so the CPU suite and the GPU box never need /root/reference.

Inputs are synthetic (include/kcpp_synth.h generator, or numpy seeded RNG); every expected
output comes from the reference library: dequantize_row_* / quantize_row_q8_K / quantize_row_q8_0
symbols via ctypes, and ggml graph ops (mul_mat, rope_ext, rms_norm, flash_attn_ext, the full
build_llama graph) via oracle/_ref/ref_llama.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

REFLIB = os.path.join(R.ROOT, "oracle", "_ref", "libggml_ref.so")


def main():
    ref = ctypes.CDLL(REFLIB)

    class InitParams(ctypes.Structure):
        _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", ctypes.c_void_p), ("no_alloc", ctypes.c_bool)]
    ref.ggml_init.argtypes = [InitParams]
    ref.ggml_init.restype = ctypes.c_void_p
    ref.ggml_init(InitParams(1 << 20, None, False))   # initializes the reference's fp16 tables
    rng = np.random.default_rng(20241016)
    out = {}
    # ---- dequantization: synthetic blocks + random bit-pattern blocks (as test_quants.py:213-226)
    names = {R.Q4_0: "q4_0", R.Q8_0: "q8_0", R.Q4_K: "q4_K", R.Q5_K: "q5_K", R.Q6_K: "q6_K"}
    for t, nm in names.items():
        e, b = R.BLOCK[t]
        k = 4096
        syn = R.synth(t, 99, 5, k, 1)
        k = 1024 if t not in (R.Q4_0, R.Q8_0) else 512
        syn = syn[:(k // e) * b]
        rnd = rng.integers(0, 256, size=(k // e) * b, dtype=np.uint8)
        # keep random fp16 scale fields finite (exponent != 31) so dequant stays finite
        blocks = rnd.reshape(-1, b)
        if t in (R.Q4_0, R.Q8_0):
            blocks[:, 1] &= 0x7B
        elif t in (R.Q4_K, R.Q5_K):
            blocks[:, 1] &= 0x7B
            blocks[:, 3] &= 0x7B
        else:
            blocks[:, 209] &= 0x7B
        for tag, data in (("syn", syn), ("rnd", rnd)):
            y = np.empty(k, np.float32)
            fn = getattr(ref, "dequantize_row_" + nm)
            fn(data.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(k))
            out["deq_%s_%s_in" % (nm, tag)] = data
            out["deq_%s_%s_out" % (nm, tag)] = y
    # ---- activation quantization (vec_dot_type from_float)
    x = (rng.standard_normal(4096) * rng.uniform(0.1, 3.0, size=4096)).astype(np.float32)
    x[256:512] = 0.0                     # an all-zero Q8_K block
    x[1000] = 7.5                        # a dominant positive max
    x[3000] = -9.25                      # a dominant negative max
    for nm, vt in (("q8_K", R.Q8_K), ("q8_0", R.Q8_0)):
        y = np.zeros(R.row_bytes(vt, 4096), np.uint8)
        getattr(ref, "quantize_row_" + nm)(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_int64(4096))
        out["quant_%s_out" % nm] = y
    out["quant_in"] = x
    # ---- mul_mat at decode / small-batch / prefill shapes (scaled down)
    for t, nm in names.items():
        for (K, N, M) in ((4096, 256, 1), (4096, 128, 8), (1024, 64, 40)):
            # weights: synth(t, seed=11, tid=t*100+M); activations: default_rng(xseed) normal
            w = R.synth(t, 11, t * 100 + M, K, N)
            xseed = 1000 + t * 10 + M
            X = np.random.default_rng(xseed).standard_normal((M, K)).astype(np.float32)
            y = R.run_ref_op("mulmat", w.tobytes() + X.tobytes(), M * N, [t, K, N, M])
            key = "mm_%s_%d_%d_%d" % (nm, K, N, M)
            out[key + "_meta"] = np.array([t, 11, t * 100 + M, xseed, K, N, M], np.int64)
            out[key + "_y"] = y.reshape(M, N)
    # ---- rms_norm, rope (bases 10000 and 500000, positions up to ~4095), flash_attn_ext
    xr = rng.standard_normal((6, 4096)).astype(np.float32) * 3
    out["rms_x"] = xr
    out["rms_y"] = R.run_ref_op("rmsnorm", xr.tobytes(), xr.size, [4096, 6, 1e-5]).reshape(xr.shape)
    xq = rng.standard_normal((13, 8, 128)).astype(np.float32)
    out["rope_x"] = xq
    for base in (10000.0, 500000.0):
        out["rope_y_%d" % int(base)] = R.run_ref_op("rope", xq.tobytes(), xq.size,
                                                    [128, 8, 13, base, 1.0, 315]).reshape(xq.shape)
    for (T, NKV) in ((1, 256), (5, 300)):
        D, H, HKV = 128, 32, 8
        q = rng.standard_normal((T, H, D)).astype(np.float32)
        k = (rng.standard_normal((NKV, HKV, D)) * 0.5).astype(np.float16)
        v = rng.standard_normal((NKV, HKV, D)).astype(np.float16)
        mask = np.zeros((T, NKV), np.float16)
        for t in range(T):
            mask[t, NKV - T + t + 1:] = -np.inf
        y = R.run_ref_op("fattn", q.tobytes() + k.tobytes() + v.tobytes() + mask.tobytes(), q.size,
                         [D, T, H, HKV, NKV])
        key = "fa_%d_%d" % (T, NKV)
        out[key + "_q"], out[key + "_k"], out[key + "_v"], out[key + "_mask"] = q, k, v, mask
        out[key + "_y"] = y.reshape(q.shape)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **out)
    # ---- end-to-end: tiny synthetic Llama (Q4_K_M policy and all-Q8_0), prefill + greedy decode
    e2e = {}
    for tag, types in (("q4km", R.q4_k_m_types(R.TINY["n_layer"])), ("q8_0", R.uniform_types(R.TINY["n_layer"], R.Q8_0))):
        prompt = [int(v) for v in rng.integers(1, R.TINY["n_vocab"], size=37)]
        L, _ = R.run_ref_llama(R.TINY, types, 1234, prompt, 8)
        e2e["%s_types" % tag] = np.array(types, np.int32)
        e2e["%s_prompt" % tag] = np.array(prompt, np.int32)
        e2e["%s_logits" % tag] = L
        e2e["%s_tokens" % tag] = np.argmax(L, axis=1).astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "e2e_tiny.npz"), **e2e)
    print("wrote", sorted(os.listdir(HERE)))


def moe():
    """tiny Mixtral-style model (TINY_MOE: 4 experts, top-2, Q5_K_M-like types): reference logits for
    prefill + 8 greedy steps; written to e2e_moe.npz (make_golden.py --moe)"""
    rng = np.random.default_rng(20241017)
    hp = R.TINY_MOE
    types = R.moe_types(hp["n_layer"])
    prompt = [int(v) for v in rng.integers(1, hp["n_vocab"], size=29)]
    L, _ = R.run_ref_llama(hp, types, 1234, prompt, 8)
    np.savez_compressed(os.path.join(HERE, "e2e_moe.npz"), types=np.array(types, np.int32),
                        prompt=np.array(prompt, np.int32), logits=L, tokens=np.argmax(L, axis=1).astype(np.int32))
    print("wrote e2e_moe.npz")


if __name__ == "__main__":
    import sys
    if "--moe" in sys.argv:
        moe()
    else:
        main()
