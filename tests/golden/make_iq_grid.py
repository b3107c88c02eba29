"""IQ2_XXS / IQ2_XS / IQ2_S / IQ3_XXS / IQ3_S / IQ1_S / IQ1_M (the lattice-grid types, ggml-common.h:340-405)
fixtures from the REFERENCE builds (run in the build container only; the output is committed): dequantize_row_iq*
(ggml-quants.c:3504-3739) on synthetic and random-bit blocks, mul_mat through the reference graph (GGML_OP_MUL_MAT,
the type . Q8_K, ggml_vec_dot_iq*_q8_K) at decode / small-batch / prefill shapes, and a tiny Llama with the type
everywhere (output Q6_K): prefill + 8 greedy steps, with the AVX2-vs-scalar build spread.

usage: python tests/golden/make_iq_grid.py   (needs `make -C oracle ref ref_scalar`)"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402


def main():
    ref = ctypes.CDLL(os.path.join(R.ROOT, "oracle", "_ref", "libggml_ref.so"))

    class InitParams(ctypes.Structure):
        _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", ctypes.c_void_p), ("no_alloc", ctypes.c_bool)]
    ref.ggml_init.argtypes = [InitParams]
    ref.ggml_init.restype = ctypes.c_void_p
    ref.ggml_init(InitParams(1 << 20, None, False))
    out = {}
    for fn, T in R.IQ_GRID.items():
        rng = np.random.default_rng(20261017 + T)
        bb = R.BLOCK[T][1]
        k = 1024
        syn = R.synth(T, 99, 5, k, 1)
        rnd = rng.integers(0, 256, size=(k // 256) * bb, dtype=np.uint8)
        blk = rnd.reshape(-1, bb)
        if T == R.IQ1_M:                              # finite f16 scale: its top nibble lives in byte 7
            blk[:, 55] &= 0x7F
            blk[:, 55] = (blk[:, 55] & 0x0F) | (((blk[:, 55] >> 4) & 0x3) << 4)
        else:
            blk[:, 1] &= 0x3B                         # finite, moderate f16 d
        for tag, data in (("syn", syn), ("rnd", rnd)):
            y = np.empty(k, np.float32)
            getattr(ref, "dequantize_row_" + fn)(data.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                                                 ctypes.c_int64(k))
            out["%s_deq_%s_in" % (fn, tag)], out["%s_deq_%s_out" % (fn, tag)] = data, y
        for (K, N, M) in ((4096, 256, 1), (4096, 128, 8), (1024, 64, 40)):
            w = R.synth(T, 11, 1200 + M, K, N)
            xseed = 1210 + M
            X = np.random.default_rng(xseed).standard_normal((M, K)).astype(np.float32)
            y = R.run_ref_op("mulmat", w.tobytes() + X.tobytes(), M * N, [T, K, N, M])
            key = "%s_mm_%d_%d_%d" % (fn, K, N, M)
            out[key + "_meta"] = np.array([T, 11, 1200 + M, xseed, K, N, M], np.int64)
            out[key + "_y"] = y.reshape(M, N)
        types = R.iq_grid_types(R.TINY["n_layer"], T)
        prompt = [int(v) for v in rng.integers(1, R.TINY["n_vocab"], size=37)]
        a, _ = R.run_ref_llama(R.TINY, types, 1234, prompt, 8)
        forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
        b, _ = R.run_ref_llama(R.TINY, types, 1234, prompt, 8, forced=forced, binary=R.REF_BIN_SCALAR)
        d = np.abs(a - b)
        out.update({fn + "_e2e_types": np.array(types, np.int32), fn + "_e2e_prompt": np.array(prompt, np.int32),
                    fn + "_e2e_logits": a, fn + "_e2e_forced": forced, fn + "_e2e_spread_max": d.max(axis=1),
                    fn + "_e2e_spread_median": np.median(d, axis=1)})
        print(fn, "tiny spread max", d.max(axis=1).max(), "median", np.median(d, axis=1).max(),
              "logit std", a.std())
    # Mixtral-shaped tiny MoE with expert weights of a grid type (and Q4_1: the other type without a fused decode
    # mat-vec), through the reference's MUL_MAT_ID
    for tag, T in (("moe_iq2_xxs", R.IQ2_XXS), ("moe_q4_1", R.Q4_1)):
        rng = np.random.default_rng(20261018 + T)
        types = R.moe_types(R.TINY_MOE["n_layer"], T)
        prompt = [int(v) for v in rng.integers(1, R.TINY_MOE["n_vocab"], size=29)]
        a, _ = R.run_ref_llama(R.TINY_MOE, types, 1234, prompt, 6)
        forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
        b, _ = R.run_ref_llama(R.TINY_MOE, types, 1234, prompt, 6, forced=forced, binary=R.REF_BIN_SCALAR)
        d = np.abs(a - b)
        out.update({tag + "_e2e_types": np.array(types, np.int32), tag + "_e2e_prompt": np.array(prompt, np.int32),
                    tag + "_e2e_logits": a, tag + "_e2e_forced": forced, tag + "_e2e_spread_max": d.max(axis=1),
                    tag + "_e2e_spread_median": np.median(d, axis=1)})
        print(tag, "tiny spread max", d.max(axis=1).max(), "median", np.median(d, axis=1).max())
    np.savez_compressed(os.path.join(HERE, "iq_grid.npz"), **out)
    print("wrote iq_grid.npz")


if __name__ == "__main__":
    main()
