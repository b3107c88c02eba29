"""IQ4_NL / IQ4_XS (non-linear 4-bit code book kvalues_iq4nl, ggml-quants.c:3741) fixtures from the REFERENCE builds
(run in the build container only; the output is committed): dequantize_row_iq4_nl / _iq4_xs on synthetic and
random-bit blocks, mul_mat at decode / small-batch / prefill shapes (the reference graph's GGML_OP_MUL_MAT through
oracle/_ref: IQ4_NL . Q8_0, IQ4_XS . Q8_K), and a tiny Llama under the type's file policy (refharness.iq4_nl_types /
iq4_xs_types): prefill + 8 greedy steps, with the AVX2-vs-scalar build spread.

usage: python tests/golden/make_iq4.py   (needs `make -C oracle ref ref_scalar`)"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

KINDS = {"iq4nl": ("IQ4_NL", 18, "iq4_nl"), "iq4xs": ("IQ4_XS", 136, "iq4_xs")}


def main():
    for tag, (tn, bb, fn) in KINDS.items():
        make(tag, getattr(R, tn), bb, fn)


def make(ftag, T, bb, fn):
    ref = ctypes.CDLL(os.path.join(R.ROOT, "oracle", "_ref", "libggml_ref.so"))

    class InitParams(ctypes.Structure):
        _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", ctypes.c_void_p), ("no_alloc", ctypes.c_bool)]
    ref.ggml_init.argtypes = [InitParams]
    ref.ggml_init.restype = ctypes.c_void_p
    ref.ggml_init(InitParams(1 << 20, None, False))
    rng = np.random.default_rng(20261017)
    out = {}
    k = 1024
    syn = R.synth(T, 99, 5, k, 1)
    rnd = rng.integers(0, 256, size=(k // R.BLOCK[T][0]) * bb, dtype=np.uint8)
    rnd.reshape(-1, bb)[:, 1] &= 0x7B              # finite f16 d
    for tag, data in (("syn", syn), ("rnd", rnd)):
        y = np.empty(k, np.float32)
        getattr(ref, "dequantize_row_" + fn)(data.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(k))
        out["deq_%s_in" % tag], out["deq_%s_out" % tag] = data, y
    for (K, N, M) in ((4096, 256, 1), (4096, 128, 8), (1024, 64, 40)):
        w = R.synth(T, 11, 1200 + M, K, N)
        xseed = 1210 + M
        X = np.random.default_rng(xseed).standard_normal((M, K)).astype(np.float32)
        y = R.run_ref_op("mulmat", w.tobytes() + X.tobytes(), M * N, [T, K, N, M])
        key = "mm_%d_%d_%d" % (K, N, M)
        out[key + "_meta"] = np.array([T, 11, 1200 + M, xseed, K, N, M], np.int64)
        out[key + "_y"] = y.reshape(M, N)
    types = getattr(R, fn + "_types")(R.TINY["n_layer"])
    prompt = [int(v) for v in rng.integers(1, R.TINY["n_vocab"], size=37)]
    a, _ = R.run_ref_llama(R.TINY, types, 1234, prompt, 8)
    forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
    b, _ = R.run_ref_llama(R.TINY, types, 1234, prompt, 8, forced=forced, binary=R.REF_BIN_SCALAR)
    d = np.abs(a - b)
    out.update(e2e_types=np.array(types, np.int32), e2e_prompt=np.array(prompt, np.int32), e2e_logits=a,
               e2e_forced=forced, e2e_spread_max=d.max(axis=1), e2e_spread_median=np.median(d, axis=1))
    print(fn, "tiny spread max", d.max(axis=1).max(), "median", np.median(d, axis=1).max())
    np.savez_compressed(os.path.join(HERE, ftag + ".npz"), **out)
    print("wrote", ftag + ".npz")


if __name__ == "__main__":
    main()
