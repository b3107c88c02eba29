"""Generate tests/golden/kshift.npz from the REFERENCE ggml (oracle/_ref/libggml_ref.so): the K-shift of llama.cpp's
build_k_shift (src/llama.cpp:10144-10190) -- ggml_rope_ext_inplace on an F16 K-cache view [D, HKV, n] with every
row's position = -diff (the cells moved down by diff), mode 0 (NORM), rope_f16 (ggml.c:14398) -- for shifts
{1, 37, 1000} at bases 1e4 and 5e5.  Run in the build container only; the fixture is committed."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

REFLIB = os.path.join(R.ROOT, "oracle", "_ref", "libggml_ref.so")
D, HKV, N_ROWS, N_CTX_ORIG = 128, 4, 24, 4096


def main():
    g = ctypes.CDLL(REFLIB)
    P, I, I64, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

    class InitParams(ctypes.Structure):
        _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", P), ("no_alloc", ctypes.c_bool)]
    for n, (a, r) in {"ggml_init": ([InitParams], P), "ggml_free": ([P], None),
                      "ggml_new_tensor_1d": ([P, I, I64], P), "ggml_new_tensor_3d": ([P, I, I64, I64, I64], P),
                      "ggml_rope_ext_inplace": ([P, P, P, P, I, I, I, F, F, F, F, F, F], P),
                      "ggml_new_graph": ([P], P), "ggml_build_forward_expand": ([P, P], None),
                      "ggml_graph_compute_with_ctx": ([P, P, I], I), "ggml_get_data": ([P], P)}.items():
        fn = getattr(g, n)
        fn.argtypes, fn.restype = a, r
    rng = np.random.default_rng(20261017)
    k = (rng.standard_normal((N_ROWS, HKV, D)) * 2).astype(np.float16)
    k[0, 0, :8] = [0.0, -0.0, 65504.0, -65504.0, 6e-8, -6e-8, 1.0, -1.0]      # zeros, extremes, subnormals
    out = {"k_in": k.view(np.uint16)}
    for base in (10000.0, 500000.0):
        for diff in (1, 37, 1000):
            ctx = g.ggml_init(InitParams(16 << 20, None, False))
            kt = g.ggml_new_tensor_3d(ctx, R.F16, D, HKV, N_ROWS)
            pos = g.ggml_new_tensor_1d(ctx, 26, N_ROWS)
            ctypes.memmove(g.ggml_get_data(kt), k.ctypes.data, k.nbytes)
            p = np.full(N_ROWS, -diff, np.int32)
            ctypes.memmove(g.ggml_get_data(pos), p.ctypes.data, p.nbytes)
            r = g.ggml_rope_ext_inplace(ctx, kt, pos, None, D, 0, N_CTX_ORIG, base, 1.0, 0.0, 1.0, 32.0, 1.0)
            gr = g.ggml_new_graph(ctx)
            g.ggml_build_forward_expand(gr, r)
            assert g.ggml_graph_compute_with_ctx(ctx, gr, 2) == 0
            res = np.empty_like(k)
            ctypes.memmove(res.ctypes.data, g.ggml_get_data(r), res.nbytes)
            out["k_shift_%d_%d" % (int(base), diff)] = res.view(np.uint16)
            g.ggml_free(ctx)
    np.savez_compressed(os.path.join(HERE, "kshift.npz"), **out)
    print("wrote", os.path.join(HERE, "kshift.npz"), sorted(out))


if __name__ == "__main__":
    main()
