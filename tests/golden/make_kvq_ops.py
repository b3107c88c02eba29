"""Generate tests/golden/kvq_ops.npz from the REFERENCE ggml build (oracle/_ref/ref_llama, build container only):
golden vectors of the quantized-KV-cache ops (koboldcpp --quantkv; gpttype_adapter.cpp:1958-1959):

  cpy_x, cpy_q8_0, cpy_q4_0  -- ggml_cpy f32 [R][N] -> Q8_0 / Q4_0 (the KV store: type_traits[t].from_float),
                               raw ggml block bytes from the reference
  fa_q, fa_kf, fa_vf, fa_mask -- flash-attention inputs (f32 q [T][H][D], f32 K/V rows quantized with the reference's
                               own cpy output, f16 causal mask with n_past), and
  fa_out_<tk>_<tv>           -- ggml_flash_attn_ext outputs with quantized K / V of those types

usage: python tests/golden/make_kvq_ops.py   (needs `make -C oracle ref`)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402


def ref_quant(t, x):
    R_, N = x.shape
    return R.run_ref_op("cpyq", np.ascontiguousarray(x, np.float32).tobytes(), R.row_bytes(t, N) * R_, [t, N, R_],
                        dtype=np.uint8).reshape(R_, R.row_bytes(t, N))


def main():
    rng = np.random.default_rng(20261016)
    out = {}
    # store: rows with a spread of magnitudes, an all-zero block, exact ties of the Q4_0 rounding
    x = (rng.standard_normal((48, 256)) * rng.uniform(0.01, 8.0, size=(48, 1))).astype(np.float32)
    x[3, 32:64] = 0.0
    x[5, :32] = np.float32(-8.0) * np.arange(32, dtype=np.float32) / 31
    out["cpy_x"] = x
    for t, name in ((R.Q8_0, "q8_0"), (R.Q4_0, "q4_0")):
        out["cpy_" + name] = ref_quant(t, x)
    # attention: D 128, 8 heads over 2 kv heads, 6 queries after 37 cached positions
    D, T, H, HKV, n_past = 128, 6, 8, 2, 37
    NKV = n_past + T
    q = rng.standard_normal((T, H, D)).astype(np.float32)
    kf = rng.standard_normal((NKV, HKV * D)).astype(np.float32)
    vf = rng.standard_normal((NKV, HKV * D)).astype(np.float32)
    mask = np.zeros((T, NKV), np.float16)
    for t in range(T):
        mask[t, n_past + t + 1:] = -np.inf
    out.update(fa_q=q, fa_kf=kf, fa_vf=vf, fa_mask=mask, fa_n_past=np.int32(n_past))
    for tk, nk in ((R.Q8_0, "q8_0"), (R.Q4_0, "q4_0")):
        for tv, nv in ((R.Q8_0, "q8_0"), (R.Q4_0, "q4_0")):
            k, v = ref_quant(tk, kf), ref_quant(tv, vf)
            res = R.run_ref_op("fattnq", q.tobytes() + k.tobytes() + v.tobytes() + mask.tobytes(), T * H * D,
                               [D, T, H, HKV, NKV, tk, tv])
            out["fa_out_%s_%s" % (nk, nv)] = res.reshape(T, H, D)
    np.savez_compressed(os.path.join(HERE, "kvq_ops.npz"), **out)
    print("wrote kvq_ops.npz")


if __name__ == "__main__":
    main()
