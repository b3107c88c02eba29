"""Generate the parity-evidence fixtures from the REFERENCE ggml builds (run in the build container only;
the outputs are committed so neither the CPU suite nor the GPU box needs /root/reference).

  ref_spread.npz  -- the reference's own build-to-build logit spread: oracle/_ref (gcc -mavx2 -mfma -mf16c)
                     vs oracle/_ref/scalar (same sources, no SIMD flags: ggml-quants.c's generic dot loops,
                     ggml.c's scalar ggml_vec_mad_f16) on identical weights, prompt and teacher-forced
                     tokens.  Per step: max and median |dlogit|.  This is what the end-to-end tolerance in
                     tests/test_gpu_model.py / test_gpu_fullwidth.py is derived from.
  e2e_full.npz    -- reference logits of a FULL-WIDTH Llama-3-8B-shape model (n_embd 4096, 32/8 heads,
                     n_ff 14336, vocab 128256, Q4_K_M policy) cut to 2 layers: a 512-token prompt plus 3
                     teacher-forced decode steps, and a 32-token prefill with the residual stream after
                     layer 0 (the reference's own input of layer 1) for the per-layer check.

usage: python tests/golden/make_fullwidth.py   (needs `make -C oracle ref ref_scalar`)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

FULL2 = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=640,
             eps=1e-5, rope_base=500000.0)
SEED = 1234
NTH = 8


def spread(a, b):
    d = np.abs(a - b)
    return d.max(axis=1), np.median(d, axis=1)


def main():
    out = {}
    g = np.load(os.path.join(HERE, "e2e_tiny.npz"))
    for tag in ("q4km", "q8_0"):
        types = [int(t) for t in g[tag + "_types"]]
        prompt, forced = g[tag + "_prompt"], g[tag + "_tokens"][:-1]
        a, _ = R.run_ref_llama(R.TINY, types, SEED, prompt, len(forced), forced=forced, nthreads=NTH)
        b, _ = R.run_ref_llama(R.TINY, types, SEED, prompt, len(forced), forced=forced, nthreads=NTH,
                               binary=R.REF_BIN_SCALAR)
        assert np.array_equal(a, g[tag + "_logits"]), "AVX2 reference no longer reproduces e2e_tiny.npz"
        out["tiny_%s_max" % tag], out["tiny_%s_median" % tag] = spread(a, b)
        print(tag, "tiny spread max", out["tiny_%s_max" % tag].max(), "median", np.median(out["tiny_%s_median" % tag]))
    g = np.load(os.path.join(HERE, "e2e_moe.npz"))
    a, _ = R.run_ref_llama(R.TINY_MOE, [int(t) for t in g["types"]], SEED, g["prompt"], len(g["tokens"]) - 1,
                           forced=g["tokens"][:-1], nthreads=NTH)
    b, _ = R.run_ref_llama(R.TINY_MOE, [int(t) for t in g["types"]], SEED, g["prompt"], len(g["tokens"]) - 1,
                           forced=g["tokens"][:-1], nthreads=NTH, binary=R.REF_BIN_SCALAR)
    out["tiny_moe_max"], out["tiny_moe_median"] = spread(a, b)
    print("moe tiny spread max", out["tiny_moe_max"].max())

    # ---- full width, 2 layers
    hp = FULL2
    types = R.q4_k_m_types(hp["n_layer"])
    rng = np.random.default_rng(20261016)
    prompt = [int(v) for v in rng.integers(1, hp["n_vocab"], size=512)]
    a, _ = R.run_ref_llama(hp, types, SEED, prompt, 3, nthreads=NTH)
    forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
    b, _ = R.run_ref_llama(hp, types, SEED, prompt, 3, forced=forced, nthreads=NTH, binary=R.REF_BIN_SCALAR)
    out["full_max"], out["full_median"] = spread(a, b)
    print("full spread max", out["full_max"], "median", out["full_median"])
    full = dict(types=np.array(types, np.int32), prompt=np.array(prompt, np.int32), forced=forced, logits=a)
    # per-layer: 32-token prefill, residual stream after layer 0 and the final logits
    p2 = [int(v) for v in rng.integers(1, hp["n_vocab"], size=32)]
    a2, info = R.run_ref_llama(hp, types, SEED, p2, 0, nthreads=NTH, hidden=True)
    b2, info_s = R.run_ref_llama(hp, types, SEED, p2, 0, nthreads=NTH, hidden=True, binary=R.REF_BIN_SCALAR)
    full.update(layer_prompt=np.array(p2, np.int32), layer_hidden0=info["hidden"][0], layer_logits=a2[0])
    dh = np.abs(info["hidden"][0] - info_s["hidden"][0])
    out["full_layer0_hidden_max"], out["full_layer0_hidden_median"] = dh.max(), np.median(dh)
    out["full_layer_logits_max"], out["full_layer_logits_median"] = spread(a2, b2)
    print("layer0 hidden spread max", dh.max(), "median", np.median(dh))
    # ---- Llama-3-70B width (BASELINE config 4), one layer + head: the spread at that width, and the reference's
    # greedy tokens for the 9-token prompt tests/test_gpu_config4.py teacher-forces
    hp70 = dict(n_vocab=128256, n_embd=8192, n_head=64, n_head_kv=8, n_layer=1, n_ff=28672, n_ctx=64, eps=1e-5,
                rope_base=500000.0)
    p70 = [int(v) for v in np.random.default_rng(71).integers(1, hp70["n_vocab"], size=9)]
    a70, _ = R.run_ref_llama(hp70, R.q4_k_m_types(1), SEED, p70, 2, nthreads=NTH)
    f70 = np.argmax(a70, axis=1)[:-1].astype(np.int32)
    b70, _ = R.run_ref_llama(hp70, R.q4_k_m_types(1), SEED, p70, 2, forced=f70, nthreads=NTH, binary=R.REF_BIN_SCALAR)
    out["l70_max"], out["l70_median"] = spread(a70, b70)
    out["l70_prompt"], out["l70_forced"] = np.array(p70, np.int32), f70
    print("70B-width 1-layer spread max", out["l70_max"], "median", out["l70_median"])
    # ---- quantized KV cache (koboldcpp --quantkv 1 / 2: q8_0 / q4_0 K and V, gpttype_adapter.cpp:1958-1959) on the
    # tiny Q4_K_M fixture, teacher-forced on its f16 run's tokens: reference logits and the build spread
    kvq = {}
    g = np.load(os.path.join(HERE, "e2e_tiny.npz"))
    types_t = [int(t) for t in g["q4km_types"]]
    for tag, kv in (("q8_0", "8 8"), ("q4_0", "2 2")):
        os.environ["REF_KV_TYPES"] = kv
        try:
            a, _ = R.run_ref_llama(R.TINY, types_t, SEED, g["q4km_prompt"], 8, forced=g["q4km_tokens"][:-1], nthreads=NTH)
            b, _ = R.run_ref_llama(R.TINY, types_t, SEED, g["q4km_prompt"], 8, forced=g["q4km_tokens"][:-1], nthreads=NTH,
                                   binary=R.REF_BIN_SCALAR)
        finally:
            del os.environ["REF_KV_TYPES"]
        kvq[tag + "_logits"] = a
        out["kv_%s_max" % tag], out["kv_%s_median" % tag] = spread(a, b)
        print("kv", tag, "spread max", out["kv_%s_max" % tag].max())
    np.savez_compressed(os.path.join(HERE, "e2e_kvq.npz"), **kvq)
    np.savez_compressed(os.path.join(HERE, "e2e_full.npz"), **full)
    np.savez_compressed(os.path.join(HERE, "ref_spread.npz"), **out)
    print("wrote e2e_full.npz, ref_spread.npz")


if __name__ == "__main__":
    main()
