"""BASELINE config 5 at full width: reference logits of a Mixtral-8x7B-shape model (n_embd 4096, 32/8 heads,
n_ff 14336, 8 experts top-2, vocab 32000, rope base 1e6) under the Q5_K_M policy (refharness.mixtral_q5_k_m_types:
Q5_K, Q8_0 attn_k / attn_v for 8 experts, Q6_K ffn_down_exps on the 'more bits' layer, F32 router), cut to 2 layers
(layer 0 plain, layer 1 'more bits'), from the REFERENCE ggml builds: a 64-token prompt plus 3 teacher-forced decode
steps, and the AVX2-vs-scalar build spread on the same inputs (the tolerance of tests/test_gpu_moe_fullwidth.py).

usage: python tests/golden/make_moe_full.py   (needs `make -C oracle ref ref_scalar`; build container only)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

MIXTRAL2 = dict(n_vocab=32000, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=128, eps=1e-5,
                rope_base=1000000.0, n_expert=8, n_expert_used=2)
SEED = 1234
NTH = 8


def main():
    hp = MIXTRAL2
    types = R.mixtral_q5_k_m_types(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(85).integers(1, hp["n_vocab"], size=64)]
    a, _ = R.run_ref_llama(hp, types, SEED, prompt, 3, nthreads=NTH, timeout=1800)
    forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
    b, _ = R.run_ref_llama(hp, types, SEED, prompt, 3, forced=forced, nthreads=NTH, binary=R.REF_BIN_SCALAR,
                           timeout=3600)
    d = np.abs(a - b)
    out = dict(types=np.array(types, np.int32), prompt=np.array(prompt, np.int32), forced=forced, logits=a,
               spread_max=d.max(axis=1), spread_median=np.median(d, axis=1))
    # the prompt alone with the residual stream after layer 0 (the reference's own input of layer 1), both builds
    a2, info = R.run_ref_llama(hp, types, SEED, prompt, 0, nthreads=NTH, hidden=True, timeout=1800)
    b2, info_s = R.run_ref_llama(hp, types, SEED, prompt, 0, nthreads=NTH, hidden=True, binary=R.REF_BIN_SCALAR,
                                 timeout=3600)
    assert np.array_equal(a2[0], a[0])
    dh = np.abs(info["hidden"][0] - info_s["hidden"][0])
    out.update(hidden0=info["hidden"][0], hidden0_spread_max=dh.max(), hidden0_spread_median=np.median(dh),
               router0=info["router"][0])
    print("layer0 hidden spread max", dh.max(), "median", np.median(dh))
    print("mixtral-width spread max", out["spread_max"], "median", out["spread_median"])
    np.savez_compressed(os.path.join(HERE, "e2e_moe_full.npz"), **out)
    print("wrote e2e_moe_full.npz")


if __name__ == "__main__":
    main()
