"""Generate the config-2-DEPTH parity fixture from the REFERENCE ggml builds (build container only; the output is
committed so neither the CPU suite nor the GPU box needs /root/reference).

BASELINE configs[1] runs a 3840-token prompt at n_ctx 4096 and decodes at positions 3840..4095; every other
reference-pinned end-to-end fixture stops at <= 640 tokens.  At 3840+ keys the reference accumulates attention's
P.V in f16 over ~4k terms (ggml.c:15788, ggml_vec_mad_f16) where the production kernels accumulate in f32, so the
depth is where the two differ most.  This fixture pins that depth:

  e2e_deep.npz -- FULL Llama-3-8B width (n_embd 4096, 32/8 heads, n_ff 14336, vocab 128256, Q4_K_M policy) cut to
                  2 layers, n_ctx 4096: a 3840-token random prompt prefilled in 512-token ubatches (7 x 512 + 256,
                  llama_decode_internal's split), then 4 teacher-forced decode steps at positions 3840..3843.
                    logits [5][V]        the AVX2 build (prompt's last token + 4 steps)
                    forced [4]           the AVX2 build's greedy tokens (teacher-forced into the scalar run)
                    hidden0_tail [64][E] residual stream after layer 0 for prompt positions 3776..3839
                    spread_max / spread_median [5]   |AVX2 - scalar| per step (the reference's own build spread)
                    hidden0_spread_max / _median     the same for hidden0_tail

usage: python tests/golden/make_deep.py     (needs `make -C oracle ref ref_scalar`; ~10 min on 8 cores)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

DEEP2 = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=4096,
             eps=1e-5, rope_base=500000.0)
SEED = 1234
N_PROMPT = 3840
N_GEN = 4
TAIL = 64
NTH = 8


def main():
    hp = DEEP2
    types = R.q4_k_m_types(hp["n_layer"])
    rng = np.random.default_rng(20261018)
    prompt = [int(v) for v in rng.integers(1, hp["n_vocab"], size=N_PROMPT)]
    t0 = time.time()
    a, ia = R.run_ref_llama(hp, types, SEED, prompt, N_GEN, nthreads=NTH, ubatch=512, timeout=7200, hidden=True)
    print("avx2 run %.1f s" % (time.time() - t0), ia["prefill_s"], ia["decode_s"], flush=True)
    forced = np.argmax(a, axis=1)[:-1].astype(np.int32)
    t0 = time.time()
    b, ib = R.run_ref_llama(hp, types, SEED, prompt, N_GEN, forced=forced, nthreads=NTH, ubatch=512, timeout=7200,
                            hidden=True, binary=R.REF_BIN_SCALAR)
    print("scalar run %.1f s" % (time.time() - t0), flush=True)
    d = np.abs(a - b)
    h_a, h_b = ia["hidden"][0][-TAIL:], ib["hidden"][0][-TAIL:]
    dh = np.abs(h_a - h_b)
    out = dict(types=np.array(types, np.int32), prompt=np.array(prompt, np.int32), forced=forced, logits=a,
               hidden0_tail=h_a.astype(np.float32), spread_max=d.max(axis=1), spread_median=np.median(d, axis=1),
               hidden0_spread_max=np.float32(dh.max()), hidden0_spread_median=np.float32(np.median(dh)),
               n_ctx=np.int32(hp["n_ctx"]), ubatch=np.int32(512))
    print("logit spread max", out["spread_max"], "median", out["spread_median"])
    print("hidden0 tail spread max %.4g median %.4g (stream std %.3g)" % (dh.max(), np.median(dh), h_a.std()))
    np.savez_compressed(os.path.join(HERE, "e2e_deep.npz"), **out)
    print("wrote e2e_deep.npz")


if __name__ == "__main__":
    main()
