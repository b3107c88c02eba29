"""Generate tests/golden/kshift_e2e.npz from the REFERENCE builds: a tiny Llama (refharness.TINY, Q4_K_M policy, seed
1234) prefills a 150-token prompt, its context is shifted (koboldcpp PurgeMissingTokens -> llama_kv_cache_seq_rm /
seq_add + build_k_shift: oracle/ref_llama.c kv_shift, REF_KSHIFT) by erasing 45 cells after the first 20, and 8
teacher-forced tokens are decoded on the shifted cache; the logits of the AVX2 build and their spread against the
scalar build (make ref_scalar).  Run in the build container only; the fixture is committed."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

P0, DIFF = 20, 45


def main():
    hp = R.TINY
    types = R.q4_k_m_types(hp["n_layer"])
    rng = np.random.default_rng(2026)
    prompt = [int(v) for v in rng.integers(1, hp["n_vocab"], size=150)]
    forced = [int(v) for v in rng.integers(1, hp["n_vocab"], size=8)]
    a, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced, kshift=(P0, DIFF))
    b, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced, kshift=(P0, DIFF),
                           binary=R.REF_BIN_SCALAR)
    # the shift is not a no-op: the same decode without it differs
    c, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced)
    d = np.abs(a - b)
    print("spread max", d.max(axis=1), "| shift effect", np.abs(a - c)[1:].max())
    np.savez_compressed(os.path.join(HERE, "kshift_e2e.npz"), types=np.array(types, np.int32),
                        prompt=np.array(prompt, np.int32), forced=np.array(forced, np.int32),
                        shift=np.array([P0, DIFF], np.int32), logits=a, spread_max=d.max(axis=1),
                        spread_median=np.median(d, axis=1), noshift_logits=c)


if __name__ == "__main__":
    main()
