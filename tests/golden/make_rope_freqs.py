"""Generate tests/golden/rope_freqs_e2e.npz from the REFERENCE builds: a tiny Llama (refharness.TINY with rope base
10000, Q4_K_M policy, seed 1234) whose ropes carry Llama-3.1 frequency factors (rope_freqs.weight as the reference's
converter computes it for rope_type "llama3": refharness.llama31_rope_freqs; fed to ggml_rope_ext as build_llama
does, src/llama.cpp:10269 build_rope_factors, :10490) prefills a 700-token prompt (n_ctx 1024), is context-shifted (100, 200: the
K-shift also takes the factors) and decodes 8 teacher-forced tokens; the AVX2 build's logits, their spread against
the scalar build (make ref_scalar) and the same run without the factors (the factors must matter).  Run in the build
container only (oracle/_ref); the fixture is committed."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import refharness as R  # noqa: E402

P0, DIFF = 100, 200


def main():
    hp = dict(R.TINY, rope_base=10000.0, n_ctx=1024)
    types = R.q4_k_m_types(hp["n_layer"])
    D = hp["n_embd"] // hp["n_head"]
    ff = R.llama31_rope_freqs(hp["rope_base"], D)
    rng = np.random.default_rng(31)
    prompt = [int(v) for v in rng.integers(1, hp["n_vocab"], size=700)]
    forced = [int(v) for v in rng.integers(1, hp["n_vocab"], size=8)]
    a, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced, kshift=(P0, DIFF), rope_freqs=ff)
    b, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced, kshift=(P0, DIFF), rope_freqs=ff,
                           binary=R.REF_BIN_SCALAR)
    c, _ = R.run_ref_llama(hp, types, 1234, prompt, len(forced), forced=forced, kshift=(P0, DIFF))
    d = np.abs(a - b)
    print("spread max", d.max(axis=1), "| factor effect", np.abs(a - c).max(axis=1))
    np.savez_compressed(os.path.join(HERE, "rope_freqs_e2e.npz"), types=np.array(types, np.int32),
                        prompt=np.array(prompt, np.int32), forced=np.array(forced, np.int32),
                        shift=np.array([P0, DIFF], np.int32), rope_freqs=ff, rope_base=np.float32(hp["rope_base"]),
                        n_ctx=np.int32(hp["n_ctx"]),
                        logits=a, spread_max=d.max(axis=1), spread_median=np.median(d, axis=1), nofreq_logits=c)


if __name__ == "__main__":
    main()
