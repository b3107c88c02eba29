"""BASELINE config 1 fixture: TinyLlama-1.1B-shape (d 2048, 22 layers, 32/4 heads of 64, ff 5632,
vocab 32000) with Q4_0 weights and a Q8_0 output head, synthetic weights (include/kcpp_synth.h, seed 1234), 512
context, a 448-token prompt and 64 greedy tokens -- run by the REFERENCE ggml CPU build (oracle/_ref/ref_llama),
plus its scalar build for the build-to-build spread.  Writes tests/golden/config1.npz:
  prompt      the 448 prompt ids: BOS + ("hello world the" x 149) in the tests' SentencePiece vocab
  tokens      the reference's 65 greedy tokens (first one from the prompt's logits)
  logits0     the prompt's logits (32000 f32)
  margin      per step: top-1 minus top-2 logit of the reference
  spread_max / spread_median   per step |AVX2 - scalar| (teacher-forced on `tokens`)
usage: python tests/golden/make_config1.py   (needs `make -C oracle ref ref_scalar`)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import gguf_writer as GW  # noqa: E402
import refharness as R  # noqa: E402

TINYLLAMA = dict(n_vocab=32000, n_embd=2048, n_head=32, n_head_kv=4, n_layer=22, n_ff=5632, n_ctx=512, eps=1e-5,
                 rope_base=10000.0)


def prompt_ids():
    toks, _, _ = GW.spm_vocab(TINYLLAMA["n_vocab"], GW.WORDS)
    words = [toks.index("▁hello"), toks.index("▁world"), toks.index("▁the")]
    return [1] + words * 149


def main():
    hp = TINYLLAMA
    types = R.uniform_types(hp["n_layer"], R.Q4_0, R.Q8_0)
    prompt = prompt_ids()
    assert len(prompt) == 448
    a, info = R.run_ref_llama(hp, types, 1234, prompt, 64, nthreads=8, timeout=1800)
    tokens = np.argmax(a, axis=1).astype(np.int32)
    b, _ = R.run_ref_llama(hp, types, 1234, prompt, 64, nthreads=8, forced=tokens[:-1], timeout=3600,
                           binary=R.REF_BIN_SCALAR)
    srt = np.sort(a, axis=1)
    d = np.abs(a - b)
    np.savez_compressed(os.path.join(HERE, "config1.npz"), prompt=np.array(prompt, np.int32), tokens=tokens,
                        logits0=a[0], margin=(srt[:, -1] - srt[:, -2]).astype(np.float32),
                        spread_max=d.max(axis=1), spread_median=np.median(d, axis=1))
    print(info, "spread max", d.max(), "min margin", (srt[:, -1] - srt[:, -2]).min())


if __name__ == "__main__":
    main()
