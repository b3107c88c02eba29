"""Decode / prefill throughput of the Llama-3-8B shape with every layer weight in one type (tools only): which
weight types ride the fused RS / unit-per-lane decode kernels and which fall back to the per-op path.
usage: python tools/decode_types.py TYPE_NAME [...]   (names as in koboldcpp_amd.lib: Q4_K, Q5_K, IQ4_XS, ...)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402
import refharness as R  # noqa: E402

HP = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=2048, eps=1e-5,
          rope_base=500000.0)


def main():
    for name in sys.argv[1:]:
        t = getattr(K, name)
        types = R.uniform_types(HP["n_layer"], t, out=K.Q6_K)
        types[0] = K.Q4_K                                   # token embedding: a row gather either way
        m = K.Model(HP, types, max_ubatch=512)
        m.synth(1234)
        prompt = [16 + (i % 2) for i in range(512)]
        m.decode(prompt[:64], 0, want_logits=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.decode(prompt, 0, want_logits=False)
        torch.cuda.synchronize()
        t_pp = time.perf_counter() - t0
        m.argmax()                                          # first token, kept on the device
        n = len(prompt)
        for _ in range(8):
            m.decode_greedy(n)
            n += 1
        torch.cuda.synchronize()
        steps = 64
        t0 = time.perf_counter()
        for _ in range(steps):
            m.decode_greedy(n)
            n += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m.close()
        print(json.dumps({"type": name, "decode_tok_s": round(steps / dt, 1), "prefill_tok_s": round(512 / t_pp, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
