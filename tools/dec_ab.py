"""A/B of single-token decode variants on the bench model (Llama-3-8B Q4_K_M synthetic, ~3.85k context): ms per
greedy token with the q|k|v + attention fusion on and off, in one process (run under rocprofv3 --kernel-trace for
per-kernel times).  usage: python tools/dec_ab.py [n_tokens] [n_layer]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import koboldcpp_amd.lib as K  # noqa: E402
import refharness as R  # noqa: E402

n_tok = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n_layer = int(sys.argv[2]) if len(sys.argv) > 2 else 32
hp = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=n_layer, n_ff=14336, n_ctx=4096, eps=1e-5,
          rope_base=500000.0)
m = K.Model(hp, R.q4_k_m_types(n_layer))
m.synth(1234)
prompt = [16 + (i % 2) for i in range(3840)]
m.decode(prompt, 0, want_logits=False)
for fused in (True, False, True, False):
    m.set_decode_fusion(fused)
    m.argmax()
    n = 3840
    for _ in range(4):
        m.decode_greedy(n)
        n += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_tok):
        m.decode_greedy(n)
        n += 1
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n_tok
    print("fused=%d  %.4f ms/token  %.1f tok/s  err=%d" % (fused, dt * 1e3, 1 / dt, m.fused_error()), flush=True)
m.close()
