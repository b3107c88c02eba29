"""Decode-step workload for rocprofv3 (kernel trace): Llama-3-8B Q4_K_M synthetic, context ~4k."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys
import torch
import koboldcpp_amd.lib as K
sys.path.insert(0, "tests")
import refharness as R

hp = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=4096, eps=1e-5,
          rope_base=500000.0)
mode = sys.argv[1] if len(sys.argv) > 1 else "decode"
m = K.Model(hp, R.q4_k_m_types(32))
m.synth(1234)
if mode == "decode":
    m.decode([1] * 512, 0, want_logits=False)
    n = 3840
    for i in range(20):
        m.decode([5], n, want_logits=False); n += 1
else:
    m.decode([1] * 512, 0, want_logits=False)
    m.decode([1] * 512, 3328, want_logits=False)
torch.cuda.synchronize()
m.close()
