"""diagnosis: 70B-width layer 0, prefill in ubatches of 12 vs one of 24, under GEMM variants / exact attention"""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import refharness as R
import koboldcpp_amd.lib as K

L70 = dict(n_vocab=128256, n_embd=8192, n_head=64, n_head_kv=8, n_layer=80, n_ff=28672, n_ctx=512, eps=1e-5,
           rope_base=500000.0)
types = R.q4_k_m_types(L70["n_layer"])
T, E = 24, L70["n_embd"]
prompt = [int(v) for v in np.random.default_rng(70).integers(1, L70["n_vocab"], size=T)]


def run(ub, variant, exact, n=24):
    old = K.raw().kcpp_gemm_set_variant(variant)
    m = K.Model(L70, types, il0=0, il1=1, has_embed=True, has_output=False, max_ubatch=ub)
    m.set_fa_exact(exact)
    m.synth(1234)
    m.decode(prompt[:n], 0, want_logits=False)
    rows = min(ub, n)
    r = m.read_hidden(rows * E).reshape(rows, E)
    m.close()
    K.raw().kcpp_gemm_set_variant(old)
    return r


for variant in (0, 3):
    a = run(24, variant, False)
    b = run(12, variant, False, n=12)
    d = np.abs(a[:12] - b).max(axis=1)
    print("variant", variant, "first 12 rows, M=24 vs M=12:", " ".join("%.2g" % v for v in d), flush=True)
    c = run(24, variant, False, n=12)
    d = np.abs(c - b).max(axis=1)
    print("variant", variant, "12-token prompt, ub 24 vs ub 12 (same M):", " ".join("%.2g" % v for v in d), flush=True)
