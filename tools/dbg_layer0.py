"""debug: layer-0 residual stream of the full-width fixture's 32-token prompt, GPU prefill vs token-by-token"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests")); sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
import koboldcpp_amd.lib as K
f = np.load("tests/golden/e2e_full.npz")
FULL2 = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=640, eps=1e-5, rope_base=500000.0)
types = [int(t) for t in f["types"]]
p2 = f["layer_prompt"]; T, E = len(p2), 4096
out = {}
for ub in (512, 1):
    m0 = K.Model(FULL2, types, il0=0, il1=1, has_embed=True, has_output=False, max_ubatch=max(ub, 8))
    m0.synth(1234)
    if ub == 512:
        m0.decode(p2, 0, want_logits=False)
        out["pre"] = m0.read_hidden(T * E).reshape(T, E)
    else:
        rows = []
        for i, t in enumerate(p2):
            m0.decode([int(t)], i, want_logits=False)
            rows.append(m0.read_hidden(E))
        out["dec"] = np.array(rows)
    m0.close()
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dbg_layer0.npz", **out)
print("ok")
