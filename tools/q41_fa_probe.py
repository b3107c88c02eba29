import sys, os, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import refharness as R
import koboldcpp_amd.lib as K
g = np.load('/root/repo/tests/golden/q41.npz')
for v in (2, 3, 4):
    K.raw().kcpp_fa_prefill_set_variant(v)
    types = [int(t) for t in g["e2e_types"]]
    m = K.Model(R.TINY, types); m.set_graphs(True); m.synth(1234)
    out = [m.decode(g["e2e_prompt"], 0)]
    n = len(g["e2e_prompt"])
    for tok in g["e2e_forced"]:
        out.append(m.decode([int(tok)], n)); n += 1
    m.close()
    d = np.abs(np.array(out) - g["e2e_logits"])
    print(v, "max", d.max(axis=1).round(4), "bar", 1.5 * g["e2e_spread_max"].max())
