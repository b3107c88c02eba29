"""Phase timeline of the persistent decode engine (dec_engine.hip ESTAMP points): the bench model (Llama-3-8B
Q4_K_M shape, synthetic weights) prefills `--prompt` tokens, then decodes a few tokens with stamps on; for each
phase interval the median over workgroups and layers (and the max over workgroups of the layer total) is printed.
Diagnostics only (never the product path)."""
import argparse
import sys
import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

NAMES = {0: "layer top", 1: "Q poll (x ready)", 2: "Q norm", 3: "Q quant", 4: "Q dots", 5: "Q epilogue+arrive",
         6: "A poll (q ready)", 7: "A q/newkv load", 8: "A consume", 9: "A merge+store", 10: "C poll", 11: "C merge",
         12: "O poll", 13: "O act copy", 14: "O dots", 15: "O store", 16: "G poll", 17: "G norm", 18: "G quant",
         19: "G dots", 20: "G store", 21: "D poll", 22: "D h copy", 23: "D quant", 24: "D dots", 25: "D store"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompt", type=int, default=3840)
    ap.add_argument("--layers", type=int, default=32)
    args = ap.parse_args()
    import torch
    import koboldcpp_amd.lib as K
    import refharness as R
    hp = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=args.layers, n_ff=14336, n_ctx=4096,
              eps=1e-5, rope_base=500000.0)
    m = K.Model(hp, R.q4_k_m_types(args.layers))
    m.synth(1234)
    m.set_engine(True)
    m.decode([16 + (i % 2) for i in range(args.prompt)], 0, want_logits=False)
    m.argmax()
    n = args.prompt
    for _ in range(4):
        m.decode_greedy(n)
        n += 1
    st = torch.zeros(256 * args.layers * 32, dtype=torch.int64, device="cuda")
    K._L.kcpp_engine_set_stamps(__import__("ctypes").c_void_p(st.data_ptr()))
    m.set_graphs(False)               # eager: the launch picks the stamp pointer up
    m.decode_greedy(n)
    torch.cuda.synchronize()
    K._L.kcpp_engine_set_stamps(None)
    assert m.engine_active() == 1
    m.close()
    s = st.cpu().numpy().reshape(256, args.layers, 32).astype(np.float64) / 100.0      # 100 MHz -> us
    print("phase intervals (us): median over workgroups and layers 1.. (layer 0 has no x poll)")
    prev = 0
    pts = sorted(NAMES)
    for k in pts[1:]:
        a = s[:, 1:, k]
        b = s[:, 1:, prev]
        ok = (a > 0) & (b > 0)
        if ok.any():
            d = (a - b)[ok]
            print("  %-22s %7.2f  (p90 %7.2f)" % (NAMES[k], np.median(d), np.percentile(d, 90)))
            prev = k
    # the critical path: each stamp against the layer's earliest top, median / max over workgroups
    print("timeline since the layer's first top (us): median over layers of [median, max] over workgroups")
    t0 = s[:, 1:, 0].min(axis=0)
    for k in pts:
        a = s[:, 1:, k]
        ok = (a > 0).all(axis=0)
        if ok.any():
            r = a[:, ok] - t0[ok]
            print("  %-22s %7.2f %7.2f" % (NAMES[k], np.median(np.median(r, axis=0)), np.median(r.max(axis=0))))
    tot = s[:, 1:, 25] - s[:, 1:, 0]
    lay = s[:, 2:, 0] - s[:, 1:-1, 0]
    print("layer (top to top): median %.2f us, max over workgroups per layer median %.2f us" %
          (np.median(lay), np.median(lay.max(axis=0))))
    print("launch: %.1f us (first stamp to last)" % (s[s > 0].max() - s[s > 0].min()))


if __name__ == "__main__":
    main()
