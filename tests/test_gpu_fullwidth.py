"""End-to-end parity at FULL Llama-3-8B width (n_embd 4096, 32/8 heads, n_ff 14336, vocab 128256, Q4_K_M
policy, 2 layers) against the reference ggml CPU build (tests/golden/e2e_full.npz, make_fullwidth.py),
with the tolerance taken from the reference's own build-to-build spread (tests/golden/ref_spread.npz:
the same sources built with AVX2/FMA/F16C vs without SIMD, identical weights/prompt/forced tokens).

Why a spread and not 1e-3: at this width the reference disagrees with itself by max |dlogit| 0.07-0.11
(median 0.010-0.016, logits std 1.35) purely from the fp32 summation order of its quantized dot products
(ggml-quants.c:7796 AVX2 vs :8223 generic) and the Q8_K re-quantization of every layer's input, which turns a
1-ulp difference into a whole quantum.  The GPU sums in a third order, so its distance from the AVX2 build
is of the same class.  Bars (per step):
  * strict mode (kcpp_model_set_fa_exact: attention in the reference's order with its f16 accumulator,
    csrc/attn_exact.hip): logits, layer-0 residual stream and layer 1 run on the REFERENCE's layer-0 output,
    each within 1.5 x the reference's own spread of that quantity (measured 0.95-1.0x on the logits, 1.4x on
    the layer-0 median).
  * production path (flash attention accumulates V*P in f32; the CPU reference in f16, ggml.c:15788):
    logits max and median <= 1.5 x the spread (measured 1.0-1.45x; the pinned C restatement with f32
    accumulation measures 1.0-1.7x); per layer max <= 1.5 x, median <= 20 x (see PROD_LAYER_MEDIAN_FACTOR).
"""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

FULL2 = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=640,
             eps=1e-5, rope_base=500000.0)
FACTOR = 1.5
EXACT_FACTOR = 1.5
# production attention accumulates in f32, the reference in f16: per layer (no re-quantization in between to
# average it out) that rounding dominates -- measured median 0.143 vs the reference's 0.0081 spread on a residual
# stream of std 23 (0.6% relative), while strict mode (same order, same f16 accumulator) is at 1.4x the spread
PROD_LAYER_MEDIAN_FACTOR = 20.0


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


@pytest.fixture(scope="module")
def fx():
    import os
    g = os.path.join(R.ROOT, "tests", "golden")
    return np.load(os.path.join(g, "e2e_full.npz")), np.load(os.path.join(g, "ref_spread.npz"))


@pytest.mark.parametrize("exact", [False, True], ids=["production", "fa_exact"])
def test_fullwidth_logits_vs_reference(K, fx, exact):
    f, s = fx
    types = [int(t) for t in f["types"]]
    m = K.Model(FULL2, types)
    m.set_fa_exact(exact)
    m.synth(1234)
    out = [m.decode(f["prompt"], 0)]
    n = len(f["prompt"])
    for tok in f["forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    d = np.abs(np.array(out) - f["logits"])
    dmax, dmed = d.max(axis=1), np.median(d, axis=1)
    print("gpu vs ref max", dmax, "median", dmed, "| ref spread max", s["full_max"], "median", s["full_median"])
    fac = EXACT_FACTOR if exact else FACTOR
    assert np.all(dmax <= fac * s["full_max"].max()), dmax
    assert np.all(dmed <= fac * s["full_median"].max()), dmed
    # greedy choice agrees with the reference at every step of this fixture
    assert np.array_equal(np.argmax(out, axis=1)[:-1], f["forced"])


@pytest.mark.parametrize("exact", [False, True], ids=["production", "fa_exact"])
def test_fullwidth_per_layer_vs_reference(K, fx, exact):
    f, s = fx
    fac = EXACT_FACTOR if exact else FACTOR
    fac_med = EXACT_FACTOR if exact else PROD_LAYER_MEDIAN_FACTOR
    types = [int(t) for t in f["types"]]
    p2 = f["layer_prompt"]
    T, E = len(p2), FULL2["n_embd"]
    # layer 0 (embedding + layer 0): its output residual stream vs the reference's
    m0 = K.Model(FULL2, types, il0=0, il1=1, has_embed=True, has_output=False)
    m0.set_fa_exact(exact)
    m0.synth(1234)
    m0.decode(p2, 0, want_logits=False)
    h0 = m0.read_hidden(T * E).reshape(T, E)
    m0.close()
    dh = np.abs(h0 - f["layer_hidden0"])
    print("layer0 hidden max %.4g median %.4g | ref spread %.4g %.4g" % (dh.max(), np.median(dh),
          s["full_layer0_hidden_max"], s["full_layer0_hidden_median"]))
    assert dh.max() <= fac * s["full_layer0_hidden_max"]
    assert np.median(dh) <= fac_med * s["full_layer0_hidden_median"]
    # layer 1 + head on the reference's own layer-0 output
    m1 = K.Model(FULL2, types, il0=1, il1=2, has_embed=False, has_output=True)
    m1.set_fa_exact(exact)
    m1.synth(1234)
    ref_in = np.ascontiguousarray(f["layer_hidden0"], np.float32)
    m1.hidden_io(ref_in.ctypes.data, T * E, 0, to_buf=False)
    lg = m1.decode(None, 0, n_tokens=T)
    m1.close()
    d = np.abs(lg - f["layer_logits"])
    print("layer1 logits max %.4g median %.4g | ref spread %.4g %.4g" % (d.max(), np.median(d),
          s["full_layer_logits_max"].max(), s["full_layer_logits_median"].max()))
    assert d.max() <= fac * s["full_layer_logits_max"].max()
    assert np.median(d) <= fac * s["full_layer_logits_median"].max()
