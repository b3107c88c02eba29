"""BASELINE config 4's shapes on one GPU: Llama-3-70B width (n_embd 8192, 64 q / 8 kv heads x 128, n_ff 28672,
vocab 128256, Q4_K_M policy).  The 8-GPU run puts 10 of the 80 layers on each GPU (tensor_split 1,...,1,
SURVEY.md 8d); this builds exactly such a stage -- layers [0, 10) with the embedding -- and a full-width
one-layer model with the head, so every kernel shape of config 4 runs here, including the K = 28672 down
projection (the long-K "XL" variant of the fused decode mat-vec, gemv_rs.hip: the activation slices read from LDS
per piece).

* 10-layer stage: finite, graph replay == eager, prefill independent of the ubatch split;
* 1-layer model with head: logits vs the C restatement of the reference CPU path (f32 attention accumulation,
  the same math as the HIP path), within 2x the reference's own build-to-build spread at this width."""
import numpy as np
import pytest

import refharness as R
from test_gpu_model import oracle_forced

pytestmark = pytest.mark.gpu

L70 = dict(n_vocab=128256, n_embd=8192, n_head=64, n_head_kv=8, n_layer=80, n_ff=28672, n_ctx=512, eps=1e-5,
           rope_base=500000.0)


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


def test_70b_stage_properties(K):
    """10-layer first stage (layers [0, 10) + embedding): no non-finite values; graph replay equals eager decode
    bit for bit; decode runs the K = 28672 down projection on the XL mat-vec in every layer.  Prefill in ubatches of 12 (attention by
    the split-KV kernel, T <= 16) vs one ubatch of 24 (MFMA flash attention, P rounded to f16) on the FIRST layer:
    with the strict-order attention (the same kernel for both splits) the last 12 rows are bit-identical; with the
    production kernels they differ by the two attention kernels' rounding, which an activation quantization
    (Q8_K before wo and the FFN) can turn into a flipped int8 rounding -- a discontinuity that moves a row by up to
    ~1% of its scale (measured: 1-2 rows in 12, under either GEMM split policy) -- so most rows must agree to 1e-5 and
    none may move beyond 2%.  (Across 10 random-weight layers such differences grow chaotically; the reference's
    own build-to-build spread does the same, tests/golden/ref_spread.npz.)"""
    types = R.q4_k_m_types(L70["n_layer"])
    T, E = 24, L70["n_embd"]
    prompt = [int(v) for v in np.random.default_rng(70).integers(1, L70["n_vocab"], size=T)]
    res = {}
    for mode in ("prefill24", "prefill12", "prefill24x", "prefill12x", "decode_graph", "decode_eager"):
        m = K.Model(L70, types, il0=0, il1=1 if mode.startswith("prefill") else 10, has_embed=True, has_output=False,
                    max_ubatch=12 if mode.startswith("prefill12") else 24)
        m.synth(1234)
        if mode.startswith("prefill"):
            m.set_fa_exact(mode.endswith("x"))
            m.decode(prompt, 0, want_logits=False)
            rows = 12 if mode.startswith("prefill12") else 24
            res[mode] = m.read_hidden(rows * E).reshape(rows, E)[-12:]
        else:
            m.set_graphs(mode == "decode_graph")
            for i, t in enumerate(prompt):
                m.decode([t], i, want_logits=False)
            res[mode] = m.read_hidden(E)
        m.close()
    for v in res.values():
        assert np.isfinite(v).all()
    assert np.array_equal(res["decode_graph"], res["decode_eager"])
    assert np.array_equal(res["prefill12x"], res["prefill24x"])
    scale = np.abs(res["prefill24"]).max()
    d = np.abs(res["prefill12"] - res["prefill24"]).max(axis=1)          # per row
    print("70B layer 0, ubatch 12 vs 24, per-row max:", " ".join("%.2g" % v for v in d), "scale %.3g" % scale)
    assert np.median(d) <= 1e-5 * scale and np.mean(d <= 1e-5 * scale) >= 0.75 and d.max() <= 0.02 * scale, d


def test_70b_width_one_layer_vs_oracle(K):
    """Llama-3-70B width, one layer (more-bits policy: Q6_K attn_v / ffn_down) + Q6_K head: prefill of the
    reference's 9-token prompt and its 2 greedy tokens teacher-forced, against the pinned C restatement with f32
    attention accumulation (the HIP path's math), per step within 2x the reference's own AVX2-vs-scalar spread
    at this width (tests/golden/ref_spread.npz l70_*: max 0.08-0.12, median 0.011-0.018, logits std 1.93)"""
    import os
    sp = np.load(os.path.join(R.ROOT, "tests", "golden", "ref_spread.npz"))
    hp = dict(L70, n_layer=1, n_ctx=64)
    types = R.q4_k_m_types(1)
    prompt, forced = [int(t) for t in sp["l70_prompt"]], [int(t) for t in sp["l70_forced"]]
    m = K.Model(hp, types)
    m.synth(1234)
    got = [m.decode(prompt, 0)]
    n = len(prompt)
    for t in forced:
        got.append(m.decode([t], n))
        n += 1
    m.close()
    ref = oracle_forced(types, prompt, forced, True, hp=hp)
    d = np.abs(np.array(got) - ref)
    print("70B-width 1 layer vs restatement: max", d.max(axis=1), "median", np.median(d, axis=1))
    assert np.all(d.max(axis=1) <= 2 * sp["l70_max"].max())
    assert np.all(np.median(d, axis=1) <= 2 * sp["l70_median"].max())


@pytest.mark.parametrize("T", [2, 5, 8])
def test_70b_width_short_prompt_vs_oracle(K, T):
    """a 2-8 token prompt (a prompt tail after context reuse) at Llama-3-70B width: M <= 8 runs the column mat-vec
    (kcpp_gemv) on every projection, including the K = 28672 ffn_down in its long-K RS layout (the XL variant with the
    activation-copy prologue); logits vs the pinned C restatement within 2x the reference's own spread at this width"""
    import os
    sp = np.load(os.path.join(R.ROOT, "tests", "golden", "ref_spread.npz"))
    hp = dict(L70, n_layer=1, n_ctx=64)
    types = R.q4_k_m_types(1)
    prompt = [int(t) for t in sp["l70_prompt"]][:T]
    m = K.Model(hp, types)
    m.synth(1234)
    got = m.decode(prompt, 0)
    m.close()
    ref = oracle_forced(types, prompt, [], True, hp=hp)
    d = np.abs(np.asarray(got) - ref[0])
    print("70B-width 1 layer, %d-token prompt vs restatement: max %.3g median %.3g" % (T, d.max(), np.median(d)))
    assert np.isfinite(got).all()
    assert d.max() <= 2 * sp["l70_max"].max()
    assert np.median(d) <= 2 * sp["l70_median"].max()
