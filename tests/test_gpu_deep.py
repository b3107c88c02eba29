"""Parity at BASELINE configs[1]'s own depth: a 3840-token prompt at n_ctx 4096 (ubatches of 512), decode at
positions 3840-3843 -- the workload bench.py times.

Reference-pinned (tests/golden/e2e_deep.npz, tests/golden/make_deep.py: the reference ggml CPU build, AVX2 and scalar,
full Llama-3-8B width cut to 2 layers, Q4_K_M policy):
  * logits of the prompt's last token and of 4 teacher-forced decode steps, production and strict-parity
    (fa_exact) attention, within FACTOR x the reference's own AVX2-vs-scalar spread at this depth (the bar of
    tests/test_gpu_fullwidth.py, where the fixture stops at 640 tokens);
  * the residual stream after layer 0 for prompt positions 3776-3839 (keys 3777-3840 per query): max within
    FACTOR x the spread; median within EXACT_FACTOR x (strict) / PROD_LAYER_MEDIAN_FACTOR x (production, whose
    attention accumulates P.V in f32 where the reference rounds every step to f16, ggml.c:15788) -- the measured
    ratios are printed.

Full size (32 layers, n_ctx 4096, the bench's exact workload), size-independent properties:
  * 3840 tokens prefilled as 512- or 256-token ubatches give the same bits (last-token logits);
  * the hipGraph decode step equals the eager one bit for bit at 3840-3850 keys;
  * greedy decode on the device (on-device argmax feeding the next step) equals the host argmax loop.
"""
import os

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

DEEP2 = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=2, n_ff=14336, n_ctx=4096,
             eps=1e-5, rope_base=500000.0)
LLAMA3_8B = dict(DEEP2, n_layer=32)
FACTOR = 1.5
EXACT_FACTOR = 1.5
PROD_LAYER_MEDIAN_FACTOR = 4.0     # measured 2.82 at this depth (the 640-token fixture needs 20: test_gpu_fullwidth.py)


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


@pytest.fixture(scope="module")
def fx():
    return np.load(os.path.join(R.ROOT, "tests", "golden", "e2e_deep.npz"))


@pytest.mark.parametrize("exact", [False, True], ids=["production", "fa_exact"])
def test_deep_logits_vs_reference(K, fx, exact):
    types = [int(t) for t in fx["types"]]
    m = K.Model(DEEP2, types, max_ubatch=int(fx["ubatch"]))
    m.set_fa_exact(exact)
    m.synth(1234)
    out = [m.decode(fx["prompt"], 0)]
    n = len(fx["prompt"])
    for tok in fx["forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    d = np.abs(np.array(out) - fx["logits"])
    dmax, dmed = d.max(axis=1), np.median(d, axis=1)
    smax, smed = fx["spread_max"], fx["spread_median"]
    print("depth 3840: gpu vs ref max", dmax, "median", dmed, "| ref spread max", smax, "median", smed,
          "| ratio max %.3f median %.3f" % (dmax.max() / smax.max(), dmed.max() / smed.max()))
    assert np.all(dmax <= FACTOR * smax.max()), dmax
    assert np.all(dmed <= FACTOR * smed.max()), dmed
    # greedy choice: equal to the reference's wherever its own top-2 margin exceeds the spread bar; at a near-tie
    # (step 1 of this fixture: 5.8776 vs 5.8646, a 0.013 margin under the 0.10 build spread) the GPU's token must be
    # one the reference scores within that bar of its maximum
    bar = 2 * FACTOR * smax.max()
    for i, ref in enumerate(fx["logits"]):
        top2 = np.sort(ref)[-2:]
        g = int(np.argmax(out[i]))
        if top2[1] - top2[0] > bar:
            assert g == int(np.argmax(ref)), (i, g)
        else:
            assert ref[g] >= top2[1] - bar, (i, g, ref[g], top2)


@pytest.mark.parametrize("exact", [False, True], ids=["production", "fa_exact"])
def test_deep_layer0_residual_vs_reference(K, fx, exact):
    types = [int(t) for t in fx["types"]]
    ub, E = int(fx["ubatch"]), DEEP2["n_embd"]
    n = len(fx["prompt"])
    last = n - (n - 1) // ub * ub                      # tokens in the prompt's last ubatch
    tail = fx["hidden0_tail"]
    m = K.Model(DEEP2, types, il0=0, il1=1, has_embed=True, has_output=False, max_ubatch=ub)
    m.set_fa_exact(exact)
    m.synth(1234)
    m.decode(fx["prompt"], 0, want_logits=False)
    h = m.read_hidden(last * E).reshape(last, E)[-len(tail):]
    m.close()
    dh = np.abs(h - tail)
    smax, smed = float(fx["hidden0_spread_max"]), float(fx["hidden0_spread_median"])
    print("depth 3840 layer0 residual max %.4g median %.4g | ref spread %.4g %.4g | ratio max %.2f median %.2f" % (
        dh.max(), np.median(dh), smax, smed, dh.max() / smax, np.median(dh) / smed))
    assert dh.max() <= FACTOR * smax
    assert np.median(dh) <= (EXACT_FACTOR if exact else PROD_LAYER_MEDIAN_FACTOR) * smed


def bench_prompt(n):
    return [16 + (i % 2) for i in range(n)]       # bench.py's synthetic prompt


def test_fullsize_depth_ubatch_invariance(K):
    types = R.q4_k_m_types(32)
    p = bench_prompt(3840)
    outs = []
    for ub in (512, 256):
        m = K.Model(LLAMA3_8B, types, max_ubatch=ub)
        m.synth(1234)
        outs.append(m.decode(p, 0))
        m.close()
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


def test_fullsize_depth_graph_eager_greedy(K):
    """graph == eager at 3840-3850 keys, and device greedy == host loop, on the bench workload"""
    types = R.q4_k_m_types(32)
    p = bench_prompt(3840)
    m = K.Model(LLAMA3_8B, types)
    m.synth(1234)
    m.decode(p, 0, want_logits=False)
    dev = [m.argmax()]
    n = len(p)
    for _ in range(10):
        dev.append(m.decode_greedy(n))
        n += 1
    # replay the same positions with the host loop: graph (decode of one token) then eager, same KV rows
    graphed, host = [], [dev[0]]
    n = len(p)
    for i in range(10):
        lg = m.decode([host[-1]], n)
        graphed.append(lg)
        host.append(int(np.argmax(lg)))
        n += 1
    m.set_graphs(False)
    n = len(p)
    for i in range(10):
        lg = m.decode([host[i]], n)
        assert np.array_equal(lg.view(np.uint32), graphed[i].view(np.uint32)), i
        n += 1
    m.close()
    assert dev == host
