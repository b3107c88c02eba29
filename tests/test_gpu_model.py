"""End-to-end GPU parity: the Llama runtime (kcpp_model_*) vs the reference ggml graph's golden
logits (tests/golden/e2e_tiny.npz, from oracle/_ref/ref_llama) and vs the C restatement."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

# Parity bar, derived from the reference's own build-to-build spread (tests/golden/ref_spread.npz,
# make_fullwidth.py: the reference sources built with AVX2/FMA/F16C vs without SIMD, same weights, prompt and
# teacher-forced tokens).  Per fixture tag:
#  * vs the reference golden: max and median |dlogit| per step <= 2 x the spread (max over steps).  One factor
#    for the summation-order class (the GPU's order is a third one), and the production attention accumulates
#    V*P in f32 where the CPU keeps an f16 accumulator (ggml.c:15788): the reference-pinned C restatement with
#    f32 accumulation measures 1.9x (max) / 1.5x (median) of the spread on these fixtures.  The strict-parity
#    mode (tests/test_gpu_fa_exact.py) is held to 1.5x.
#  * vs the C restatement with f32 accumulation (same attention math as the HIP path): the same spread class.
#  * HIP-vs-HIP self-consistency (ubatch split, fused vs unfused): 2x the largest spread.
_SP = np.load(R.ROOT + "/tests/golden/ref_spread.npz")
SPREAD_MAX = {t: float(_SP["tiny_%s_max" % t].max()) for t in ("q4km", "q8_0", "moe")}
SPREAD_MED = {t: float(_SP["tiny_%s_median" % t].max()) for t in ("q4km", "q8_0", "moe")}
TOL_MAX = 2 * max(SPREAD_MAX.values())
TOL_MEDIAN_F32 = 2 * max(SPREAD_MED.values())


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


def run_gpu(K, types, prompt, n_gen, ub=512, graphs=True, hp=R.TINY):
    m = K.Model(hp, types, max_ubatch=ub)
    m.set_graphs(graphs)
    m.synth(1234)
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for _ in range(n_gen):
        tok = int(np.argmax(out[-1]))
        assert m.argmax() == tok
        out.append(m.decode([tok], n))
        n += 1
    m.close()
    return np.array(out)


def run_gpu_forced(K, types, prompt, forced, hp=R.TINY):
    """prefill, then decode the given tokens (teacher forcing) -> logits per step"""
    m = K.Model(hp, types)
    m.synth(1234)
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in forced:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    return np.array(out)


def oracle_forced(types, prompt, forced, f32_accum, hp=R.TINY):
    R.lib().orc_set_fa_f32_accum(int(f32_accum))
    try:
        o = R.OracleLlama(hp, types, 1234)
        out = [o.eval(prompt, 0)]
        n = len(prompt)
        for tok in forced:
            out.append(o.eval([int(tok)], n))
            n += 1
    finally:
        R.lib().orc_set_fa_f32_accum(0)
    return np.array(out)


@pytest.mark.parametrize("tag", ["q4km", "q8_0"])
def test_e2e_vs_reference_golden(K, golden_e2e, tag):
    types = [int(t) for t in golden_e2e[tag + "_types"]]
    prompt = golden_e2e[tag + "_prompt"]
    L = golden_e2e[tag + "_logits"]
    forced = golden_e2e[tag + "_tokens"][:-1]          # the reference's own greedy tokens
    got = run_gpu_forced(K, types, prompt, forced)
    d = np.abs(got - L)
    assert np.all(d.max(axis=1) <= 2 * SPREAD_MAX[tag]), d.max(axis=1)
    assert np.all(np.median(d, axis=1) <= 2 * SPREAD_MED[tag]), np.median(d, axis=1)
    # the same comparison for the restatement with f32 attention accumulation shows the same spread
    orc32 = oracle_forced(types, prompt, forced, True)
    d32 = np.abs(orc32 - L)
    assert np.median(d) < 2 * np.median(d32) + 1e-4
    # and the HIP path equals that restatement up to fp32 summation order
    e = np.abs(got - orc32)
    assert np.median(e) < TOL_MEDIAN_F32 and e.max() < TOL_MAX, (np.median(e), e.max())


def test_graph_replay_matches_eager(K):
    types = R.q4_k_m_types(R.TINY["n_layer"])
    prompt = list(range(3, 20))
    a = run_gpu(K, types, prompt, 6, graphs=True)
    b = run_gpu(K, types, prompt, 6, graphs=False)
    assert np.array_equal(a, b)


def test_ubatch_split_matches_single_batch(K):
    types = R.q4_k_m_types(R.TINY["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(2).integers(1, 500, size=150)]
    a = run_gpu(K, types, prompt, 2, ub=512)
    b = run_gpu(K, types, prompt, 2, ub=64)
    np.testing.assert_allclose(a, b, rtol=0, atol=TOL_MAX)


@pytest.mark.parametrize("types_fn", [lambda n: R.uniform_types(n, R.Q4_0, R.Q6_K),
                                      lambda n: R.uniform_types(n, R.Q5_K, R.Q8_0)])
def test_e2e_vs_oracle_other_types(K, types_fn):
    hp = dict(R.TINY)
    types = types_fn(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(7).integers(1, 500, size=45)]
    got = run_gpu(K, types, prompt, 4)
    forced = np.argmax(got, axis=1)[:-1]
    orc32 = oracle_forced(types, prompt, forced, True)
    d = np.abs(got - orc32)
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))


def test_q8_0_batch32_prefill_vs_oracle(K):
    """BASELINE config 3 at test size: all-Q8_0 weights, prompt prefilled in ubatches of 32 tokens (the
    batched Q8_0 GEMM path at M = 32, plus a ragged last ubatch), teacher-forced vs the restatement"""
    types = R.uniform_types(R.TINY["n_layer"], R.Q8_0)
    prompt = [int(v) for v in np.random.default_rng(5).integers(1, 500, size=77)]
    got = run_gpu(K, types, prompt, 3, ub=32)
    forced = np.argmax(got, axis=1)[:-1]
    orc32 = oracle_forced(types, prompt, forced, True)
    d = np.abs(got - orc32)
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))


@pytest.mark.parametrize("types_fn", [lambda n: R.q4_k_m_types(n), lambda n: R.uniform_types(n, R.Q8_0),
                                      lambda n: R.uniform_types(n, R.Q4_0, R.Q5_K)])
def test_fused_decode_matches_unfused(K, types_fn):
    """gemv_dec fusions (norm/quant prologue, RoPE/KV epilogue) vs one-kernel-per-op decode."""
    types = types_fn(R.TINY["n_layer"])
    prompt = list(range(5, 30))
    outs = []
    for fused in (True, False):
        m = K.Model(R.TINY, types)
        m.set_fused_decode(fused)
        m.synth(1234)
        lg = [m.decode(prompt, 0)]
        n = len(prompt)
        for tok in (7, 100, 3, 250):
            lg.append(m.decode([tok], n))
            n += 1
        m.close()
        outs.append(np.array(lg))
    d = np.abs(outs[0] - outs[1])
    assert d.max() < TOL_MAX and np.median(d) < 1e-5, (d.max(), np.median(d))


@pytest.mark.parametrize("graphs", [True, False])
def test_decode_greedy_matches_host_loop(K, graphs):
    """kcpp_model_decode_greedy (token fed back on device) == decode([tok]) + argmax on the host"""
    types = R.q4_k_m_types(R.TINY["n_layer"])
    prompt = [(5 * i + 1) % R.TINY["n_vocab"] for i in range(21)]

    def run(greedy):
        m = K.Model(R.TINY, types)
        m.set_graphs(graphs)
        m.synth(1234)
        m.decode(prompt, 0, want_logits=False)
        tok = m.argmax()
        toks, n = [tok], len(prompt)
        for i in range(12):
            if greedy == "lagged":           # the host one token behind (bench.py's decode loop)
                prev = m.decode_greedy_lagged(n)
                assert (prev == -1) == (i == 0)
                if i:
                    toks.append(prev)
            elif greedy:
                tok = m.decode_greedy(n)
            else:
                logits = m.decode([tok], n)
                tok = m.argmax()
                assert tok == int(np.argmax(logits))
            if greedy != "lagged":
                toks.append(tok)
            n += 1
        if greedy == "lagged":
            toks.append(m.greedy_drain())
            assert m.greedy_drain() == -1
        m.close()
        return toks
    want = run(False)
    assert run(True) == want
    assert run("lagged") == want


def test_q8_0_decode_copy(K, monkeypatch):
    """all-Q8_0 model: prefill on the tile layout (KT_Q8_0_T), single tokens on the fused row-major chain over the
    KT_Q8_0 decode copies (round 6).  Weights given as GGUF bytes (kcpp_model_set_tensor fills both copies) equal the
    synthetic ones; decode with the copies vs without (KCPP_Q80_DEC=0: the tile GEMM at M = 1) within the GEMM bar, and
    both vs the C restatement"""
    hp = dict(R.TINY)
    types = R.uniform_types(hp["n_layer"], R.Q8_0)
    prompt = [int(v) for v in np.random.default_rng(9).integers(1, 500, size=40)]
    outs = {}
    for mode in ("copies", "set_tensor", "tile"):
        if mode == "tile":
            monkeypatch.setenv("KCPP_Q80_DEC", "0")
        m = K.Model(hp, types)
        if mode == "set_tensor":
            for idx, t in enumerate(types):
                m.set_tensor(idx, R.synth_tensor(hp, t, 1234, idx))
        else:
            m.synth(1234)
        lg = [m.decode(prompt, 0)]
        n = len(prompt)
        for tok in (7, 100, 3, 250, 11):
            lg.append(m.decode([tok], n))
            n += 1
        m.close()
        outs[mode] = np.array(lg)
    assert np.array_equal(outs["copies"].view(np.uint32), outs["set_tensor"].view(np.uint32))
    d = np.abs(outs["copies"] - outs["tile"])
    assert d.max() < TOL_MAX and np.median(d) < 1e-5, (d.max(), np.median(d))
    orc32 = oracle_forced(types, prompt, [7, 100, 3, 250, 11], True)
    d = np.abs(outs["copies"] - orc32)
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))
