"""The fused single-token q|k|v + attention launch (koboldcpp_amd/csrc/dec_fused.hip) against the two-launch path it
replaces (k_gemv_rs / k_gemv_rs_qkv + k_fa_dec4 + k_fa_comb4): every result is computed by the same arithmetic in the
same order, so the logits must be identical bit for bit -- at every offset of the new key inside its 16-key group
and split, at short contexts (empty splits) and long ones (keys streamed after the prefetched groups), on the
plain Q4_K_M layers (q|k|v all Q4_K) and the more-bits layers (v in Q6_K).  The hand-off's timeout flag stays 0."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

HP = dict(n_vocab=4096, n_embd=4096, n_head=32, n_head_kv=8, n_layer=4, n_ff=2048, n_ctx=4608, eps=1e-5,
          rope_base=500000.0)


@pytest.fixture(scope="module")
def model():
    import koboldcpp_amd.lib as K
    types = R.q4_k_m_types(HP["n_layer"])          # layers 2, 3 keep attn_v in Q6_K (use_more_bits)
    m = K.Model(HP, types, max_ubatch=512)
    m.synth(77)
    yield m
    m.close()


def _steps(m, toks, n_past, fused):
    m.set_decode_fusion(fused)
    out = []
    for i, t in enumerate(toks):
        out.append(m.decode([t], n_past + i))
    return np.stack(out)


@pytest.mark.parametrize("n_prompt,n_steps", [(1, 40), (200, 24), (4000, 24)])
def test_fused_qkv_attention_bitwise(model, n_prompt, n_steps):
    m = model
    rng = np.random.default_rng(n_prompt)
    prompt = rng.integers(0, HP["n_vocab"], n_prompt).tolist()
    toks = rng.integers(0, HP["n_vocab"], n_steps).tolist()
    m.decode(prompt, 0, want_logits=False)
    a = _steps(m, toks, n_prompt, True)
    assert m.fused_error() == 0
    b = _steps(m, toks, n_prompt, False)          # rewrites the same K/V rows with the same values
    assert np.isfinite(a).all()
    bad = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, ("steps differ", bad[:8].tolist(), float(np.abs(a - b).max()))


def test_fused_greedy_graph_replay(model):
    """the graph-replayed greedy loop (position advanced on the device) through the fused launch equals the
    two-launch loop token for token"""
    m = model
    prompt = list(range(3, 300))
    runs = []
    for fused in (True, False):
        m.set_decode_fusion(fused)
        m.decode(prompt, 0, want_logits=False)
        toks = [m.argmax()]
        n = len(prompt)
        for _ in range(16):
            toks.append(m.decode_greedy(n))
            n += 1
        runs.append(toks)
    m.set_decode_fusion(False)
    assert runs[0] == runs[1]
    assert m.fused_error() == 0
