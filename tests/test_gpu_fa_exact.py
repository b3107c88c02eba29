"""Strict-parity attention (csrc/attn_exact.hip, kcpp_flash_attn_exact): the reference CPU's
flash_attn_ext_f16 arithmetic order with its f16 V accumulator (ggml.c:15667-15875).

* kernel vs the reference build's own outputs (tests/golden/ops.npz fa_*, from oracle/_ref): equal up to
  the rounding of exp (the reference calls glibc expf, the kernel rounds a double exp -- both correctly
  rounded except in rare ties); measured bit-exact on these fixtures, asserted within 1 f32 ulp of the
  output scale;
* end to end, a model in this mode vs the reference golden logits: within the reference's own AVX2-vs-scalar
  build spread (tests/golden/ref_spread.npz) -- tiny models here, full width in test_gpu_fullwidth.py."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


@pytest.mark.parametrize("key", ["fa_1_256", "fa_5_300"])
def test_fa_exact_vs_reference_golden(env, golden_ops, key):
    torch, K = env
    q, k, v = (golden_ops[key + s] for s in ("_q", "_k", "_v"))
    T, H, D = q.shape
    n_kv, HKV, _ = k.shape
    qd = torch.from_numpy(q.astype(np.float16).view(np.int16)).cuda()
    kd = torch.from_numpy(np.ascontiguousarray(k).view(np.int16)).cuda()
    vd = torch.from_numpy(np.ascontiguousarray(v).view(np.int16)).cuda()
    out = torch.full((T, H, D), float("nan"), device="cuda")
    K.call("kcpp_flash_attn_exact", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), T, H, HKV, D,
           n_kv - T, None, float(np.float32(1) / np.sqrt(np.float32(D))),   # 1.0f / sqrtf(D), as ref_llama
           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got, ref = out.cpu().numpy(), golden_ops[key + "_y"]
    n_diff = int((got.view(np.uint32) != ref.view(np.uint32)).sum())
    print("%s: %d of %d outputs differ in any bit" % (key, n_diff, got.size))
    assert np.abs(got - ref).max() <= np.spacing(np.abs(ref).max())


def _forced(K, hp, types, prompt, forced, exact):
    m = K.Model(hp, types)
    m.set_fa_exact(exact)
    m.synth(1234)
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in forced:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    return np.array(out)


@pytest.mark.parametrize("tag", ["q4km", "q8_0"])
def test_e2e_exact_within_reference_spread(env, golden_e2e, tag):
    """strict mode end to end (prefill + teacher-forced decode) vs the reference golden: per step within the
    reference's own AVX2-vs-scalar spread on the same fixture (max over steps, x1.5: the GPU sums the
    quantized dots in a third order, so its distance to the AVX2 build is a spread of the same class)"""
    torch, K = env
    sp = np.load(R.ROOT + "/tests/golden/ref_spread.npz")
    types = [int(t) for t in golden_e2e[tag + "_types"]]
    L = golden_e2e[tag + "_logits"]
    got = _forced(K, R.TINY, types, golden_e2e[tag + "_prompt"], golden_e2e[tag + "_tokens"][:-1], True)
    d = np.abs(got - L)
    print(tag, "exact-mode vs ref max", d.max(axis=1), "median", np.median(d, axis=1))
    assert np.all(d.max(axis=1) <= 1.5 * sp["tiny_%s_max" % tag].max())
    assert np.all(np.median(d, axis=1) <= 1.5 * sp["tiny_%s_median" % tag].max())


def test_exact_mode_graph_replay_equals_eager(env):
    """the strict kernel reads n_past from the device in the captured decode graph"""
    torch, K = env
    types = R.q4_k_m_types(R.TINY["n_layer"])
    prompt = list(range(3, 40))
    outs = []
    for graphs in (True, False):
        m = K.Model(R.TINY, types)
        m.set_fa_exact(True)
        m.set_graphs(graphs)
        m.synth(1234)
        lg = [m.decode(prompt, 0)]
        n = len(prompt)
        for tok in (5, 9, 200):
            lg.append(m.decode([tok], n))
            n += 1
        m.close()
        outs.append(np.array(lg))
    assert np.array_equal(outs[0], outs[1])
