"""Row split (koboldcpp --rowsplit -> LLAMA_SPLIT_MODE_ROW, gpttype_adapter.cpp:1892): every layer matrix and the
output matrix spread by rows over several lanes (ggml_backend_cuda_split_buffer / ggml_cuda_op_mul_mat's split
branch, ggml/src/ggml-cuda.cu:659-955,1403-1700).  The test box has one GPU, so the lanes are all on it: every lane
but the first runs the full protocol (own stream, peer copy of the activations and residual rows, its slice's
mat-vec / GEMM, rows copied back, event fence).  Checked against the reference's golden logits at the same bar as
the unsplit model, and against the unsplit model on the same (unfused, graph-less) kernels."""
import numpy as np
import pytest

import refharness as R
from test_gpu_model import SPREAD_MAX, SPREAD_MED, TOL_MAX

pytestmark = pytest.mark.gpu

SPLIT = (0.5, 0.3, 0.2)


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


def run(K, types, prompt, forced, split=None, hp=R.TINY, ub=512):
    m = K.Model(hp, types, max_ubatch=ub)
    if split:
        m.set_row_split([0] * len(split), split)
    else:
        m.set_graphs(False)
        m.set_fused_decode(False)
    m.synth(1234)
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in forced:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    return np.array(out)


@pytest.mark.parametrize("tag", ["q4km", "q8_0"])
def test_rowsplit_vs_reference_golden(K, golden_e2e, tag):
    types = [int(t) for t in golden_e2e[tag + "_types"]]
    prompt = golden_e2e[tag + "_prompt"]
    L = golden_e2e[tag + "_logits"]
    forced = golden_e2e[tag + "_tokens"][:-1]
    got = run(K, types, prompt, forced, SPLIT)
    d = np.abs(got - L)
    assert np.all(d.max(axis=1) <= 2 * SPREAD_MAX[tag]), d.max(axis=1)
    assert np.all(np.median(d, axis=1) <= 2 * SPREAD_MED[tag]), np.median(d, axis=1)
    whole = run(K, types, prompt, forced)
    e = np.abs(got - whole)
    print("rowsplit vs whole", tag, e.max())
    assert e.max() <= 1e-4 * max(1.0, np.abs(whole).max()), e.max()


@pytest.mark.parametrize("types_fn,split", [
    (lambda n: R.q2_k_types(n), (1.0, 1.0)),
    (lambda n: R.q3_k_m_types(n), (0.25, 0.25, 0.5)),
    (lambda n: R.uniform_types(n, R.Q6_K, R.Q4_0), (2.0, 1.0)),
    (lambda n: R.uniform_types(n, R.Q5_K, R.Q8_0), (0.0, 0.0, 0.0, 0.0)),
    (lambda n: R.uniform_types(n, R.Q8_0), (1.0, 1.0)),          # the Q8_0 tile layout (gemm_q80t.hip) sliced by rows
])
def test_rowsplit_matches_whole_model(K, types_fn, split):
    """every device layout (row-major Q4_K/Q5_K, RS, SoA Q6_K/Q3_K/Q2_K, Q4_0/Q8_0 repacks) sliced by rows; a
    150-token prompt in 64-token ubatches (GEMM path) and 4 decode steps (mat-vec path)"""
    hp = dict(R.TINY)
    types = types_fn(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(3).integers(1, 500, size=150)]
    whole = run(K, types, prompt, [], ub=64)
    forced = [int(np.argmax(whole[-1]))] + [5, 77, 301]
    whole = run(K, types, prompt, forced, ub=64)
    got = run(K, types, prompt, forced, split, ub=64)
    e = np.abs(got - whole)
    print("rowsplit vs whole", split, e.max())
    assert e.max() <= 1e-4 * max(1.0, np.abs(whole).max()), e.max()
    assert np.median(e) <= TOL_MAX


def test_rowsplit_refuses_moe(K):
    m = K.Model(R.TINY_MOE, R.moe_types(R.TINY_MOE["n_layer"]))
    with pytest.raises(K.KcppError):
        m.set_row_split([0, 0], (1.0, 1.0))
    m.close()
