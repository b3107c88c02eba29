"""The residual GEMM carrying the next rms_norm (kcpp_gemm_rms_norm / kcpp_gemm_q6p_rms_norm / kcpp_reduce_rms_norm):
the split-K reduce forms x = sum of the partials (split order) + res AND the rms_norm * w -> Q8_K activation of x in one
launch (ops.hip k_rms_norm with partials).  Bar: bit-identical to kcpp_gemm followed by kcpp_rms_norm -- x and every
byte of the Q8_K activation -- for split shapes (wo 4096 -> 4096, down 14336 -> 4096: Q4_K_RS on the int8 GEMM v4,
Q6_K_RS on the prefill image) and unsplit ones (q|k|v 4096 -> 6144, where the norm runs as its own launch), at full
and ragged token counts.  The model-level tests (prefill ubatch invariance, deep parity vs the reference build) run the
folded path as the runtime's default."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

Q4_K_RS, Q6_K_RS = 112, 114


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("t", [Q4_K_RS, Q6_K_RS])
@pytest.mark.parametrize("Kd,N,M", [(4096, 4096, 512), (14336, 4096, 300), (4096, 4096, 37), (4096, 6144, 200)])
def test_gemm_rms_norm_bitwise(env, t, Kd, N, M):
    torch, K = env
    s = sptr(torch)
    w = torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", t, 3, 17, w.data_ptr(), Kd, N, s)
    img = None
    if t == Q6_K_RS:
        img = torch.empty(int(K.raw().kcpp_q6p_image_bytes(Kd, N)), dtype=torch.uint8, device="cuda")
        K.call("kcpp_q6p_build", w.data_ptr(), Kd, N, img.data_ptr(), s)
    rng = np.random.default_rng(M + Kd)
    x = torch.from_numpy(rng.standard_normal((M, Kd)).astype(np.float32)).cuda()
    act = torch.empty(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", R.Q8_K, x.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda()
    nw = torch.from_numpy((1.0 + 0.1 * rng.standard_normal(N)).astype(np.float32)).cuda()
    ws = torch.empty(int(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M)), dtype=torch.uint8, device="cuda")
    qb = K.act_bytes(R.Q4_K, N, M)
    y0, y1 = torch.full((M, N), float("nan"), device="cuda"), torch.full((M, N), float("nan"), device="cuda")
    q0, q1 = torch.zeros(qb, dtype=torch.uint8, device="cuda"), torch.ones(qb, dtype=torch.uint8, device="cuda")
    eps = 1e-5
    # reference pair: the GEMM (+ residual), then the norm into Q8_K
    if img is not None:
        K.call("kcpp_gemm_q6p", img.data_ptr(), w.data_ptr(), None, None, Kd, N, act.data_ptr(), M, y0.data_ptr(), N,
               res.data_ptr(), N, 0, ws.data_ptr(), s)
    else:
        K.call("kcpp_gemm", t, w.data_ptr(), None, Kd, N, act.data_ptr(), M, y0.data_ptr(), N, res.data_ptr(), N, 0,
               ws.data_ptr(), s)
    K.call("kcpp_rms_norm", y0.data_ptr(), N, nw.data_ptr(), None, 0, q0.data_ptr(), N, M, eps, s)
    # folded
    if img is not None:
        K.call("kcpp_gemm_q6p_rms_norm", img.data_ptr(), w.data_ptr(), Kd, N, act.data_ptr(), M, y1.data_ptr(), N,
               res.data_ptr(), N, ws.data_ptr(), s, nw.data_ptr(), eps, q1.data_ptr())
    else:
        K.call("kcpp_gemm_rms_norm", t, w.data_ptr(), Kd, N, act.data_ptr(), M, y1.data_ptr(), N, res.data_ptr(), N,
               ws.data_ptr(), s, nw.data_ptr(), eps, q1.data_ptr())
    torch.cuda.synchronize()
    a0, a1 = y0.cpu().numpy(), y1.cpu().numpy()
    assert np.isfinite(a1).all()
    assert np.array_equal(a0.view(np.uint32), a1.view(np.uint32))
    assert np.array_equal(q0.cpu().numpy(), q1.cpu().numpy())


def test_reduce_rms_norm_matches_reduce_then_norm(env):
    """the kernel alone on hand-made partials: three splits, a residual, Mp > M"""
    torch, K = env
    s = sptr(torch)
    KS, M, Mp, N = 3, 70, 128, 2048
    rng = np.random.default_rng(5)
    part = torch.from_numpy(rng.standard_normal((KS, Mp, N)).astype(np.float32)).cuda()
    res = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda()
    nw = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    x = torch.empty((M, N), device="cuda")
    q = torch.empty(K.act_bytes(R.Q4_K, N, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_reduce_rms_norm", part.data_ptr(), KS, Mp, res.data_ptr(), N, x.data_ptr(), N, nw.data_ptr(), q.data_ptr(),
           N, M, 1e-5, s)
    torch.cuda.synchronize()
    p = part.cpu().numpy()
    want = p[0, :M].copy()
    for k in range(1, KS):
        want = (want + p[k, :M]).astype(np.float32)
    want = (want + res.cpu().numpy()).astype(np.float32)
    assert np.array_equal(x.cpu().numpy().view(np.uint32), want.view(np.uint32))
    q2 = torch.empty_like(q)
    K.call("kcpp_rms_norm", x.data_ptr(), N, nw.data_ptr(), None, 0, q2.data_ptr(), N, M, 1e-5, s)
    torch.cuda.synchronize()
    assert np.array_equal(q.cpu().numpy(), q2.cpu().numpy())
