"""The one-launch q|k (Q4_K) + v (Q6_K) decode projection (gemv_rs.hip k_gemv_rs_qkv, used on the Q4_K_M "more
bits" layers) against the two launches it replaces (kcpp_gemv_dec mode 2 for q|k in Q4_K_RS, then for v in
Q6_K_RS): the rope'd f16 q, the K and V cache rows must be equal bit for bit, at Llama-3-8B / 70B / 2048 widths
(Q6_K_RS needs K / 256 % 8 == 0, so narrower models keep two launches)."""
import ctypes

import numpy as np
import pytest

from test_gpu_kernels import dev, host, sptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


@pytest.mark.parametrize("E,H,HKV,pos", [(4096, 32, 8, 3000), (8192, 64, 8, 17), (2048, 16, 4, 5)])
def test_qkv_mixed_equals_two_launches(env, E, H, HKV, pos):
    torch, K = env
    D = E // H
    EKV = HKV * D
    n_ctx = pos + 8
    sp = sptr(torch)
    wq = torch.empty(K.row_bytes(K.Q4_K_RS, E) * E, dtype=torch.uint8, device="cuda")
    wk = torch.empty(K.row_bytes(K.Q4_K_RS, E) * EKV, dtype=torch.uint8, device="cuda")
    wv = torch.empty(K.row_bytes(K.Q6_K_RS, E) * EKV, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", K.Q4_K_RS, 7, 1, wq.data_ptr(), E, E, sp)
    K.call("kcpp_weight_synth", K.Q4_K_RS, 7, 2, wk.data_ptr(), E, EKV, sp)
    K.call("kcpp_weight_synth", K.Q6_K_RS, 7, 3, wv.data_ptr(), E, EKV, sp)
    rng = np.random.default_rng(E + pos)
    x = dev(torch, rng.standard_normal(E).astype(np.float32))
    nw = dev(torch, (1.0 + 0.1 * rng.standard_normal(E)).astype(np.float32))
    tab = np.zeros((n_ctx, D // 2, 2), np.float32)
    K.raw().kcpp_rope_table(tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, ctypes.c_float(500000.0), ctypes.c_float(1.0),
                            None, ctypes.c_float(0.0), ctypes.c_float(1.0), ctypes.c_float(32.0), ctypes.c_float(1.0), n_ctx)
    rt = dev(torch, tab)
    posd = dev(torch, np.array([pos], np.int32))
    outs = []
    for mixed in (False, True):
        q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
        kc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
        vc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")

        def args(ws, ns, roles):
            a = K.DecArgs()
            a.K, a.x, a.nw, a.eps = E, x.data_ptr(), nw.data_ptr(), 1e-5
            a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), EKV, D, \
                posd.data_ptr(), rt.data_ptr()
            for i, (w, n, r) in enumerate(zip(ws, ns, roles)):
                a.W[i], a.N[i], a.role[i] = w.data_ptr(), n, r
            a.nseg = len(ws)
            return a
        if mixed:
            a = args([wq, wk, wv], [E, EKV, EKV], [0, 1, 2])
            assert K.raw().kcpp_gemv_rs_qkv_mixed(ctypes.byref(a), ctypes.c_void_p(sp)) == 0
        else:
            assert K.gemv_dec(K.Q4_K_RS, args([wq, wk], [E, EKV], [0, 1]), 2, 1, 2, sp) == 0
            assert K.gemv_dec(K.Q6_K_RS, args([wv], [EKV], [2]), 2, 1, 2, sp) == 0
        outs.append([host(torch, t, np.int16) for t in (q16, kc, vc)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert np.abs(outs[1][2][pos * EKV:(pos + 1) * EKV]).max() > 0      # V row written at pos


@pytest.mark.parametrize("qt", [113, 112])     # Q5_K_RS (Mixtral Q5_K_M: attn_q), Q4_K_RS
@pytest.mark.parametrize("pos", [0, 517, 4000])
def test_qkv_dual_equals_two_launches(env, qt, pos):
    """q in an RS layout + k|v in Q8_0 (Mixtral's Q5_K_M policy, n_expert == 8) as one grid (kcpp_gemv_qkv_dual)
    against the two kcpp_gemv_dec launches: rope'd f16 q and the K / V cache rows bit for bit"""
    torch, K = env
    E, H, HKV = 4096, 32, 8
    D = E // H
    EKV = HKV * D
    n_ctx = pos + 8
    sp = sptr(torch)
    Q8_0 = 8
    wq = torch.empty(K.row_bytes(qt, E) * E, dtype=torch.uint8, device="cuda")
    wk = torch.empty(K.row_bytes(Q8_0, E) * EKV, dtype=torch.uint8, device="cuda")
    wv = torch.empty(K.row_bytes(Q8_0, E) * EKV, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", qt, 9, 1, wq.data_ptr(), E, E, sp)
    K.call("kcpp_weight_synth", Q8_0, 9, 2, wk.data_ptr(), E, EKV, sp)
    K.call("kcpp_weight_synth", Q8_0, 9, 3, wv.data_ptr(), E, EKV, sp)
    rng = np.random.default_rng(pos + qt)
    x = dev(torch, rng.standard_normal(E).astype(np.float32))
    nw = dev(torch, (1.0 + 0.1 * rng.standard_normal(E)).astype(np.float32))
    tab = np.zeros((n_ctx, D // 2, 2), np.float32)
    K.raw().kcpp_rope_table(tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, ctypes.c_float(1000000.0), ctypes.c_float(1.0),
                            None, ctypes.c_float(0.0), ctypes.c_float(1.0), ctypes.c_float(32.0), ctypes.c_float(1.0), n_ctx)
    rt = dev(torch, tab)
    posd = dev(torch, np.array([pos], np.int32))
    outs = []
    for dual in (False, True):
        q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
        kc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
        vc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")

        def args(ws, ns, roles):
            a = K.DecArgs()
            a.K, a.x, a.nw, a.eps = E, x.data_ptr(), nw.data_ptr(), 1e-5
            a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), EKV, D, \
                posd.data_ptr(), rt.data_ptr()
            for i, (w, n, r) in enumerate(zip(ws, ns, roles)):
                a.W[i], a.N[i], a.role[i] = w.data_ptr(), n, r
            a.nseg = len(ws)
            return a
        aq, akv = args([wq], [E], [0]), args([wk, wv], [EKV, EKV], [1, 2])
        if dual:
            assert K.raw().kcpp_gemv_qkv_dual(ctypes.byref(aq), ctypes.c_int(qt), ctypes.byref(akv),
                                              ctypes.c_void_p(sp)) == 0
        else:
            assert K.gemv_dec(qt, aq, 2, 1, 2, sp) == 0
            assert K.gemv_dec(Q8_0, akv, 2, 1, 2, sp) == 0
        outs.append([host(torch, t, np.int16) for t in (q16, kc, vc)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert np.abs(outs[1][0]).max() > 0 and np.abs(outs[1][2][pos * EKV:(pos + 1) * EKV]).max() > 0
