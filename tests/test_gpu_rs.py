"""Row-major decode layouts KT_Q4_K_RS / KT_Q5_K_RS / KT_Q6_K_RS (include/kcpp_synth.h, csrc/gemv_rs.hip).

* layout: ggml bytes -> RS -> ggml is the identity; the device synth and dequant of an RS tensor equal
  those of the base type (bit-exact);
* mat-vec (every mode / prologue the decode step uses, masked-piece shapes, MoE-free) vs kcpp_gemv on the
  base type, whose parity with the reference CPU dot is pinned in test_gpu_kernels.py -- integer parts are
  exact, only the fp32 combination order differs (rtol 1e-4, as test_gpu_gemv_dec.py);
* the M-column kcpp_gemv path and the MFMA GEMM (prefill) read the RS planes: GEMM results are
  bit-identical to the base layout (same kernel, same arithmetic, other addresses)."""
import ctypes

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

RS = {R.Q4_K: 112, R.Q5_K: 113, R.Q6_K: 114}


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


def _synth(torch, K, t, Kd, N, tid):
    w = torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", t, 7, tid, w.data_ptr(), Kd, N, sptr(torch))
    return w


def _close(a, b, rtol=1e-4):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err < rtol, "max rel err %.3g" % err


@pytest.mark.parametrize("base", [R.Q4_K, R.Q5_K, R.Q6_K])
@pytest.mark.parametrize("Kd", [2048, 5632, 14336])
def test_rs_layout_roundtrip_synth_dequant(env, base, Kd):
    torch, K = env
    t = RS[base]
    if not K.raw().kcpp_rs_supported(t, Kd):
        pytest.skip("K not held in the RS layout")
    N = 6
    w = R.synth(base, 5, 77, Kd, N)
    src = torch.from_numpy(w).cuda()
    rs = torch.empty_like(src)
    K.call("kcpp_weight_repack", t, src.data_ptr(), rs.data_ptr(), Kd, N, 0, sptr(torch))
    back = torch.empty_like(src)
    K.call("kcpp_weight_repack", t, rs.data_ptr(), back.data_ptr(), Kd, N, 1, sptr(torch))
    torch.cuda.synchronize()
    assert np.array_equal(back.cpu().numpy(), w)
    assert not np.array_equal(rs.cpu().numpy(), w)            # really re-arranged
    syn = _synth(torch, K, t, Kd, N, 77)
    syn_b = _synth(torch, K, base, Kd, N, 77)
    # synth(RS) is the RS image of synth(base): dequantize both
    y_rs = torch.empty(N * Kd, device="cuda")
    y_b = torch.empty(N * Kd, device="cuda")
    K.call("kcpp_dequantize", t, syn.data_ptr(), y_rs.data_ptr(), Kd, N, sptr(torch))
    K.call("kcpp_dequantize", base, syn_b.data_ptr(), y_b.data_ptr(), Kd, N, sptr(torch))
    torch.cuda.synchronize()
    assert np.array_equal(y_rs.cpu().numpy().view(np.uint32), y_b.cpu().numpy().view(np.uint32))
    # and the RS image of the ggml bytes dequantizes like the oracle
    y2 = torch.empty(N * Kd, device="cuda")
    K.call("kcpp_dequantize", t, rs.data_ptr(), y2.data_ptr(), Kd, N, sptr(torch))
    torch.cuda.synchronize()
    assert np.array_equal(y2.cpu().numpy().view(np.uint32), R.dequant(base, w, Kd * N).view(np.uint32))


CASES = [  # name, base, K, N, mode, pro
    ("wo", R.Q4_K, 4096, 4096, 0, 0),
    ("glu", R.Q4_K, 4096, 14336, 1, 1),
    ("down", R.Q4_K, 14336, 4096, 0, 2),
    ("down_pro0", R.Q4_K, 14336, 4096, 0, 0),
    ("head", R.Q4_K, 4096, 8192, 0, 1),
    ("k2048", R.Q4_K, 2048, 512, 0, 1),
    ("k5632_masked", R.Q4_K, 5632, 2048, 0, 2),
    ("k8192_glu", R.Q4_K, 8192, 1024, 1, 1),
    ("wo_q6k", R.Q6_K, 4096, 4096, 0, 0),
    ("v_q6k", R.Q6_K, 4096, 1024, 0, 1),
    ("down_q6k", R.Q6_K, 14336, 4096, 0, 2),
    ("glu_q6k", R.Q6_K, 4096, 2048, 1, 1),
    ("head_q6k_big", R.Q6_K, 4096, 128256, 0, 1),
    ("k2048_q6k", R.Q6_K, 2048, 256, 0, 0),
    ("wo_q5k", R.Q5_K, 4096, 4096, 0, 0),
    ("glu_q5k", R.Q5_K, 4096, 14336, 1, 1),
    ("down_q5k", R.Q5_K, 14336, 4096, 0, 2),
    ("qkv_q5k", R.Q5_K, 4096, 6144, 0, 1),
    ("k5632_q5k_masked", R.Q5_K, 5632, 2048, 0, 2),
    ("head_q5k", R.Q5_K, 4096, 32768, 0, 1),
    # long K (the XL variants: activation slices read from LDS per piece): every prologue of mode 0 -- 0 is the column
    # path (kcpp_gemv / the ggml plugin's few-row MUL_MAT) on the 70B ffn_down --, GLU for n_embd past 14336
    ("down70_pro0", R.Q4_K, 28672, 512, 0, 0),
    ("down70_pro2", R.Q4_K, 28672, 512, 0, 2),
    ("glu_xl", R.Q4_K, 16384, 256, 1, 1),
    ("glu_xl_pro0", R.Q4_K, 16384, 256, 1, 0),
    ("down_q5k_xl_pro0", R.Q5_K, 20480, 256, 0, 0),
    ("down_q6k_xl_pro0", R.Q6_K, 32768, 256, 0, 0),
    ("glu_q6k_xl", R.Q6_K, 16384, 128, 1, 1),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_gemv_rs_vs_base(env, case):
    torch, K = env
    name, base, Kd, N, mode, pro = case
    t = RS[base]
    s = sptr(torch)
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(Kd, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(Kd, generator=g)).cuda()
    res = torch.randn(N, generator=g).cuda()
    Wb, Wr = _synth(torch, K, base, Kd, N, 1), _synth(torch, K, t, Kd, N, 1)
    W2b = _synth(torch, K, base, Kd, N, 2) if mode == 1 else None
    W2r = _synth(torch, K, t, Kd, N, 2) if mode == 1 else None
    y1 = torch.empty(Kd, device="cuda")
    if pro == 1:
        K.call("kcpp_rms_norm", x.data_ptr(), Kd, nw.data_ptr(), y1.data_ptr(), Kd, None, Kd, 1, 1e-5, s)
    else:
        y1.copy_(x)
    act = torch.zeros(K.act_bytes(base, Kd, 1) + 64, dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(base), y1.data_ptr(), Kd, act.data_ptr(), Kd, 1, s)
    use_res = mode == 0 and pro != 1
    yref = torch.empty(N, device="cuda")
    K.call("kcpp_gemv", base, Wb.data_ptr(), W2b.data_ptr() if W2b is not None else None, Kd, N, act.data_ptr(), 1,
           yref.data_ptr(), N, res.data_ptr() if use_res else None, N, mode, s)
    y = torch.full((N,), float("nan"), device="cuda")
    a = K.DecArgs()
    a.K, a.nseg, a.x, a.nw, a.eps, a.act = Kd, 1, x.data_ptr(), nw.data_ptr(), 1e-5, act.data_ptr()
    a.W[0], a.N[0], a.Y[0] = Wr.data_ptr(), N, y.data_ptr()
    a.res = res.data_ptr() if use_res else None
    a.W2 = W2r.data_ptr() if W2r is not None else None
    rc = K.gemv_dec(t, a, mode, pro, 1, s)
    assert rc == 0
    torch.cuda.synchronize()
    _close(y.cpu().numpy(), yref.cpu().numpy())


@pytest.mark.parametrize("pos", [0, 4000])
def test_gemv_rs_qkv_rope_kv(env, pos):
    """mode 2 (q|k|v + RoPE + f16 stores) on Q4_K_RS, against the same fused mode on the base layout"""
    torch, K = env
    E, EKV, D, n_ctx = 4096, 1024, 128, 4096
    s = sptr(torch)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(E, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(E, generator=g)).cuda()
    tab = np.empty(n_ctx * D, np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tab_d = torch.from_numpy(tab).cuda()
    posd = torch.tensor([pos], dtype=torch.int32, device="cuda")
    outs = []
    for t in (R.Q4_K, 112):
        Ws = [_synth(torch, K, t, E, n, 3 + i) for i, n in enumerate((E, EKV, EKV))]
        q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
        kc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
        vc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
        a = K.DecArgs()
        a.K, a.nseg, a.x, a.nw, a.eps = E, 3, x.data_ptr(), nw.data_ptr(), 1e-5
        for i, (w, n) in enumerate(zip(Ws, (E, EKV, EKV))):
            a.W[i], a.N[i], a.role[i] = w.data_ptr(), n, i
        a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = (q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), EKV, D,
                                                           posd.data_ptr(), tab_d.data_ptr())
        assert K.gemv_dec(t, a, 2, 1, 2, s) == 0
        torch.cuda.synchronize()
        f = lambda z: z.cpu().numpy().view(np.float16).astype(np.float32)
        sl = slice(pos * EKV, (pos + 1) * EKV)
        outs.append((f(q16), f(kc[sl]), f(vc[sl])))
    for a_, b_ in zip(*outs):
        _close(a_, b_, rtol=2e-3)


def test_gemv_rs_qkv_rope_kv_xl(env):
    """mode 2 at n_embd 16384 (past the register-resident activation: the XL variant) on Q4_K_RS, against the per-op
    path on the base layout: rms_norm, Q8_K, the column mat-vec, then NORM RoPE of q / k from the same table (adjacent
    pairs, ggml_rope_cache_init's cos / sin) and f16 rounding"""
    torch, K = env
    E, EKV, D, n_ctx, pos = 16384, 4096, 128, 256, 77
    s = sptr(torch)
    g = torch.Generator(device="cpu").manual_seed(6)
    x = torch.randn(E, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(E, generator=g)).cuda()
    tab = np.empty(n_ctx * D, np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tab_d = torch.from_numpy(tab).cuda()
    posd = torch.tensor([pos], dtype=torch.int32, device="cuda")
    Ns = (E, EKV, EKV)
    Wr = [_synth(torch, K, 112, E, n, 3 + i) for i, n in enumerate(Ns)]
    Wb = [_synth(torch, K, R.Q4_K, E, n, 3 + i) for i, n in enumerate(Ns)]
    q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
    kc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    vc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    a = K.DecArgs()
    a.K, a.nseg, a.x, a.nw, a.eps = E, 3, x.data_ptr(), nw.data_ptr(), 1e-5
    for i, (w, n) in enumerate(zip(Wr, Ns)):
        a.W[i], a.N[i], a.role[i] = w.data_ptr(), n, i
    a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = (q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), EKV, D,
                                                       posd.data_ptr(), tab_d.data_ptr())
    assert K.gemv_dec(112, a, 2, 1, 2, s) == 0
    y1 = torch.empty(E, device="cuda")
    K.call("kcpp_rms_norm", x.data_ptr(), E, nw.data_ptr(), y1.data_ptr(), E, None, E, 1, 1e-5, s)
    act = torch.zeros(K.act_bytes(R.Q4_K, E, 1) + 64, dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(R.Q4_K), y1.data_ptr(), E, act.data_ptr(), E, 1, s)
    ref = []
    for w, n in zip(Wb, Ns):
        y = torch.empty(n, device="cuda")
        K.call("kcpp_gemv", R.Q4_K, w.data_ptr(), None, E, n, act.data_ptr(), 1, y.data_ptr(), n, None, n, 0, s)
        ref.append(y)
    torch.cuda.synchronize()
    cs = tab.reshape(n_ctx, D // 2, 2)[pos]

    def rope(v):
        p = v.reshape(-1, D // 2, 2)
        c, sn = cs[None, :, 0], cs[None, :, 1]
        return np.stack([p[..., 0] * c - p[..., 1] * sn, p[..., 0] * sn + p[..., 1] * c], -1).reshape(-1)
    want = [rope(ref[0].cpu().numpy()), rope(ref[1].cpu().numpy()), ref[2].cpu().numpy()]
    f = lambda z: z.cpu().numpy().view(np.float16).astype(np.float32)
    sl = slice(pos * EKV, (pos + 1) * EKV)
    for got, w_ in zip((f(q16), f(kc[sl]), f(vc[sl])), want):
        assert np.isfinite(got).all()
        _close(got, w_, rtol=2e-3)


@pytest.mark.parametrize("base", [R.Q4_K, R.Q5_K, R.Q6_K])
@pytest.mark.parametrize("M", [3, 37])
def test_rs_columns_and_gemm(env, base, M):
    """kcpp_gemv (M <= 8, one RS launch per column) and kcpp_gemm (MFMA, RS planes) vs the base layout"""
    torch, K = env
    t = RS[base]
    Kd, N = 4096, 512
    s = sptr(torch)
    X = torch.randn(M, Kd, generator=torch.Generator(device="cpu").manual_seed(M)).cuda()
    act = torch.zeros(K.act_bytes(base, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(base), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.randn(M, N).cuda()
    ys = []
    K.raw().kcpp_gemm_set_variant(3)       # the unsplit kernels: Q6_K's base layout runs v2, its RS layout v3
    for tt in (base, t):
        W, W2 = _synth(torch, K, tt, Kd, N, 8), _synth(torch, K, tt, Kd, N, 9)
        for mode in (0, 1):
            Y = torch.empty(M, N, device="cuda")
            r = res.data_ptr() if mode == 0 else None
            w2 = W2.data_ptr() if mode == 1 else None
            if M <= 8:
                K.call("kcpp_gemv", tt, W.data_ptr(), w2, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, r, N, mode, s)
            else:
                ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(tt, Kd, N, M), dtype=torch.uint8, device="cuda")
                K.call("kcpp_gemm", tt, W.data_ptr(), w2, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, r, N, mode,
                       ws.data_ptr(), s)
            torch.cuda.synchronize()
            ys.append(Y.cpu().numpy())
    K.raw().kcpp_gemm_set_variant(0)
    for a_, b_ in zip(ys[:2], ys[2:]):
        if M > 8:
            assert np.array_equal(a_.view(np.uint32), b_.view(np.uint32))
        else:
            _close(b_, a_)


@pytest.mark.parametrize("base,Kd", [(R.Q4_K, 28672), (R.Q5_K, 20480), (R.Q6_K, 32768)])
@pytest.mark.parametrize("M", [1, 2, 5, 8])
def test_rs_columns_long_k(env, base, Kd, M):
    """kcpp_gemv at M <= 8 on a long-K RS tensor (Llama-3-70B ffn_down K = 28672: a 2-8 token prompt tail, the ggml
    plugin's few-row MUL_MAT): one XL launch per column with the activation-copy prologue, vs the base layout's
    column mat-vec -- plain + residual and GLU"""
    torch, K = env
    t = RS[base]
    assert K.raw().kcpp_rs_supported(t, Kd)
    N = 384
    s = sptr(torch)
    X = torch.randn(M, Kd, generator=torch.Generator(device="cpu").manual_seed(M + Kd)).cuda()
    act = torch.zeros(K.act_bytes(base, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(base), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.randn(M, N).cuda()
    ys = []
    for tt in (base, t):
        W, W2 = _synth(torch, K, tt, Kd, N, 21), _synth(torch, K, tt, Kd, N, 22)
        for mode in (0, 1):
            Y = torch.full((M, N), float("nan"), device="cuda")
            K.call("kcpp_gemv", tt, W.data_ptr(), W2.data_ptr() if mode == 1 else None, Kd, N, act.data_ptr(), M,
                   Y.data_ptr(), N, res.data_ptr() if mode == 0 else None, N, mode, s)
            torch.cuda.synchronize()
            ys.append(Y.cpu().numpy())
    for a_, b_ in zip(ys[:2], ys[2:]):
        assert np.isfinite(b_).all()
        _close(b_, a_)


@pytest.mark.parametrize("base", [R.Q4_K, "rs", "rs6"])
@pytest.mark.parametrize("Kd,N,M", [(4096, 512, 37), (4096, 640, 128), (2048, 1024, 300), (14336, 256, 512),
                                    (4096, 192, 17)])
def test_gemm_v3_matches_v2_bitwise(env, base, Kd, N, M):
    """Q4_K GEMM v3 (128x128 tiles, LDS-DMA activation, register-dequantized weights, permuted k order)
    against v2 (LDS weight tiles, natural k order): every integer partial sum is exact in fp32, so the two
    must agree bit for bit, for both layouts, plain+residual and GLU modes, ragged M and N"""
    torch, K = env
    t = {"rs": RS[R.Q4_K], "rs6": RS[R.Q6_K]}.get(base, R.Q4_K)
    s = sptr(torch)
    X = torch.randn(M, Kd, generator=torch.Generator(device="cpu").manual_seed(M + Kd)).cuda()
    act = torch.zeros(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(R.Q4_K), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.randn(M, N).cuda()
    W, W2 = _synth(torch, K, t, Kd, N, 3), _synth(torch, K, t, Kd, N, 4)
    ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
    outs = {}
    try:
        for v in (2, 3):
            K.raw().kcpp_gemm_set_variant(v)
            for mode in (0, 1):
                Y = torch.full((M, N), float("nan"), device="cuda")
                K.call("kcpp_gemm", t, W.data_ptr(), W2.data_ptr() if mode == 1 else None, Kd, N, act.data_ptr(), M,
                       Y.data_ptr(), N, res.data_ptr() if mode == 0 else None, N, mode, ws.data_ptr(), s)
                torch.cuda.synchronize()
                outs[v, mode] = Y.cpu().numpy()
    finally:
        K.raw().kcpp_gemm_set_variant(0)
    for mode in (0, 1):
        assert np.isfinite(outs[3, mode]).all()
        assert np.array_equal(outs[2, mode].view(np.uint32), outs[3, mode].view(np.uint32)), mode


@pytest.mark.parametrize("base", [R.Q4_K, "rs", "rs6"])
@pytest.mark.parametrize("Kd,N,M", [(4096, 512, 37), (14336, 256, 512), (2048, 384, 300)])
def test_gemm_v3_split_k(env, base, Kd, N, M):
    """v3 with the K range split in two (kcpp_gemm_set_variant(4); the default for grids under 384 workgroups):
    each half's fp32 partial is the unsplit kernel's running sum over its super-blocks, added in split order and
    then to the residual -- equal to the unsplit result up to that one re-association (<= 2e-6 of the output
    scale) and to the oracle within the GEMM bar"""
    torch, K = env
    t = {"rs": RS[R.Q4_K], "rs6": RS[R.Q6_K]}.get(base, R.Q4_K)
    bt = R.Q6_K if base == "rs6" else R.Q4_K
    s = sptr(torch)
    Xh = np.random.default_rng(M + Kd + 1).standard_normal((M, Kd)).astype(np.float32)
    X = torch.from_numpy(Xh).cuda()
    act = torch.zeros(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(R.Q4_K), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    resh = np.random.default_rng(M + N).standard_normal((M, N)).astype(np.float32)
    res = torch.from_numpy(resh).cuda()
    W = _synth(torch, K, t, Kd, N, 5)
    ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
    outs = {}
    try:
        for v in (3, 4):
            K.raw().kcpp_gemm_set_variant(v)
            Y = torch.full((M, N), float("nan"), device="cuda")
            K.call("kcpp_gemm", t, W.data_ptr(), None, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, res.data_ptr(), N, 0,
                   ws.data_ptr(), s)
            torch.cuda.synchronize()
            outs[v] = Y.cpu().numpy()
    finally:
        K.raw().kcpp_gemm_set_variant(0)
    assert np.isfinite(outs[4]).all()
    scale = max(1.0, float(np.abs(outs[3]).max()))
    assert np.abs(outs[4] - outs[3]).max() <= 2e-6 * scale
    want = R.mul_mat(bt, R.synth(bt, 7, 5, Kd, N), Kd, N, Xh) + resh
    assert np.abs(outs[4] - want).max() <= 3e-6 * max(1.0, float(np.abs(want).max())) + 1e-5


@pytest.mark.parametrize("base", [R.Q4_K, "rs", R.Q5_K, "rs5"])
@pytest.mark.parametrize("Kd,N,M", [(4096, 512, 37), (4096, 640, 128), (2048, 1024, 300), (14336, 256, 512),
                                    (4096, 384, 200)])
def test_gemm_v4_int8_matches_v2_bitwise(env, base, Kd, N, M):
    """Q4_K GEMM v4 (v_mfma_i32_32x32x32_i8 on the Q8_K bytes, isum = 8 acc(q*(sc>>3)) + acc(q*(sc&7)) in int32,
    operands by LDS-DMA straight from the Q8_K buffer): the same integer sumi as v2's exact fp32 sums and the same
    per-super-block epilogue, so bit-identical unsplit (kcpp_gemm_set_variant(13)), plain+residual and GLU, ragged M
    (token rows past M clamp to M - 1 and are not stored) and N; the split-K default (11) within the GEMM bar.
    Q5_K (base and RS layouts): the fifth bit as a third MFMA, hb*2sc into acc_h -- the same exact sumi"""
    torch, K = env
    t = {"rs": RS[R.Q4_K], "rs5": RS[R.Q5_K]}.get(base, base)
    s = sptr(torch)
    Xh = np.random.default_rng(M + Kd + 7).standard_normal((M, Kd)).astype(np.float32)
    X = torch.from_numpy(Xh).cuda()
    act = torch.zeros(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(R.Q4_K), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.randn(M, N).cuda()
    W, W2 = _synth(torch, K, t, Kd, N, 3), _synth(torch, K, t, Kd, N, 4)
    ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
    outs = {}
    try:
        for v in (2, 13, 11):
            K.raw().kcpp_gemm_set_variant(v)
            for mode in (0, 1):
                Y = torch.full((M, N), float("nan"), device="cuda")
                K.call("kcpp_gemm", t, W.data_ptr(), W2.data_ptr() if mode == 1 else None, Kd, N, act.data_ptr(), M,
                       Y.data_ptr(), N, res.data_ptr() if mode == 0 else None, N, mode, ws.data_ptr(), s)
                torch.cuda.synchronize()
                outs[v, mode] = Y.cpu().numpy()
    finally:
        K.raw().kcpp_gemm_set_variant(0)
    for mode in (0, 1):
        assert np.isfinite(outs[13, mode]).all()
        assert np.array_equal(outs[2, mode].view(np.uint32), outs[13, mode].view(np.uint32)), mode
        scale = max(1.0, float(np.abs(outs[2, mode]).max()))
        assert np.abs(outs[11, mode] - outs[2, mode]).max() <= 2e-6 * scale


@pytest.mark.parametrize("Kd,N,M", [(4096, 28672, 512), (4096, 1000, 300), (2048, 512, 129), (14336, 4096, 256),
                                    (4096, 14336, 64)])
def test_gemm_v5_matches_v4_bitwise(env, Kd, N, M):
    """Q4_K GEMM v5 (256-row tiles, every wave against all 128 tokens) against v4 (128-row tiles): the same
    per-element integer MFMAs and f32 epilogue in the same order, and the same split-K rule, so the outputs must be
    equal bit for bit -- RS layout, plain+residual and GLU modes, ragged M and N (a partial 256-row tile)"""
    torch, K = env
    t = RS[R.Q4_K]
    s = sptr(torch)
    X = torch.randn(M, Kd, generator=torch.Generator(device="cpu").manual_seed(M + N)).cuda()
    act = torch.zeros(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(R.Q4_K), X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    res = torch.randn(M, N).cuda()
    W, W2 = _synth(torch, K, t, Kd, N, 13), _synth(torch, K, t, Kd, N, 14)
    ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
    outs = {}
    try:
        for v in (11, 14):
            K.raw().kcpp_gemm_set_variant(v)
            for mode in (0, 1):
                Y = torch.full((M, N), float("nan"), device="cuda")
                K.call("kcpp_gemm", t, W.data_ptr(), W2.data_ptr() if mode == 1 else None, Kd, N, act.data_ptr(), M,
                       Y.data_ptr(), N, res.data_ptr() if mode == 0 else None, N, mode, ws.data_ptr(), s)
                torch.cuda.synchronize()
                outs[v, mode] = Y.cpu().numpy()
    finally:
        K.raw().kcpp_gemm_set_variant(0)
    for mode in (0, 1):
        assert np.isfinite(outs[14, mode]).all()
        assert np.array_equal(outs[11, mode].view(np.uint32), outs[14, mode].view(np.uint32)), mode
