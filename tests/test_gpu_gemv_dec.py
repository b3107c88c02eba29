"""Fused single-token mat-vec (kcpp_gemv_dec: gemv_dec_impl.h unit-per-lane kernel, and the
coalesced-streaming Q4_K kernel kcpp_gemv_stream) against the unfused composition of kernels that
are themselves pinned bit-exact / to the oracle in test_gpu_kernels.py:
rms_norm(+Q8_K quant) -> kcpp_gemv (+res / silu-GLU) -> rope_kv.
Only the fp32 summation order differs (per-chunk vs per-unit partial sums), hence rtol 1e-4."""
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


def _w(torch, K, t, Kd, N, tid):
    w = torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", t, 7, tid, w.data_ptr(), Kd, N, torch.cuda.current_stream().cuda_stream)
    return w


def _close(a, b, rtol=1e-4):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err < rtol, "max rel err %.3g" % err


def _ref_act(torch, K, t, x, nw, Kd, eps=1e-5, norm=True):
    s = torch.cuda.current_stream().cuda_stream
    vt = K.vec_dot_type(t)
    y = torch.empty(Kd, device="cuda")
    if norm:
        K.call("kcpp_rms_norm", x.data_ptr(), Kd, nw.data_ptr(), y.data_ptr(), Kd, None, Kd, 1, eps, s)
    else:
        y.copy_(x)
    act = torch.zeros(K.act_bytes(t, Kd, 1) + 64, dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", vt, y.data_ptr(), Kd, act.data_ptr(), Kd, 1, s)
    return act


def _args(lib, **kw):
    d = lib.DecArgs()
    for k, v in kw.items():
        if k in ("W", "Y", "N", "role"):
            for i, e in enumerate(v):
                getattr(d, k)[i] = e
        else:
            setattr(d, k, v)
    return d


CASES = [  # name, type, K, N, mode, pro
    ("wo", R.Q4_K, 4096, 4096, 0, 0),
    ("wo_q6k", R.Q6_K, 4096, 4096, 0, 0),
    ("glu", R.Q4_K, 4096, 14336, 1, 1),
    ("down_q4k", R.Q4_K, 14336, 4096, 0, 2),
    ("down_q6k", R.Q6_K, 14336, 4096, 0, 2),
    ("head_q4k", R.Q4_K, 4096, 8192, 0, 1),
    ("head_q6k", R.Q6_K, 4096, 8192, 0, 1),
    ("glu_q80", R.Q8_0, 4096, 2048, 1, 1),
    ("glu_q6k", R.Q6_K, 4096, 2048, 1, 1),
    ("head_q6k_big", R.Q6_K, 4096, 128256, 0, 1),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("entry", ["dec", "stream", "q4k"])
def test_gemv_dec_vs_unfused(env, case, entry):
    torch, K = env
    name, t, Kd, N, mode, pro = case
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(Kd, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(Kd, generator=g)).cuda()
    res = torch.randn(N, generator=g).cuda()
    W = _w(torch, K, t, Kd, N, 1)
    W2 = _w(torch, K, t, Kd, N, 2) if mode == 1 else None
    act = _ref_act(torch, K, t, x, nw, Kd, norm=(pro == 1))
    yref = torch.empty(N, device="cuda")
    use_res = mode == 0 and pro != 1
    K.call("kcpp_gemv", t, W.data_ptr(), W2.data_ptr() if W2 is not None else None, Kd, N, act.data_ptr(), 1,
           yref.data_ptr(), N, res.data_ptr() if use_res else None, N, mode, s)
    y = torch.full((N,), float("nan"), device="cuda")
    a = _args(K, K=Kd, nseg=1, W=[W.data_ptr()], N=[N], Y=[y.data_ptr()], x=x.data_ptr(), nw=nw.data_ptr(), eps=1e-5,
              act=act.data_ptr(), res=res.data_ptr() if use_res else None,
              W2=W2.data_ptr() if W2 is not None else None)
    if entry == "stream":
        rc = int(K.raw().kcpp_gemv_stream(t, __import__("ctypes").byref(a), mode, pro, s))
        if rc == -3:
            pytest.skip("shape/type not covered by the streaming kernel")
    elif entry == "q4k":
        if t != R.Q4_K:
            pytest.skip("type-specific kernel")
        rc = int(K.raw().kcpp_gemv_q4k(__import__("ctypes").byref(a), mode, pro, s))
        if rc == -3:
            pytest.skip("shape not covered")
    else:
        rc = K.gemv_dec(t, a, mode, pro, 1, s)
    assert rc == 0
    torch.cuda.synchronize()
    _close(y.cpu().numpy(), yref.cpu().numpy())


@pytest.mark.parametrize("entry", ["dec", "stream", "q4k"])
@pytest.mark.parametrize("pos", [0, 77, 4000])
def test_gemv_dec_qkv_rope_kv(env, entry, pos):
    """mode 2: q|k|v mat-vec + RoPE + f16 stores, vs kcpp_gemv + kcpp_rope_kv"""
    torch, K = env
    import ctypes
    t, E, EKV, D, H, HKV, n_ctx = R.Q4_K, 4096, 1024, 128, 32, 8, 4096
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(E, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(E, generator=g)).cuda()
    Wq, Wk, Wv = _w(torch, K, t, E, E, 3), _w(torch, K, t, E, EKV, 4), _w(torch, K, t, E, EKV, 5)
    tab = np.empty(n_ctx * D, np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tab_d = torch.from_numpy(tab).cuda()
    act = _ref_act(torch, K, t, x, nw, E)
    qkv = torch.empty(E + 2 * EKV, device="cuda")
    for W, off, n in ((Wq, 0, E), (Wk, E, EKV), (Wv, E + EKV, EKV)):
        K.call("kcpp_gemv", t, W.data_ptr(), None, E, n, act.data_ptr(), 1, qkv[off:].data_ptr(), n, None, 0, 0, s)
    posd = torch.tensor([pos], dtype=torch.int32, device="cuda")
    q16r = torch.zeros(E, dtype=torch.int16, device="cuda")
    kcr = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    vcr = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    K.call("kcpp_rope_kv", qkv.data_ptr(), E + 2 * EKV, None, q16r.data_ptr(), kcr.data_ptr(), vcr.data_ptr(), 1, H, HKV,
           D, 0, posd.data_ptr(), tab_d.data_ptr(), s)
    q16 = torch.zeros_like(q16r)
    kc = torch.zeros_like(kcr)
    vc = torch.zeros_like(vcr)
    a = _args(K, K=E, nseg=3, W=[Wq.data_ptr(), Wk.data_ptr(), Wv.data_ptr()], N=[E, EKV, EKV], role=[0, 1, 2],
              x=x.data_ptr(), nw=nw.data_ptr(), eps=1e-5, q16=q16.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(),
              ekv=EKV, D=D, pos=posd.data_ptr(), rope_tab=tab_d.data_ptr())
    if entry == "stream":
        rc = int(K.raw().kcpp_gemv_stream(t, ctypes.byref(a), 2, 1, s))
        if rc == -3:
            pytest.skip("shape/type not covered by the streaming kernel")
    elif entry == "q4k":
        rc = int(K.raw().kcpp_gemv_q4k(ctypes.byref(a), 2, 1, s))
    else:
        rc = K.gemv_dec(t, a, 2, 1, 2, s)
    assert rc == 0
    torch.cuda.synchronize()
    f = lambda z: z.cpu().numpy().view(np.float16).astype(np.float32)
    _close(f(q16), f(q16r), rtol=2e-3)          # f16 outputs: allow one f16 ulp flips
    sl = slice(pos * EKV, (pos + 1) * EKV)
    _close(f(kc[sl]), f(kcr[sl]), rtol=2e-3)
    _close(f(vc[sl]), f(vcr[sl]), rtol=2e-3)
    assert f(kc).any() and np.count_nonzero(f(kc)) == np.count_nonzero(f(kc[sl]))
