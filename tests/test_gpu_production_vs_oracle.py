"""Direct oracle parity of the PRODUCTION decode and prefill kernels at BASELINE config-2 shapes
(Llama-3-8B: n_embd 4096, n_ff 14336, n_head_kv 8, vocab 128256).

Each case launches exactly what the runtime launches (csrc/runtime.cpp forward_layers_dec / forward_layers)
-- k_gemv_rs through kcpp_gemv_dec on the row-major Q4_K_RS / Q6_K_RS layouts, and kcpp_gemm on the same
layouts at M = 512 (the v3 MFMA kernels) -- and compares with the C restatement of the reference CPU path
(oracle/ggml_oracle.c: quantize_row_q8_K_ref, ggml_vec_dot_q4_K_q8_K / q6_K, ggml-quants.c:3786,7714,8919;
rms_norm ggml.c:12059; rope ggml.c:14272), which tests/test_oracle_golden.py pins to the reference build.

Tolerance: the integer block dots are exact on both sides; only the order of the fp32 combination of the
per-superblock terms differs, so outputs agree to a few fp32 ulps of the row's magnitude:
    max |gpu - oracle| <= RTOL * max |oracle|,   RTOL = 3e-6
f16 outputs (q, K/V cache rows) may differ by the f16 rounding of such an ulp: <= 1 f16 ulp.
For the GEMMs the full production grid runs; the oracle recomputes a row subset (both ends + a random
sample) to stay within seconds on the host."""
import ctypes

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

RTOL = 3e-6
RS = {R.Q4_K: 112, R.Q6_K: 114}
E, F, EKV, D, V = 4096, 14336, 1024, 128, 128256
SEED = 21


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


def dev_synth(torch, K, t, Kd, N, tid):
    w = torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", t, SEED, tid, w.data_ptr(), Kd, N, sptr(torch))
    return w


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def f16_ulp_ok(a16, b16):
    """|a - b| <= one f16 ulp of the larger magnitude (f16 arrays)"""
    a, b = a16.astype(np.float32), b16.astype(np.float32)
    m = np.maximum(np.abs(a), np.abs(b))
    ulp = np.spacing(m.astype(np.float16)).astype(np.float32)
    return np.all(np.abs(a - b) <= ulp)


def silu(x):
    return x / (np.float32(1) + np.exp(-x, dtype=np.float32))


def vecs(Kd, n_extra, seed):
    g = np.random.default_rng(seed)
    x = g.standard_normal(Kd).astype(np.float32)
    nw = (1 + 0.01 * g.standard_normal(Kd)).astype(np.float32)
    extra = g.standard_normal(n_extra).astype(np.float32)
    return x, nw, extra


def test_glu_gate_up_q4k(env):
    """ffn_norm -> Q8_K -> gate|up -> silu(g)*u: k_gemv_rs<Q4_K_RS, GLU, norm prologue>, 4096 -> 2 x 14336"""
    torch, K = env
    x, nw, _ = vecs(E, 0, 1)
    Wg, Wu = dev_synth(torch, K, RS[R.Q4_K], E, F, 1), dev_synth(torch, K, RS[R.Q4_K], E, F, 2)
    y = torch.full((F,), float("nan"), device="cuda")
    xd, nwd = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    a = K.DecArgs()
    a.K, a.nseg, a.x, a.nw, a.eps = E, 1, xd.data_ptr(), nwd.data_ptr(), 1e-5
    a.W[0], a.W2, a.N[0], a.Y[0] = Wg.data_ptr(), Wu.data_ptr(), F, y.data_ptr()
    assert K.gemv_dec(RS[R.Q4_K], a, 1, 1, 1, sptr(torch)) == 0
    torch.cuda.synchronize()
    h = R.rms_norm(x, nw, 1e-5)
    g = R.mul_mat(R.Q4_K, R.synth(R.Q4_K, SEED, 1, E, F), E, F, h)[0]
    u = R.mul_mat(R.Q4_K, R.synth(R.Q4_K, SEED, 2, E, F), E, F, h)[0]
    ref = silu(g) * u
    assert rel_err(y.cpu().numpy(), ref) < RTOL


@pytest.mark.parametrize("base", [R.Q4_K, R.Q6_K])
def test_down_residual(env, base):
    """x += down . Q8_K(h): k_gemv_rs<.., quantize prologue, residual>, 14336 -> 4096 (Q4_K and the
    more-bits layers' Q6_K)"""
    torch, K = env
    h, _, res = vecs(F, E, 2)
    W = dev_synth(torch, K, RS[base], F, E, 3)
    hd, y = torch.from_numpy(h).cuda(), torch.from_numpy(res).cuda()
    a = K.DecArgs()
    a.K, a.nseg, a.x = F, 1, hd.data_ptr()
    a.W[0], a.N[0], a.Y[0], a.res = W.data_ptr(), E, y.data_ptr(), y.data_ptr()
    assert K.gemv_dec(RS[base], a, 0, 2, 1, sptr(torch)) == 0
    torch.cuda.synchronize()
    ref = R.mul_mat(base, R.synth(base, SEED, 3, F, E), F, E, h)[0] + res
    assert rel_err(y.cpu().numpy(), ref) < RTOL


@pytest.mark.parametrize("base,Kd,N", [(R.Q4_K, 28672, 8192), (R.Q6_K, 28672, 8192), (R.Q5_K, 20480, 4096)],
                         ids=["q4k-70b-down", "q6k-70b-down", "q5k-long"])
def test_down_residual_long_k(env, base, Kd, N):
    """x += down . Q8_K(h) beyond the register-resident activation budget: Llama-3-70B's ffn_down (K = n_ff = 28672,
    Q4_K and the more-bits layers' Q6_K) and a long-K Q5_K (MoE experts with a large n_ff) on the XL variant of
    k_gemv_rs (activation slices read from the LDS image per piece)"""
    torch, K = env
    rs = {R.Q4_K: 112, R.Q5_K: 113, R.Q6_K: 114}[base]
    assert K.raw().kcpp_rs_supported(rs, Kd) == 1
    h, _, res = vecs(Kd, N, 7)
    W = dev_synth(torch, K, rs, Kd, N, 8)
    hd, y = torch.from_numpy(h).cuda(), torch.from_numpy(res).cuda()
    a = K.DecArgs()
    a.K, a.nseg, a.x = Kd, 1, hd.data_ptr()
    a.W[0], a.N[0], a.Y[0], a.res = W.data_ptr(), N, y.data_ptr(), y.data_ptr()
    assert K.gemv_dec(rs, a, 0, 2, 1, sptr(torch)) == 0
    torch.cuda.synchronize()
    ref = R.mul_mat(base, R.synth(base, SEED, 8, Kd, N), Kd, N, h)[0] + res
    assert rel_err(y.cpu().numpy(), ref) < RTOL


def test_wo_residual(env):
    """x += wo . attn (attn already Q8_K, written by the flash-attention combine)"""
    torch, K = env
    at, _, res = vecs(E, E, 3)
    W = dev_synth(torch, K, RS[R.Q4_K], E, E, 4)
    s = sptr(torch)
    atd = torch.from_numpy(at).cuda()
    act = torch.zeros(K.act_bytes(R.Q4_K, E, 1) + 64, dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", R.Q8_K, atd.data_ptr(), E, act.data_ptr(), E, 1, s)
    y = torch.from_numpy(res).cuda()
    a = K.DecArgs()
    a.K, a.nseg, a.act = E, 1, act.data_ptr()
    a.W[0], a.N[0], a.Y[0], a.res = W.data_ptr(), E, y.data_ptr(), y.data_ptr()
    assert K.gemv_dec(RS[R.Q4_K], a, 0, 0, 1, s) == 0
    torch.cuda.synchronize()
    ref = R.mul_mat(R.Q4_K, R.synth(R.Q4_K, SEED, 4, E, E), E, E, at)[0] + res
    assert rel_err(y.cpu().numpy(), ref) < RTOL


@pytest.mark.parametrize("vtype", [R.Q4_K, R.Q6_K])
@pytest.mark.parametrize("pos", [0, 3971])
def test_qkv_rope_kv_store(env, vtype, pos):
    """attn_norm -> Q8_K -> q|k|v -> RoPE (base 500000) -> f16 q and K/V cache rows at `pos`, exactly the
    launches forward_layers_dec makes (one per weight type present: q|k Q4_K_RS, v Q4_K_RS or Q6_K_RS)"""
    torch, K = env
    n_ctx = 4096
    x, nw, _ = vecs(E, 0, 4 + pos)
    s = sptr(torch)
    tab = np.empty(n_ctx * D, np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tab_d = torch.from_numpy(tab).cuda()
    posd = torch.tensor([pos], dtype=torch.int32, device="cuda")
    xd, nwd = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    types = [R.Q4_K, R.Q4_K, vtype]
    Ns = [E, EKV, EKV]
    Ws = [dev_synth(torch, K, RS[t], E, n, 10 + i) for i, (t, n) in enumerate(zip(types, Ns))]
    q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
    kc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    vc = torch.zeros(n_ctx * EKV, dtype=torch.int16, device="cuda")
    j = 0
    while j < 3:
        a = K.DecArgs()
        a.K, a.x, a.nw, a.eps = E, xd.data_ptr(), nwd.data_ptr(), 1e-5
        a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = (q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), EKV, D,
                                                           posd.data_ptr(), tab_d.data_ptr())
        t0 = types[j]
        while j < 3 and types[j] == t0:
            a.W[a.nseg], a.N[a.nseg], a.role[a.nseg] = Ws[j].data_ptr(), Ns[j], j
            a.nseg += 1
            j += 1
        assert K.gemv_dec(RS[t0], a, 2, 1, 2, s) == 0
    torch.cuda.synchronize()
    h = R.rms_norm(x, nw, 1e-5)
    q = R.mul_mat(R.Q4_K, R.synth(R.Q4_K, SEED, 10, E, E), E, E, h)[0]
    k = R.mul_mat(R.Q4_K, R.synth(R.Q4_K, SEED, 11, E, EKV), E, EKV, h)[0]
    v = R.mul_mat(vtype, R.synth(vtype, SEED, 12, E, EKV), E, EKV, h)[0]
    qr = R.rope(q.reshape(1, 32, D), [pos], 500000.0)[0].reshape(-1)
    kr = R.rope(k.reshape(1, 8, D), [pos], 500000.0)[0].reshape(-1)
    sl = slice(pos * EKV, (pos + 1) * EKV)
    f16 = lambda z: z.cpu().numpy().view(np.float16)
    assert f16_ulp_ok(f16(q16), qr.astype(np.float16))
    assert f16_ulp_ok(f16(kc[sl]), kr.astype(np.float16))
    assert f16_ulp_ok(f16(vc[sl]), v.astype(np.float16))


def test_output_head_q6k(env):
    """output_norm -> Q8_K -> logits: k_gemv_rs<Q6_K_RS, norm prologue>, 4096 -> 128256"""
    torch, K = env
    x, nw, _ = vecs(E, 0, 5)
    W = dev_synth(torch, K, RS[R.Q6_K], E, V, 6)
    y = torch.full((V,), float("nan"), device="cuda")
    xd, nwd = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    a = K.DecArgs()
    a.K, a.nseg, a.x, a.nw, a.eps = E, 1, xd.data_ptr(), nwd.data_ptr(), 1e-5
    a.W[0], a.N[0], a.Y[0] = W.data_ptr(), V, y.data_ptr()
    assert K.gemv_dec(RS[R.Q6_K], a, 0, 1, 4, sptr(torch)) == 0
    torch.cuda.synchronize()
    ref = R.mul_mat(R.Q6_K, R.synth(R.Q6_K, SEED, 6, E, V), E, V, R.rms_norm(x, nw, 1e-5))[0]
    assert rel_err(y.cpu().numpy(), ref) < RTOL


def _row_sample(N, n, seed):
    g = np.random.default_rng(seed)
    return np.unique(np.concatenate([np.arange(64), np.arange(N - 64, N), g.choice(N, n, replace=False)]))


@pytest.mark.parametrize("case", [("gate_up_q4k", R.Q4_K, E, 2 * F, False),
                                  ("down_q6k", R.Q6_K, F, E, True),
                                  ("down_q4k", R.Q4_K, F, E, True),
                                  ("wq_q4k", R.Q4_K, E, E + EKV, False)],
                         ids=lambda c: c[0])
def test_prefill_gemm_m512(env, case):
    """kcpp_gemm at ubatch 512 on the RS layouts (the v3 MFMA kernels the prefill dispatches): gate|up as
    one 4096 x 28672 GEMM, down 14336 x 4096 (+ residual), q|k 4096 x 5120"""
    torch, K = env
    name, base, Kd, N, with_res = case
    M = 512
    t = RS[base]
    s = sptr(torch)
    X = np.random.default_rng(Kd + N).standard_normal((M, Kd)).astype(np.float32)
    res = np.random.default_rng(7).standard_normal((M, N)).astype(np.float32) if with_res else None
    Xd = torch.from_numpy(X).cuda()
    act = torch.zeros(K.act_bytes(base, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", R.Q8_K, Xd.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    W = dev_synth(torch, K, t, Kd, N, 20)
    Y = torch.from_numpy(res).cuda() if with_res else torch.full((M, N), float("nan"), device="cuda")
    ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_gemm", t, W.data_ptr(), None, Kd, N, act.data_ptr(), M, Y.data_ptr(), N,
           Y.data_ptr() if with_res else None, N, 0, ws.data_ptr(), s)
    torch.cuda.synchronize()
    got = Y.cpu().numpy()
    assert np.isfinite(got).all()
    rows = _row_sample(N, 384, N)
    wb = R.synth(base, SEED, 20, Kd, N).reshape(N, -1)[rows]
    ref = R.mul_mat(base, wb, Kd, len(rows), X)
    if with_res:
        ref = ref + res[:, rows]
    assert rel_err(got[:, rows], ref) < RTOL
