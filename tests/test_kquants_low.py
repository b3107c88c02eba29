"""Q2_K, Q3_K, Q5_0, Q4_1, Q5_1, IQ4_NL and IQ4_XS weights (Q2_K / Q3_K_S / Q3_K_M / Q5_0 / Q4_1 / Q5_1 / IQ4_NL /
IQ4_XS models; block_q2_K / block_q3_K / block_q5_0 / block_q4_1 / block_q5_1 / block_iq4_nl / block_iq4_xs,
ggml-common.h:250,267,161,149,168,407,413; Q4_1 / Q5_1 dot Q8_1 activations, block_q8_1.s = f16(d * sum qs); IQ4_NL
dot Q8_0, IQ4_XS dot Q8_K through the kvalues_iq4nl code book): the CPU oracle and the HIP kernels against the reference
builds' own outputs (tests/golden/q2k.npz / q3k.npz / q50.npz / q41.npz / q51.npz / iq4nl.npz / iq4xs.npz,
make_q2k.py / make_q3k.py / make_legacy32.py / make_iq4.py).

* oracle (CPU): dequantize_row_q3_K bit-exact on synthetic and random-bit blocks; mul_mat at decode / small-batch /
  prefill shapes within 3e-6 of the output scale (a different fp32 summation order than ggml_vec_dot_q3_K_q8_K);
* GPU: the SoA device layout round-trips and dequantizes bit-exactly; the generic mat-vec (kcpp_gemv), the fused
  decode mat-vec (kcpp_gemv_dec: plain + residual, SiLU-GLU, rms_norm prologue) and the MFMA GEMM (exact integer
  f16 operands: Q3_K (sc - 32)(v - 4), Q2_K (sc & 15) q with the mins through the bsum MFMA, Q5_0 (q | h << 4) - 16,
  Q4_1 / Q5_1 q (| h << 4) with the m_w s_a term as an fp32 MFMA over the block scales, IQ4_NL code-book values, IQ4_XS
  (ls - 32) kv split over two planes; past 16 tokens) against the golden and
  the oracle at 3e-6; a tiny Llama under the Q3_K_M / Q2_K / Q5_0 policy end to end (prefill + teacher-forced decode, graph
  and eager) within 1.5x the reference's AVX2-vs-scalar spread."""
import os

import numpy as np
import pytest

import refharness as R

KINDS = {"q3_k": (R.Q3_K, "q3k.npz"), "q2_k": (R.Q2_K, "q2k.npz"), "q5_0": (R.Q5_0, "q50.npz"),
         "q4_1": (R.Q4_1, "q41.npz"), "q5_1": (R.Q5_1, "q51.npz"), "iq4_nl": (R.IQ4_NL, "iq4nl.npz"),
         "iq4_xs": (R.IQ4_XS, "iq4xs.npz")}


@pytest.fixture(scope="module", params=sorted(KINDS))
def kq(request):
    t, f = KINDS[request.param]
    return t, np.load(os.path.join(R.ROOT, "tests", "golden", f))


def test_oracle_dequant_bit_exact(kq):
    T, g = kq
    for tag in ("syn", "rnd"):
        got = R.dequant(T, g["deq_%s_in" % tag], g["deq_%s_out" % tag].size)
        assert np.array_equal(got.view(np.uint32), g["deq_%s_out" % tag].view(np.uint32)), tag


@pytest.mark.parametrize("shape", [(4096, 256, 1), (4096, 128, 8), (1024, 64, 40)])
def test_oracle_mul_mat_vs_reference(kq, shape):
    T, g = kq
    key = "mm_%d_%d_%d" % shape
    t, seed, tid, xseed, K, N, M = [int(v) for v in g[key + "_meta"]]
    w = R.synth(t, seed, tid, K, N)
    X = np.random.default_rng(xseed).standard_normal((M, K)).astype(np.float32)
    want = g[key + "_y"]
    np.testing.assert_allclose(R.mul_mat(t, w, K, N, X), want, rtol=0, atol=3e-6 * max(1.0, np.abs(want).max()))


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import koboldcpp_amd.lib as K
    return torch, K


def _sp(torch):
    return torch.cuda.current_stream().cuda_stream


def _upload(torch, K, data, Kd, N, T):
    src = torch.from_numpy(np.ascontiguousarray(data)).cuda()
    dst = torch.empty_like(src)
    K.call("kcpp_weight_repack", T, src.data_ptr(), dst.data_ptr(), Kd, N, 0, _sp(torch))
    return dst


@pytest.mark.gpu
def test_gpu_layout_and_dequant(env, kq):
    torch, K = env
    T, g = kq
    for tag in ("syn", "rnd"):
        data, want = g["deq_%s_in" % tag], g["deq_%s_out" % tag]
        d = _upload(torch, K, data, want.size, 1, T)
        back = torch.empty_like(d)
        K.call("kcpp_weight_repack", T, d.data_ptr(), back.data_ptr(), want.size, 1, 1, _sp(torch))
        y = torch.empty(want.size, dtype=torch.float32, device="cuda")
        K.call("kcpp_dequantize", T, d.data_ptr(), y.data_ptr(), want.size, 1, _sp(torch))
        torch.cuda.synchronize()
        assert np.array_equal(back.cpu().numpy(), data)
        assert np.array_equal(y.cpu().numpy().view(np.uint32), want.view(np.uint32)), tag
    # device synth == host synth, through the layout
    Kd, N = 2048, 8
    w = R.synth(T, 5, 77, Kd, N)
    s = torch.empty(w.nbytes, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", T, 5, 77, s.data_ptr(), Kd, N, _sp(torch))
    torch.cuda.synchronize()
    assert np.array_equal(s.cpu().numpy(), _upload(torch, K, w, Kd, N, T).cpu().numpy())


def _gpu_mul_mat(torch, K, T, w, Kd, N, X, mode=0, w2=None, res=None):
    M = X.shape[0]
    wd = _upload(torch, K, w, Kd, N, T)
    w2d = _upload(torch, K, w2, Kd, N, T) if w2 is not None else None
    xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).cuda()
    act = torch.zeros(K.act_bytes(T, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(T), xd.data_ptr(), Kd, act.data_ptr(), Kd, M, _sp(torch))
    Y = torch.empty((M, N), dtype=torch.float32, device="cuda")
    rd = torch.from_numpy(np.ascontiguousarray(res, np.float32)).cuda() if res is not None else None
    w2p = w2d.data_ptr() if w2d is not None else None
    rp = rd.data_ptr() if rd is not None else None
    if M <= 8:
        K.call("kcpp_gemv", T, wd.data_ptr(), w2p, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, rp, N, mode, _sp(torch))
    else:
        ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(T, Kd, N, M), dtype=torch.uint8, device="cuda")
        K.call("kcpp_gemm", T, wd.data_ptr(), w2p, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, rp, N, mode,
               ws.data_ptr(), _sp(torch))
    torch.cuda.synchronize()
    return Y.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4096, 256, 1), (4096, 128, 8), (1024, 64, 40)])
def test_gpu_mul_mat_vs_reference_golden(env, kq, shape):
    torch, K = env
    T, g = kq
    key = "mm_%d_%d_%d" % shape
    t, seed, tid, xseed, Kd, N, M = [int(v) for v in g[key + "_meta"]]
    w = R.synth(t, seed, tid, Kd, N)
    X = np.random.default_rng(xseed).standard_normal((M, Kd)).astype(np.float32)
    want = g[key + "_y"]
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, T, w, Kd, N, X), want, rtol=0, atol=3e-6 * max(1.0, np.abs(want).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 17, 64, 300])
def test_gpu_mul_mat_modes_vs_oracle(env, kq, M):
    torch, K = env
    T, _ = kq
    Kd, N = 2048, 96
    rng = np.random.default_rng(M)
    w, w2 = R.synth(T, 9, 1011, Kd, N), R.synth(T, 9, 2011, Kd, N)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float32)
    a, b = R.mul_mat(T, w, Kd, N, X), R.mul_mat(T, w2, Kd, N, X)
    tol = 3e-6 * max(1.0, np.abs(a).max())
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, T, w, Kd, N, X, res=res), a + res, rtol=0, atol=tol + 1e-6)
    glu = (a / (1 + np.exp(-a))) * b
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, T, w, Kd, N, X, mode=1, w2=w2), glu, rtol=1e-5, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,pro", [(0, 0), (0, 2), (1, 1)])
def test_gpu_fused_decode_matvec(env, kq, mode, pro):
    """kcpp_gemv_dec (the single-token decode step's fused mat-vec) on Q3_K vs the oracle: plain + residual with the
    activation given (PRO 0) or quantized in the prologue (PRO 2), SiLU-GLU with the rms_norm prologue (PRO 1)"""
    torch, K = env
    T, _ = kq
    if T in (R.Q4_1, R.Q5_1, R.IQ4_NL, R.IQ4_XS):
        pytest.skip("Q8_1-activation and code-book types have no fused decode mat-vec: the runtime decodes them per op")
    Kd, N = 4096, 512
    rng = np.random.default_rng(7 + mode + pro)
    x = rng.standard_normal(Kd).astype(np.float32)
    nw = (1 + 0.01 * rng.standard_normal(Kd)).astype(np.float32)
    res = rng.standard_normal(N).astype(np.float32)
    w, w2 = R.synth(T, 3, 31, Kd, N), R.synth(T, 3, 32, Kd, N)
    xin = R.rms_norm(x[None], nw, 1e-5)[0] if pro == 1 else x
    a = R.mul_mat(T, w, Kd, N, xin[None])[0]
    want = (a / (1 + np.exp(-a))) * R.mul_mat(T, w2, Kd, N, xin[None])[0] if mode == 1 else a + res
    s = _sp(torch)
    xd, nwd, rd = (torch.from_numpy(v).cuda() for v in (x, nw, res))
    act = torch.zeros(K.act_bytes(T, Kd, 1), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(T), xd.data_ptr(), Kd, act.data_ptr(), Kd, 1, s)
    wd, w2d = _upload(torch, K, w, Kd, N, T), _upload(torch, K, w2, Kd, N, T)
    y = torch.full((N,), float("nan"), device="cuda")
    a_ = K.DecArgs()
    a_.K, a_.nseg, a_.x, a_.nw, a_.eps, a_.act = Kd, 1, xd.data_ptr(), nwd.data_ptr(), 1e-5, act.data_ptr()
    a_.W[0], a_.N[0], a_.Y[0] = wd.data_ptr(), N, y.data_ptr()
    a_.res = rd.data_ptr() if mode == 0 else None
    a_.W2 = w2d.data_ptr() if mode == 1 else None
    assert K.gemv_dec(T, a_, mode, pro, 1, s) == 0
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), want, rtol=1e-5, atol=3e-6 * max(1.0, np.abs(want).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [True, False], ids=["graph", "eager"])
def test_gpu_model_vs_reference(env, kq, graphs):
    """tiny Llama, Q3_K_M policy (Q3_K embedding / q / k / gate / up, Q5_K / Q4_K v, Q4_K wo, Q3_K / Q4_K down, Q6_K
    head) or Q2_K policy (Q2_K embedding / q / k / gate / up, Q3_K v / wo / down, Q6_K head): prefill + 8
    teacher-forced decode steps vs the reference logits, within 1.5x its own build spread"""
    torch, K = env
    T, g = kq
    types = [int(t) for t in g["e2e_types"]]
    m = K.Model(R.TINY, types)
    m.set_graphs(graphs)
    m.synth(1234)
    out = [m.decode(g["e2e_prompt"], 0)]
    n = len(g["e2e_prompt"])
    for tok in g["e2e_forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    d = np.abs(np.array(out) - g["e2e_logits"])
    print("gpu vs ref max", d.max(axis=1), "| spread", g["e2e_spread_max"])
    assert np.all(d.max(axis=1) <= 1.5 * g["e2e_spread_max"].max())
    assert np.all(np.median(d, axis=1) <= 1.5 * g["e2e_spread_median"].max())
