"""The Q8_0 tile layout KT_Q8_0_T and its GEMM (koboldcpp_amd/csrc/gemm_q80t.hip): every batch size of a Q8_0 model's
layer matrices (BASELINE config 3: Llama-3-8B Q8_0, ubatches of 32).

* layout: synthetic weights written in the tile layout and repacked back equal the ggml bytes (the reference's
  block_q8_0, ggml-common.h:223) byte for byte;
* kcpp_rms_norm_q80t / kcpp_quantize_act(KT_Q8_0_TA) hold exactly the Q8_0 quantization of kcpp_quantize_act(Q8_0)
  (the AVX2 quantize_row_q8_0 semantics, pinned in test_gpu_kernels.py) in the fragment order;
* GEMM vs the C restatement of ggml_vec_dot_q8_0_q8_0 / ggml_compute_forward_mul_mat (oracle/ggml_oracle.c) at the
  config-3 shapes and ragged / small / large batches: max |gpu - oracle| <= 3e-6 x max |oracle| (the integer block dots
  are exact; only the fp32 combination order of the per-block terms differs), plain, + residual, silu GLU;
* the GLU epilogue's quantization of h equals kcpp_quantize_act(KT_Q8_0_TA) of the f32 h byte for byte;
* batch invariance: a token's output does not depend on how many tokens share the launch (M = 1 vs 32 vs 100, bit for
  bit), and a second launch on the same workspace gives the same bits (split-K tickets left at zero)."""
import ctypes

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

RTOL = 3e-6


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


def dev_t(torch, K, Kd, N, tid):
    w = torch.empty(K.row_bytes(R.Q8_0, Kd) * N, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", K.Q8_0_T, 5, tid, w.data_ptr(), Kd, N, sptr(torch))
    return w


def quant_ta(torch, K, X):
    M, Kd = X.shape
    xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).cuda()
    act = torch.zeros(K.act_bytes(K.Q8_0_T, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.Q8_0_TA, xd.data_ptr(), Kd, act.data_ptr(), Kd, M, sptr(torch))
    return act


def ws_for(torch, K, Kd, N, M):
    return torch.zeros(int(K.raw().kcpp_gemm_workspace_bytes(K.Q8_0_T, Kd, N, M)), dtype=torch.uint8, device="cuda")


def gemm(torch, K, Ws, Ns, Kd, act, M, mode=0, W2=None, res=None, qout=None, ws=None):
    N = sum(Ns) if mode == 0 else Ns[0]
    Y = torch.full((M, N), float("nan"), dtype=torch.float32, device="cuda")
    wp = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in Ws])
    np_ = (ctypes.c_int64 * 3)(*Ns)
    ws = ws if ws is not None else ws_for(torch, K, Kd, N, M)
    K.call("kcpp_gemm_q80t", wp, np_, len(Ws), W2.data_ptr() if W2 is not None else None, Kd, act.data_ptr(), M,
           Y.data_ptr(), N, res.data_ptr() if res is not None else None, N, mode,
           qout.data_ptr() if qout is not None else None, ws.data_ptr(), sptr(torch))
    torch.cuda.synchronize()
    return Y.cpu().numpy()


def test_layout_roundtrip(env):
    torch, K = env
    Kd, N = 1024, 96
    w = dev_t(torch, K, Kd, N, 3)
    back = torch.empty_like(w)
    K.call("kcpp_weight_repack", K.Q8_0_T, w.data_ptr(), back.data_ptr(), Kd, N, 1, sptr(torch))
    torch.cuda.synchronize()
    assert np.array_equal(back.cpu().numpy(), R.synth(R.Q8_0, 5, 3, Kd, N))
    fwd = torch.empty_like(w)
    src = torch.from_numpy(R.synth(R.Q8_0, 5, 3, Kd, N)).cuda()
    K.call("kcpp_weight_repack", K.Q8_0_T, src.data_ptr(), fwd.data_ptr(), Kd, N, 0, sptr(torch))
    torch.cuda.synchronize()
    assert torch.equal(fwd, w)


@pytest.mark.parametrize("M", [1, 5, 32, 45])
def test_ta_quantization_matches_q8_0(env, M):
    """the TA layout holds kcpp_quantize_act(Q8_0)'s bytes and f16-rounded scales, in fragment order; the fused
    rms_norm variant equals rms_norm then the TA quantization"""
    torch, K = env
    Kd = 1024
    X = np.random.default_rng(M).standard_normal((M, Kd)).astype(np.float32)
    ta = quant_ta(torch, K, X).cpu().numpy()
    xd = torch.from_numpy(X).cuda()
    q0 = torch.zeros(K.act_bytes(R.Q8_0, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", R.Q8_0, xd.data_ptr(), Kd, q0.data_ptr(), Kd, M, sptr(torch))
    torch.cuda.synchronize()
    q0 = q0.cpu().numpy()
    nb, G = Kd // 32, (M + 31) // 32
    qs = q0[:M * Kd].reshape(M, nb, 2, 16)
    d = q0[M * Kd:M * Kd + M * nb * 4].view(np.float32).reshape(M, nb)
    tq = ta[:G * 32 * Kd].reshape(G, nb, 2, 32, 16)
    td = ta[G * 32 * Kd:G * 32 * Kd + G * nb * 32 * 4].view(np.float32).reshape(G, nb, 32)
    for m in range(M):
        g, t = divmod(m, 32)
        assert np.array_equal(tq[g, :, :, t, :], qs[m]), m
        assert np.array_equal(td[g, :, t], d[m]), m
    w = (1 + 0.1 * np.random.default_rng(7).standard_normal(Kd)).astype(np.float32)
    wd = torch.from_numpy(w).cuda()
    fused = torch.zeros_like(torch.from_numpy(ta)).cuda()
    K.call("kcpp_rms_norm_q80t", xd.data_ptr(), Kd, wd.data_ptr(), fused.data_ptr(), Kd, M, 1e-5, sptr(torch))
    sep = quant_ta(torch, K, R.rms_norm(X, w, 1e-5)).cpu().numpy()
    fz = fused.cpu().numpy()
    nq = G * 32 * Kd
    for m in range(M):
        g, t = divmod(m, 32)
        assert np.array_equal(fz[:nq].reshape(G, nb, 2, 32, 16)[g, :, :, t], sep[:nq].reshape(G, nb, 2, 32, 16)[g, :, :, t])
        assert np.array_equal(fz[nq:nq + G * nb * 128].view(np.float32).reshape(G, nb, 32)[g, :, t],
                              sep[nq:nq + G * nb * 128].view(np.float32).reshape(G, nb, 32)[g, :, t])


SHAPES = [(4096, 14336, 32), (14336, 4096, 32), (4096, 4096, 32), (4096, 1024, 1), (512, 128, 7), (4096, 4096, 45),
          (1024, 2048, 100)]


@pytest.mark.parametrize("Kd,N,M", SHAPES)
def test_gemm_vs_oracle(env, Kd, N, M):
    torch, K = env
    rng = np.random.default_rng(Kd + N + M)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float32)
    W = dev_t(torch, K, Kd, N, 11)
    ref = R.mul_mat(R.Q8_0, R.synth(R.Q8_0, 5, 11, Kd, N), Kd, N, X)
    act = quant_ta(torch, K, X)
    tol = RTOL * max(1.0, np.abs(ref).max())
    got = gemm(torch, K, [W], [N], Kd, act, M)
    assert np.abs(got - ref).max() <= tol, np.abs(got - ref).max()
    rd = torch.from_numpy(res).cuda()
    got = gemm(torch, K, [W], [N], Kd, act, M, res=rd)
    assert np.abs(got - (ref + res)).max() <= tol + 1e-6


@pytest.mark.parametrize("Kd,N,M", [(4096, 14336, 32), (512, 1024, 9), (1024, 512, 70)])
def test_gemm_glu_vs_oracle_and_quantized_h(env, Kd, N, M):
    torch, K = env
    rng = np.random.default_rng(Kd * 3 + N + M)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    Wg, Wu = dev_t(torch, K, Kd, N, 21), dev_t(torch, K, Kd, N, 22)
    g = R.mul_mat(R.Q8_0, R.synth(R.Q8_0, 5, 21, Kd, N), Kd, N, X)
    u = R.mul_mat(R.Q8_0, R.synth(R.Q8_0, 5, 22, Kd, N), Kd, N, X)
    ref = (g / (1 + np.exp(-g))) * u
    act = quant_ta(torch, K, X)
    h = gemm(torch, K, [Wg], [N], Kd, act, M, mode=1, W2=Wu)
    assert np.abs(h - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    # the epilogue's TA quantization of h == kcpp_quantize_act(TA) of that f32 h, for every token < M
    q = torch.full((K.act_bytes(K.Q8_0_T, N, M),), 0xA5, dtype=torch.uint8, device="cuda")
    gemm(torch, K, [Wg], [N], Kd, act, M, mode=1, W2=Wu, qout=q)
    want = quant_ta(torch, K, h).cpu().numpy()
    got = q.cpu().numpy()
    nb, G = N // 32, (M + 31) // 32
    for m in range(M):
        gi, t = divmod(m, 32)
        assert np.array_equal(got[:G * 32 * N].reshape(G, nb, 2, 32, 16)[gi, :, :, t],
                              want[:G * 32 * N].reshape(G, nb, 2, 32, 16)[gi, :, :, t]), m
        off = G * 32 * N
        assert np.array_equal(got[off:off + G * nb * 128].view(np.float32).reshape(G, nb, 32)[gi, :, t],
                              want[off:off + G * nb * 128].view(np.float32).reshape(G, nb, 32)[gi, :, t]), m


def test_qkv_segments(env):
    """q|k|v as one launch over three segments equals one matrix of the concatenated rows bit for bit (the split is a
    function of the launch's total shape), and the three separate mat-muls (their own splits) to f32 summation-order
    rounding"""
    torch, K = env
    Kd, Ns, M = 4096, [4096, 1024, 1024], 32
    X = np.random.default_rng(9).standard_normal((M, Kd)).astype(np.float32)
    Ws = [dev_t(torch, K, Kd, n, 30 + i) for i, n in enumerate(Ns)]
    act = quant_ta(torch, K, X)
    one = gemm(torch, K, Ws, Ns, Kd, act, M)
    # KT_Q8_0_T of the stacked rows: the tile planes in order, then the scale planes in order
    cat = torch.cat([w[:n * Kd] for w, n in zip(Ws, Ns)] + [w[n * Kd:] for w, n in zip(Ws, Ns)])
    whole = gemm(torch, K, [cat], [sum(Ns)], Kd, act, M)
    assert np.array_equal(one.view(np.uint32), whole.view(np.uint32))
    parts = np.concatenate([gemm(torch, K, [w], [n], Kd, act, M) for w, n in zip(Ws, Ns)], axis=1)
    assert np.abs(one - parts).max() <= 1e-5 * np.abs(parts).max()


@pytest.mark.parametrize("Kd,N", [(4096, 4096), (14336, 4096), (4096, 14336)])
def test_batch_invariance_and_ticket_reset(env, Kd, N):
    """token t's row is the same bits whether it is computed alone, in a 32-token or in a 100-token launch; the
    same launch twice on one workspace gives the same bits (the split-K tickets are left at zero)"""
    torch, K = env
    X = np.random.default_rng(N).standard_normal((100, Kd)).astype(np.float32)
    W = dev_t(torch, K, Kd, N, 41)
    ws = ws_for(torch, K, Kd, N, 100)
    full = gemm(torch, K, [W], [N], Kd, quant_ta(torch, K, X), 100, ws=ws)
    again = gemm(torch, K, [W], [N], Kd, quant_ta(torch, K, X), 100, ws=ws)
    assert np.array_equal(full.view(np.uint32), again.view(np.uint32))
    b32 = gemm(torch, K, [W], [N], Kd, quant_ta(torch, K, X[40:72]), 32, ws=ws)
    assert np.array_equal(b32.view(np.uint32), full[40:72].view(np.uint32))
    for t in (0, 57, 99):
        one = gemm(torch, K, [W], [N], Kd, quant_ta(torch, K, X[t:t + 1]), 1, ws=ws)
        assert np.array_equal(one[0].view(np.uint32), full[t].view(np.uint32)), t


@pytest.mark.parametrize("M,n_past,dev_pos", [(32, 1000, False), (7, 4000, False), (1, 3839, True), (45, 17, True)])
def test_qkv_rope_epilogue(env, M, n_past, dev_pos):
    """q|k|v with the rope + f16 K/V stores in the GEMM epilogue == the GEMM then kcpp_rope_kv, bit for bit (q16, the
    cache rows at the positions, nothing else written)"""
    torch, K = env
    Kd, H, HKV, D, n_ctx = 4096, 32, 8, 128, 4096
    Ns = [H * D, HKV * D, HKV * D]
    X = np.random.default_rng(M).standard_normal((M, Kd)).astype(np.float32)
    Ws = [dev_t(torch, K, Kd, n, 60 + i) for i, n in enumerate(Ns)]
    act = quant_ta(torch, K, X)
    tab = np.empty((n_ctx, D // 2, 2), np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tabd = torch.from_numpy(tab).cuda()
    pos = np.arange(n_past, n_past + M, dtype=np.int32)
    if dev_pos:
        pos = np.random.default_rng(1).permutation(n_ctx)[:M].astype(np.int32)   # scattered positions
    posd = torch.from_numpy(pos).cuda()
    qkv = torch.from_numpy(gemm(torch, K, Ws, Ns, Kd, act, M)).cuda()
    outs = []
    for fused in (False, True):
        q16 = torch.zeros((M, H * D), dtype=torch.int16, device="cuda")
        kc = torch.zeros((n_ctx, HKV * D), dtype=torch.int16, device="cuda")
        vc = torch.zeros((n_ctx, HKV * D), dtype=torch.int16, device="cuda")
        if fused:
            wp = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in Ws])
            np_ = (ctypes.c_int64 * 3)(*Ns)
            K.call("kcpp_gemm_q80t_qkv_rope", wp, np_, Kd, act.data_ptr(), M, tabd.data_ptr(), n_past,
                   posd.data_ptr() if dev_pos else None, D, q16.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                   ws_for(torch, K, Kd, sum(Ns), M).data_ptr(), sptr(torch))
        else:
            K.call("kcpp_rope_kv", qkv.data_ptr(), sum(Ns), None, q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), M, H,
                   HKV, D, n_past, posd.data_ptr() if dev_pos else None, tabd.data_ptr(), sptr(torch))
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in (q16, kc, vc)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert np.count_nonzero(outs[1][1].any(axis=1)) == M       # exactly the M positions' rows written
