"""Q6_K prefill image + int8-MFMA GEMM (kcpp_q6p_build / kcpp_gemm_q6p, csrc/gemm.hip k_gemm_q6p).

The image holds each weight's exact integer sc*(q-32) as two int8 planes (64 A + C); the GEMM multiplies them with
the Q8_K bytes on v_mfma_i32_32x32x32_i8 and applies q6v3's per-super-block epilogue in q6v3's order, under
q6v3's K-split rule.  So:
* its results equal kcpp_gemm(KT_Q6_K_RS) (q6v3, f16 MFMA) bit for bit -- plain, + residual, GLU (mode 1), split
  and unsplit shapes, ragged token counts (padding rows clamped);
* against the oracle (the reference CPU mul_mat, tests/refharness.py orc_mul_mat = ggml_vec_dot_q6_K_q8_K) within
  the fp32-order bar of test_gpu_kernels.py (3e-6 of the output scale);
* random scale / quant bytes (every sc in [-128, 127], every q in [0, 63]) reach the planes' extremes:
  A in [-64, 64], C in [-32, 31]."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

Q6_K_RS = 114


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


def _weights(torch, K, Kd, N, seed, rnd=False):
    """Q6_K_RS weights on the device: synthetic (include/kcpp_synth.h) or uniformly random ggml bytes with a sane d"""
    if rnd:
        rng = np.random.default_rng(seed)
        w = rng.integers(0, 256, size=(N * Kd // 256, 210), dtype=np.uint8)
        w[:, 208:210] = np.frombuffer(np.float16(0.01).tobytes(), np.uint8)   # d = 0.01 (finite, no overflow)
        w = w.ravel()
    else:
        w = R.synth(R.Q6_K, 11, seed, Kd, N)
    src = torch.from_numpy(w).cuda()
    rs = torch.empty_like(src)
    K.call("kcpp_weight_repack", Q6_K_RS, src.data_ptr(), rs.data_ptr(), Kd, N, 0, sptr(torch))
    return w, rs


def _image(torch, K, rs, Kd, N):
    nb = int(K.raw().kcpp_q6p_image_bytes(Kd, N))
    assert nb == N * Kd * 2
    img = torch.empty(nb, dtype=torch.uint8, device="cuda")
    K.call("kcpp_q6p_build", rs.data_ptr(), Kd, N, img.data_ptr(), sptr(torch))
    return img


def _act(torch, K, X):
    M, Kd = X.shape
    xd = torch.from_numpy(np.ascontiguousarray(X, np.float32)).cuda()
    act = torch.empty(K.act_bytes(R.Q6_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", R.Q8_K, xd.data_ptr(), Kd, act.data_ptr(), Kd, M, sptr(torch))
    return act


def _both(torch, K, rs, img, Kd, N, act, M, res=None, mode=0, rs2=None, img2=None):
    ws = torch.empty(int(K.raw().kcpp_gemm_workspace_bytes(Q6_K_RS, Kd, N, M)), dtype=torch.uint8, device="cuda")
    rp = res.data_ptr() if res is not None else None
    y3 = torch.full((M, N), float("nan"), device="cuda")
    y4 = torch.full((M, N), float("nan"), device="cuda")
    K.call("kcpp_gemm", Q6_K_RS, rs.data_ptr(), rs2.data_ptr() if rs2 is not None else None, Kd, N, act.data_ptr(), M,
           y3.data_ptr(), N, rp, N, mode, ws.data_ptr(), sptr(torch))
    K.call("kcpp_gemm_q6p", img.data_ptr(), rs.data_ptr(), img2.data_ptr() if img2 is not None else None,
           rs2.data_ptr() if rs2 is not None else None, Kd, N, act.data_ptr(), M, y4.data_ptr(), N, rp, N, mode,
           ws.data_ptr(), sptr(torch))
    torch.cuda.synchronize()
    return y3.cpu().numpy(), y4.cpu().numpy()


# (K, N, M): attn_v 4096 -> 1024 (split, small grid), wo-like 4096 -> 4096, ffn_down 14336 -> 4096 (long K, split),
# ragged token counts (partial 128-token tiles), one token tile
@pytest.mark.parametrize("Kd,N,M", [(4096, 1024, 512), (4096, 1024, 37), (4096, 4096, 200), (14336, 4096, 512),
                                    (14336, 4096, 129), (2048, 384, 64), (4096, 14336, 300)])
def test_q6p_bitwise_vs_q6v3(env, Kd, N, M):
    torch, K = env
    _, rs = _weights(torch, K, Kd, N, 3)
    img = _image(torch, K, rs, Kd, N)
    X = np.random.default_rng(M).standard_normal((M, Kd)).astype(np.float32)
    act = _act(torch, K, X)
    y3, y4 = _both(torch, K, rs, img, Kd, N, act, M)
    assert np.isfinite(y4).all()
    assert np.array_equal(y3.view(np.uint32), y4.view(np.uint32))


def test_q6p_residual_and_glu_bitwise(env):
    torch, K = env
    Kd, N, M = 4096, 1024, 150
    _, rs = _weights(torch, K, Kd, N, 4)
    _, rs2 = _weights(torch, K, Kd, N, 5)
    img, img2 = _image(torch, K, rs, Kd, N), _image(torch, K, rs2, Kd, N)
    rng = np.random.default_rng(9)
    act = _act(torch, K, rng.standard_normal((M, Kd)).astype(np.float32))
    res = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda()
    y3, y4 = _both(torch, K, rs, img, Kd, N, act, M, res=res)
    assert np.array_equal(y3.view(np.uint32), y4.view(np.uint32))
    y3, y4 = _both(torch, K, rs, img, Kd, N, act, M, mode=1, rs2=rs2, img2=img2)
    assert np.array_equal(y3.view(np.uint32), y4.view(np.uint32))


@pytest.mark.parametrize("rnd", [False, True])
def test_q6p_vs_oracle(env, rnd):
    torch, K = env
    Kd, N, M = 2048, 256, 48
    w, rs = _weights(torch, K, Kd, N, 6, rnd=rnd)
    img = _image(torch, K, rs, Kd, N)
    X = np.random.default_rng(2).standard_normal((M, Kd)).astype(np.float32)
    act = _act(torch, K, X)
    y3, y4 = _both(torch, K, rs, img, Kd, N, act, M)
    want = R.mul_mat(R.Q6_K, w, Kd, N, X)
    np.testing.assert_allclose(y4, want, rtol=0, atol=3e-6 * max(1.0, np.abs(want).max()))
    assert np.array_equal(y3.view(np.uint32), y4.view(np.uint32))


def test_q6p_image_planes(env):
    """the image's planes: 64 A + C = sc * (q - 32) for every weight (random bytes: the extremes of both planes)"""
    torch, K = env
    Kd, N = 512, 128
    w, rs = _weights(torch, K, Kd, N, 8, rnd=True)
    img = _image(torch, K, rs, Kd, N)
    torch.cuda.synchronize()
    im = img.cpu().numpy().view(np.int8).astype(np.int32)
    # the exact integers from the ggml bytes (dequantize_row_q6_K's decoding, ggml-quants.c:2978)
    blocks = w.reshape(N, Kd // 256, 210)
    v = np.zeros((N, Kd), np.int32)
    for sb in range(Kd // 256):
        ql, qh, sc = blocks[:, sb, :128].astype(np.int32), blocks[:, sb, 128:192].astype(np.int32), \
            blocks[:, sb, 192:208].view(np.int8).astype(np.int32)
        for half in range(2):
            for l in range(32):
                base = 256 * sb + 128 * half
                is_ = l // 16
                q1 = (ql[:, 64 * half + l] & 0xF) | (((qh[:, 32 * half + l] >> 0) & 3) << 4)
                q2 = (ql[:, 64 * half + l + 32] & 0xF) | (((qh[:, 32 * half + l] >> 2) & 3) << 4)
                q3 = (ql[:, 64 * half + l] >> 4) | (((qh[:, 32 * half + l] >> 4) & 3) << 4)
                q4 = (ql[:, 64 * half + l + 32] >> 4) | (((qh[:, 32 * half + l] >> 6) & 3) << 4)
                v[:, base + l] = sc[:, 8 * half + is_ + 0] * (q1 - 32)
                v[:, base + l + 32] = sc[:, 8 * half + is_ + 2] * (q2 - 32)
                v[:, base + l + 64] = sc[:, 8 * half + is_ + 4] * (q3 - 32)
                v[:, base + l + 96] = sc[:, 8 * half + is_ + 6] * (q4 - 32)
    n = np.arange(N)[:, None]
    k = np.arange(Kd)[None, :]
    nsb = Kd // 256
    kk = k % 256
    off = (((n >> 5) * nsb + (k >> 8)) * 16 + 2 * (kk >> 5)) * 1024 + 16 * ((n & 31) + 32 * ((kk >> 4) & 1)) + (kk & 15)
    A, C = im[off], im[off + 1024]
    assert np.array_equal(64 * A + C, v)
    assert A.min() >= -64 and A.max() <= 64 and C.min() >= -32 and C.max() <= 31
    assert A.min() < -60 and A.max() > 60        # the random bytes reach the extremes
