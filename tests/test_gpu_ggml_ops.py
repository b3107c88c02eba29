"""General-layout ggml node kernels (csrc/ggml_ops.hip, kcpp_flash_attn_ext) -- the ops a ggml backend
plugin dispatches besides the fused Llama path -- against the reference's semantics:
* bit-exact where the CPU op is exact fp32 elementwise work (add/sub/mul/div with broadcast, scale,
  f32<->f16 copies, get_rows, argsort order incl. ties);
* the reference golden vectors (tests/golden/ops.npz, from the reference ggml build) for rope and
  flash_attn_ext with its own causal mask;
* the C restatement (oracle) for rms_norm, rope with YaRN parameters, and flash attention under
  explicit non-causal masks; fp64 numpy for soft_max / sum_rows / F16 mul_mat (tolerances in-line)."""
import ctypes

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


def s_(torch):
    return torch.cuda.current_stream().cuda_stream


def run(torch, K, name, *args):
    """args: torch tensors become data pointers; ('desc', t) becomes a kcpp_tdesc*"""
    keep, conv = [], []
    for a in args:
        if isinstance(a, tuple) and a[0] == "desc":
            d = K.tdesc(a[1])
            keep.append(d)
            conv.append(ctypes.addressof(d))
        elif hasattr(a, "data_ptr"):
            conv.append(a.data_ptr())
        else:
            conv.append(a)
    K.call(name, *conv, s_(torch))
    torch.cuda.synchronize()


@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("bshape", ["full", "row", "bcast2"])
def test_binary_broadcast_bit_exact(env, op, bshape):
    torch, K = env
    g = torch.Generator().manual_seed(op)
    a = torch.randn(3, 5, 300, generator=g)
    b = {"full": torch.randn(3, 5, 300, generator=g), "row": torch.randn(300, generator=g) + 2,
         "bcast2": torch.randn(1, 5, 300, generator=g) + 2}[bshape]
    at = a.cuda().transpose(0, 1)                   # non-contiguous source view
    bt = b.cuda()
    bt = bt.transpose(0, 1) if bt.dim() == 3 else bt
    d = torch.empty(at.shape, device="cuda")
    run(torch, K, "kcpp_ggml_binary", op, at, ("desc", at), bt, ("desc", bt), d, ("desc", d))
    an, bn = at.cpu().numpy(), bt.cpu().numpy()
    want = [np.add, np.subtract, np.multiply, np.divide][op](an, bn).astype(np.float32)
    assert np.array_equal(d.cpu().numpy(), want)


def test_unary_scale_cpy_get_rows(env):
    torch, K = env
    g = torch.Generator().manual_seed(3)
    x = (4 * torch.randn(7, 1000, generator=g)).cuda()
    y = torch.empty_like(x)
    run(torch, K, "kcpp_ggml_unary", 0, x, ("desc", x), y, ("desc", y), 0.0)
    xn = x.cpu().numpy()
    np.testing.assert_allclose(y.cpu().numpy(), xn / (1 + np.exp(-xn.astype(np.float64))), rtol=2e-6, atol=1e-7)
    run(torch, K, "kcpp_ggml_unary", 1, x, ("desc", x), y, ("desc", y), 0.125)
    assert np.array_equal(y.cpu().numpy(), (xn * np.float32(0.125)).astype(np.float32))
    # f32 -> f16 into a strided view (the KV-cache store), f16 -> f32, and a reshaping copy
    cache = torch.zeros(20, 8, 128, dtype=torch.float16, device="cuda")
    src = torch.randn(5, 8, 128, generator=g).cuda()
    view = cache[10:15]
    run(torch, K, "kcpp_ggml_cpy", 0, src, ("desc", src), 1, view, ("desc", view))
    assert np.array_equal(cache[10:15].cpu().numpy(), src.cpu().numpy().astype(np.float16))
    assert not cache[:10].cpu().numpy().any()
    back = torch.empty(5, 1024, device="cuda")      # other shape, same element order
    run(torch, K, "kcpp_ggml_cpy", 1, view, ("desc", view), 0, back, ("desc", back))
    assert np.array_equal(back.cpu().numpy().reshape(5, 8, 128), src.cpu().numpy().astype(np.float16).astype(np.float32))
    # get_rows: dst[:, i] = src[:, ids[i]]
    tab = torch.randn(50, 64, generator=g).cuda()
    ids = torch.tensor([3, 49, 0, 3], dtype=torch.int32, device="cuda")
    out = torch.empty(4, 64, device="cuda")
    run(torch, K, "kcpp_ggml_get_rows", 0, tab, ("desc", tab), ids, ("desc", ids), out, ("desc", out))
    assert np.array_equal(out.cpu().numpy(), tab.cpu().numpy()[[3, 49, 0, 3]])
    tab16 = tab.half()
    run(torch, K, "kcpp_ggml_get_rows", 1, tab16, ("desc", tab16), ids, ("desc", ids), out, ("desc", out))
    assert np.array_equal(out.cpu().numpy(), tab16.cpu().numpy()[[3, 49, 0, 3]].astype(np.float32))


@pytest.mark.parametrize("ne0", [4096, 5120, 100])
def test_rms_norm_generic_vs_oracle(env, ne0):
    torch, K = env
    x = np.random.default_rng(ne0).standard_normal((9, ne0)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    y = torch.empty_like(xd)
    run(torch, K, "kcpp_ggml_rms_norm", xd, ("desc", xd), y, ("desc", y), 1e-5)
    want = np.empty_like(x)
    R.lib().orc_rms_norm(R.ptr(x), None, R.ptr(want), ne0, 9, ctypes.c_float(1e-5))
    np.testing.assert_allclose(y.cpu().numpy(), want, rtol=1e-6, atol=0)


def test_rope_golden_and_yarn(env, golden_ops):
    torch, K = env
    x = golden_ops["rope_x"]                      # [T=13][H=8][D=128], positions t * 315
    T = x.shape[0]
    pos = torch.tensor([t * 315 for t in range(T)], dtype=torch.int32, device="cuda")
    xd = torch.from_numpy(x).cuda()
    y = torch.empty_like(xd)
    for base in (10000, 500000):
        run(torch, K, "kcpp_ggml_rope", xd, ("desc", xd), y, ("desc", y), pos, None, 128, 0, 4096, float(base), 1.0,
            0.0, 1.0, 32.0, 1.0)
        np.testing.assert_allclose(y.cpu().numpy(), golden_ops["rope_y_%d" % base], rtol=0, atol=2e-5)
    # YaRN-scaled (ext_factor, freq_scale) and partial n_dims vs the restatement
    p_np = np.array([0, 7, 1000, 4000], np.int32)
    x2 = np.random.default_rng(1).standard_normal((4, 4, 128)).astype(np.float32)
    want = np.empty_like(x2)
    R.lib().orc_rope(R.ptr(x2), R.ptr(want), 128, 4, 4, R.ptr(p_np), 128, ctypes.c_float(10000.0),
                     ctypes.c_float(0.25), None, ctypes.c_float(1.0), ctypes.c_float(1.0), ctypes.c_float(32.0),
                     ctypes.c_float(1.0), 4096)
    xd2 = torch.from_numpy(x2).cuda()
    y2 = torch.empty_like(xd2)
    pd = torch.from_numpy(p_np).cuda()
    run(torch, K, "kcpp_ggml_rope", xd2, ("desc", xd2), y2, ("desc", y2), pd, None, 128, 0, 4096, 10000.0, 0.25, 1.0,
        1.0, 32.0, 1.0)
    np.testing.assert_allclose(y2.cpu().numpy(), want, rtol=0, atol=5e-5)


def _rope_neox_ref(x, pos, n_dims, base):
    y = x.astype(np.float64).copy()
    half = n_dims // 2
    for t, p in enumerate(pos):
        th = p * base ** (-2.0 * np.arange(half) / n_dims)
        c, s = np.cos(th), np.sin(th)
        x0, x1 = x[t, :, :half].astype(np.float64), x[t, :, half:n_dims].astype(np.float64)
        y[t, :, :half] = x0 * c - x1 * s
        y[t, :, half:n_dims] = x0 * s + x1 * c
    return y


def test_rope_neox_partial_dims(env):
    torch, K = env
    x = np.random.default_rng(2).standard_normal((3, 2, 128)).astype(np.float32)
    pos = np.array([0, 5, 300], np.int32)
    xd, pd = torch.from_numpy(x).cuda(), torch.from_numpy(pos).cuda()
    y = torch.empty_like(xd)
    run(torch, K, "kcpp_ggml_rope", xd, ("desc", xd), y, ("desc", y), pd, None, 64, 2, 4096, 10000.0, 1.0, 0.0, 1.0,
        32.0, 1.0)
    np.testing.assert_allclose(y.cpu().numpy(), _rope_neox_ref(x, pos, 64, 10000.0), rtol=0, atol=5e-5)


@pytest.mark.parametrize("mask", [None, "f16", "f32"])
def test_soft_max(env, mask):
    torch, K = env
    rng = np.random.default_rng(4)
    x = rng.standard_normal((2, 6, 300)).astype(np.float32)
    m = np.where(rng.random((6, 300)) < 0.3, -np.inf, rng.standard_normal((6, 300))).astype(np.float32)
    m[:, 0] = 0.0
    xd = torch.from_numpy(x).cuda()
    y = torch.empty_like(xd)
    md = None if mask is None else torch.from_numpy(m.astype(np.float16 if mask == "f16" else np.float32)).cuda()
    mt = 1 if mask == "f16" else 0
    run(torch, K, "kcpp_ggml_soft_max", xd, ("desc", xd), md, mt, 300, 6, y, ("desc", y), 0.5)
    mm = 0 if mask is None else (m.astype(np.float16).astype(np.float64) if mask == "f16" else m.astype(np.float64))
    w = x.astype(np.float64) * 0.5 + mm
    e = np.exp(w - w.max(-1, keepdims=True))
    np.testing.assert_allclose(y.cpu().numpy(), e / e.sum(-1, keepdims=True), rtol=2e-6, atol=1e-9)


def _exchange_argsort(row, desc):
    idx = list(range(len(row)))
    for j in range(len(row)):
        for k in range(j + 1, len(row)):
            a, b = row[idx[j]], row[idx[k]]
            if (a < b) if desc else (a > b):
                idx[j], idx[k] = idx[k], idx[j]
    return idx


@pytest.mark.parametrize("desc", [0, 1])
def test_argsort_and_sum_rows(env, desc):
    torch, K = env
    rng = np.random.default_rng(desc)
    x = np.round(rng.standard_normal((33, 8)), 1).astype(np.float32)     # many ties
    xd = torch.from_numpy(x).cuda()
    d = torch.empty(33, 8, dtype=torch.int32, device="cuda")
    run(torch, K, "kcpp_ggml_argsort", xd, ("desc", xd), d, 8, desc)
    assert d.cpu().numpy().tolist() == [_exchange_argsort(r, desc) for r in x]
    s = torch.empty(33, 1, device="cuda")
    run(torch, K, "kcpp_ggml_sum_rows", xd, ("desc", xd), s, ("desc", s))
    np.testing.assert_allclose(s.cpu().numpy()[:, 0], x.astype(np.float64).sum(1), rtol=1e-7, atol=1e-7)


@pytest.mark.parametrize("wt", [R.F16, R.F32])
def test_mul_mat_f(env, wt):
    torch, K = env
    rng = np.random.default_rng(5)
    w = (0.05 * rng.standard_normal((2, 24, 512))).astype(np.float16 if wt == R.F16 else np.float32)
    x = rng.standard_normal((4, 7, 512)).astype(np.float32)              # batch 4 broadcasts over 2 weights
    wd, xd = torch.from_numpy(w).cuda(), torch.from_numpy(x).cuda()
    d = torch.empty(4, 7, 24, device="cuda")
    run(torch, K, "kcpp_ggml_mul_mat_f", wt, wd, ("desc", wd), xd, ("desc", xd), d, ("desc", d))
    xr = x.astype(np.float16).astype(np.float64) if wt == R.F16 else x.astype(np.float64)
    want = np.stack([xr[b] @ w[b // 2].astype(np.float64).T for b in range(4)])
    np.testing.assert_allclose(d.cpu().numpy(), want, rtol=1e-5, atol=1e-5)


def _fa_ext(torch, K, q, k, v, mask, scale):
    """q [T][H][D] f32 given as the permuted ggml view; k/v [n_kv][HKV][D] f16; mask [T][n_kv] f16"""
    T, H, D = q.shape
    n_kv, HKV, _ = k.shape
    qd = torch.from_numpy(np.ascontiguousarray(q)).cuda()
    kd, vd = torch.from_numpy(k).cuda(), torch.from_numpy(v).cuda()
    md = None if mask is None else torch.from_numpy(np.ascontiguousarray(mask)).cuda()
    out = torch.full((T, H, D), float("nan"), device="cuda")
    ws = torch.zeros(K.fa_ext_workspace_bytes(T, H, n_kv), dtype=torch.uint8, device="cuda")
    K.call("kcpp_flash_attn_ext", qd.data_ptr(), H * D * 4, D * 4, kd.data_ptr(), vd.data_ptr(),
           md.data_ptr() if md is not None else None, n_kv if md is not None else -1, out.data_ptr(), ws.data_ptr(),
           T, H, HKV, D, n_kv, scale, s_(torch))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("key", ["fa_1_256", "fa_5_300"])
def test_flash_attn_ext_golden(env, golden_ops, key):
    torch, K = env
    q, k, v, m = (golden_ops[key + s] for s in ("_q", "_k", "_v", "_mask"))
    got = _fa_ext(torch, K, q, k, v, m, 1.0 / np.sqrt(q.shape[2]))
    np.testing.assert_allclose(got, golden_ops[key + "_y"], rtol=4e-3, atol=4e-3)


@pytest.mark.parametrize("T,n_kv", [(1, 700), (7, 300), (40, 257), (130, 600)])
def test_flash_attn_ext_explicit_mask_vs_oracle(env, T, n_kv):
    """a mask with holes (not causal): both the split-KV (T <= 16) and the tiled path must apply it;
    V rows of fully-masked keys hold NaN and must never reach the output (the CPU skips them)"""
    torch, K = env
    rng = np.random.default_rng(T + n_kv)
    H, HKV, D = 8, 2, 128
    q = rng.standard_normal((T, H, D)).astype(np.float32)
    k = rng.standard_normal((n_kv, HKV, D)).astype(np.float16)
    v = rng.standard_normal((n_kv, HKV, D)).astype(np.float16)
    mask = np.where(rng.random((T, n_kv)) < 0.4, np.float16(-np.inf), np.float16(0)).astype(np.float16)
    mask[:, 3] = 0
    mask[:, -5:] = -np.inf                          # keys nobody may see
    v[-5:] = np.nan
    want = np.empty((T, H, D), np.float32)
    R.lib().orc_set_fa_f32_accum(1)
    try:
        R.lib().orc_flash_attn_ext(R.ptr(q), R.ptr(k), R.ptr(v), HKV * D, R.ptr(mask), R.ptr(want), D, T, H, n_kv, HKV,
                                   ctypes.c_float(1.0 / np.sqrt(D)), 4)
    finally:
        R.lib().orc_set_fa_f32_accum(0)
    got = _fa_ext(torch, K, q, k, v, mask, 1.0 / np.sqrt(D))
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)
