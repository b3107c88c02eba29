"""GPU parity tests: every HIP kernel vs the C restatement of the reference CPU path (oracle) on
identical seeded inputs, plus the reference's own golden vectors (tests/golden).  Calls go through
the C ABI (koboldcpp_amd/lib.py -> koboldcpp_hipblas.so).  Bars: bit-exact for integer/byte work
(dequant, activation quantization, repack, rope table), fp32-order tolerance for dots."""
import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

TYPES = [R.Q4_K, R.Q5_K, R.Q6_K, R.Q4_0, R.Q8_0]


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import koboldcpp_amd.lib as K
    return torch, K


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def empty(torch, nbytes):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device="cuda")


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


def host(torch, t, dtype):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(dtype)


def upload_weight(torch, K, t, data, Kd, N):
    src = dev(torch, data)
    dst = empty(torch, data.nbytes)
    K.call("kcpp_weight_repack", t, src.data_ptr(), dst.data_ptr(), Kd, N, 0, sptr(torch))
    return dst


@pytest.mark.parametrize("t", TYPES)
def test_repack_roundtrip_and_synth(env, t):
    torch, K = env
    Kd, N = 1024, 24
    w = R.synth(t, 5, 77, Kd, N)
    d = upload_weight(torch, K, t, w, Kd, N)
    back = empty(torch, w.nbytes)
    K.call("kcpp_weight_repack", t, d.data_ptr(), back.data_ptr(), Kd, N, 1, sptr(torch))
    assert np.array_equal(host(torch, back, np.uint8), w)
    # device-side synthetic generator == host generator, bit for bit
    s = empty(torch, w.nbytes)
    K.call("kcpp_weight_synth", t, 5, 77, s.data_ptr(), Kd, N, sptr(torch))
    assert np.array_equal(host(torch, s, np.uint8), host(torch, d, np.uint8))


@pytest.mark.parametrize("t", TYPES)
def test_dequant_bit_exact(env, golden_ops, t):
    torch, K = env
    nm = {R.Q4_0: "q4_0", R.Q8_0: "q8_0", R.Q4_K: "q4_K", R.Q5_K: "q5_K", R.Q6_K: "q6_K"}[t]
    for tag in ("syn", "rnd"):
        data = golden_ops["deq_%s_%s_in" % (nm, tag)]
        want = golden_ops["deq_%s_%s_out" % (nm, tag)]
        Kd = want.size
        d = upload_weight(torch, K, t, data, Kd, 1)
        y = torch.empty(Kd, dtype=torch.float32, device="cuda")
        K.call("kcpp_dequantize", t, d.data_ptr(), y.data_ptr(), Kd, 1, sptr(torch))
        got = host(torch, y, np.float32)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (nm, tag)


def _adversarial_acts(rng, n):
    x = (rng.standard_normal(n) * np.exp(rng.uniform(-4, 4, size=n))).astype(np.float32)
    x[256:512] = 0.0
    x[700] = 5.0; x[701] = -5.0          # equal |max| with opposite signs: first index wins
    # exact .5 ties after scaling by -127/max (round-half-even path of nearest_int)
    blk = x[1024:1280]
    blk[:] = np.float32(0.01)
    blk[0] = np.float32(127.0)
    blk[1:9] = np.array([0.5, 1.5, 2.5, -0.5, -1.5, 100.5, -126.5, 3.5], np.float32)
    # |max| reached in several lanes of a block, the first occurrence negative, in a later lane and element
    b2 = x[1536:1792]
    b2[:] = (rng.standard_normal(256) * 0.1).astype(np.float32)
    b2[37] = -7.0; b2[40] = 7.0; b2[200] = 7.0; b2[38] = -7.0
    # and positive first, ties inside one lane only
    b3 = x[2048:2304]
    b3[:] = (rng.standard_normal(256) * 0.1).astype(np.float32)
    b3[129] = 3.25; b3[130] = -3.25; b3[143] = 3.25
    return x


@pytest.mark.parametrize("vt", [R.Q8_K, R.Q8_0])
def test_quantize_act_bit_exact(env, golden_ops, vt):
    torch, K = env
    rng = np.random.default_rng(3)
    for x in (golden_ops["quant_in"], _adversarial_acts(rng, 8192), rng.standard_normal(4096 * 3).astype(np.float32)):
        M = x.size // 4096 if x.size % 4096 == 0 else 1
        Kd = x.size // M
        xd = dev(torch, x)
        wt = R.Q4_K if vt == R.Q8_K else R.Q8_0
        out = empty(torch, K.act_bytes(wt, Kd, M))
        K.call("kcpp_quantize_act", vt, xd.data_ptr(), Kd, out.data_ptr(), Kd, M, sptr(torch))
        got = host(torch, out, np.uint8)
        for m in range(M):
            ref = R.quantize(vt, x[m * Kd:(m + 1) * Kd])
            if vt == R.Q8_K:
                blocks = ref.reshape(-1, 292)
                qs = got[m * Kd:(m + 1) * Kd]
                d = got[M * Kd:M * Kd + M * (Kd // 256) * 4].view(np.float32)[m * (Kd // 256):(m + 1) * (Kd // 256)]
                off = M * Kd + M * (Kd // 256) * 4
                bs = got[off:off + M * (Kd // 16) * 2].view(np.int16)[m * (Kd // 16):(m + 1) * (Kd // 16)]
                assert np.array_equal(qs.reshape(-1, 256), blocks[:, 4:260])
                assert np.array_equal(d.view(np.uint32), blocks[:, :4].copy().view(np.uint32).ravel())
                assert np.array_equal(bs.reshape(-1, 16), blocks[:, 260:].copy().view(np.int16))
            else:
                blocks = ref.reshape(-1, 34)
                qs = got[m * Kd:(m + 1) * Kd]
                d = got[M * Kd:M * Kd + M * (Kd // 32) * 4].view(np.float32)[m * (Kd // 32):(m + 1) * (Kd // 32)]
                assert np.array_equal(qs.reshape(-1, 32), blocks[:, 2:])
                want_d = np.array([R.dequant(R.F16, blocks[i, :2], 1)[0] for i in range(blocks.shape[0])], np.float32)
                assert np.array_equal(d, want_d)


def _gpu_mul_mat(torch, K, t, w, Kd, N, X, mode=0, w2=None, res=None, force_gemm=False):
    M = X.shape[0]
    wd = upload_weight(torch, K, t, w, Kd, N)
    w2d = upload_weight(torch, K, t, w2, Kd, N) if w2 is not None else None
    xd = dev(torch, X.astype(np.float32))
    act = empty(torch, K.act_bytes(t, Kd, M))
    K.call("kcpp_quantize_act", K.vec_dot_type(t), xd.data_ptr(), Kd, act.data_ptr(), Kd, M, sptr(torch))
    Y = torch.empty((M, N), dtype=torch.float32, device="cuda")
    rd = dev(torch, res.astype(np.float32)) if res is not None else None
    if M <= 8 and not force_gemm:
        K.call("kcpp_gemv", t, wd.data_ptr(), w2d.data_ptr() if w2d is not None else None, Kd, N, act.data_ptr(), M,
               Y.data_ptr(), N, rd.data_ptr() if rd is not None else None, N, mode, sptr(torch))
    else:
        ws = empty(torch, K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M))
        K.call("kcpp_gemm", t, wd.data_ptr(), w2d.data_ptr() if w2d is not None else None, Kd, N, act.data_ptr(), M,
               Y.data_ptr(), N, rd.data_ptr() if rd is not None else None, N, mode, ws.data_ptr(), sptr(torch))
    return host(torch, Y, np.float32).reshape(M, N)


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("shape", [(4096, 256, 1), (4096, 128, 8), (1024, 64, 40)])
def test_mul_mat_vs_reference_golden(env, golden_ops, t, shape):
    torch, K = env
    nm = {R.Q4_0: "q4_0", R.Q8_0: "q8_0", R.Q4_K: "q4_K", R.Q5_K: "q5_K", R.Q6_K: "q6_K"}[t]
    key = "mm_%s_%d_%d_%d" % ((nm,) + shape)
    tt, seed, tid, xseed, Kd, N, M = [int(v) for v in golden_ops[key + "_meta"]]
    w = R.synth(tt, seed, tid, Kd, N)
    X = np.random.default_rng(xseed).standard_normal((M, Kd)).astype(np.float32)
    got = _gpu_mul_mat(torch, K, tt, w, Kd, N, X)
    want = golden_ops[key + "_y"]
    np.testing.assert_allclose(got, want, rtol=0, atol=3e-6 * max(1.0, np.abs(want).max()))


@pytest.mark.parametrize("t", TYPES)
@pytest.mark.parametrize("M", [1, 3, 8, 17, 64])
def test_mul_mat_modes_vs_oracle(env, t, M):
    torch, K = env
    rng = np.random.default_rng(M * 31 + t)
    Kd, N = 2048, 96
    w = R.synth(t, 9, 1000 + t, Kd, N)
    w2 = R.synth(t, 9, 2000 + t, Kd, N)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float32)
    a = R.mul_mat(t, w, Kd, N, X)
    b = R.mul_mat(t, w2, Kd, N, X)
    tol = 3e-6 * max(1.0, np.abs(a).max())
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X), a, rtol=0, atol=tol)
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, res=res), a + res, rtol=0, atol=tol + 1e-6)
    glu = (a / (1 + np.exp(-a))) * b
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, mode=1, w2=w2), glu, rtol=1e-5, atol=tol)


def test_rms_norm_and_fused_quant(env, golden_ops):
    torch, K = env
    x = golden_ops["rms_x"]
    rows, E = x.shape
    w = (1 + 0.01 * np.random.default_rng(1).standard_normal(E)).astype(np.float32)
    xd, wd = dev(torch, x), dev(torch, w)
    y = torch.empty_like(xd)
    q = empty(torch, K.act_bytes(R.Q4_K, E, rows))
    K.call("kcpp_rms_norm", xd.data_ptr(), E, None, y.data_ptr(), E, None, E, rows, 1e-5, sptr(torch))
    assert np.array_equal(host(torch, y, np.float32).reshape(rows, E), golden_ops["rms_y"])
    K.call("kcpp_rms_norm", xd.data_ptr(), E, wd.data_ptr(), y.data_ptr(), E, q.data_ptr(), E, rows, 1e-5, sptr(torch))
    yn = R.rms_norm(x, w, 1e-5)
    assert np.array_equal(host(torch, y, np.float32).reshape(rows, E), yn)
    got = host(torch, q, np.uint8)
    for r in range(rows):
        ref = R.quantize(R.Q8_K, yn[r]).reshape(-1, 292)
        assert np.array_equal(got[r * E:(r + 1) * E].reshape(-1, 256), ref[:, 4:260])


def test_rope_kv(env, golden_ops):
    import ctypes
    torch, K = env
    T, H, HKV, D = 5, 8, 2, 128
    n_past, n_ctx = 3000, 4096
    rng = np.random.default_rng(5)
    qkv = rng.standard_normal((T, (H + 2 * HKV) * D)).astype(np.float32)
    tab = np.empty((n_ctx, D // 2, 2), np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data_as(ctypes.c_void_p), n_ctx, D, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0,
           n_ctx)
    tabd = dev(torch, tab)
    qd = dev(torch, qkv)
    qo = torch.empty((T, H, D), dtype=torch.float32, device="cuda")
    q16 = torch.empty((T, H, D), dtype=torch.float16, device="cuda")
    kc = torch.zeros((n_ctx, HKV * D), dtype=torch.float16, device="cuda")
    vc = torch.zeros((n_ctx, HKV * D), dtype=torch.float16, device="cuda")
    K.call("kcpp_rope_kv", qd.data_ptr(), qkv.shape[1], qo.data_ptr(), q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), T,
           H, HKV, D, n_past, None, tabd.data_ptr(), sptr(torch))
    pos = np.arange(n_past, n_past + T)
    qr = R.rope(qkv[:, :H * D].reshape(T, H, D), pos, 500000.0)
    kr = R.rope(qkv[:, H * D:(H + HKV) * D].reshape(T, HKV, D), pos, 500000.0)
    assert np.array_equal(host(torch, qo, np.float32).reshape(T, H, D), qr)
    assert np.array_equal(host(torch, q16, np.float16).reshape(T, H, D), qr.astype(np.float16))
    kch = host(torch, kc, np.float16).reshape(n_ctx, HKV * D)
    vch = host(torch, vc, np.float16).reshape(n_ctx, HKV * D)
    assert np.array_equal(kch[n_past:n_past + T], kr.reshape(T, -1).astype(np.float16))
    assert np.array_equal(vch[n_past:n_past + T], qkv[:, (H + HKV) * D:].astype(np.float16))
    # golden: reference ggml rope at base 500000 / 10000 (positions 0,315,...)
    x = golden_ops["rope_x"]
    for base in (10000, 500000):
        tabb = np.empty((4096, 64, 2), np.float32)
        K.call("kcpp_rope_table", tabb.ctypes.data_as(ctypes.c_void_p), 4096, 128, float(base), 1.0, None, 0.0, 1.0,
               32.0, 1.0, 4096)
        want = golden_ops["rope_y_%d" % base]
        for t_ in range(x.shape[0]):
            p = t_ * 315
            c, s = tabb[p, :, 0], tabb[p, :, 1]
            x0, x1 = x[t_, :, 0::2], x[t_, :, 1::2]
            np.testing.assert_allclose(x0 * c - x1 * s, want[t_, :, 0::2], rtol=0, atol=1e-5)


@pytest.mark.parametrize("T,n_past,path", [(1, 0, 1), (1, 255, 1), (1, 1000, 1), (3, 700, 1), (5, 295, 1),
                                           (40, 0, 2), (70, 130, 2), (16, 300, 2),
                                           (40, 0, 3), (70, 130, 3), (16, 300, 3), (200, 700, 3), (1, 5, 3)])
def test_flash_attn_vs_oracle(env, T, n_past, path):
    torch, K = env
    H, HKV, D = 32, 8, 128
    n_ctx = 2048
    rng = np.random.default_rng(T * 1000 + n_past)
    n_kv = n_past + T
    q = rng.standard_normal((T, H, D)).astype(np.float32)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    mask = np.zeros((T, n_kv), np.float16)
    for t in range(T):
        mask[t, n_past + t + 1:] = -np.inf
    want = R.flash_attn(q, kcache[:n_kv], vcache[:n_kv], mask)
    q16 = dev(torch, q.astype(np.float16))
    kd, vd = dev(torch, kcache), dev(torch, vcache)
    out = torch.empty((T, H, D), dtype=torch.float32, device="cuda")
    ws = torch.zeros(K.fa_workspace_bytes(max(T, 16), H, n_ctx), dtype=torch.uint8, device="cuda")
    K.call("kcpp_flash_attn", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), None, ws.data_ptr(), T, H,
           HKV, D, n_past, None, n_ctx, 1.0 / np.sqrt(D), path, sptr(torch))
    got = host(torch, out, np.float32).reshape(T, H, D)
    # oracle accumulates V in fp16 like the reference CPU: tolerance = a few f16 ulps of |out|
    np.testing.assert_allclose(got, want, rtol=4e-3, atol=4e-3)


@pytest.mark.parametrize("key", ["fa_1_256", "fa_5_300"])
def test_flash_attn_golden(env, golden_ops, key):
    torch, K = env
    q, k, v = (golden_ops[key + s] for s in ("_q", "_k", "_v"))
    T, H, D = q.shape
    n_kv, HKV, _ = k.shape
    n_past = n_kv - T
    out = torch.empty((T, H, D), dtype=torch.float32, device="cuda")
    ws = torch.zeros(K.fa_workspace_bytes(16, H, n_kv), dtype=torch.uint8, device="cuda")
    qd, kd, vd = dev(torch, q.astype(np.float16)), dev(torch, k), dev(torch, v)   # keep alive across the call
    K.call("kcpp_flash_attn", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), None, ws.data_ptr(), T, H,
           HKV, D, n_past, None, n_kv, 1.0 / np.sqrt(D), 0, sptr(torch))
    np.testing.assert_allclose(host(torch, out, np.float32).reshape(q.shape), golden_ops[key + "_y"], rtol=4e-3, atol=4e-3)


@pytest.mark.parametrize("T,n_past,path", [(1, 0, 1), (1, 1000, 1), (5, 295, 1), (16, 300, 1), (16, 300, 2),
                                           (17, 0, 2), (37, 0, 2), (40, 0, 2), (70, 130, 2), (200, 60, 2),
                                           (17, 0, 3), (37, 0, 3), (70, 130, 3), (200, 60, 3), (512, 300, 3)])
def test_flash_attn_vs_oracle_f32_accum(env, T, n_past, path):
    """Same math as the HIP kernels (f32 V accumulation): must agree to fp32 rounding.  Path 3 (MFMA
    prefill) rounds the probabilities to f16 for the P.V product: a 2^-11 relative error per weight."""
    torch, K = env
    H, HKV, D = 32, 8, 128
    n_ctx = 1024
    rng = np.random.default_rng(T * 7 + n_past)
    n_kv = n_past + T
    q = rng.standard_normal((T, H, D)).astype(np.float32)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    mask = np.zeros((T, n_kv), np.float16)
    for t in range(T):
        mask[t, n_past + t + 1:] = -np.inf
    R.lib().orc_set_fa_f32_accum(1)
    try:
        want = R.flash_attn(q, kcache[:n_kv], vcache[:n_kv], mask)
    finally:
        R.lib().orc_set_fa_f32_accum(0)
    q16 = dev(torch, q.astype(np.float16))
    kd, vd = dev(torch, kcache), dev(torch, vcache)
    out = torch.empty((T, H, D), dtype=torch.float32, device="cuda")
    ws = torch.zeros(K.fa_workspace_bytes(max(T, 16), H, n_ctx), dtype=torch.uint8, device="cuda")
    K.call("kcpp_flash_attn", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), None, ws.data_ptr(), T, H,
           HKV, D, n_past, None, n_ctx, 1.0 / np.sqrt(D), path, sptr(torch))
    got = host(torch, out, np.float32).reshape(T, H, D)
    if path == 3:
        np.testing.assert_allclose(got, want, rtol=2e-3, atol=2e-3)
    else:
        np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("variant", [3, 5, 8])
@pytest.mark.parametrize("H,HKV", [(32, 8), (32, 32), (64, 8), (16, 8), (32, 4), (8, 4), (64, 64)])
def test_fa_dec4_split_counts(env, H, HKV, variant):
    """the decode pairs (5: k_fa_dec5 + k_fa_comb4, production: 64-key chunks dealt round-robin over the splits, rows
    clamped to the cache; 3: round 5's k_fa_dec4, contiguous key ranges; 8: the short-context single launch, one
    workgroup per kv head over every key) over split counts 4..64 (256 / HKV rounded down
    to a power of two) and GQA groups 1..8: back-to-back calls whose key counts differ (empty, partial and full splits,
    a cache whose rows past the keys hold NaN / inf, which must not leak into the result) are reproducible bit for bit
    and match the f32-accumulation oracle."""
    torch, K = env
    D, n_ctx = 128, 4200
    rng = np.random.default_rng(H * 100 + HKV)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    kd, vd = dev(torch, kcache), dev(torch, vcache)
    ws = torch.zeros(K.fa_workspace_bytes(16, H, n_ctx), dtype=torch.uint8, device="cuda")
    npd = torch.zeros(1, dtype=torch.int32, device="cuda")
    for n_past in (0, 5, 100, 3850, 7, 4095):
        npd.fill_(n_past)
        # rows past the keys: stale cache contents may be anything (v5 loads them, masked by score)
        kd.copy_(dev(torch, kcache))
        vd.copy_(dev(torch, vcache))
        kd.view(n_ctx, HKV, D)[n_past + 1:] = float("nan")
        vd.view(n_ctx, HKV, D)[n_past + 1:] = float("inf")
        q = rng.standard_normal((1, H, D)).astype(np.float32)
        q16 = dev(torch, q.astype(np.float16))
        outs = []
        for _ in range(2):
            out = torch.full((1, H, D), float("nan"), dtype=torch.float32, device="cuda")
            K.call("kcpp_fa_decode_ex", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), HKV * D, D, out.data_ptr(), None,
                   ws.data_ptr(), H, HKV, 0, npd.data_ptr(), n_ctx, 1.0 / np.sqrt(D), variant, sptr(torch))
            outs.append(host(torch, out, np.float32).reshape(1, H, D))
        assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32)), f"n_past {n_past}"
        n_kv = n_past + 1
        R.lib().orc_set_fa_f32_accum(1)
        try:
            want = R.flash_attn(q, kcache[:n_kv], vcache[:n_kv], np.zeros((1, n_kv), np.float16))
        finally:
            R.lib().orc_set_fa_f32_accum(0)
        np.testing.assert_allclose(outs[0], want, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("path", [1, 6])
@pytest.mark.parametrize("n_past", [63, 2047, 4095])
def test_flash_attn_decode_long_ctx(env, n_past, path):
    """decode (1: the production k_fa_dec4 splits + k_fa_comb4; 6: 64-key chunks + combine) at 4k context,
    graph-style device n_past, vs the f32-accumulation oracle; twice in a row with the same workspace."""
    torch, K = env
    H, HKV, D, n_ctx = 32, 8, 128, 4096
    rng = np.random.default_rng(n_past)
    n_kv = n_past + 1
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    kd, vd = dev(torch, kcache), dev(torch, vcache)
    ws = torch.zeros(K.fa_workspace_bytes(16, H, n_ctx), dtype=torch.uint8, device="cuda")
    npd = dev(torch, np.array([n_past], np.int32))
    for rep in range(2):
        q = rng.standard_normal((1, H, D)).astype(np.float32)
        q16 = dev(torch, q.astype(np.float16))
        out = torch.empty((1, H, D), dtype=torch.float32, device="cuda")
        K.call("kcpp_flash_attn", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), None, ws.data_ptr(), 1, H,
               HKV, D, 0, npd.data_ptr(), n_ctx, 1.0 / np.sqrt(D), path, sptr(torch))
        got = host(torch, out, np.float32).reshape(1, H, D)
        R.lib().orc_set_fa_f32_accum(1)
        try:
            want = R.flash_attn(q, kcache[:n_kv], vcache[:n_kv], np.zeros((1, n_kv), np.float16))
        finally:
            R.lib().orc_set_fa_f32_accum(0)
        np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("t", TYPES)
# (2048, 96) at M = 17: the shape of test_mul_mat_modes_vs_oracle[17-13] (Q5_K) that faulted once in round 1
@pytest.mark.parametrize("Kd,N", [(512, 128), (512, 512), (512, 1024), (1024, 512), (2048, 96)])
@pytest.mark.parametrize("M", [17, 37])
def test_gemm_small_shapes(env, t, Kd, N, M):
    torch, K = env
    rng = np.random.default_rng(Kd + N + M + t)
    w = R.synth(t, 3, 500 + t, Kd, N)
    w2 = R.synth(t, 3, 600 + t, Kd, N)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float32)
    a = R.mul_mat(t, w, Kd, N, X)
    b = R.mul_mat(t, w2, Kd, N, X)
    tol = 3e-6 * max(1.0, np.abs(a).max())
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X), a, rtol=0, atol=tol)
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, res=res), a + res, rtol=0, atol=tol + 1e-6)
    glu = (a / (1 + np.exp(-a))) * b
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, mode=1, w2=w2), glu, rtol=1e-5, atol=tol)


@pytest.mark.parametrize("t", [R.Q5_K, R.Q6_K, R.Q4_K, R.Q8_0])
@pytest.mark.parametrize("Kd,N", [(4096, 256), (14336, 128)])
def test_mul_mat_every_batch_size(env, t, Kd, N):
    """every token count 1..64 (the MoE prefill runs each expert's GEMMs on however many tokens the router sent
    it) at the Mixtral expert widths, plain and GLU, vs the oracle"""
    torch, K = env
    rng = np.random.default_rng(Kd + N + t)
    w = R.synth(t, 4, 700 + t, Kd, N)
    w2 = R.synth(t, 4, 800 + t, Kd, N)
    X = rng.standard_normal((64, Kd)).astype(np.float32)
    a_all = R.mul_mat(t, w, Kd, N, X)
    b_all = R.mul_mat(t, w2, Kd, N, X)
    bad = []
    for M in range(1, 65):
        a, b = a_all[:M], b_all[:M]
        tol = 3e-6 * max(1.0, np.abs(a).max())
        g = _gpu_mul_mat(torch, K, t, w, Kd, N, X[:M])
        if not np.allclose(g, a, rtol=0, atol=tol):
            bad.append(("plain", M, float(np.abs(g - a).max())))
        glu = (a / (1 + np.exp(-a))) * b
        g = _gpu_mul_mat(torch, K, t, w, Kd, N, X[:M], mode=1, w2=w2)
        if not np.allclose(g, glu, rtol=1e-5, atol=tol):
            bad.append(("glu", M, float(np.abs(g - glu).max())))
    assert not bad, bad


@pytest.mark.parametrize("H,HKV", [(32, 8), (8, 8), (64, 8), (16, 8)])
def test_flash_attn_decode_fused_quant(env, H, HKV):
    """decode FA with the combine quantizing its output to Q8_K vs the oracle and vs the separate quantizer,
    over repeated calls on one workspace."""
    torch, K = env
    D, n_ctx = 128, 1024
    rng = np.random.default_rng(H)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    kd, vd = dev(torch, kcache), dev(torch, vcache)
    ws = torch.zeros(K.fa_workspace_bytes(16, H, n_ctx), dtype=torch.uint8, device="cuda")
    for n_past in (0, 127, 128, 700):
        q = rng.standard_normal((1, H, D)).astype(np.float32)
        q16 = dev(torch, q.astype(np.float16))
        out = torch.empty((1, H, D), dtype=torch.float32, device="cuda")
        qa = empty(torch, K.act_bytes(R.Q4_K, H * D, 1))
        K.call("kcpp_flash_attn", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), qa.data_ptr(),
               ws.data_ptr(), 1, H, HKV, D, n_past, None, n_ctx, 1.0 / np.sqrt(D), 1, sptr(torch))
        got = host(torch, out, np.float32).reshape(1, H, D)
        n_kv = n_past + 1
        R.lib().orc_set_fa_f32_accum(1)
        try:
            want = R.flash_attn(q, kcache[:n_kv], vcache[:n_kv], None)
        finally:
            R.lib().orc_set_fa_f32_accum(0)
        np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-6)
        ref = R.quantize(R.Q8_K, got.ravel()).reshape(-1, 292)
        gq = host(torch, qa, np.uint8)
        assert np.array_equal(gq[:H * D].reshape(-1, 256), ref[:, 4:260])


@pytest.mark.parametrize("Kd,N,M", [(4096, 1024, 32), (14336, 256, 32), (4096, 4096, 9), (2048, 300, 31)])
def test_gemm_q8_0_small_batch(env, Kd, N, M):
    """BASELINE config 3's batched Q8_0 path (M <= 32: int8 MFMA block dots, split-K, ordered reduction)
    vs the C restatement of ggml_vec_dot_q8_0_q8_0 (plain, + residual, silu GLU)"""
    torch, K = env
    t = R.Q8_0
    rng = np.random.default_rng(Kd + N + M)
    w = R.synth(t, 5, 700, Kd, N)
    w2 = R.synth(t, 5, 701, Kd, N)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float32)
    a = R.mul_mat(t, w, Kd, N, X)
    b = R.mul_mat(t, w2, Kd, N, X)
    tol = 3e-6 * max(1.0, np.abs(a).max())
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X), a, rtol=0, atol=tol)
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, res=res), a + res, rtol=0, atol=tol + 1e-6)
    glu = (a / (1 + np.exp(-a))) * b
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, t, w, Kd, N, X, mode=1, w2=w2), glu, rtol=1e-5, atol=tol)


@pytest.mark.parametrize("Kd,N,M", [(4096, 14336, 32), (4096, 1024, 9), (256, 96, 1)])
def test_gemm_q80_glu_q80_bitwise(env, Kd, N, M):
    """config 3's gate|up GEMM with the Q8_0 quantization of silu(g) * u in its reduce must equal kcpp_gemm(mode 1)
    followed by kcpp_quantize_act(Q8_0) byte for byte"""
    torch, K = env
    t = R.Q8_0
    rng = np.random.default_rng(Kd + N + M)
    wd = upload_weight(torch, K, t, R.synth(t, 5, 710, Kd, N), Kd, N)
    w2d = upload_weight(torch, K, t, R.synth(t, 5, 711, Kd, N), Kd, N)
    xd = dev(torch, rng.standard_normal((M, Kd)).astype(np.float32))
    act = empty(torch, K.act_bytes(t, Kd, M))
    K.call("kcpp_quantize_act", K.vec_dot_type(t), xd.data_ptr(), Kd, act.data_ptr(), Kd, M, sptr(torch))
    ws = empty(torch, K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M))
    Y = torch.empty((M, N), dtype=torch.float32, device="cuda")
    K.call("kcpp_gemm", t, wd.data_ptr(), w2d.data_ptr(), Kd, N, act.data_ptr(), M, Y.data_ptr(), N, None, N, 1,
           ws.data_ptr(), sptr(torch))
    nbytes = K.act_bytes(t, N, M)
    qa = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    qb = torch.full((nbytes,), 0xA5, dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.vec_dot_type(t), Y.data_ptr(), N, qa.data_ptr(), N, M, sptr(torch))
    K.call("kcpp_gemm_q80_glu_q80", wd.data_ptr(), w2d.data_ptr(), Kd, N, act.data_ptr(), M, qb.data_ptr(), ws.data_ptr(),
           sptr(torch))
    torch.cuda.synchronize()
    used = M * N + M * (N // 32) * 6                   # qs, d (f32), block sums (i16)
    np.testing.assert_array_equal(host(torch, qb, np.uint8)[:used], host(torch, qa, np.uint8)[:used])


@pytest.mark.parametrize("ne0,nrows", [(4096, 9), (4096, 32), (256, 3), (14336, 5)])
def test_rms_norm_q80_fused_bitwise(env, ne0, nrows):
    """rms_norm with the Q8_0 quantization in its epilogue (config 3's norm -> Q8_0 step) must equal
    kcpp_rms_norm followed by kcpp_quantize_act(Q8_0) byte for byte (qs, d, block sums)"""
    torch, K = env
    rng = np.random.default_rng(ne0 + nrows)
    x = (rng.standard_normal((nrows, ne0)) * 3).astype(np.float32)
    x[0, :32] = 0.0                                    # an all-zero block: d = 0, id = 0
    w = rng.standard_normal(ne0).astype(np.float32)
    xd, wd = dev(torch, x), dev(torch, w)
    nb = ne0 // 32
    nbytes = nrows * ne0 + nrows * nb * 4 + nrows * nb * 2
    y = torch.empty((nrows, ne0), dtype=torch.float32, device="cuda")
    qa = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    qb = torch.full((nbytes,), 0xA5, dtype=torch.uint8, device="cuda")
    K.call("kcpp_rms_norm", xd.data_ptr(), ne0, wd.data_ptr(), y.data_ptr(), ne0, None, ne0, nrows, 1e-5, sptr(torch))
    K.call("kcpp_quantize_act", R.Q8_0, y.data_ptr(), ne0, qa.data_ptr(), ne0, nrows, sptr(torch))
    K.call("kcpp_rms_norm_q80", xd.data_ptr(), ne0, wd.data_ptr(), qb.data_ptr(), ne0, nrows, 1e-5, sptr(torch))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(torch, qb, np.uint8), host(torch, qa, np.uint8))


@pytest.mark.parametrize("T,n_past", [(16, 0), (37, 0), (200, 60), (512, 300), (512, 3328), (70, 130)])
def test_flash_attn_prefill_mfma_v2_bitwise(env, T, n_past):
    """MFMA prefill v2 (next-tile prefetch, V through ds_read_b64_tr_b16) keeps v1's key order and summation
    order: outputs must be identical bit for bit"""
    torch, K = env
    H, HKV, D = 32, 8, 128
    n_ctx = n_past + T + 64
    rng = np.random.default_rng(T + 7 * n_past)
    q = rng.standard_normal((T, H, D)).astype(np.float16)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    q16, kd, vd = dev(torch, q), dev(torch, kcache), dev(torch, vcache)
    outs = []
    try:
        for v in (1, 2):
            K.raw().kcpp_fa_prefill_set_variant(v)
            out = torch.full((T, H, D), float("nan"), dtype=torch.float32, device="cuda")
            K.call("kcpp_flash_attn_prefill_mfma", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), T, H, HKV,
                   D, n_past, float(1.0 / np.sqrt(D)), sptr(torch))
            outs.append(host(torch, out, np.float32))
    finally:
        K.raw().kcpp_fa_prefill_set_variant(0)
    assert np.isfinite(outs[1]).all()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("T,n_past", [(16, 0), (37, 0), (200, 60), (512, 300), (512, 3328), (70, 130), (512, 0)])
@pytest.mark.parametrize("v", [3, 4, 5])
def test_flash_attn_prefill_mfma_v3_vs_v2(env, T, n_past, v):
    """MFMA prefill v3 (LDS-DMA K/V ring, swizzled LDS, exp2-domain softmax, mask only on diagonal / end tiles; v = 4:
    two waves per head over the two key halves of each tile, merged at the end) against v2 and an exact float64
    softmax(Q K^T / sqrt(D)) V of the same f16 inputs (4 of the 32 heads): both round P to f16 (the reference CPU
    accumulates V*P in f16 itself), v3 relative to an exp2-domain maximum (and v4 per key half), so the bar is v2's
    own error -- v3/v4 within 1.5x of v2's worst and 1.25x of its mean error against the exact result"""
    torch, K = env
    H, HKV, D = 32, 8, 128
    n_ctx = n_past + T + 64
    rng = np.random.default_rng(T + 11 * n_past)
    q = rng.standard_normal((T, H, D)).astype(np.float16)
    kcache = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
    vcache = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
    vcache[n_past + T:] = np.float16(np.inf)           # never visible: must not leak (P = 0 rows are clamped copies)
    q16, kd, vd = dev(torch, q), dev(torch, kcache), dev(torch, vcache)
    outs = []
    try:
        for vv in (2, v):
            K.raw().kcpp_fa_prefill_set_variant(vv)
            out = torch.full((T, H, D), float("nan"), dtype=torch.float32, device="cuda")
            K.call("kcpp_flash_attn_prefill_mfma", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), T, H, HKV,
                   D, n_past, float(1.0 / np.sqrt(D)), sptr(torch))
            outs.append(host(torch, out, np.float32))
    finally:
        K.raw().kcpp_fa_prefill_set_variant(0)
    assert np.isfinite(outs[1]).all()
    heads = [0, 5, 18, 31]
    ref = np.empty((T, len(heads), D))
    kf, vf = kcache.astype(np.float64), vcache[:n_past + T].astype(np.float64)
    for j, hh in enumerate(heads):
        s_ = q[:, hh].astype(np.float64) @ kf[:n_past + T, hh // 4].T / np.sqrt(D)
        s_[np.arange(n_past + T)[None, :] > (n_past + np.arange(T))[:, None]] = -np.inf
        pr = np.exp(s_ - s_.max(1, keepdims=True))
        ref[:, j] = (pr @ vf[:, hh // 4]) / pr.sum(1, keepdims=True)
    e_old = np.abs(outs[0][:, heads] - ref)
    e_new = np.abs(outs[1][:, heads] - ref)
    assert e_new.max() <= 1.5 * e_old.max() + 1e-6, (e_new.max(), e_old.max())
    assert e_new.mean() <= 1.25 * e_old.mean() + 1e-7, (e_new.mean(), e_old.mean())
