"""Mixture-of-experts FFN on the GPU (GGML_OP_MUL_MAT_ID as used by
llm_build_moe_ffn, src/llama.cpp:9416-9514; BASELINE config 5, Mixtral-style top-2).

* router kernel (kcpp_moe_route) vs a numpy restatement of the reference's router math
  (F16 mul_mat with src1 rounded to f16, ggml_vec_soft_max_f32 with a ggml_float sum, argsort
  descending, weights / sum_rows): ids exact, weights to fp32 summation order;
* expert-indexed mat-vecs (DecArgs.eid / escale: the expert id read on the device) are bit-identical
  to the same kernel run on that expert's slice, times the routing weight;
* the whole model (TINY_MOE: 4 experts, top-2, Q5_K_M-like mix, F16 router) vs the reference graph's
  golden logits (tests/golden/e2e_moe.npz, oracle/_ref/ref_llama) and vs the C restatement; graph
  replay vs eager; ubatch split; fused vs unfused decode."""
import ctypes

import numpy as np
import pytest

import refharness as R
from test_gpu_model import SPREAD_MAX, SPREAD_MED, TOL_MAX, TOL_MEDIAN_F32, oracle_forced, run_gpu, run_gpu_forced

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def _route_ref(x, w, wtype, k):
    """llm_build_moe_ffn router (src/llama.cpp:9435-9470) for one token, in the reference's precision"""
    if wtype == R.F16:
        lg = (x.astype(np.float16).astype(np.float64) @ w.astype(np.float64).T)
    else:
        lg = x.astype(np.float64) @ w.astype(np.float64).T
    lg = lg.astype(np.float32)
    out_ids, out_w, gaps = [], [], []
    for p in lg:
        e = np.exp((p - p.max()).astype(np.float32)).astype(np.float32)
        pr = (e * np.float32(1.0 / e.astype(np.float64).sum())).astype(np.float32)
        order = sorted(range(len(pr)), key=lambda i: (-pr[i], i))
        sel = order[:k]
        srt = np.sort(pr)[::-1]
        gaps.append(srt[k - 1] - srt[k] if k < len(pr) else 1.0)
        ws = np.float32(pr[sel].astype(np.float64).sum())
        out_ids.append(sel)
        out_w.append(pr[sel] / ws)
    return np.array(out_ids), np.array(out_w, np.float32), np.array(gaps)


@pytest.mark.parametrize("wtype", [R.F16, R.F32])
@pytest.mark.parametrize("NE,k", [(8, 2), (4, 2), (16, 4), (64, 6)])
def test_router_vs_restatement(env, wtype, NE, k):
    torch, K = env
    E, T = 512, 37
    rng = np.random.default_rng(NE * 10 + k)
    x = rng.standard_normal((T, E)).astype(np.float32)
    w = (0.05 * rng.standard_normal((NE, E))).astype(np.float16 if wtype == R.F16 else np.float32)
    xd, wd = torch.from_numpy(x).cuda(), torch.from_numpy(w.view(np.uint8).copy()).cuda()
    ids = torch.full((T, k), -1, dtype=torch.int32, device="cuda")
    wts = torch.zeros((T, k), device="cuda")
    K.call("kcpp_moe_route", xd.data_ptr(), E, wd.data_ptr(), wtype, E, NE, k, ids.data_ptr(), wts.data_ptr(), T,
           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rid, rw, gaps = _route_ref(x, w, wtype, k)
    gid, gw = ids.cpu().numpy(), wts.cpu().numpy()
    clear = gaps > 1e-5                          # near-ties may legitimately swap under fp32 sum order
    assert clear.sum() > T // 2
    np.testing.assert_array_equal(gid[clear], rid[clear])
    np.testing.assert_allclose(gw[clear], rw[clear], rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(gw.sum(1), 1.0, atol=1e-5)


def test_router_rejects_bad_shapes(env):
    torch, K = env
    rc = K.raw().kcpp_moe_route(None, 512, None, R.F16, 512, 65, 2, None, None, 1, None)
    assert rc != 0
    rc = K.raw().kcpp_moe_route(None, 512, None, R.F16, 512, 8, 9, None, None, 1, None)
    assert rc != 0


EXPERT_CASES = [  # type, K, N, mode, pro
    (R.Q4_K, 4096, 2048, 1, 1),      # gate|up + silu (lean Q4_K GLU kernel)
    (R.Q5_K, 4096, 2048, 1, 1),
    (R.Q4_K, 14336, 4096, 0, 2),     # down, quantizing the f32 input in the prologue
    (R.Q5_K, 14336, 4096, 0, 2),
    (R.Q6_K, 14336, 4096, 0, 2),
    (R.Q8_0, 4096, 1024, 1, 1),
    (R.Q4_0, 4096, 1024, 0, 2),
]


@pytest.mark.parametrize("case", EXPERT_CASES, ids=lambda c: "t%d_%dx%d_m%d" % c[:4])
def test_expert_indexed_matvec_bit_identical(env, case):
    torch, K = env
    t, Kd, N, mode, pro = case
    NE = 4
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(Kd, generator=g).cuda()
    nw = (1 + 0.01 * torch.randn(Kd, generator=g)).cuda()
    sb = K.row_bytes(t, Kd) * N
    W = torch.empty(NE * sb, dtype=torch.uint8, device="cuda")
    W2 = torch.empty(NE * sb, dtype=torch.uint8, device="cuda")
    for e in range(NE):
        K.call("kcpp_weight_synth", t, 9, 100 + e, W[e * sb:].data_ptr(), Kd, N, s)
        K.call("kcpp_weight_synth", t, 9, 200 + e, W2[e * sb:].data_ptr(), Kd, N, s)
    for e in (2, 0, 3):
        eid = torch.tensor([e], dtype=torch.int32, device="cuda")
        wt = torch.tensor([0.3125 + 0.1 * e], dtype=torch.float32, device="cuda")
        y0 = torch.full((N,), float("nan"), device="cuda")
        y1 = torch.full((N,), float("nan"), device="cuda")
        a0 = K.DecArgs()
        a1 = K.DecArgs()
        for a, y, wp, w2p in ((a0, y0, W[e * sb:].data_ptr(), W2[e * sb:].data_ptr()),
                              (a1, y1, W.data_ptr(), W2.data_ptr())):
            a.K, a.nseg, a.x, a.nw, a.eps = Kd, 1, x.data_ptr(), nw.data_ptr(), 1e-5
            a.N[0], a.Y[0], a.W[0] = N, y.data_ptr(), wp
            if mode == 1:
                a.W2 = w2p
        a1.eid, a1.ebytes = eid.data_ptr(), sb
        if mode == 0:
            a1.escale = wt.data_ptr()
        assert K.gemv_dec(t, a0, mode, pro, 1, s) == 0
        assert K.gemv_dec(t, a1, mode, pro, 1, s) == 0
        torch.cuda.synchronize()
        ref = y0.cpu().numpy()
        if mode == 0:
            ref = (ref * np.float32(wt.item())).astype(np.float32)
        got = y1.cpu().numpy()
        assert np.isfinite(got).all()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (t, e, np.abs(got - ref).max())


def test_scatter_combine_order(env):
    """x = ((s0 + s1) + s2) + x, slots written as w * out (ggml_mul then the ggml_add chain)"""
    torch, K = env
    s = torch.cuda.current_stream().cuda_stream
    T, E, k = 5, 256, 3
    rng = np.random.default_rng(1)
    x = rng.standard_normal((T, E)).astype(np.float32)
    outs = rng.standard_normal((T * k, E)).astype(np.float32)
    w = rng.random(T * k).astype(np.float32)
    rows = rng.permutation(T * k).astype(np.int32)       # entry i -> slot row rows[i] (= j * T + t)
    slots = torch.zeros(k * T * E, device="cuda")
    xd = torch.from_numpy(x.copy()).cuda()
    od, wd, rd = torch.from_numpy(outs).cuda(), torch.from_numpy(w).cuda(), torch.from_numpy(rows).cuda()
    K.call("kcpp_moe_scatter", slots.data_ptr(), E, od.data_ptr(), rd.data_ptr(), wd.data_ptr(), T * k, E, s)
    K.call("kcpp_moe_combine", xd.data_ptr(), slots.data_ptr(), T * E, k, T * E, s)
    torch.cuda.synchronize()
    sl = np.zeros((k * T, E), np.float32)
    sl[rows] = outs * w[:, None]
    sl = sl.reshape(k, T, E)
    acc = sl[0].copy()
    for j in range(1, k):
        acc = acc + sl[j]
    want = acc + x
    assert np.array_equal(xd.cpu().numpy(), want)
    # gather
    src = torch.from_numpy(x).cuda()
    g = torch.zeros((3, E), device="cuda")
    idx = torch.tensor([4, 0, 2], dtype=torch.int32, device="cuda")
    K.call("kcpp_moe_gather", src.data_ptr(), E, idx.data_ptr(), 3, E, g.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), x[[4, 0, 2]])


@pytest.fixture(scope="module")
def golden_moe():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "e2e_moe.npz"))


def test_moe_e2e_vs_reference_golden(env, golden_moe):
    """teacher-forced on the reference's own greedy tokens; the dense model's bar (2 x the reference's own
    AVX2-vs-scalar spread on this MoE fixture, tests/golden/ref_spread.npz tiny_moe_*)"""
    torch, K = env
    types = [int(t) for t in golden_moe["types"]]
    prompt = golden_moe["prompt"]
    L = golden_moe["logits"]
    forced = golden_moe["tokens"][:-1]
    got = run_gpu_forced(K, types, prompt, forced, hp=R.TINY_MOE)
    d = np.abs(got - L)
    assert np.all(d.max(axis=1) <= 2 * SPREAD_MAX["moe"]), d.max(axis=1)
    assert np.all(np.median(d, axis=1) <= 2 * SPREAD_MED["moe"]), np.median(d, axis=1)
    orc32 = oracle_forced(types, prompt, forced, True, hp=R.TINY_MOE)
    e = np.abs(got - orc32)
    assert np.median(e) < TOL_MEDIAN_F32 and e.max() < TOL_MAX, (np.median(e), e.max())


@pytest.mark.parametrize("t", [R.Q4_K, R.Q8_0])
def test_moe_e2e_vs_oracle_other_types(env, t):
    torch, K = env
    hp = R.TINY_MOE
    types = R.moe_types(hp["n_layer"], t=t, router=R.F32 if t == R.Q8_0 else R.F16)
    prompt = [int(v) for v in np.random.default_rng(7).integers(1, 500, size=45)]
    got = run_gpu(K, types, prompt, 4, hp=hp)
    forced = np.argmax(got, axis=1)[:-1]
    orc32 = oracle_forced(types, prompt, forced, True, hp=hp)
    d = np.abs(got - orc32)
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))


def test_moe_graph_replay_and_ubatch(env):
    torch, K = env
    types = R.moe_types(R.TINY_MOE["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(2).integers(1, 500, size=150)]
    a = run_gpu(K, types, prompt, 5, graphs=True, hp=R.TINY_MOE)
    b = run_gpu(K, types, prompt, 5, graphs=False, hp=R.TINY_MOE)
    assert np.array_equal(a, b)
    c = run_gpu(K, types, prompt, 2, ub=64, hp=R.TINY_MOE)
    np.testing.assert_allclose(a[:3], c, rtol=0, atol=TOL_MAX)


def test_moe_fused_decode_matches_unfused(env):
    torch, K = env
    types = R.moe_types(R.TINY_MOE["n_layer"])
    prompt = list(range(5, 30))
    outs = []
    for fused in (True, False):
        m = K.Model(R.TINY_MOE, types)
        m.set_fused_decode(fused)
        m.synth(1234)
        lg = [m.decode(prompt, 0)]
        n = len(prompt)
        for tok in (7, 100, 3, 250):
            lg.append(m.decode([tok], n))
            n += 1
        m.close()
        outs.append(np.array(lg))
    d = np.abs(outs[0] - outs[1])
    assert d.max() < TOL_MAX and np.median(d) < 1e-5, (d.max(), np.median(d))


@pytest.mark.gpu
def test_moe_mixtral_q5_k_m_policy_vs_oracle(env):
    """BASELINE config 5's exact type mix (Q5_K, Q8_0 attn_k/attn_v, Q6_K down on more-bits layers, F32
    router, Q6_K output) on the tiny MoE shape, teacher-forced vs the f32-accumulation restatement"""
    torch, K = env
    hp = R.TINY_MOE                     # 2 layers: layer 1 is a "more bits" layer (Q6_K ffn_down_exps)
    types = R.mixtral_q5_k_m_types(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(11).integers(1, 500, size=37)]
    got = run_gpu(K, types, prompt, 4, hp=hp)
    forced = np.argmax(got, axis=1)[:-1]
    orc32 = oracle_forced(types, prompt, forced, True, hp=hp)
    d = np.abs(got - orc32)
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))


@pytest.mark.parametrize("wtype", [R.F16, R.F32])
@pytest.mark.parametrize("E", [4096, 512])
def test_route_norm_fused_matches_norm_then_route(env, wtype, E):
    """decode router with ffn_norm fused in (kcpp_moe_route_norm) == kcpp_rms_norm then kcpp_moe_route, bit for bit"""
    torch, K = env
    NE, k, T = 8, 2, 5
    rng = np.random.default_rng(E + wtype)
    x = (3 * rng.standard_normal((T, E))).astype(np.float32)
    nw = (1 + 0.1 * rng.standard_normal(E)).astype(np.float32)
    w = (0.05 * rng.standard_normal((NE, E))).astype(np.float16 if wtype == R.F16 else np.float32)
    xd, nd = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    wd = torch.from_numpy(w.view(np.uint8).copy()).cuda()
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for fused in (True, False):
        ids = torch.full((T, k), -1, dtype=torch.int32, device="cuda")
        wts = torch.zeros((T, k), device="cuda")
        if fused:
            K.call("kcpp_moe_route_norm", xd.data_ptr(), E, nd.data_ptr(), 1e-5, wd.data_ptr(), wtype, E, NE, k,
                   ids.data_ptr(), wts.data_ptr(), T, s)
        else:
            xn = torch.empty_like(xd)
            K.call("kcpp_rms_norm", xd.data_ptr(), E, nd.data_ptr(), xn.data_ptr(), E, None, E, T, 1e-5, s)
            K.call("kcpp_moe_route", xn.data_ptr(), E, wd.data_ptr(), wtype, E, NE, k, ids.data_ptr(), wts.data_ptr(), T, s)
        torch.cuda.synchronize()
        outs.append((ids.cpu().numpy(), wts.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))


@pytest.mark.parametrize("policy", ["q5_k_f16_router", "mixtral_q5_k_m_f32_router"])
@pytest.mark.parametrize("graphs", [True, False])
def test_moe_routing_inside_glu_launch_bitwise(env, policy, graphs):
    """single-token MoE decode with the router inside the two-slot gate|up launch (k_gemv_rs ROUTE: k_moe_route's
    element map, fma order and sums on the prologue's normalised row) and both slots' down projections in one launch
    (MODE 3, at n_ff 14336) == the separate router launch + two chained down launches: the same expert ids every
    layer and step, logits bit for bit"""
    torch, K = env
    hp = dict(R.TINY_MOE, n_ff=14336)       # the two-slot down launch covers the Mixtral class (n_ff 14336)
    types = R.moe_types(hp["n_layer"]) if policy.startswith("q5_k_f16") else R.mixtral_q5_k_m_types(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(21).integers(1, 500, size=29)]
    outs, traces = [], []
    for fused in (True, False):
        m = K.Model(hp, types)
        m.set_graphs(graphs)
        m.set_fused_route(fused)
        m.synth(1234)
        m.moe_trace(True)
        lg = [m.decode(prompt, 0)]
        tr = []
        n = len(prompt)
        for tok in (7, 100, 3, 250, 11, 42):
            lg.append(m.decode([tok], n))
            tr.append(m.moe_trace_read(hp["n_layer"], hp["n_expert_used"]))
            n += 1
        routed, paired = m.fused_route_count()
        assert (routed > 0) == fused and (paired > 0) == fused     # the fused launches really ran (only when asked)
        m.close()
        outs.append(np.array(lg))
        traces.append(np.array(tr))
    assert np.array_equal(traces[0], traces[1])
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("t,mode", [(R.Q4_K, 0), (R.Q5_K, 0), (113, 0), (R.Q4_K, 1), (R.Q5_K, 1), (113, 1), (114, 0)])
def test_gemm_grouped_matches_per_expert_bitwise(env, t, mode):
    """kcpp_gemm_grouped (every expert's GEMM in one launch: the MoE prefill of ggml_cuda_mul_mat_id,
    ggml-cuda.cu:2003-2139) == kcpp_gemm on each expert's own rows with the unsplit kernels
    (kcpp_gemm_set_variant(13)), bit for bit, plain and GLU, over ragged counts (empty experts, 1 row, > 256 rows);
    Q6_K (RS layout, plain) through its 128-row-padded virtual layout"""
    torch, K = env
    s = torch.cuda.current_stream().cuda_stream
    Kd, N = 2048, 640
    cnt = [37, 0, 1, 129, 300, 31, 64, 5]
    NE, M = len(cnt), sum(cnt)
    rb = K.row_bytes(t, Kd) * N
    W = torch.empty(NE * rb, dtype=torch.uint8, device="cuda")
    W2 = torch.empty(NE * rb, dtype=torch.uint8, device="cuda")
    for e in range(NE):
        K.call("kcpp_weight_synth", t, 1, 50 + e, W.data_ptr() + e * rb, Kd, N, s)
        K.call("kcpp_weight_synth", t, 1, 80 + e, W2.data_ptr() + e * rb, Kd, N, s)
    X = torch.randn(M, Kd, generator=torch.Generator(device="cpu").manual_seed(M + t + mode)).cuda()
    vt = K.vec_dot_type(R.Q4_K)
    act = torch.zeros(K.act_bytes(R.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", vt, X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
    cnt_dev = torch.tensor(cnt, dtype=torch.int32, device="cuda")
    cnt_host = (ctypes.c_int32 * NE)(*cnt)
    Y = torch.full((M, N), float("nan"), device="cuda")
    up = torch.empty(M, N, device="cuda")
    gws = torch.empty(max(1, int(K.raw().kcpp_gemm_grouped_ws_bytes(t, Kd, M, NE))), dtype=torch.uint8, device="cuda")
    K.call("kcpp_gemm_grouped", t, W.data_ptr(), W2.data_ptr() if mode else None, rb, Kd, N, act.data_ptr(), M,
           cnt_host, cnt_dev.data_ptr(), NE, Y.data_ptr(), up.data_ptr() if mode else None, mode, gws.data_ptr(), s)
    torch.cuda.synchronize()
    got = Y.cpu().numpy()
    bad = []
    try:
        K.raw().kcpp_gemm_set_variant(13)
        r0 = 0
        for e, n in enumerate(cnt):
            if n:
                ae = torch.zeros(K.act_bytes(R.Q4_K, Kd, n), dtype=torch.uint8, device="cuda")
                K.call("kcpp_quantize_act", vt, X[r0:r0 + n].contiguous().data_ptr(), Kd, ae.data_ptr(), Kd, n, s)
                ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, n), dtype=torch.uint8, device="cuda")
                Ye = torch.empty(n, N, device="cuda")
                K.call("kcpp_gemm", t, W.data_ptr() + e * rb, W2.data_ptr() + e * rb if mode else None, Kd, N,
                       ae.data_ptr(), n, Ye.data_ptr(), N, None, N, mode, ws.data_ptr(), s)
                torch.cuda.synchronize()
                want = Ye.cpu().numpy()
                if not np.array_equal(got[r0:r0 + n].view(np.uint32), want.view(np.uint32)):
                    bad.append((e, n, float(np.nanmax(np.abs(got[r0:r0 + n] - want)))))
            r0 += n
    finally:
        K.raw().kcpp_gemm_set_variant(0)
    assert not bad, bad


@pytest.mark.parametrize("policy", ["q5_k_f16router", "mixtral_q5_k_m"])
def test_moe_grouped_prefill_matches_per_expert(env, policy):
    """MoE prefill with the grouped expert GEMMs (default) vs the per-expert loop: gate|up bitwise (unsplit v4 on
    both), down within split-K re-association, so logits within the GEMM bar; the grouped path really ran (and the
    Q6_K down of the 'more bits' layers took its per-expert fallback)"""
    torch, K = env
    hp = R.TINY_MOE
    types = R.moe_types(hp["n_layer"]) if policy.startswith("q5_k") else R.mixtral_q5_k_m_types(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(5).integers(1, 500, size=150)]
    outs = []
    for grouped in (True, False):
        m = K.Model(hp, types)
        m.set_moe_grouped(grouped)
        m.synth(77)
        lg = [m.decode(prompt, 0), m.decode([9], len(prompt))]
        assert (m.moe_grouped_count() > 0) == grouped
        m.close()
        outs.append(np.array(lg))
    assert np.isfinite(outs[0]).all()
    d = np.abs(outs[0] - outs[1]).max()
    assert d < TOL_MAX, d


def test_moe_grouped_prefill_unaligned_bsums_falls_back(env):
    """n_ff with an odd super-block count (768 = 3 x 256, as K 11008 / 6400 of real MoE merges) and an odd prompt: the
    routed rows x (F / 256) is not a multiple of 4, so the grouped int8 GEMM cannot stream the down projection's Q8_K
    bsums plane (kcpp_gemm_grouped: -3); that layer's down runs per expert while gate|up (K = 512) stays grouped.
    Prefill succeeds and matches the all-per-expert path within the GEMM bar"""
    torch, K = env
    hp = dict(R.TINY_MOE, n_ff=768)
    types = R.moe_types(hp["n_layer"])
    prompt = [int(v) for v in np.random.default_rng(6).integers(1, 500, size=151)]
    outs = []
    for grouped in (True, False):
        m = K.Model(hp, types)
        m.set_moe_grouped(grouped)
        m.synth(78)
        lg = [m.decode(prompt, 0), m.decode([9], len(prompt))]
        assert (m.moe_grouped_count() > 0) == grouped
        m.close()
        outs.append(np.array(lg))
    assert np.isfinite(outs[0]).all()
    d = np.abs(outs[0] - outs[1]).max()
    assert d < TOL_MAX, d
