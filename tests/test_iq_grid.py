"""The lattice-grid weight types IQ2_XXS / IQ2_XS / IQ2_S / IQ3_XXS / IQ3_S / IQ1_S / IQ1_M (block_iq2_xxs ..
block_iq1_m, ggml-common.h:340-405; dot Q8_K through the code books, ggml_vec_dot_iq*_q8_K ggml-quants.c:9606-12468):
the CPU oracle and the HIP kernels against the reference builds' own outputs (tests/golden/iq_grid.npz,
make_iq_grid.py; the code books themselves are recovered from the reference's dequantization by
tools/gen_iq_grids.py).

* oracle (CPU): dequantize_row_iq* bit-exact on synthetic and random-bit blocks; mul_mat at decode / small-batch /
  prefill shapes within 3e-6 of the output scale;
* GPU: the (identity) device layout round-trips and dequantizes bit-exactly (kcpp_dequantize and get_rows); the
  mat-vec (kcpp_gemv, M <= 8) and the MFMA GEMM (kcpp_gemm past 16 tokens: codes x integer group scales as exact f16
  fragments) against the golden and the oracle at 3e-6; a tiny Llama with the type everywhere (output Q6_K) end to
  end (prefill + teacher-forced decode, graph and eager) within 2x the reference's AVX2-vs-scalar spread (the bar
  of tests/test_gpu_model.py), and against the C restatement with the HIP path's f32 attention accumulation."""
import os

import numpy as np
import pytest

import refharness as R

G = None


def golden():
    global G
    if G is None:
        G = np.load(os.path.join(R.ROOT, "tests", "golden", "iq_grid.npz"))
    return G


@pytest.fixture(scope="module", params=sorted(R.IQ_GRID))
def kq(request):
    return request.param, R.IQ_GRID[request.param], golden()


def test_oracle_dequant_bit_exact(kq):
    fn, T, g = kq
    for tag in ("syn", "rnd"):
        want = g["%s_deq_%s_out" % (fn, tag)]
        got = R.dequant(T, g["%s_deq_%s_in" % (fn, tag)], want.size)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), tag


@pytest.mark.parametrize("shape", [(4096, 256, 1), (4096, 128, 8), (1024, 64, 40)])
def test_oracle_mul_mat_vs_reference(kq, shape):
    fn, T, g = kq
    key = "%s_mm_%d_%d_%d" % ((fn,) + shape)
    t, seed, tid, xseed, K, N, M = [int(v) for v in g[key + "_meta"]]
    w = R.synth(t, seed, tid, K, N)
    X = np.random.default_rng(xseed).standard_normal((M, K)).astype(np.float32)
    want = g[key + "_y"]
    np.testing.assert_allclose(R.mul_mat(t, w, K, N, X), want, rtol=0, atol=3e-6 * max(1.0, np.abs(want).max()))


def test_code_books_generated():
    """the generated header holds every table at its size (tools/gen_iq_grids.py)"""
    src = open(os.path.join(R.ROOT, "koboldcpp_amd", "csrc", "iq_grids.h")).read()
    for name, n in (("kcpp_iq2xxs_grid", 512), ("kcpp_iq2xs_grid", 1024), ("kcpp_iq2s_grid", 2048),
                    ("kcpp_iq3xxs_grid", 256), ("kcpp_iq3s_grid", 512), ("kcpp_iq1s_grid", 4096)):
        assert "KCPP_IQ_TABLE(%s, %d)" % (name, n) in src


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
    fn, T, g = kq
    for tag in ("syn", "rnd"):
        data, want = g["%s_deq_%s_in" % (fn, tag)], g["%s_deq_%s_out" % (fn, tag)]
        d = _upload(torch, K, data, want.size, 1, T)
        back = torch.empty_like(d)
        K.call("kcpp_weight_repack", T, d.data_ptr(), back.data_ptr(), want.size, 1, 1, _sp(torch))
        y = torch.empty(want.size, dtype=torch.float32, device="cuda")
        K.call("kcpp_dequantize", T, d.data_ptr(), y.data_ptr(), want.size, 1, _sp(torch))
        # get_rows of row 0 of the same bytes seen as a [1][K] matrix
        ids = torch.zeros(1, dtype=torch.int32, device="cuda")
        yr = torch.empty(want.size, dtype=torch.float32, device="cuda")
        K.call("kcpp_get_rows", T, d.data_ptr(), want.size, 1, ids.data_ptr(), 1, yr.data_ptr(), want.size, _sp(torch))
        torch.cuda.synchronize()
        assert np.array_equal(back.cpu().numpy(), data)
        assert np.array_equal(y.cpu().numpy().view(np.uint32), want.view(np.uint32)), tag
        assert np.array_equal(yr.cpu().numpy().view(np.uint32), want.view(np.uint32)), tag
    Kd, N = 2048, 8
    w = R.synth(T, 5, 77, Kd, N)
    s = torch.empty(w.nbytes, dtype=torch.uint8, device="cuda")
    K.call("kcpp_weight_synth", T, 5, 77, s.data_ptr(), Kd, N, _sp(torch))
    torch.cuda.synchronize()
    assert np.array_equal(s.cpu().numpy(), w)


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
    fn, T, g = kq
    key = "%s_mm_%d_%d_%d" % ((fn,) + shape)
    t, seed, tid, xseed, Kd, N, M = [int(v) for v in g[key + "_meta"]]
    w = R.synth(t, seed, tid, Kd, N)
    X = np.random.default_rng(xseed).standard_normal((M, Kd)).astype(np.float32)
    want = g[key + "_y"]
    np.testing.assert_allclose(_gpu_mul_mat(torch, K, T, w, Kd, N, X), want, rtol=0,
                               atol=3e-6 * max(1.0, np.abs(want).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 17, 64, 300])
def test_gpu_mul_mat_modes_vs_oracle(env, kq, M):
    torch, K = env
    fn, T, _ = kq
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


# the tiny-model parity bar of tests/test_gpu_model.py: the reference's own AVX2-vs-scalar spread (the larger of this
# fixture's and the standard tiny fixtures', tests/golden/ref_spread.npz), x2 -- one factor for the GPU's summation
# order, and the production attention accumulates V*P in f32 where the CPU keeps f16 (ggml.c:15788)
_SP = np.load(os.path.join(R.ROOT, "tests", "golden", "ref_spread.npz"))
SPREAD_MAX = max(float(_SP["tiny_%s_max" % t].max()) for t in ("q4km", "q8_0", "moe"))
SPREAD_MED = max(float(_SP["tiny_%s_median" % t].max()) for t in ("q4km", "q8_0", "moe"))


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [True, False], ids=["graph", "eager"])
def test_gpu_model_vs_reference(env, kq, graphs):
    """tiny Llama with the grid type everywhere (output Q6_K): prefill + 8 teacher-forced decode steps vs the
    reference logits within 2x the reference's build spread, and vs the C restatement with f32 attention
    accumulation (the HIP path's math) within the same bar"""
    torch, K = env
    fn, T, g = kq
    types = [int(t) for t in g[fn + "_e2e_types"]]
    m = K.Model(R.TINY, types)
    m.set_graphs(graphs)
    m.synth(1234)
    prompt = [int(v) for v in g[fn + "_e2e_prompt"]]
    forced = [int(t) for t in g[fn + "_e2e_forced"]]
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in forced:
        out.append(m.decode([tok], n))
        n += 1
    m.close()
    got = np.array(out)
    d = np.abs(got - g[fn + "_e2e_logits"])
    tmax = 2 * max(float(g[fn + "_e2e_spread_max"].max()), SPREAD_MAX)
    tmed = 2 * max(float(g[fn + "_e2e_spread_median"].max()), SPREAD_MED)
    print(fn, "gpu vs ref max", d.max(axis=1), "| spread", g[fn + "_e2e_spread_max"])
    assert np.all(d.max(axis=1) <= tmax), d.max(axis=1)
    assert np.all(np.median(d, axis=1) <= tmed), np.median(d, axis=1)
    R.lib().orc_set_fa_f32_accum(1)
    try:
        o = R.OracleLlama(R.TINY, types, 1234)
        ref32 = [o.eval(prompt, 0)]
        n = len(prompt)
        for tok in forced:
            ref32.append(o.eval([tok], n))
            n += 1
    finally:
        R.lib().orc_set_fa_f32_accum(0)
    e = np.abs(got - np.array(ref32))
    print(fn, "gpu vs oracle(f32 accumulation) max", e.max(), "median", np.median(e))
    assert e.max() <= 2 * SPREAD_MAX and np.median(e) <= 2 * SPREAD_MED


@pytest.mark.gpu
@pytest.mark.parametrize("fn", ["iq2_xxs", "iq1_m", "iq3_s"])
def test_gpu_gguf_load_and_generate(env, tmp_path, fn):
    """a GGUF file with the grid type (tests/gguf_writer.py; the same synthetic weights) through the drop-in ABI:
    load_model accepts it and generate()'s greedy text equals the in-process model's greedy decode"""
    torch, K = env
    import gguf_writer as GW
    from koboldcpp_amd import expose as X
    T = R.IQ_GRID[fn]
    types = R.iq_grid_types(R.TINY["n_layer"], T)
    path = str(tmp_path / (fn + ".gguf"))
    toks = GW.llama_gguf(path, R.TINY, types, 1234, GW.WORDS)
    _, _, ttypes = GW.spm_vocab(R.TINY["n_vocab"], GW.WORDS)
    h = X.init_library()
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 512
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0
    assert h.load_model(li)
    prompt = b"hello world the"
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.memory = b""
    gi.max_context_length = 248
    gi.max_length = 8
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 7
    out = h.generate(gi)
    m = K.Model(dict(R.TINY, n_ctx=256), types)
    m.synth(1234)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(7):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()

    def piece(t):
        s = toks[t]
        if ttypes[t] in (2, 3, 5):
            return b""
        if ttypes[t] == 6:
            return bytes([int(s[3:5], 16)])
        return s.replace("▁", " ").encode()
    assert out.status == 1 and out.text == b"".join(piece(t) for t in want)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["moe_iq2_xxs", "moe_q4_1"])
@pytest.mark.parametrize("graphs", [True, False], ids=["graph", "eager"])
def test_gpu_moe_experts_without_fused_matvec(env, tag, graphs):
    """Mixtral-shaped tiny MoE whose expert weights have no fused decode mat-vec (IQ2_XXS, Q4_1): decode routes each
    top-k slot through the generic mat-vec on the expert slice its device-resident id selects (kcpp_gemv_expert,
    the router weight applied to down's product), prefill groups tokens by expert; vs the reference's MUL_MAT_ID
    logits (prefill + 6 teacher-forced steps) within 2x the reference's build spread"""
    torch, K = env
    g = golden()
    types = [int(t) for t in g[tag + "_e2e_types"]]
    m = K.Model(R.TINY_MOE, types)
    m.set_graphs(graphs)
    m.synth(1234)
    prompt = [int(v) for v in g[tag + "_e2e_prompt"]]
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in g[tag + "_e2e_forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    d = np.abs(np.array(out) - g[tag + "_e2e_logits"])
    tmax = 2 * max(float(g[tag + "_e2e_spread_max"].max()), SPREAD_MAX)
    tmed = 2 * max(float(g[tag + "_e2e_spread_median"].max()), SPREAD_MED)
    print(tag, "gpu vs ref max", d.max(axis=1))
    assert np.all(d.max(axis=1) <= tmax), d.max(axis=1)
    assert np.all(np.median(d, axis=1) <= tmed), np.median(d, axis=1)
