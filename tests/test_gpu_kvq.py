"""Quantized KV cache (koboldcpp --quantkv 1 / 2 = Q8_0 / Q4_0 K and V; gpttype_adapter.cpp:1958-1959) on the GPU
(koboldcpp_amd/csrc/attn_kvq.hip):

* the store kernel's cache bytes equal the REFERENCE's ggml_cpy f32 -> Q8_0 / Q4_0 bytes (tests/golden/kvq_ops.npz);
* the attention kernel vs the reference's ggml_flash_attn_ext on quantized K / V (same fixture), and vs the pinned
  C restatement over random shapes (decode with a device position, prefill tiles, GQA, head dims 128 / 64);
* the tiny Q4_K_M model with quantized caches vs the reference's logits (tests/golden/e2e_kvq.npz), decode graph
  replay == eager, context shift refused;
* load_model(quant_k, quant_v) -> generate() equals the in-process runtime with the same cache types."""
import numpy as np
import pytest

import refharness as R
from test_gpu_kernels import dev, host, sptr

pytestmark = pytest.mark.gpu

KVQ = {"q8_0": R.Q8_0, "q4_0": R.Q4_0}


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import koboldcpp_amd.lib as K
    return torch, K


@pytest.fixture(scope="module")
def gkv():
    return np.load(R.ROOT + "/tests/golden/kvq_ops.npz")


def cache_bytes(K, t, n_ctx, ekv):
    return int(K._L.kcpp_kv_cache_bytes(t, n_ctx, ekv))


def soa_to_blocks(t, c, n_ctx, ekv):
    """device cache layout (qs [n_ctx][ekv or ekv/2] ++ d f16 [n_ctx][ekv/32]) -> ggml block rows [n_ctx][row bytes]"""
    nb = ekv // 32
    qb = 32 if t == R.Q8_0 else 16
    qs = c[:n_ctx * nb * qb].reshape(n_ctx, nb, qb)
    d = c[n_ctx * nb * qb:n_ctx * nb * qb + n_ctx * nb * 2].reshape(n_ctx, nb, 2)
    return np.concatenate([d, qs], axis=2).reshape(n_ctx, nb * (qb + 2))


def blocks_to_soa(t, rows):
    """ggml block rows [n][row bytes] -> the device layout"""
    qb = 32 if t == R.Q8_0 else 16
    n = rows.shape[0]
    b = rows.reshape(n, -1, qb + 2)
    return np.concatenate([b[:, :, 2:].ravel(), b[:, :, :2].ravel()])


def store(torch, K, tk, tv, kf, vf, n_ctx, n_past, pos_dev=None):
    """K rows kf / V rows vf ([T][ekv] f32) through kcpp_kv_store_q from q|k|v-shaped staging rows"""
    T, ekv = kf.shape
    E = 96                                              # a q block in front, as in the runtime's staging rows
    ld = E + 2 * ekv
    st = np.zeros((T, ld), np.float32)
    st[:, E:E + ekv], st[:, E + ekv:] = kf, vf
    sd = dev(torch, st)
    kc = torch.zeros(cache_bytes(K, tk, n_ctx, ekv), dtype=torch.uint8, device="cuda")
    vc = torch.zeros(cache_bytes(K, tv, n_ctx, ekv), dtype=torch.uint8, device="cuda")
    pd = dev(torch, np.array([pos_dev], np.int32)) if pos_dev is not None else None
    K.call("kcpp_kv_store_q", tk, tv, sd.data_ptr(), ld, E, E + ekv, T, ekv, kc.data_ptr(), vc.data_ptr(), n_ctx,
           n_past, pd.data_ptr() if pd is not None else None, sptr(torch))
    return host(torch, kc, np.uint8), host(torch, vc, np.uint8)


@pytest.mark.parametrize("nk", list(KVQ))
@pytest.mark.parametrize("nv", list(KVQ))
def test_kv_store_equals_reference_bytes(env, gkv, nk, nv):
    """48 rows of 256 (zero block, exact Q4_0 ties included) at positions 5..52: byte-equal to the reference's
    ggml_cpy output; the V rows in reverse order; untouched rows stay zero"""
    torch, K = env
    x = gkv["cpy_x"]
    n_ctx, n_past = 64, 5
    kc, vc = store(torch, K, KVQ[nk], KVQ[nv], x, x[::-1].copy(), n_ctx, n_past)
    kb, vb = soa_to_blocks(KVQ[nk], kc, n_ctx, 256), soa_to_blocks(KVQ[nv], vc, n_ctx, 256)
    for name, got, want in (("K", kb[n_past:n_past + 48], gkv["cpy_" + nk]), ("V", vb[n_past:n_past + 48], gkv["cpy_" + nv][::-1])):
        bad = np.argwhere(got != want)
        assert bad.size == 0, (name, nk, nv, len(bad), bad[:8].tolist(), got[tuple(bad[0])], want[tuple(bad[0])])
    assert not kb[:n_past].any() and not kb[n_past + 48:].any()


def test_kv_store_device_position(env, gkv):
    """graph decode form: one row at pos_dev[0] (n_past ignored)"""
    torch, K = env
    x = gkv["cpy_x"][:1]
    kc, vc = store(torch, K, R.Q8_0, R.Q4_0, x, x, 16, 0, pos_dev=11)
    assert np.array_equal(soa_to_blocks(R.Q8_0, kc, 16, 256)[11], gkv["cpy_q8_0"][0])
    assert np.array_equal(soa_to_blocks(R.Q4_0, vc, 16, 256)[11], gkv["cpy_q4_0"][0])


def attend(torch, K, tk, tv, q, kblocks, vblocks, n_ctx, n_past, dev_pos=False):
    T, H, D = q.shape
    ekv = kblocks.shape[1] // R.row_bytes(tk, 32) * 32
    HKV = ekv // D
    kpad = np.zeros((n_ctx, kblocks.shape[1]), np.uint8)
    vpad = np.zeros((n_ctx, vblocks.shape[1]), np.uint8)
    kpad[:kblocks.shape[0]], vpad[:vblocks.shape[0]] = kblocks, vblocks
    kc, vc = dev(torch, blocks_to_soa(tk, kpad)), dev(torch, blocks_to_soa(tv, vpad))
    assert kc.numel() == cache_bytes(K, tk, n_ctx, ekv)
    qd = dev(torch, q.reshape(T, H * D))
    out = torch.empty((T, H, D), dtype=torch.float32, device="cuda")
    pd = dev(torch, np.array([n_past], np.int32)) if dev_pos else None
    K.call("kcpp_flash_attn_q", tk, tv, qd.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), out.data_ptr(), T, H, HKV,
           D, n_ctx, 0 if dev_pos else n_past, pd.data_ptr() if pd is not None else None,
           float(np.float32(1) / np.sqrt(np.float32(D))), sptr(torch))
    return host(torch, out, np.float32).reshape(T, H, D)


@pytest.mark.parametrize("nk", list(KVQ))
@pytest.mark.parametrize("nv", list(KVQ))
def test_flash_attn_q_vs_reference(env, gkv, nk, nv):
    """against the reference's ggml_flash_attn_ext outputs (6 queries after 37 positions, 8 heads over 2 kv heads):
    integer block dots exact, fp32 order only (GPU: per-block d_k d_q fma, 64-key online-softmax tiles)"""
    torch, K = env
    g = gkv
    k = np.stack([R.quantize(KVQ[nk], r) for r in g["fa_kf"]])
    v = np.stack([R.quantize(KVQ[nv], r) for r in g["fa_vf"]])
    got = attend(torch, K, KVQ[nk], KVQ[nv], g["fa_q"], k, v, 64, int(g["fa_n_past"]))
    want = g["fa_out_%s_%s" % (nk, nv)]
    d = np.abs(got - want).max()
    print(nk, nv, "vs reference: max", d, "scale", np.abs(want).max())
    assert d <= 2e-6 * np.abs(want).max()


@pytest.mark.parametrize("T,n_past,D,H,HKV,dev_pos", [(1, 0, 128, 32, 8, True), (1, 700, 128, 32, 8, True),
                                                      (5, 61, 128, 32, 8, False), (64, 0, 128, 32, 8, False),
                                                      (100, 130, 128, 32, 8, False), (1, 300, 64, 32, 4, True),
                                                      (77, 20, 64, 32, 4, False)])
@pytest.mark.parametrize("nm", list(KVQ))
def test_flash_attn_q_vs_oracle(env, T, n_past, D, H, HKV, dev_pos, nm):
    torch, K = env
    t = KVQ[nm]
    rng = np.random.default_rng(T * 13 + n_past + D)
    n_kv, n_ctx = n_past + T, 1024
    q = rng.standard_normal((T, H, D)).astype(np.float32)
    kf = (rng.standard_normal((n_kv, HKV * D)) * 0.7).astype(np.float32)
    vf = rng.standard_normal((n_kv, HKV * D)).astype(np.float32)
    k = np.stack([R.quantize(t, r) for r in kf])
    v = np.stack([R.quantize(t, r) for r in vf])
    mask = np.zeros((T, n_kv), np.float16)
    for i in range(T):
        mask[i, n_past + i + 1:] = -np.inf
    want = R.flash_attn_q(q, k, v, t, t, mask)
    got = attend(torch, K, t, t, q, k, v, n_ctx, n_past, dev_pos)
    d = np.abs(got - want).max()
    assert d <= 2e-6 * np.abs(want).max(), d


def _forced(K, hp, types, kv, prompt, forced, graphs=True):
    m = K.Model(hp, types)
    m.synth(1234)
    if kv is not None:
        m.set_kv_types(kv, kv)
    m.set_graphs(graphs)
    out = [m.decode(prompt, 0)]
    n = len(prompt)
    for tok in forced:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    return np.array(out)


@pytest.mark.parametrize("nm", list(KVQ))
def test_e2e_quantized_kv_vs_reference(env, nm):
    """tiny Q4_K_M model, Q8_0 / Q4_0 caches, prompt + 8 teacher-forced steps vs the reference's logits.
    Q4_0: equal to ~1e-7 (measured 2-5e-7; bar 1e-5, as the restatement's).  Q8_0: per step within 2x the
    reference's own build-to-build spread of that run (0.017 max; measured 0.006-0.019): a few K/V/Q values sit
    within an ulp of a Q8_0 rounding boundary, so ~1e-7 upstream differences flip single quanta -- the
    amplification that makes the AVX2 and scalar reference builds differ by 0.017 (tests/test_oracle_golden.py)"""
    torch, K = env
    g = np.load(R.ROOT + "/tests/golden/e2e_tiny.npz")
    L = np.load(R.ROOT + "/tests/golden/e2e_kvq.npz")[nm + "_logits"]
    sp = np.load(R.ROOT + "/tests/golden/ref_spread.npz")
    types = [int(t) for t in g["q4km_types"]]
    got = _forced(K, R.TINY, types, KVQ[nm], g["q4km_prompt"], g["q4km_tokens"][:L.shape[0] - 1])
    d = np.abs(got - L)
    print(nm, "kv vs reference max", d.max(axis=1), "median", np.median(d, axis=1))
    if nm == "q4_0":
        assert d.max() <= 1e-5
    else:
        assert np.all(d.max(axis=1) <= 2 * sp["kv_q8_0_max"].max())
        assert np.all(np.median(d, axis=1) <= 2 * sp["kv_q8_0_median"].max())


def test_quantized_kv_graph_equals_eager_and_no_shift(env):
    torch, K = env
    g = np.load(R.ROOT + "/tests/golden/e2e_tiny.npz")
    types = [int(t) for t in g["q4km_types"]]
    forced = g["q4km_tokens"][:6]
    a = _forced(K, R.TINY, types, R.Q8_0, g["q4km_prompt"], forced, graphs=True)
    b = _forced(K, R.TINY, types, R.Q8_0, g["q4km_prompt"], forced, graphs=False)
    assert np.array_equal(a, b)
    m = K.Model(R.TINY, types)
    m.synth(1234)
    m.set_kv_types(R.Q4_0, R.Q4_0)
    m.decode(list(g["q4km_prompt"]), 0, want_logits=False)
    with pytest.raises(RuntimeError):
        m.kv_shift(1, 4, len(g["q4km_prompt"]))
    with pytest.raises(RuntimeError):
        m.set_kv_types(R.Q8_0, R.F16)                 # mixed F16 / quantized is refused
    m.close()


def test_load_model_quantkv_generate(env, tmp_path):
    """load_model(quant_k = quant_v = 1) -> Q8_0 caches in every stage; generate()'s greedy tokens equal the
    in-process runtime's with the same caches"""
    torch, K = env
    import gguf_writer as GW
    from koboldcpp_amd import expose as X
    from test_gpu_expose import piece
    types = R.q4_k_m_types(R.TINY["n_layer"])
    path = str(tmp_path / "tiny.gguf")
    toks = GW.llama_gguf(path, R.TINY, types, 1234, GW.WORDS)
    _, _, ttypes = GW.spm_vocab(R.TINY["n_vocab"], GW.WORDS)
    h = X.init_library()
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 512
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
    li.flash_attention = True
    li.use_contextshift = True                        # turned off by the quantized cache
    li.quant_k = li.quant_v = 1
    assert h.load_model(li)
    prompt = b"hello world the"
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.memory = b""
    gi.max_context_length = 248
    gi.max_length = 12
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 7
    out = h.generate(gi)
    assert out.status == 1 and h.get_last_token_count() == 12
    m = K.Model(dict(R.TINY, n_ctx=256), types)
    m.synth(1234)
    m.set_kv_types(R.Q8_0, R.Q8_0)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(11):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()
    assert out.text == b"".join(piece(toks, ttypes, t) for t in want)
