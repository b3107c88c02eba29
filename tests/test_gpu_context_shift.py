"""Context shifting (koboldcpp PurgeMissingTokens, gpttype_adapter.cpp:1504-1571, and the K-shift of
llama.cpp's build_k_shift): a middle span of the context leaves the KV cache, the rows behind it move down and
their K is re-rotated by the shift distance (ggml_compute_forward_rope_f16, mode NORM).

* kernel: kcpp_kv_shift_rows vs a numpy restatement of rope_f16 with the library's own (cos, sin) row -- bit-exact;
* runtime (one layer, whose K/V rows depend only on their own tokens): prefill A, shift out a span, decode new
  tokens  vs  prefill the shortened context from scratch -- equal up to the K-shift's extra f16 rounding;
* drop-in ABI: load_model(use_contextshift) + generate() with a prompt whose middle was cut runs the shift path;
* against the reference: the K-shift kernel bit for bit vs build_k_shift's rope (tests/golden/kshift.npz), and a
  2-layer model's decode on the shifted cache vs the reference's logits (tests/golden/kshift_e2e.npz)."""
import ctypes

import numpy as np
import pytest

import refharness as R
from test_gpu_model import TOL_MAX, TOL_MEDIAN_F32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def rope_row(K, p, D, base):
    row = np.zeros(D, np.float32)
    K.call("kcpp_rope_row", row.ctypes.data, p, D, base, 1.0, 0.0, 1.0, 32.0, 1.0, 256)
    return row


@pytest.mark.parametrize("diff", [1, 37, 1000])
def test_kv_shift_rows_bitexact(env, diff):
    torch, K = env
    D, HKV, n = 128, 8, 50
    rng = np.random.default_rng(diff)
    k = (rng.standard_normal((n, HKV, D)) * 2).astype(np.float16)
    v = rng.standard_normal((n, HKV, D)).astype(np.float16)
    cs = rope_row(K, -diff, D, 500000.0)
    kd, vd = torch.from_numpy(k.view(np.uint16).astype(np.int16)).cuda(), torch.from_numpy(v.view(np.uint16).astype(np.int16)).cuda()
    ks, vs = torch.empty_like(kd), torch.empty_like(vd)
    csd = torch.from_numpy(cs).cuda()
    s = torch.cuda.current_stream().cuda_stream
    K.call("kcpp_kv_shift_rows", kd.data_ptr(), vd.data_ptr(), ks.data_ptr(), vs.data_ptr(), n * HKV, D, csd.data_ptr(), s)
    torch.cuda.synchronize()
    got_k = ks.cpu().numpy().astype(np.uint16).view(np.float16).reshape(n, HKV, D)
    got_v = vs.cpu().numpy().astype(np.uint16).view(np.float16).reshape(n, HKV, D)
    x0, x1 = k[..., 0::2].astype(np.float32), k[..., 1::2].astype(np.float32)
    c, sn = cs[0::2], cs[1::2]
    want = np.empty_like(k)
    want[..., 0::2] = (x0 * c - x1 * sn).astype(np.float16)
    want[..., 1::2] = (x0 * sn + x1 * c).astype(np.float16)
    assert np.array_equal(got_k.view(np.uint16), want.view(np.uint16))
    assert np.array_equal(got_v.view(np.uint16), v.view(np.uint16))


@pytest.mark.parametrize("types_fn", [lambda n: R.q4_k_m_types(n), lambda n: R.uniform_types(n, R.Q8_0)])
def test_model_kv_shift_vs_recompute(env, types_fn):
    """one layer: its K/V rows depend on their own token only, so the shifted cache must equal a recompute of the
    shortened context up to the K-shift's extra f16 rounding (f16(rope(f16(rope(k, p)), -diff)) vs
    f16(rope(k, p - diff))).  With more layers the moved rows still carry what they attended to in the erased
    span -- as in the reference, context shifting is not a recompute -- so only the first layer is comparable."""
    torch, K = env
    hp = dict(R.TINY, n_layer=1)
    types = types_fn(hp["n_layer"])
    rng = np.random.default_rng(3)
    A = [int(v) for v in rng.integers(1, 500, size=150)]
    new = [int(v) for v in rng.integers(1, 500, size=5)]
    p0, diff = 20, 45
    shortened = A[:p0] + A[p0 + diff:]

    def run(prefill, shift):
        m = K.Model(hp, types)
        m.synth(1234)
        m.decode(prefill, 0, want_logits=False)
        if shift:
            m.kv_shift(p0, diff, len(A))
        out = [m.decode(new[:1], len(shortened))]
        for i, t in enumerate(new[1:]):
            out.append(m.decode([t], len(shortened) + 1 + i))
        m.close()
        return np.array(out)

    d = np.abs(run(A, True) - run(shortened, False))
    # the e2e bar (test_gpu_model): an f16-ulp change of a key can flip one Q8_K rounding of wo's input
    assert d.max() < TOL_MAX and np.median(d) < TOL_MEDIAN_F32, (d.max(), np.median(d))


def test_model_kv_shift_rejects_bad_ranges(env):
    torch, K = env
    m = K.Model(R.TINY, R.q4_k_m_types(R.TINY["n_layer"]))
    for p0, diff, n_past in [(-1, 3, 10), (5, 0, 10), (5, 6, 10), (0, 1, R.TINY["n_ctx"] + 1)]:
        assert K.raw().kcpp_model_kv_shift(m.m, p0, diff, n_past) < 0
    m.close()


def test_generate_with_context_shift(tmp_path, capfd):
    """load_model(use_contextshift) + a second prompt = first prompt with 30 words cut after a 20-word head and 30
    new words (226 -> 236 tokens: past koboldcpp's 208-token shortfall threshold at n_ctx 248):
    generate() erases the span from the KV cache (K-shift) and continues; the continuation equals the one
    generated without context shifting for the first tokens (the shift only perturbs f16 rounding)"""
    import gguf_writer as GW
    from koboldcpp_amd import expose as X
    from test_gpu_expose import WORDS
    path = str(tmp_path / "tiny.gguf")
    GW.llama_gguf(path, R.TINY, R.q4_k_m_types(R.TINY["n_layer"]), 1234, WORDS)
    h = X.init_library()
    words = ["hello", "world", "the"]            # one SentencePiece token each (test_gpu_expose.test_token_count_spm)
    rng = np.random.default_rng(11)
    A = [words[i] for i in rng.integers(0, len(words), size=235)]
    new = [words[i] for i in rng.integers(0, len(words), size=30)]
    B = A[:20] + A[50:] + new
    outs = []
    for shift in (True, False):
        li = X.load_model_inputs()
        li.model_filename = path.encode()
        li.max_context_length = 248
        li.blasbatchsize = 512
        li.gpulayers = 999
        li.rope_freq_base = 10000.0
        li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
        li.use_contextshift = shift
        assert h.load_model(li)
        res = []
        for words_ in (A, B):
            gi = X.generation_inputs()
            gi.prompt = " ".join(words_).encode()
            r = h.token_count(gi.prompt, True)
            assert r.count == len(words_) + 1
            gi.memory = b""
            gi.max_context_length = 248
            gi.max_length = 8
            gi.temperature = 0.0
            gi.top_k = 1
            gi.rep_pen = 1.0
            gi.bypass_eos_token = True
            gi.seed = 5
            out = h.generate(gi)
            assert out.status == 1
            res.append([h.new_token(i) for i in range(h.get_stream_count())])
        outs.append(res)
    err = capfd.readouterr().err
    assert err.count("Context Shifting: Erased") == 1, err
    assert outs[0][0] == outs[1][0]                  # first request: identical paths
    assert outs[0][1][:1] == outs[1][1][:1]          # after the shift: same next token


def _kshift_fixture():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kshift.npz"))


@pytest.mark.parametrize("base", [10000, 500000])
@pytest.mark.parametrize("diff", [1, 37, 1000])
def test_kv_shift_rows_vs_reference_k_shift(env, base, diff):
    """the K-shift pinned to the reference: llama.cpp's build_k_shift graph (ggml_rope_ext_inplace on the F16 K-cache
    view at position -diff, rope_f16, src/llama.cpp:10144-10190) run by the reference library
    (tests/golden/make_kshift.py)  ==  kcpp_kv_shift_rows with the runtime's (cos, sin) row, bit for bit"""
    torch, K = env
    fx = _kshift_fixture()
    k = fx["k_in"]
    n, HKV, D = k.shape
    cs = rope_row(K, -diff, D, float(base))
    kd = torch.from_numpy(k.view(np.int16).copy()).cuda()
    vd = torch.zeros_like(kd)
    ks, vs = torch.empty_like(kd), torch.empty_like(vd)
    csd = torch.from_numpy(cs).cuda()
    K.call("kcpp_kv_shift_rows", kd.data_ptr(), vd.data_ptr(), ks.data_ptr(), vs.data_ptr(), n * HKV, D, csd.data_ptr(),
           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = ks.cpu().numpy().astype(np.uint16)
    assert np.array_equal(got, fx["k_shift_%d_%d" % (base, diff)])


@pytest.mark.parametrize("strict", [False, True], ids=["production", "strict"])
def test_model_kv_shift_vs_reference_logits(env, strict):
    """context shift end to end against the REFERENCE: a 2-layer tiny Llama (Q4_K_M policy) prefills 150 tokens,
    45 cells after the first 20 are erased (kcpp_model_kv_shift  vs  the reference's seq_rm / seq_add +
    build_k_shift, run by oracle/ref_llama.c on its own graph: tests/golden/make_kshift_e2e.py) and 8 teacher-forced
    tokens are decoded on the shifted cache.  Bars: with the strict-parity attention every step
    within 1.5x this fixture's AVX2-vs-scalar spread; with the production attention (f32 V*P accumulator) the tiny
    e2e bar of test_gpu_model (TOL_MAX / TOL_MEDIAN_F32).  The shift moves the logits by up to 1.6, so a missing or
    wrong shift fails either bar."""
    import os
    torch, K = env
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kshift_e2e.npz"))
    p0, diff = (int(v) for v in g["shift"])
    prompt = [int(v) for v in g["prompt"]]
    m = K.Model(R.TINY, [int(t) for t in g["types"]])
    m.synth(1234)
    m.set_fa_exact(strict)
    out = [m.decode(prompt, 0)]
    m.kv_shift(p0, diff, len(prompt))
    n = len(prompt) - diff
    for tok in g["forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    d = np.abs(np.array(out) - g["logits"])
    print("gpu vs ref max", d.max(axis=1), "| spread", g["spread_max"])
    if strict:
        assert np.all(d.max(axis=1) <= 1.5 * g["spread_max"].max())
        assert np.all(np.median(d, axis=1) <= 1.5 * g["spread_median"].max())
    else:
        assert np.all(d.max(axis=1) <= TOL_MAX) and np.all(np.median(d, axis=1) <= TOL_MEDIAN_F32)
    # and not the unshifted continuation
    assert np.abs(np.array(out)[1:] - g["noshift_logits"][1:]).max() > 10 * g["spread_max"].max()
