"""RoPE configuration of real Llama-3.x GGUFs in the drop-in path, against the reference:
* rope_freqs.weight (Llama-3.1 / 3.2 frequency factors, src/llama.cpp:7171 + build_rope_factors :10269): a tiny
  Llama (rope base 10000, n_ctx 1024) with Llama-3.1 factors prefills 700 tokens, is context-shifted (the K-shift
  takes the factors too) and decodes 8 teacher-forced tokens; logits vs the reference build's
  (tests/golden/make_rope_freqs.py -> rope_freqs_e2e.npz) within 1.5x its AVX2-vs-scalar spread with the
  strict-parity attention and within the tiny e2e bar of test_gpu_model with the production attention; the same run
  without the factors is 10x the spread away (so a dropped tensor fails);
* load_model reads rope_freqs.weight from the GGUF and applies it (generate() == the in-process model with the
  factors set), and applies koboldcpp's automatic RoPE base (GradientAI, gpttype_adapter.cpp:1926-1949) when the
  requested context exceeds llama.context_length;
* gpulayers below n_layer (a partial CPU offload, src/llama.cpp:6977-7036) is refused, not silently ignored."""
import os

import numpy as np
import pytest

import gguf_writer as GW
import refharness as R
from test_gpu_model import TOL_MAX, TOL_MEDIAN_F32

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


@pytest.mark.parametrize("strict", [True, False])
def test_rope_freqs_vs_reference(K, strict):
    g = np.load(os.path.join(HERE, "golden", "rope_freqs_e2e.npz"))
    hp = dict(R.TINY, rope_base=float(g["rope_base"]), n_ctx=int(g["n_ctx"]))
    p0, diff = (int(v) for v in g["shift"])
    prompt = [int(v) for v in g["prompt"]]
    m = K.Model(hp, [int(t) for t in g["types"]])
    m.synth(1234)
    m.set_rope_freqs(g["rope_freqs"])
    m.set_fa_exact(strict)
    out = [m.decode(prompt, 0)]
    m.kv_shift(p0, diff, len(prompt))
    n = len(prompt) - diff
    for tok in g["forced"]:
        out.append(m.decode([int(tok)], n))
        n += 1
    m.close()
    out = np.array(out)
    d = np.abs(out - g["logits"])
    print("gpu vs ref max", d.max(axis=1), "| spread", g["spread_max"])
    if strict:
        assert np.all(d.max(axis=1) <= 1.5 * g["spread_max"].max())
        assert np.all(np.median(d, axis=1) <= 1.5 * g["spread_median"].max())
    else:
        assert np.all(d.max(axis=1) <= TOL_MAX) and np.all(np.median(d, axis=1) <= TOL_MEDIAN_F32)
    assert np.abs(out - g["nofreq_logits"]).max() > 10 * g["spread_max"].max()


def _load(X, path, max_ctx, gpulayers=999):
    h = X.init_library()
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = max_ctx
    li.blasbatchsize = 512
    li.gpulayers = gpulayers
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0                      # koboldcpp.py default --ropeconfig: automatic
    return h, h.load_model(li)


def _greedy(h, X, prompt, n):
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.memory = b""
    gi.max_context_length = 200
    gi.max_length = n
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 7
    out = h.generate(gi)
    assert out.status == 1
    return out.text


def _runtime_text(K, hp, types, ids, n, toks, ttypes, ff=None):
    from test_gpu_expose import piece
    m = K.Model(hp, types)
    m.synth(1234)
    if ff is not None:
        m.set_rope_freqs(ff)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    p = len(ids)
    for _ in range(n - 1):
        want.append(m.decode_greedy(p))
        p += 1
    m.close()
    return b"".join(piece(toks, ttypes, t) for t in want)


def test_load_model_reads_rope_freqs(K, tmp_path):
    from koboldcpp_amd import expose as X
    hp = dict(R.TINY, rope_base=10000.0, n_ctx=1024)
    types = R.q4_k_m_types(hp["n_layer"])
    ff = R.llama31_rope_freqs(10000.0, hp["n_embd"] // hp["n_head"])
    path = str(tmp_path / "rf.gguf")
    toks = GW.llama_gguf(path, hp, types, 1234, GW.WORDS, rope_freqs=ff)
    _, _, ttypes = GW.spm_vocab(hp["n_vocab"], GW.WORDS)
    h, ok = _load(X, path, 1000)
    assert ok
    prompt = b"hello world the " * 40
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    text = _greedy(h, X, prompt, 10)
    assert text == _runtime_text(K, dict(hp, n_ctx=1008), types, ids, 10, toks, ttypes, ff)


def test_load_model_auto_rope_base(K, tmp_path):
    from koboldcpp_amd import expose as X
    hp = dict(R.TINY, n_ctx=1024)                 # trained context 1024, base 500000 (auto-scaled family)
    types = R.q4_k_m_types(hp["n_layer"])
    path = str(tmp_path / "auto.gguf")
    toks = GW.llama_gguf(path, hp, types, 1234, GW.WORDS)
    _, _, ttypes = GW.spm_vocab(hp["n_vocab"], GW.WORDS)
    base = float(K._L.kcpp_gradient_ai_rope_base(500000.0, 1024, 3000, 0))
    assert base > 700000.0
    h, ok = _load(X, path, 3000)
    assert ok
    prompt = b"hello world the " * 40
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    text = _greedy(h, X, prompt, 10)
    assert text == _runtime_text(K, dict(hp, rope_base=base, n_ctx=3008), types, ids, 10, toks, ttypes)


def test_load_model_refuses_partial_offload(tmp_path):
    from koboldcpp_amd import expose as X
    path = str(tmp_path / "t.gguf")
    GW.llama_gguf(path, R.TINY, R.q4_k_m_types(R.TINY["n_layer"]), 1234, GW.WORDS)
    _, ok = _load(X, path, 248, gpulayers=1)
    assert not ok
