"""The koboldcpp drop-in ABI end to end on the GPU: a synthetic Llama GGUF (tests/gguf_writer.py,
weights = the runtime's synthetic weights) is loaded through load_model(), generate() runs greedy,
and the text, token count, stop reason and stream must equal the same model built in-process
(kcpp_model_* with kcpp_model_synth_weights) decoding the same prompt ids."""
import ctypes

import numpy as np
import pytest

import gguf_writer as GW
import refharness as R

pytestmark = pytest.mark.gpu

# SentencePiece merges only through pieces that exist: give every word its whole prefix chain
WORDS = GW.WORDS


def piece(toks, types, t):
    """llama_token_to_piece_impl with special=false (src/llama-vocab.cpp:2014-2064, SPM): UNKNOWN / CONTROL
    are suppressed, UNUSED falls through to an empty piece, USER_DEFINED is copied raw."""
    s = toks[t]
    if types[t] in (2, 3, 5):
        return b""
    if types[t] == 4:
        return s.encode()
    if types[t] == 6:
        return bytes([int(s[3:5], 16)])
    return s.replace("▁", " ").encode()


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    import torch
    assert torch.cuda.is_available()
    from koboldcpp_amd import expose as X
    path = str(tmp_path_factory.mktemp("gguf") / "tiny.gguf")
    types = R.q4_k_m_types(R.TINY["n_layer"])
    toks = GW.llama_gguf(path, R.TINY, types, 1234, WORDS)
    h = X.init_library()
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 512
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
    assert h.load_model(li)
    _TINY.update(li=li, path=path)
    _, _, ttypes = GW.spm_vocab(R.TINY["n_vocab"], WORDS)
    return h, X, toks, ttypes, types


_TINY = {}


def _reload_tiny(model):
    """load the module's tiny GGUF again: the MoE / split tests above replace the loaded model"""
    h = model[0]
    assert h.load_model(_TINY["li"])


def test_token_count_spm(model):
    h, X, toks, ttypes, _ = model
    r = h.token_count(b"hello world the", True)
    ids = [r.ids[i] for i in range(r.count)]
    assert ids == [1, toks.index("▁hello"), toks.index("▁world"), toks.index("▁the")]
    r = h.token_count(b"hellab", False)        # merges stop at "▁hell" ("▁hella" is no piece)
    ids = [r.ids[i] for i in range(r.count)]
    assert ids == [toks.index("▁hell"), toks.index("ab")]
    r = h.token_count("zé".encode(), False)  # no pieces: byte fallback for every byte
    ids = [r.ids[i] for i in range(r.count)]
    assert [toks[i] for i in ids] == ["<0xE2>", "<0x96>", "<0x81>", "<0x7A>", "<0xC3>", "<0xA9>"]


def test_generate_greedy_matches_runtime(model):
    import koboldcpp_amd.lib as K
    h, X, toks, ttypes, types = model
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
    assert out.status == 1 and out.stopreason == 0
    assert h.get_last_token_count() == 12 and h.has_finished() and h.get_stream_count() == 12
    # the same model in-process
    hp = dict(R.TINY, n_ctx=256)
    m = K.Model(hp, types)
    m.synth(1234)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(11):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()
    text = b"".join(piece(toks, ttypes, t) for t in want)
    assert out.text == text
    assert b"".join(h.new_token(i) for i in range(12)) == text
    assert h.get_last_process_time() > 0 and h.get_last_eval_time() > 0
    # a second request sharing the prefix reuses the KV cache and gives the same continuation
    out2 = h.generate(gi)
    assert out2.text == text


def test_generate_stop_sequence_and_sampling(model):
    h, X, toks, ttypes, _ = model
    gi = X.generation_inputs()
    gi.prompt = b"the a b"
    gi.max_context_length = 248
    gi.max_length = 16
    gi.temperature = 0.8
    gi.top_k = 40
    gi.top_p = 0.9
    gi.rep_pen = 1.1
    gi.rep_pen_range = 64
    gi.bypass_eos_token = True
    gi.seed = 42
    a = h.generate(gi).text
    b = h.generate(gi).text
    assert a == b                               # seeded sampling is reproducible
    full = a
    if len(full) > 3:                            # stop on a substring of the known output
        stop = full[1:3]
        gi.stop_sequence[0] = stop
        o = h.generate(gi)
        assert o.stopreason == 2 and o.text == full[:full.find(stop)]


@pytest.mark.parametrize("split", [False, True])
def test_moe_gguf_generate_matches_runtime(model, tmp_path, split):
    """Mixtral-style GGUF (expert_count / expert_used_count, ffn_*_exps or per-expert tensors,
    ffn_gate_inp) through load_model + greedy generate == the in-process runtime.  Runs last: it
    replaces the module's loaded model."""
    import koboldcpp_amd.lib as K
    h, X, _, _, _ = model
    hp = dict(R.TINY_MOE, n_ctx=256)
    types = R.moe_types(hp["n_layer"])
    path = str(tmp_path / "moe.gguf")
    toks = GW.llama_gguf(path, hp, types, 99, WORDS, split_experts=split)
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 512
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
    assert h.load_model(li)
    _, _, ttypes = GW.spm_vocab(hp["n_vocab"], WORDS)
    prompt = b"hello world the a b of to the"
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.max_context_length = 248
    gi.max_length = 10
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    out = h.generate(gi)
    assert out.status == 1
    m = K.Model(hp, types)
    m.synth(99)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(9):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()
    assert out.text == b"".join(piece(toks, ttypes, t) for t in want)


def test_greedy_respects_logit_bias(model):
    """Greedy with a logit bias: the reference adds biases before any sampler (gpttype_adapter.cpp:1349-1353),
    token ids >= 0 accepted (:2576-2584).  Checked on tokens with visible pieces (the random weights may pick an
    unused token, whose piece is empty): a +1000 bias forces its token, a ban beside another +1000 moves the pick,
    and token 0 (<unk>, empty piece) at +1000 beats a visible token at +999."""
    h, X, toks, ttypes, _ = model
    _reload_tiny(model)
    gi = X.generation_inputs()
    gi.prompt = b"hello world"
    gi.max_context_length = 248
    gi.max_length = 1
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 3
    vis = [t for t in range(len(toks)) if ttypes[t] == 1 and piece(toks, ttypes, t)]
    v, w = vis[3], vis[7]
    gi.logit_biases[0].token_id = v
    gi.logit_biases[0].bias = 1000.0
    assert h.generate(gi).text == piece(toks, ttypes, v)
    gi.logit_biases[0].bias = -1000.0
    gi.logit_biases[1].token_id = w
    gi.logit_biases[1].bias = 1000.0
    assert h.generate(gi).text == piece(toks, ttypes, w)
    gi.logit_biases[0].token_id = 0                       # token 0 may be biased too (>= 0)
    gi.logit_biases[0].bias = 1000.0
    gi.logit_biases[1].bias = 999.0
    assert h.generate(gi).text == piece(toks, ttypes, 0) == b""


def test_long_context_decode_matches_short_context():
    """n_ctx beyond 16384 keys (the combine's old chunk table) builds, graph-replays and gives the same logits as
    a short-context model with the same weights (every decode failed at graph capture)."""
    import koboldcpp_amd.lib as K
    types = R.q4_k_m_types(R.TINY["n_layer"])
    prompt = list(range(3, 40))
    outs = []
    for n_ctx in (256, 20008):
        m = K.Model(dict(R.TINY, n_ctx=n_ctx), types)
        m.synth(1234)
        m.decode(prompt, 0, want_logits=False)
        t = m.argmax()
        lg = m.decode([t], len(prompt))
        outs.append(lg)
        m.close()
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("handoff,split", [("linked", (1.0, 2.0, 1.0)), ("copy", (1.0, 2.0, 1.0)),
                                           ("linked", (1.0, 1.0, 3.0, 1.0, 1.0))])
def test_generate_layer_split_pipeline_matches_single_stage(model, tmp_path, monkeypatch, handoff, split):
    """--tensorsplit through load_model: 3 or 5 stages (KCPP_VIRTUAL_DEVICES puts them all on the one GPU of the
    test box), prefill in 16-token ubatches pipelined across the stages, the residual stream handed stage to stage
    on the stage streams with event ordering and no host synchronisation (RCCL send/recv when the stages sit on
    distinct GPUs); greedy decode steps with the hand-off inside the stage graphs (link.hip: each stage's first
    kernel pulls its input once the producer's flag is up, stage 0 pulls the last stage's token; KCPP_HANDOFF=copy:
    the event-ordered copies, as in prefill), uneven stages -- greedy text equal to a single in-process stage with
    the same ubatch size.  Runs last: it replaces the module's loaded model."""
    import koboldcpp_amd.lib as K
    h, X, _, _, _ = model
    hp = dict(R.TINY, n_layer=5, n_ctx=256)
    types = R.q4_k_m_types(hp["n_layer"])
    path = str(tmp_path / "split.gguf")
    toks = GW.llama_gguf(path, hp, types, 1234, WORDS)
    monkeypatch.setenv("KCPP_VIRTUAL_DEVICES", str(len(split)))
    if handoff == "copy":
        monkeypatch.setenv("KCPP_HANDOFF", "copy")
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 16
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
    for i, v in enumerate(split):
        li.tensor_split[i] = v
    assert h.load_model(li)
    _, _, ttypes = GW.spm_vocab(hp["n_vocab"], WORDS)
    prompt = b" ".join([b"hello world the a b of to"] * 6)
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    assert len(ids) > 32                                       # at least three ubatches of 16
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.max_context_length = 248
    gi.max_length = 24
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    out = h.generate(gi)
    assert out.status == 1
    m = K.Model(hp, types, max_ubatch=16)
    m.synth(1234)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(23):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()
    assert out.text == b"".join(piece(toks, ttypes, t) for t in want)


def test_generate_row_split_matches_in_process(model, tmp_path, monkeypatch):
    """--rowsplit through load_model (use_rowsplit, tensor_split 1:2; KCPP_VIRTUAL_DEVICES=2 puts both row lanes on
    the test box's GPU): one stage owning every layer, each matrix's rows split over the lanes -- greedy text equal
    to the same row split built in-process"""
    import koboldcpp_amd.lib as K
    h, X, _, _, _ = model
    hp = dict(R.TINY, n_layer=3, n_ctx=256)
    types = R.q4_k_m_types(hp["n_layer"])
    path = str(tmp_path / "rows.gguf")
    toks = GW.llama_gguf(path, hp, types, 1234, WORDS)
    monkeypatch.setenv("KCPP_VIRTUAL_DEVICES", "2")
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 248
    li.blasbatchsize = 512
    li.gpulayers = 999
    li.rope_freq_base = 10000.0
    li.rope_freq_scale = 0.0     # koboldcpp.py default --ropeconfig 0: automatic RoPE
    li.use_rowsplit = True
    for i, v in enumerate((1.0, 2.0)):
        li.tensor_split[i] = v
    assert h.load_model(li)
    _, _, ttypes = GW.spm_vocab(hp["n_vocab"], WORDS)
    prompt = b" ".join([b"hello world the a b of to"] * 3)
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.max_context_length = 248
    gi.max_length = 8
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    out = h.generate(gi)
    assert out.status == 1
    m = K.Model(hp, types)
    m.set_row_split([0, 0], (1.0, 2.0))
    m.synth(1234)
    m.decode(ids, 0, want_logits=False)
    want = [m.argmax()]
    n = len(ids)
    for _ in range(7):
        want.append(m.decode_greedy(n))
        n += 1
    m.close()
    assert out.text == b"".join(piece(toks, ttypes, t) for t in want)


def test_engine_bench_virtual_stages(monkeypatch):
    """bench.py --gpus N's path (kcpp_engine_bench): load_model's layer-split stages (3 on the one test GPU via
    KCPP_VIRTUAL_DEVICES), event-ordered hand-off, pipelined prefill, generate()'s greedy loop -- runs and reports
    the token count it decoded"""
    import koboldcpp_amd.lib as K
    monkeypatch.setenv("KCPP_VIRTUAL_DEVICES", "3")
    hp = dict(R.TINY, n_layer=5, n_ctx=256)
    types = R.q4_k_m_types(hp["n_layer"])
    r = K.engine_bench(hp, types, 3, 64, 16, 2, 8)
    assert r["n_past"] == 64 + 2 + 8 and not r["rccl"]
    assert r["prefill_s"] > 0 and r["decode_s"] > 0
    # the linked single-token steps: 200 of them back to back on 8 stages (every hand-off flag reused 200 times)
    monkeypatch.setenv("KCPP_VIRTUAL_DEVICES", "8")
    hp8 = dict(R.TINY, n_layer=8, n_ctx=300)
    r = K.engine_bench(hp8, R.q4_k_m_types(8), 8, 32, 16, 4, 200)
    assert r["n_past"] == 32 + 4 + 200 and r["decode_s"] > 0


def test_generate_process_time_includes_the_prefill(model):
    """last_process_time covers the prompt's device time (the stream is drained before the clock stops): the
    prompt's ms/token x tokens is at least a third of the same prompt's synchronous in-process decode"""
    import time
    import koboldcpp_amd.lib as K
    h, X, _, _, types = model
    prompt = b" ".join([b"hello world the a b of to"] * 12)
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.max_context_length = 248
    gi.max_length = 2
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    h.generate(gi)                                   # warm (and fills the cache: the next call fast-forwards)
    gi.prompt = b"the " + prompt                    # a different first token: the whole prompt is processed again
    out = h.generate(gi)
    assert out.status == 1
    np_ = h.token_count(gi.prompt, True).count
    t_proc = h.get_last_process_time() * np_ / 1e3
    m = K.Model(dict(R.TINY, n_ctx=512), types, max_ubatch=512)
    m.synth(1234)
    m.decode(ids, 0, want_logits=False)
    t0 = time.perf_counter()
    m.decode(ids, 0, want_logits=False)
    t_ref = time.perf_counter() - t0
    m.close()
    assert t_proc >= 0.3 * t_ref, (t_proc, t_ref)


def _antislop_script(m, prompt_ids, phrases, limit, max_len, piece_of):
    """the reference's generation loop with antislop, restated from gpttype_adapter.cpp:3218-3341 + ContextRewind
    (:424-480) for greedy sampling on the in-process model: the sampled token's piece enters a delay line of `limit`
    entries; when the held-back text contains a banned phrase (lower case), the context is rewound to just before
    the shortest tail holding it, that tail's first token is banned at that position, and the new last context
    token is evaluated again.  Returns the streamed text and the number of sampled tokens."""
    import numpy as np
    ctx = list(prompt_ids)
    logits = m.decode(ctx, 0)
    delayed, out, slop, n_gen = [], [], {}, 0
    while n_gen < max_len:
        lg = logits.copy()
        for b in slop.get(len(ctx), []):
            lg[b] = -np.inf
        t = int(np.argmax(lg))
        n_gen += 1
        delayed.append(piece_of(t))
        while len(delayed) > limit:
            out.append(delayed.pop(0))
        scan = b"".join(delayed).lower()
        rewound = False
        for ph in phrases:
            if ph not in scan:
                continue
            check, r = b"", 0
            for d in reversed(delayed):
                check = d + check
                r += 1
                if ph in check.lower():
                    break
            full = ctx + [t]
            if r > 0 and len(full) - r > 0:
                last_tok = full[len(full) - r]
                delayed = delayed[:len(delayed) - r]
                ctx = full[:len(full) - r]
                logits = m.decode([ctx[-1]], len(ctx) - 1)
                slop.setdefault(len(ctx), []).append(last_tok)
                rewound = True
                break
        if rewound:
            continue
        logits = m.decode([t], len(ctx))
        ctx.append(t)
    return b"".join(out + delayed), n_gen


def test_generate_antislop_phrase_ban(model):
    """antislop phrase banning (gpttype_adapter.cpp:2514-2545 classification, :3218-3341 detection and rewind) against
    the loop restated in Python on the in-process model (_antislop_script; parity unpinned: ref_sampler has no
    generation loop, so these are scripted expectations derived from those lines): a phrase spanning two generated
    tokens is never streamed, the text before it is unchanged, the result equals the script's, and the delay line
    holds the text back only by the phrase's token count + 3."""
    import koboldcpp_amd.lib as K
    h, X, toks, ttypes, types = model
    _reload_tiny(model)
    prompt = b"hello world the"
    r = h.token_count(prompt, True)
    ids = [r.ids[i] for i in range(r.count)]
    gi = X.generation_inputs()
    gi.prompt = prompt
    gi.memory = b""
    gi.max_context_length = 248
    gi.max_length = 16
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 7
    base = h.generate(gi).text
    hp = dict(R.TINY, n_ctx=256)
    m = K.Model(hp, types)
    m.synth(1234)
    pf = lambda t: piece(toks, ttypes, t)
    import numpy as np
    lg = m.decode(ids, 0)
    first = m.argmax()
    lg1 = m.decode([first], len(ids))
    second = m.argmax()
    assert int(np.argmax(lg)) == first and int(np.argmax(lg1)) == second, (int(np.argmax(lg)), first, int(np.argmax(lg1)), second)
    plain, _ = _antislop_script(m, ids, [], 0, 16, pf)
    assert plain == base
    # greedy tokens of the plain run; a phrase made of two consecutive visible pieces that first occurs there
    m.decode(ids, 0, want_logits=False)
    seq = [m.argmax()]
    n = len(ids)
    for _ in range(15):
        seq.append(m.decode_greedy(n))
        n += 1
    phrase = None
    for i in range(2, 12):
        a, b = pf(seq[i]), pf(seq[i + 1])
        cand = (a + b).lower()
        if len(a) >= 1 and len(b) >= 1 and len(cand) >= 2 and cand not in b"".join(pf(t) for t in seq[:i + 1]).lower() \
                and cand not in b.lower():
            phrase = cand
            break
    if phrase is None:
        pytest.skip("the synthetic model's greedy text has no two-piece phrase to ban")
    gi.banned_tokens[0] = phrase
    got = h.generate(gi)
    ntok = h.token_count(phrase, False).count
    want, n_sampled = _antislop_script(m, ids, [phrase], ntok + 3, 16, pf)
    m.close()
    assert phrase not in got.text.lower()
    assert got.text == want
    assert got.text[:base.lower().find(phrase)] == base[:base.lower().find(phrase)]
    assert h.get_last_token_count() == n_sampled
    gi.banned_tokens[0] = None


def test_generate_render_special(model):
    """render_special (gpttype_adapter.cpp:3253-3257): a forced EOS (bypassed, so generation continues) renders as
    its text with render_special and as nothing without (the piece of a CONTROL token, llama_token_to_piece special)"""
    h, X, toks, ttypes, _ = model
    _reload_tiny(model)
    gi = X.generation_inputs()
    gi.prompt = b"hello world"
    gi.max_context_length = 248
    gi.max_length = 1
    gi.temperature = 0.0
    gi.top_k = 1
    gi.rep_pen = 1.0
    gi.bypass_eos_token = True
    gi.seed = 3
    gi.logit_biases[0].token_id = 2                       # </s>
    gi.logit_biases[0].bias = 1000.0
    gi.render_special = False
    assert h.generate(gi).text == b""
    gi.render_special = True
    assert h.generate(gi).text == b"</s>"
