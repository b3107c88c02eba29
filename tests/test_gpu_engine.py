"""The persistent single-token decode engine (koboldcpp_amd/csrc/dec_engine.hip: every layer of the stage in ONE launch,
in-launch hand-offs) against the launch chain it replaces (six fused launches per layer, runtime.cpp
forward_layers_dec), on Llama-3-8B-width layers with the Q4_K_M type policy (attn_v / ffn_down in Q6_K on the
"more bits" layers, Q4_K elsewhere).

The engine is a scheduling change only: every mat-vec computes its rows exactly as the stand-alone k_gemv_rs (same
lane -> piece map, same per-lane order, same wave reduction), the attention splits and assigns keys to waves exactly
as k_fa_dec4 and merges them as fadec::finish, and the split merge repeats k_fa_comb4's order -- so its logits are
the launch chain's BIT FOR BIT, at contexts that leave most splits empty (5 keys), prefetch every key of a split
(1k) and stream chunks through the LDS ring (12k keys), at full depth (32 layers), through the graph and eagerly, and
for a greedy loop.  The launch chain itself is pinned to the oracle / the reference (test_gpu_production_vs_oracle,
test_gpu_fullwidth), so these equalities carry that parity over to the engine."""
import ctypes

import numpy as np
import pytest

import refharness as R

pytestmark = pytest.mark.gpu

HP = dict(n_vocab=32000, n_embd=4096, n_head=32, n_head_kv=8, n_layer=4, n_ff=14336, n_ctx=512, eps=1e-5,
          rope_base=500000.0)


@pytest.fixture(scope="module")
def K():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return K


def prompt(n, seed=3):
    return [int(v) for v in np.random.default_rng(seed).integers(1, 32000, size=n)]


@pytest.mark.parametrize("n_ctx,n_prompt", [(512, 5), (2048, 1000), (16384, 12000)])
def test_engine_matches_launch_chain(K, n_ctx, n_prompt):
    hp = dict(HP, n_ctx=n_ctx)
    m = K.Model(hp, R.q4_k_m_types(hp["n_layer"]))
    m.synth(77)
    m.decode(prompt(n_prompt), 0, want_logits=False)
    nxt = [11, 2222, 31999, 7]
    outs = {}
    for eng in (True, False):
        m.set_engine(eng)
        outs[eng] = [m.decode([t], n_prompt + i) for i, t in enumerate(nxt)]   # same positions: same K/V rows
        assert m.engine_active() == int(eng)
    m.close()
    for a, b in zip(outs[True], outs[False]):
        assert np.isfinite(a).all()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), np.abs(a - b).max()


def test_engine_eager_equals_graph_and_greedy(K):
    """graph replay vs eager launch of the engine step: bit-identical; on-device greedy loop == the chain's tokens"""
    hp = dict(HP, n_ctx=1024)
    m = K.Model(hp, R.q4_k_m_types(hp["n_layer"]))
    m.synth(5)
    m.set_engine(True)
    p = prompt(300, 9)
    m.decode(p, 0, want_logits=False)
    g = [m.decode([t], 300 + i) for i, t in enumerate([3, 4, 5])]
    assert m.engine_active() == 1
    m.set_graphs(False)
    e = [m.decode([t], 300 + i) for i, t in enumerate([3, 4, 5])]
    for a, b in zip(g, e):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    m.set_graphs(True)
    toks = {}
    for eng in (True, False):
        m.set_engine(eng)
        m.decode(p, 0, want_logits=False)
        m.argmax()
        toks[eng] = [m.decode_greedy(300 + i) for i in range(24)]
    m.close()
    assert toks[True] == toks[False]


def test_engine_full_depth_first_token(K):
    """32 layers (the bench model): the first decode token's logits after a 512-token prompt, engine vs chain"""
    hp = dict(HP, n_layer=32, n_ctx=1024)
    m = K.Model(hp, R.q4_k_m_types(32))
    m.synth(1234)
    p = prompt(512, 4)
    m.decode(p, 0, want_logits=False)
    outs = []
    for eng in (True, False):
        m.set_engine(eng)
        outs.append(m.decode([42], 512))
    m.close()
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32)), np.abs(outs[0] - outs[1]).max()


@pytest.mark.parametrize("v6,d6,NP", [(False, False, 300), (True, True, 300), (False, True, 12000)])
def test_engine_phases_vs_kernels(K, v6, d6, NP):
    """one layer through kcpp_engine_decode vs the launch chain's kernels on the same inputs (8B shapes, 300 or
    12000 cached keys), every hand-off checked bit for bit: q (RoPE'd, f16) and the new K / V cache rows, the split
    partials (m, l, O), the attention's merged f32 rows and their Q8_K image, gate|up's h and the layer output."""
    import torch
    E_, F_, H_, HKV_, D_ = 4096, 14336, 32, 8, 128
    NCTX = 512 if NP < 500 else 16384
    EKV_ = HKV_ * D_
    s = torch.cuda.current_stream().cuda_stream
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if not K._L.kcpp_engine_supported(E_, F_, H_, HKV_, D_, ncu):
        pytest.skip("engine geometry not compiled for %d CUs" % ncu)
    Q4, Q6 = 112, 114
    g = np.random.default_rng(11)

    def synth(t, Kd, N, tid):
        w = torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", t, 5, tid, w.data_ptr(), Kd, N, s)
        return w
    tv, td = (Q6 if v6 else Q4), (Q6 if d6 else Q4)
    wq, wk, wv = synth(Q4, E_, E_, 1), synth(Q4, E_, EKV_, 2), synth(tv, E_, EKV_, 3)
    wo, wg, wu, wd = synth(Q4, E_, E_, 4), synth(Q4, E_, F_, 5), synth(Q4, E_, F_, 6), synth(td, F_, E_, 7)
    an = torch.from_numpy((1 + 0.1 * g.standard_normal(E_)).astype(np.float32)).cuda()
    fn = torch.from_numpy((1 + 0.1 * g.standard_normal(E_)).astype(np.float32)).cuda()
    x0 = (3 * g.standard_normal(E_)).astype(np.float32)
    kc0 = torch.from_numpy(g.standard_normal((NCTX, EKV_)).astype(np.float16)).cuda()
    vc0 = torch.from_numpy(g.standard_normal((NCTX, EKV_)).astype(np.float16)).cuda()
    tab = np.zeros(NCTX * D_, np.float32)
    K.call("kcpp_rope_table", tab.ctypes.data, NCTX, D_, 500000.0, 1.0, None, 0.0, 1.0, 32.0, 1.0, NCTX)
    rope = torch.from_numpy(tab).cuda()
    pos = torch.tensor([NP, 1], dtype=torch.int32, device="cuda")
    ws_bytes = int(K._L.kcpp_fa_workspace_bytes(16, H_, NCTX))
    scale = 1.0 / np.sqrt(D_)

    def bufs():
        return dict(x=torch.from_numpy(x0.copy()).cuda(), kc=kc0.clone(), vc=vc0.clone(),
                    q16=torch.zeros(H_ * D_, dtype=torch.float16, device="cuda"),
                    ws=torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda"),
                    act=torch.zeros(K.act_bytes(12, F_, 1) + 256, dtype=torch.uint8, device="cuda"),
                    h=torch.zeros(F_, device="cuda"), attn=torch.zeros(E_, device="cuda"))
    # ---- engine, one layer
    A = bufs()
    rec = np.zeros(int(K._L.kcpp_engine_layer_bytes()), np.uint8)
    K._L.kcpp_engine_layer(rec.ctypes.data, wq.data_ptr(), wk.data_ptr(), wv.data_ptr(), wo.data_ptr(), wg.data_ptr(),
                           wu.data_ptr(), wd.data_ptr(), an.data_ptr(), fn.data_ptr(), A["kc"].data_ptr(),
                           A["vc"].data_ptr(), int(v6), int(d6))
    lay = torch.from_numpy(rec).cuda()
    sync = torch.zeros(int(K._L.kcpp_engine_sync_bytes(1)), dtype=torch.uint8, device="cuda")
    dbg = torch.zeros(E_ + 64, device="cuda")
    K._L.kcpp_engine_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    rc = K._L.kcpp_engine_decode(lay.data_ptr(), 1, A["x"].data_ptr(), A["q16"].data_ptr(), A["ws"].data_ptr(),
                                 A["act"].data_ptr(), A["h"].data_ptr(), sync.data_ptr(), pos.data_ptr(),
                                 rope.data_ptr(), 1e-5, scale, E_, F_, H_, HKV_, s)
    torch.cuda.synchronize()
    K._L.kcpp_engine_set_debug(None)
    assert rc == 0
    assert int(sync.view(torch.int32)[-32].item()) == 0, "hand-off timeout"
    # ---- the launch chain's kernels
    B = bufs()
    a = K.DecArgs()
    a.K, a.x, a.nw, a.eps = E_, B["x"].data_ptr(), an.data_ptr(), 1e-5
    a.q16, a.kc, a.vc, a.ekv, a.D, a.pos, a.rope_tab = B["q16"].data_ptr(), B["kc"].data_ptr(), B["vc"].data_ptr(), EKV_, D_, pos.data_ptr(), rope.data_ptr()
    a.nseg = 3
    for j, (w, n) in enumerate([(wq, E_), (wk, EKV_), (wv, EKV_)]):
        a.W[j], a.N[j], a.role[j] = w.data_ptr(), n, j
    if v6:
        assert K._L.kcpp_gemv_rs_qkv_mixed(ctypes.byref(a), ctypes.c_void_p(s)) == 0
    else:
        assert K.gemv_dec(Q4, a, 2, 1, 2, s) == 0
    K.call("kcpp_flash_attn", B["q16"].data_ptr(), B["kc"].data_ptr(), B["vc"].data_ptr(), B["attn"].data_ptr(), None,
           B["ws"].data_ptr(), 1, H_, HKV_, D_, 0, pos.data_ptr(), NCTX, scale, 1, s)
    K.call("kcpp_quantize_act", 15, B["attn"].data_ptr(), E_, B["act"].data_ptr(), E_, 1, s)
    torch.cuda.synchronize()
    assert torch.equal(A["q16"].view(torch.int16), B["q16"].view(torch.int16)), "q"
    assert torch.equal(A["kc"][NP].view(torch.int16), B["kc"][NP].view(torch.int16)), "K row"
    assert torch.equal(A["vc"][NP].view(torch.int16), B["vc"][NP].view(torch.int16)), "V row"

    # the split partials (both sides use k_fa_dec4's partition: 32 splits per kv head): O [H][32][D], (M, L) [H][32]
    NS = 32
    off = 2048                                   # KCPP_FA_WS_HEADER
    def parts(ws):
        b = ws.cpu().numpy()
        po = b[off:off + H_ * NS * D_ * 4].view(np.float32).reshape(H_, NS, D_)
        pml = b[off + H_ * NS * D_ * 4:off + H_ * NS * D_ * 4 + H_ * NS * 8].view(np.float32).reshape(H_, NS, 2)
        return po, pml
    poA, pmlA = parts(A["ws"])
    poB, pmlB = parts(B["ws"])
    assert np.array_equal(poA.view(np.uint32), poB.view(np.uint32)), "split partials O"
    assert np.array_equal(pmlA.view(np.uint32), pmlB.view(np.uint32)), "split partials (m, l)"
    dd = dbg.cpu().numpy()
    attn_ref = B["attn"].cpu().numpy()
    assert np.array_equal(dd[:E_].view(np.uint32), attn_ref.view(np.uint32)), "merged attention"
    K.call("kcpp_quantize_act", 15, B["attn"].data_ptr(), E_, B["act"].data_ptr(), E_, 1, s)
    torch.cuda.synchronize()
    nb = E_ + E_ // 64 + E_ // 8
    assert torch.equal(A["act"][:nb], B["act"][:nb]), "attention Q8_K image"
    a2 = K.DecArgs()
    a2.K, a2.nseg, a2.act = E_, 1, B["act"].data_ptr()
    a2.W[0], a2.N[0], a2.Y[0], a2.res = wo.data_ptr(), E_, B["x"].data_ptr(), B["x"].data_ptr()
    assert K.gemv_dec(Q4, a2, 0, 0, 1, s) == 0
    a3 = K.DecArgs()
    a3.K, a3.x, a3.nw, a3.eps, a3.nseg = E_, B["x"].data_ptr(), fn.data_ptr(), 1e-5, 1
    a3.W[0], a3.W2, a3.N[0], a3.Y[0] = wg.data_ptr(), wu.data_ptr(), F_, B["h"].data_ptr()
    assert K.gemv_dec(Q4, a3, 1, 1, 1, s) == 0
    a4 = K.DecArgs()
    a4.K, a4.x, a4.nseg = F_, B["h"].data_ptr(), 1
    a4.W[0], a4.N[0], a4.Y[0], a4.res = wd.data_ptr(), E_, B["x"].data_ptr(), B["x"].data_ptr()
    assert K.gemv_dec(td, a4, 0, 2, 1, s) == 0
    torch.cuda.synchronize()
    hA, hB = A["h"].cpu().numpy(), B["h"].cpu().numpy()
    xA, xB = A["x"].cpu().numpy(), B["x"].cpu().numpy()
    assert np.array_equal(hA.view(np.uint32), hB.view(np.uint32)), "h"
    assert np.array_equal(xA.view(np.uint32), xB.view(np.uint32)), "x"
