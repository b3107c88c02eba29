"""The key-split MFMA prefill attention (attn_mfma.hip k_fa_prefill_mfma3<8, true>: ubatches <= 64 tokens, keys split
over ~512 workgroups, the last split of each (query block, kv head) merging in split order) and its KT_Q8_0_TA
epilogue (attn_output's activation for KT_Q8_0_T weights).

  * split == unsplit (k_fa_prefill_mfma3<8, false>, pinned against the reference elsewhere: test_gpu_fullwidth.py,
    test_gpu_deep.py) to the f16 rounding of P (taken against each split's own maximum); the split launch is deterministic and leaves its tickets at
    zero (same bits twice on one workspace);
  * the TA output is bit-identical to kcpp_quantize_act(KT_Q8_0_TA) of the same launch's f32 output.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available()
    import koboldcpp_amd.lib as K
    return torch, K


def sptr(torch):
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("T,n_past", [(32, 992), (32, 0), (17, 3000), (64, 200), (48, 4000)])
def test_split_prefill_vs_unsplit_and_ta(env, T, n_past):
    torch, K = env
    H, HKV, D, n_ctx = 32, 8, 128, 4096 + 64
    E = H * D
    g = torch.Generator(device="cuda").manual_seed(T * 7 + n_past)
    q16 = torch.randn(T, H, D, device="cuda", generator=g).half()
    kc = torch.randn(n_ctx, HKV * D, device="cuda", generator=g).half()
    vc = torch.randn(n_ctx, HKV * D, device="cuda", generator=g).half()
    scale = 1.0 / np.sqrt(D)
    ref = torch.empty(T, E, device="cuda")
    K.call("kcpp_flash_attn_prefill_mfma", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), ref.data_ptr(), T, H, HKV, D,
           n_past, scale, sptr(torch))
    ws = torch.zeros(int(K.raw().kcpp_fa_workspace_bytes(16, H, n_ctx)), dtype=torch.uint8, device="cuda")
    assert ws.numel() >= K.raw().kcpp_fa_split_ws_bytes(H)
    outs, qtas = [], []
    for _ in range(2):
        out = torch.full((T, E), float("nan"), device="cuda")
        qta = torch.zeros(K.act_bytes(K.Q8_0_T, E, T), dtype=torch.uint8, device="cuda")
        K.call("kcpp_flash_attn_prefill_mfma_ex", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), out.data_ptr(),
               qta.data_ptr(), ws.data_ptr(), T, H, HKV, D, n_past, scale, sptr(torch))
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        qtas.append(qta.cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    assert np.array_equal(qtas[0], qtas[1])
    assert not ws[:2048].any().item()                       # header untouched
    r = ref.cpu().numpy()
    err = np.abs(outs[0] - r).max()
    print("T %d n_past %d: split vs unsplit max |d| %.3g (max |o| %.3g)" % (T, n_past, err, np.abs(r).max()))
    # P is rounded to f16 against each split's own running maximum (unsplit: the whole row's): f16-ulp-level drift
    assert err <= 2e-3 * np.abs(r).max() + 1e-5
    # the epilogue's TA bytes == kcpp_quantize_act of the same f32 output
    sep = torch.zeros_like(torch.from_numpy(qtas[0])).cuda()
    outd = torch.from_numpy(outs[0]).cuda()
    K.call("kcpp_quantize_act", K.Q8_0_TA, outd.data_ptr(), E, sep.data_ptr(), E, T, sptr(torch))
    torch.cuda.synchronize()
    assert np.array_equal(qtas[0], sep.cpu().numpy())


def test_unsplit_ta_epilogue(env):
    """T > 64 (no split): the TA epilogue alone, out = NULL, equals quantize_act of the plain kernel's output"""
    torch, K = env
    T, H, HKV, D, n_past = 80, 32, 8, 128, 500
    E = H * D
    g = torch.Generator(device="cuda").manual_seed(3)
    q16 = torch.randn(T, H, D, device="cuda", generator=g).half()
    kc = torch.randn(1024, HKV * D, device="cuda", generator=g).half()
    vc = torch.randn(1024, HKV * D, device="cuda", generator=g).half()
    ref = torch.empty(T, E, device="cuda")
    K.call("kcpp_flash_attn_prefill_mfma", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), ref.data_ptr(), T, H, HKV, D,
           n_past, 0.088, sptr(torch))
    want = torch.zeros(K.act_bytes(K.Q8_0_T, E, T), dtype=torch.uint8, device="cuda")
    K.call("kcpp_quantize_act", K.Q8_0_TA, ref.data_ptr(), E, want.data_ptr(), E, T, sptr(torch))
    qta = torch.zeros_like(want)
    ws = torch.zeros(int(K.raw().kcpp_fa_workspace_bytes(16, H, 1024)), dtype=torch.uint8, device="cuda")
    K.call("kcpp_flash_attn_prefill_mfma_ex", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), None, qta.data_ptr(),
           ws.data_ptr(), T, H, HKV, D, n_past, 0.088, sptr(torch))
    torch.cuda.synchronize()
    assert torch.equal(qta, want)


@pytest.mark.parametrize("n_past,dev", [(3840, False), (100, True)])
def test_decode_ta_combine(env, n_past, dev):
    """single-token decode with the combine writing the KT_Q8_0_TA activation: out bit-identical to the plain pair,
    TA bytes == kcpp_quantize_act(KT_Q8_0_TA) of that output"""
    import ctypes
    torch, K = env
    H, HKV, D, n_ctx = 32, 8, 128, 4096
    E = H * D
    g = torch.Generator(device="cuda").manual_seed(n_past)
    q16 = torch.randn(1, H, D, device="cuda", generator=g).half()
    kc = torch.randn(n_ctx, HKV * D, device="cuda", generator=g).half()
    vc = torch.randn(n_ctx, HKV * D, device="cuda", generator=g).half()
    ws = torch.zeros(int(K.raw().kcpp_fa_workspace_bytes(16, H, n_ctx)), dtype=torch.uint8, device="cuda")
    npd = torch.tensor([n_past], dtype=torch.int32, device="cuda")
    ref = torch.empty(1, E, device="cuda")
    K.call("kcpp_flash_attn", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), ref.data_ptr(), None, ws.data_ptr(), 1, H,
           HKV, D, 0 if dev else n_past, npd.data_ptr() if dev else None, n_ctx, 0.088, 0, sptr(torch))
    out = torch.empty(1, E, device="cuda")
    qta = torch.zeros(K.act_bytes(K.Q8_0_T, E, 1), dtype=torch.uint8, device="cuda")
    K.call("kcpp_flash_attn_dec_ta", q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), out.data_ptr(), qta.data_ptr(),
           ws.data_ptr(), H, HKV, D, 0 if dev else n_past, npd.data_ptr() if dev else None, n_ctx, 0.088, sptr(torch))
    want = torch.zeros_like(qta)
    K.call("kcpp_quantize_act", K.Q8_0_TA, ref.data_ptr(), E, want.data_ptr(), E, 1, sptr(torch))
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(qta, want)
