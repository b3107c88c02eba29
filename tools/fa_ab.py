"""Prefill flash-attention A/B (tools only): kcpp_flash_attn_prefill_mfma variants (default 2 vs 3) at the bench's
ubatch-512 shapes (Llama-3-8B: 32 q heads, 8 kv heads, D 128), HIP-event timed.
usage: python tools/fa_ab.py [variants...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402


def main():
    s = torch.cuda.current_stream()
    H, HKV, D, T = 32, 8, 128, 512
    n_ctx = 4096
    q = torch.randn(T, H, D, device="cuda").half()
    kc = (torch.randn(n_ctx, HKV, D, device="cuda") * 0.5).half()
    vc = torch.randn(n_ctx, HKV, D, device="cuda").half()
    out = torch.empty(T, H, D, device="cuda")
    for n_past in [int(x) for x in os.environ.get("FA_NPAST", "0,1536,3328").split(",")]:
        for v in [int(a) for a in sys.argv[1:]] or [2, 3]:
            K.raw().kcpp_fa_prefill_set_variant(v)
            run = lambda: K.call("kcpp_flash_attn_prefill_mfma", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), out.data_ptr(),
                                 T, H, HKV, D, n_past, 1.0 / D ** 0.5, s.cuda_stream)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for _ in range(10):
                run()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            fl = 4.0 * H * D * sum(n_past + t + 1 for t in range(T))       # causal QK^T + PV
            print(json.dumps({"n_past": n_past, "T": T, "variant": v, "us": round(us, 1), "TFLOPs": round(fl / us / 1e6, 1)}),
                  flush=True)
    K.raw().kcpp_fa_prefill_set_variant(0)


if __name__ == "__main__":
    main()
