"""Kernel micro-benchmarks (HIP-event timed) for the hot path: mat-vec (decode), MFMA GEMM (prefill),
flash attention.  Prints one JSON line per kernel.  Not part of the driver contract."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import sys

import numpy as np
import torch

import koboldcpp_amd.lib as K


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    s = torch.cuda.current_stream().cuda_stream
    out = []
    shapes = [(12, 4096, 14336, 512), (12, 4096, 4096, 512), (12, 4096, 1024, 512), (14, 4096, 1024, 512),
              (12, 4096, 6144, 512), (12, 4096, 28672, 512), (14, 14336, 4096, 512), (12, 14336, 4096, 512),
              (8, 4096, 14336, 32), (8, 4096, 4096, 512), (2, 4096, 4096, 512), (13, 4096, 4096, 512)]
    if os.environ.get("MB_SHAPES") == "prefill":
        shapes = shapes[:8]
    if os.environ.get("MB_SHAPES") == "fa":
        shapes = []
    for (t, Kd, N, M) in shapes:
        wb = Kd // K.BLOCK[t][0] * K.BLOCK[t][1] * N
        w = torch.empty(wb, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", t, 1, 1, w.data_ptr(), Kd, N, s)
        x = torch.randn(M, Kd, device="cuda")
        act = torch.empty(K.act_bytes(t, Kd, M), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", K.vec_dot_type(t), x.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
        y = torch.empty(M, N, device="cuda")
        ws = torch.empty(max(1, K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M)), dtype=torch.uint8, device="cuda")
        if M > 8:
            f = lambda: K.call("kcpp_gemm", t, w.data_ptr(), None, Kd, N, act.data_ptr(), M, y.data_ptr(), N, None, 0, 0, ws.data_ptr(), s)
        else:
            f = lambda: K.call("kcpp_gemv", t, w.data_ptr(), None, Kd, N, act.data_ptr(), M, y.data_ptr(), N, None, 0, 0, s)
        ms = timeit(f)
        flop = 2.0 * Kd * N * M
        out.append({"kernel": "gemm" if M > 8 else "gemv", "type": t, "K": Kd, "N": N, "M": M, "ms": round(ms, 4),
                    "TFLOPs": round(flop / ms / 1e9, 1), "weight_GBps": round(wb / ms / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    # flash attention prefill / decode
    H, HKV, D, n_ctx = 32, 8, 128, 4096
    kc = torch.randn(n_ctx, HKV * D, device="cuda").half()
    vc = torch.randn(n_ctx, HKV * D, device="cuda").half()
    for (T, n_past) in [(512, 0), (512, 3328), (1, 4095), (1, 1024)]:
        q = torch.randn(T, H, D, device="cuda").half()
        o = torch.empty(T, H, D, device="cuda")
        ws = torch.zeros(K.fa_workspace_bytes(max(T, 16), H, n_ctx), dtype=torch.uint8, device="cuda")
        f = lambda: K.call("kcpp_flash_attn", q.data_ptr(), kc.data_ptr(), vc.data_ptr(), o.data_ptr(), None, ws.data_ptr(),
                           T, H, HKV, D, n_past, None, n_ctx, 1 / np.sqrt(D), 0, s)
        ms = timeit(f)
        pairs = sum(n_past + t + 1 for t in range(T))
        flop = 4.0 * D * H * pairs
        kvb = 2 * (n_past + T) * HKV * D * 2
        print(json.dumps({"kernel": "flash_attn", "T": T, "n_past": n_past, "ms": round(ms, 4),
                          "TFLOPs": round(flop / ms / 1e9, 2), "kv_GBps": round(kvb / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
