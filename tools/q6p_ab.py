"""A/B timing of the Q6_K prefill GEMM: kcpp_gemm(KT_Q6_K_RS) (q6v3, f16 MFMA) vs kcpp_gemm_q6p (int8 image) at
the bench's prefill shapes (M = 512): ffn_down 14336 -> 4096 and attn_v 4096 -> 1024, plus an all-Q6_K gate|up.
Prints one JSON line per shape.   python3 tools/q6p_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import koboldcpp_amd.lib as K  # noqa: E402

Q6_K_RS = 114


def main():
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(14336, 4096, 512), (4096, 1024, 512), (4096, 4096, 512), (4096, 28672, 512), (14336, 4096, 128)]
    if os.environ.get("Q6P_AB_SHAPES"):          # e.g. "0" or "0,3": a subset (PMC passes)
        shapes = [shapes[int(i)] for i in os.environ["Q6P_AB_SHAPES"].split(",")]
    for Kd, N, M in shapes:
        w = torch.empty(N * Kd // 256 * 210, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", Q6_K_RS, 7, 1, w.data_ptr(), Kd, N, s)
        img = torch.empty(int(K.raw().kcpp_q6p_image_bytes(Kd, N)), dtype=torch.uint8, device="cuda")
        K.call("kcpp_q6p_build", w.data_ptr(), Kd, N, img.data_ptr(), s)
        x = torch.randn(M, Kd, device="cuda")
        act = torch.empty(K.act_bytes(12, Kd, M), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", 15, x.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
        ws = torch.empty(int(K.raw().kcpp_gemm_workspace_bytes(Q6_K_RS, Kd, N, M)), dtype=torch.uint8, device="cuda")
        y = torch.empty(M, N, device="cuda")
        out = {"K": Kd, "N": N, "M": M}
        for name, fn in [("q6v3", lambda: K.call("kcpp_gemm", Q6_K_RS, w.data_ptr(), None, Kd, N, act.data_ptr(), M,
                                                    y.data_ptr(), N, None, N, 0, ws.data_ptr(), s)),
                         ("q6p", lambda: K.call("kcpp_gemm_q6p", img.data_ptr(), w.data_ptr(), None, None, Kd, N,
                                                   act.data_ptr(), M, y.data_ptr(), N, None, N, 0, ws.data_ptr(), s))]:
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / n
            out[name + "_us"] = round(us, 2)
            out[name + "_tflops"] = round(2.0 * M * N * Kd / us / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
