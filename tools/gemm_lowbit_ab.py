"""Prefill GEMM A/B for the Q8_1-activation and code-book weight types (tools only): kcpp_gemm's MFMA GEMM (variant 0)
vs the column-group mat-vec (variant 20) and the unsplit GEMM (21) for Q4_1 / Q5_1 / IQ4_NL / IQ4_XS at several batch sizes, HIP-event timed over
weights rotated past the Infinity Cache; prints the max |difference| relative to the output scale.
usage: python tools/gemm_lowbit_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402


def main():
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    variants = [int(v) for v in os.environ.get("LOWBIT_VARIANTS", "0,20").split(",")]
    types = [int(v) for v in os.environ.get("LOWBIT_TYPES", "%d,%d,%d,%d" % (K.Q4_1, K.Q5_1, K.IQ4_NL, K.IQ4_XS)).split(",")]
    Ms = [int(v) for v in os.environ.get("LOWBIT_M", "16,37,64,128,512").split(",")]
    for t in types:
        for Kd, N in ((4096, 4096), (4096, 14336)):
            nrot = 3
            ws_ = [torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda") for _ in range(nrot)]
            for i, w in enumerate(ws_):
                K.call("kcpp_weight_synth", t, 1, 40 + i, w.data_ptr(), Kd, N, sp)
            for M in Ms:
                X = torch.randn(M, Kd, device="cuda")
                vt = K.vec_dot_type(t)
                act = torch.zeros(K.act_bytes(t, Kd, M), dtype=torch.uint8, device="cuda")
                K.call("kcpp_quantize_act", vt, X.data_ptr(), Kd, act.data_ptr(), Kd, M, sp)
                Y = torch.empty(M, N, device="cuda")
                ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
                res = {}
                for v in variants:
                    K.raw().kcpp_gemm_set_variant(v)
                    run = lambda i: K.call("kcpp_gemm", t, ws_[i % nrot].data_ptr(), None, Kd, N, act.data_ptr(), M,
                                           Y.data_ptr(), N, None, N, 0, ws.data_ptr(), sp)
                    for i in range(3):
                        run(i)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    it = 10
                    e0.record(s)
                    for i in range(it):
                        run(i)
                    e1.record(s)
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / it * 1e3
                    run(0)
                    torch.cuda.synchronize()
                    res[v] = (us, Y.clone())
                r0 = res[variants[0]][1]
                out = {"type": t, "K": Kd, "N": N, "M": M}
                for v in variants:
                    out["us_v%d" % v] = round(res[v][0], 1)
                    out["rel_diff_v%d" % v] = float((res[v][1] - r0).abs().max() / r0.abs().max().clamp_min(1.0))
                print(json.dumps(out), flush=True)
            K.raw().kcpp_gemm_set_variant(-1)


if __name__ == "__main__":
    main()
