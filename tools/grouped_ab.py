"""Grouped expert GEMM A/B (tools only): kcpp_gemm_grouped at the Mixtral expert shapes, 8 experts with a ragged
~128-row routing (ubatch 512, top-2), per kernel variant (kcpp_gemm_set_variant); HIP-event timed.
usage: python tools/grouped_ab.py [variants...]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1:]] or [0]
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    cnt = [131, 97, 160, 118, 142, 125, 109, 142]
    NE, M = len(cnt), sum(cnt)
    for name, t, Kd, N, mode in [("down6", K.Q6_K_RS, 14336, 4096, 0), ("down5", K.Q5_K_RS, 14336, 4096, 0),
                                 ("glu5", K.Q5_K_RS, 4096, 14336, 1)]:
        rb = K.row_bytes(t, Kd) * N
        W = torch.empty(NE * rb, dtype=torch.uint8, device="cuda")
        W2 = torch.empty(NE * rb, dtype=torch.uint8, device="cuda")
        for e in range(NE):
            K.call("kcpp_weight_synth", t, 1, 40 + e, W.data_ptr() + e * rb, Kd, N, sp)
            K.call("kcpp_weight_synth", t, 1, 60 + e, W2.data_ptr() + e * rb, Kd, N, sp)
        X = torch.randn(M, Kd, device="cuda")
        act = torch.zeros(K.act_bytes(K.Q4_K, Kd, M), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", K.vec_dot_type(K.Q4_K), X.data_ptr(), Kd, act.data_ptr(), Kd, M, sp)
        cd = torch.tensor(cnt, dtype=torch.int32, device="cuda")
        ch = (ctypes.c_int32 * NE)(*cnt)
        Y = torch.empty(M, N, device="cuda")
        up = torch.empty(M, N, device="cuda")
        ws = torch.empty(max(1, int(K.raw().kcpp_gemm_grouped_ws_bytes(t, Kd, M, NE))), dtype=torch.uint8, device="cuda")
        y0 = None
        for v in variants:
            K.raw().kcpp_gemm_set_variant(v)
            run = lambda: K.call("kcpp_gemm_grouped", t, W.data_ptr(), W2.data_ptr() if mode else None, rb, Kd, N,
                                 act.data_ptr(), M, ch, cd.data_ptr(), NE, Y.data_ptr(), up.data_ptr() if mode else None,
                                 mode, ws.data_ptr(), sp)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 10
            e0.record(s)
            for _ in range(it):
                run()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / it * 1e3
            same = None if y0 is None else bool(torch.equal(Y, y0))
            if y0 is None:
                y0 = Y.clone()
            fl = 2.0 * M * N * Kd * (2 if mode else 1)
            print(json.dumps({"shape": name, "type": t, "M": M, "experts": NE, "variant": v, "us": round(us, 1),
                              "TFLOPs": round(fl / us / 1e6, 1), "bitwise_equal_first": same}), flush=True)
    K.raw().kcpp_gemm_set_variant(0)


if __name__ == "__main__":
    main()
