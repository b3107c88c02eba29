"""Prefill GEMM A/B (tools only): kcpp_gemm Q4_K_RS / Q6_K_RS at the Llama-3-8B ubatch-512 shapes and Q5_K at the
Mixtral expert shapes (GEMM_M tokens, GEMM_ONLY one shape): kernel variants (kcpp_gemm_set_variant, default 2 vs 3),
HIP-event timed over weights rotated past the Infinity Cache.
usage: python tools/gemm_ab.py [variants...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1:]] or [2, 3]
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    M = int(os.environ.get("GEMM_M", "512"))
    for name, t, Kd, N, mode in [("gate|up", K.Q4_K_RS, 4096, 28672, 0), ("qkv", K.Q4_K_RS, 4096, 6144, 0),
                                 ("wo", K.Q4_K_RS, 4096, 4096, 0), ("down", K.Q4_K_RS, 14336, 4096, 0),
                                 ("glu2", K.Q4_K_RS, 4096, 14336, 1), ("down6", K.Q6_K_RS, 14336, 4096, 0),
                                 ("v6", K.Q6_K_RS, 4096, 1024, 0), ("glu5", K.Q5_K, 4096, 14336, 1),
                                 ("down5", K.Q5_K, 14336, 4096, 0), ("glu5rs", K.Q5_K_RS, 4096, 14336, 1),
                                 ("wo5", K.Q5_K, 4096, 4096, 0), ("gu5", K.Q5_K_RS, 4096, 28672, 0),
                                 ("qkv5", K.Q5_K_RS, 4096, 6144, 0)]:
        if os.environ.get("GEMM_ONLY") and name != os.environ["GEMM_ONLY"]:
            continue
        nrot = 3
        ws_ = [torch.empty(K.row_bytes(t, Kd) * N, dtype=torch.uint8, device="cuda") for _ in range(nrot)]
        for i, w in enumerate(ws_):
            K.call("kcpp_weight_synth", t, 1, 40 + i, w.data_ptr(), Kd, N, sp)
        X = torch.randn(M, Kd, device="cuda")
        act = torch.zeros(K.act_bytes(12, Kd, M), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", K.vec_dot_type(12), X.data_ptr(), Kd, act.data_ptr(), Kd, M, sp)
        Y = torch.empty(M, N, device="cuda")
        ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(t, Kd, N, M), dtype=torch.uint8, device="cuda")
        y0 = None
        for v in variants:
            K.raw().kcpp_gemm_set_variant(v)
            run = lambda i: K.call("kcpp_gemm", t, ws_[i % nrot].data_ptr(), ws_[(i + 1) % nrot].data_ptr() if mode else None,
                                   Kd, N, act.data_ptr(), M, Y.data_ptr(), N, None, N, mode, ws.data_ptr(), sp)
            for i in range(3):
                run(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            it = 12
            e0.record(s)
            for i in range(it):
                run(i)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / it * 1e3
            run(0)
            torch.cuda.synchronize()
            same = None
            if y0 is None:
                y0 = Y.clone()
                if os.environ.get("GEMM_DUMP"):      # the first variant's output, for a cross-build bitwise check
                    os.makedirs(os.environ["GEMM_DUMP"], exist_ok=True)
                    Y.cpu().numpy().tofile(os.path.join(os.environ["GEMM_DUMP"], name.replace("|", "_") + ".f32"))
            else:
                same = bool(torch.equal(Y, y0))
            fl = 2.0 * M * N * Kd * (2 if mode else 1)
            print(json.dumps({"shape": name, "type": t, "M": M, "K": Kd, "N": N, "variant": v, "us": round(us, 1),
                              "TFLOPs": round(fl / us / 1e6, 1), "bitwise_equal_first": same}), flush=True)
    K.raw().kcpp_gemm_set_variant(0)


if __name__ == "__main__":
    main()
