"""One KT_Q8_0_T GEMM shape of BASELINE config 3 (Llama-3-8B, M = 32 tokens), launched 64 times over 8 weight copies
(rotated past the 256 MiB Infinity Cache) for rocprofv3 --pmc passes; prints the HIP-event time per launch and the
algorithmic bytes (weights + activation + output).  usage: python3 tools/q80t_shapes.py qkv|wo|down|gate_up [M] [--warm]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import koboldcpp_amd.lib as K  # noqa: E402

SHAPES = {"qkv": (4096, [4096, 1024, 1024], 0), "wo": (4096, [4096], 0), "down": (14336, [4096], 0),
          "gate_up": (4096, [14336], 1)}
name = sys.argv[1]
M = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 32
NC = 1 if "--warm" in sys.argv else 8      # --warm: one weight copy, re-read from the Infinity Cache every launch
Kd, Ns, mode = SHAPES[name]
s = torch.cuda.current_stream().cuda_stream
N = sum(Ns)
wb = [K.row_bytes(K.Q8_0, Kd) * n for n in Ns]
copies = []
for c in range(NC):
    ws = []
    for i, (n, b) in enumerate(zip(Ns, wb)):
        w = torch.empty(b, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", K.Q8_0_T, 5, 100 * c + i, w.data_ptr(), Kd, n, s)
        ws.append(w)
    if mode == 1:
        w2 = torch.empty(wb[0], dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", K.Q8_0_T, 5, 100 * c + 9, w2.data_ptr(), Kd, Ns[0], s)
        ws.append(w2)
    copies.append(ws)
X = torch.randn(M, Kd, device="cuda")
act = torch.zeros(K.act_bytes(K.Q8_0_T, Kd, M), dtype=torch.uint8, device="cuda")
K.call("kcpp_quantize_act", K.Q8_0_TA, X.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
wsb = torch.zeros(int(K.raw().kcpp_gemm_workspace_bytes(K.Q8_0_T, Kd, N, M)), dtype=torch.uint8, device="cuda")
Y = torch.empty(M, N, device="cuda")
q = torch.empty(K.act_bytes(K.Q8_0_T, Ns[0], M), dtype=torch.uint8, device="cuda")


def launch(ws):
    segs = ws[:-1] if mode == 1 else ws
    wp = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in segs])
    npp = (ctypes.c_int64 * 3)(*Ns)
    K.call("kcpp_gemm_q80t", wp, npp, len(segs), ws[-1].data_ptr() if mode == 1 else None, Kd, act.data_ptr(), M,
           Y.data_ptr(), N, None, N, mode, q.data_ptr() if mode == 1 else None, wsb.data_ptr(), s)


for c in copies:
    launch(c)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 64
e0.record()
for i in range(it):
    launch(copies[i % NC])
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / it
wbytes = sum(wb) * (2 if mode == 1 else 1)
abytes = int(act.numel())
obytes = int(q.numel()) if mode == 1 else M * N * 4
print(json.dumps({"shape": name, "M": M, "copies": NC, "us": round(us, 2), "weight_bytes": wbytes, "act_bytes": abytes,
                  "out_bytes": obytes, "algo_bytes": wbytes + abytes + obytes,
                  "GBps": round((wbytes + abytes + obytes) / us / 1e3, 1)}))
