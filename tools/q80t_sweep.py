"""Sweep of the KT_Q8_0_T GEMM's split (S K ranges per tile, WV waves per workgroup) at BASELINE config 3's shapes
(Llama-3-8B, M = 32 and M = 1): HIP-event time per launch with 8 weight copies rotated past the Infinity Cache.
Each setting runs in its own process (KCPP_Q80T_SHAPE is read once).  Diagnostics only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"qkv": (4096, [4096, 1024, 1024]), "wo": (4096, [4096]), "down": (14336, [4096]), "gate_up": (4096, [14336])}

CHILD = r'''
import ctypes, json, os, sys
import numpy as np, torch
sys.path.insert(0, ROOT_)
import koboldcpp_amd.lib as K
name, Kd, Ns, M, mode = ARGS_
s = torch.cuda.current_stream().cuda_stream
N = sum(Ns)
wbytes = [K.row_bytes(K.Q8_0, Kd) * n for n in Ns]
copies = []
for c in range(8):
    ws = []
    for i, (n, b) in enumerate(zip(Ns, wbytes)):
        w = torch.empty(b, dtype=torch.uint8, device="cuda")
        K.call("kcpp_weight_synth", K.Q8_0_T, 5, 100 * c + i, w.data_ptr(), Kd, n, s)
        ws.append(w)
    if mode == 1:
        w2 = torch.empty(wbytes[0], dtype=torch.uint8, device="cuda")
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
for c in copies: launch(c)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 64
e0.record()
for i in range(it): launch(copies[i % 8])
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / it
b = sum(wbytes) * (2 if mode == 1 else 1)
print(json.dumps({"shape": name, "M": M, "us": round(us, 2), "GBps": round(b / us / 1e3, 1),
                  "ov": os.environ.get("KCPP_Q80T_GLU" if mode == 1 else "KCPP_Q80T_SHAPE")}))
'''

FULL = "--full" in sys.argv          # the (S, WV) grid at M = 32; default: the built-in choice at M = 32 and 1
for name, (Kd, Ns) in SHAPES.items():
    mode = 1 if name == "gate_up" else 0
    grid = [None]
    if FULL:
        grid = ["4", "8"] if mode == 1 else ["%d,%d" % (S, W) for S in (1, 2, 4, 8) for W in (2, 4, 8)]
    for M in ((32,) if FULL else (32, 1)):
        for ov in grid:
            env = dict(os.environ)
            if ov:
                env["KCPP_Q80T_GLU" if mode == 1 else "KCPP_Q80T_SHAPE"] = ov
            code = CHILD.replace("ROOT_", repr(ROOT)).replace("ARGS_", repr((name, Kd, Ns, M, mode)))
            r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
            print(r.stdout.strip().splitlines()[-1] if r.returncode == 0 else "FAIL %s %s %s" % (name, ov, r.stderr[-300:]),
                  flush=True)
