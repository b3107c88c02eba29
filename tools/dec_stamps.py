"""Phase stamps of the fused q|k|v + attention launch (layer 5 of a decode token; probe build KCPP_FUSED_PROBE=5:
make -C koboldcpp_amd/csrc stamps PROBE_DEFS=-DKCPP_FUSED_PROBE=5 PROBE_DIR=build_probe5
STAMPS_OUT=../koboldcpp_hipblas_p5.so; run with KCPP_LIB=koboldcpp_amd/koboldcpp_hipblas_p5.so).
q|k|v workgroups: start, prologue done, streaming done, stores drained; attention splits: start, compute done,
wait done, partials drained (us from the launch's first stamp)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import koboldcpp_amd.lib as K  # noqa: E402
import refharness as R  # noqa: E402

hp = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=8, n_ff=14336, n_ctx=4096, eps=1e-5,
          rope_base=500000.0)
m = K.Model(hp, R.q4_k_m_types(8))
m.synth(1234)
m.decode([16 + (i % 2) for i in range(3840)], 0, want_logits=False)
buf = torch.zeros(8192 + 2048, dtype=torch.int64, device="cuda")
L = K.raw()
L.kcpp_dec_set_stamps.argtypes = [ctypes.c_void_p]
assert L.kcpp_dec_set_stamps(buf.data_ptr()) == 0
m.argmax()
n = 3840
for _ in range(6):
    m.decode_greedy(n)
    n += 1
torch.cuda.synchronize()
st = buf.cpu().numpy().astype(np.float64)
q = st[:4096].reshape(-1, 4)
q = q[q[:, 0] > 0]
a = st[4096:4096 + 4 * 256].reshape(-1, 4)
a = a[a[:, 0] > 0]
t0 = min(q[:, 0].min(), a[:, 0].min())
q = (q - t0) / 100.0
a = (a - t0) / 100.0   # s_memrealtime: 100 MHz
pc = lambda x: "p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))
print("q|k|v wgs %d  attention wgs %d" % (len(q), len(a)))
for i, nm in enumerate(["qkv start", "qkv prologue", "qkv stream done", "qkv stores drained"]):
    print("%-22s %s" % (nm, pc(q[:, i])))
for i, nm in enumerate(["att start", "att compute done", "att wait done", "att partials drained"]):
    print("%-22s %s" % (nm, pc(a[:, i])))
m.close()
