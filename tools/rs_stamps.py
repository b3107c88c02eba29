"""Phase stamps of the RS decode mat-vecs inside one graph-replayed decode step (tools only).
Needs the instrumented build: make -C koboldcpp_amd/csrc stamps; run with
KCPP_LIB=koboldcpp_amd/koboldcpp_hipblas_stamps.so python tools/rs_stamps.py
Per kernel (grid, K, mode, prologue, rows): median over workgroups of each phase, microseconds after the
kernel's earliest workgroup entry: act = activation in registers, g0 = first group reduced, loop = streaming
done, st = results stored; 'span' = last workgroup done - first entry.  Kernels in launch order of layer 1."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402
import refharness as R  # noqa: E402

hp = dict(n_vocab=128256, n_embd=4096, n_head=32, n_head_kv=8, n_layer=32, n_ff=14336, n_ctx=4096, eps=1e-5,
          rope_base=500000.0)
m = K.Model(hp, R.q4_k_m_types(32))
m.synth(1234)
m.decode([1] * 512, 0, want_logits=False)
n = 3840
for _ in range(4):
    m.decode_greedy(n)
    n += 1
buf = torch.zeros(131072 * 16, dtype=torch.int64, device="cuda")
L = K.raw()
L.kcpp_rs_set_stamps.argtypes = [ctypes.c_void_p]
torch.cuda.synchronize()
assert L.kcpp_rs_set_stamps(buf.data_ptr()) == 0
m.decode_greedy(n)
torch.cuda.synchronize()
L.kcpp_rs_set_stamps(None)
a = buf.view(-1, 16).cpu().numpy().astype(np.int64)
a = a[a[:, 0] > 0]
# launches: consecutive slots with the same signature (every 8th workgroup records, in start order)
rows, i = [], 0
while i < len(a):
    n_rec = (int(a[i, 5] >> 32) + 7) // 8
    rows.append(a[i:i + n_rec])
    i += n_rec
t_first = min(int(b[:, 0].min()) for b in rows)
out = []
for b in rows:
    e0 = int(b[:, 0].min())
    dl = lambda c1, c0: round(float(np.median((b[:, c1] - b[:, c0]) / 100.0)), 2)
    sig = int(b[0, 6])
    out.append({"t0": round((e0 - t_first) / 100.0, 2), "grid": int(b[0, 5] >> 32), "K": sig & 0xFFFFFF,
                "mode": (sig >> 24) & 15, "pro": (sig >> 28) & 15, "rows": int(b[0, 7]),
                "entry_spread": round(float((b[:, 0].max() - e0) / 100.0), 2), "d_act": dl(1, 0), "d_g0": dl(2, 1),
                "d_loop": dl(3, 2), "d_st": dl(4, 3), "wg_total": dl(4, 0),
                "pro_x": dl(8, 0) if (b[:, 8] > 0).all() else None,
                "pro_red": dl(9, 8) if (b[:, 9] > 0).all() else None, "pro_sync": dl(10, 9) if (b[:, 10] > 0).all() else None,
                "pro_q": dl(11, 10) if (b[:, 10] > 0).all() else (dl(11, 8) if (b[:, 11] > 0).all() else None),
                "pro_sync2": dl(12, 11) if (b[:, 12] > 0).all() else None, "act_lds": dl(1, 12) if (b[:, 12] > 0).all() else None,
                "span": round(float((b[:, 4].max() - e0) / 100.0), 2)})
print(json.dumps({"launches": len(out)}))
for r in out[:16]:
    print(json.dumps(r))
m.close()
