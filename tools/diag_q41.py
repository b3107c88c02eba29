"""diagnosis: Q4_1 mat-mul at M = 64 vs the oracle, per token; Q8_1 activation s vs the oracle's"""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch
import refharness as R
import koboldcpp_amd.lib as K

T, Kd, N, M = R.Q4_1, 2048, 96, 64
rng = np.random.default_rng(M)
w = R.synth(T, 9, 1011, Kd, N)
X = rng.standard_normal((M, Kd)).astype(np.float32)
a = R.mul_mat(T, w, Kd, N, X)
s = torch.cuda.current_stream().cuda_stream
xd = torch.from_numpy(X).cuda()
act = torch.zeros(K.act_bytes(T, Kd, M), dtype=torch.uint8, device="cuda")
K.call("kcpp_quantize_act", K.vec_dot_type(T), xd.data_ptr(), Kd, act.data_ptr(), Kd, M, s)
torch.cuda.synchronize()
ab = act.cpu().numpy()
nb = Kd // 32
sg = ab[M * Kd + M * nb * 4 + M * nb * 2:].view(np.float32)[:M * nb].reshape(M, nb)
qg = ab[:M * Kd].view(np.int8).reshape(M, Kd)
for m in range(M):
    q = R.quantize(R.Q8_1, X[m]).reshape(nb, 36)
    so = q[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
    qo = q[:, 4:].view(np.int8).reshape(-1)
    bad_s = np.nonzero(so != sg[m])[0]
    bad_q = np.nonzero(qo != qg[m])[0]
    if len(bad_s) or len(bad_q):
        print("token", m, "s mismatches", bad_s[:5], so[bad_s[:3]], sg[m][bad_s[:3]], "q mismatches", bad_q[:5])
wd = torch.from_numpy(w).cuda()
dst = torch.empty_like(wd)
K.call("kcpp_weight_repack", T, wd.data_ptr(), dst.data_ptr(), Kd, N, 0, s)
Y = torch.empty((M, N), dtype=torch.float32, device="cuda")
ws = torch.empty(K.raw().kcpp_gemm_workspace_bytes(T, Kd, N, M), dtype=torch.uint8, device="cuda")
K.call("kcpp_gemm", T, dst.data_ptr(), None, Kd, N, act.data_ptr(), M, Y.data_ptr(), N, None, N, 0, ws.data_ptr(), s)
torch.cuda.synchronize()
d = np.abs(Y.cpu().numpy() - a).max(axis=1)
print("per-token max diff:", " ".join("%.1e" % v for v in d))
