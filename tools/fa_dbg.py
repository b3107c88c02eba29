import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
import koboldcpp_amd.lib as K
T, n_past = int(sys.argv[1]), int(sys.argv[2])
H, HKV, D = 32, 8, 128
n_ctx = n_past + T + 64
rng = np.random.default_rng(T + 11 * n_past)
q = rng.standard_normal((T, H, D)).astype(np.float16)
kc = (rng.standard_normal((n_ctx, HKV, D)) * 0.5).astype(np.float16)
vc = rng.standard_normal((n_ctx, HKV, D)).astype(np.float16)
inf = len(sys.argv) > 3
if inf: vc[n_past + T:] = np.float16(np.inf)
q16, kd, vd = [torch.from_numpy(x.view(np.int16)).cuda() for x in (q, kc, vc)]
for v in (2, 3, 4):
    K.raw().kcpp_fa_prefill_set_variant(v)
    out = torch.full((T, H, D), float("nan"), dtype=torch.float32, device="cuda")
    K.call("kcpp_flash_attn_prefill_mfma", q16.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), T, H, HKV, D, n_past, float(1/np.sqrt(D)), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    bad = np.argwhere(~np.isfinite(o))
    print(v, "nonfinite", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:20], "heads", sorted(set(bad[:, 1].tolist()))[:40], "dims", sorted(set(bad[:, 2].tolist()))[:10])
