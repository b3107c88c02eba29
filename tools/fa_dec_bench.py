"""Decode flash-attention A/B (tools only): kcpp_fa_decode_ex variants x KV layouts at Llama-3-8B shapes
(32 q heads, 8 kv heads, D 128), 32 layers' caches rotated so the Infinity Cache cannot serve them, each
variant captured in one graph of 32 calls (as the decode step replays them), HIP-event timed.
usage: python tools/fa_dec_bench.py [n_past ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import koboldcpp_amd.lib as K  # noqa: E402

H, HKV, D, L = 32, 8, 128, 32


def main():
    n_ctx = 4176
    npasts = [int(a) for a in sys.argv[1:]] or [3850, 1000, 16000]
    n_ctx = max(n_ctx, max(npasts) + 8)
    torch.manual_seed(0)
    # one big cache per layout; layer l = slice l
    kc = (torch.randn(L, n_ctx * HKV * D, device="cuda") * 0.5).half()
    vc = torch.randn(L, n_ctx * HKV * D, device="cuda").half()
    q = torch.randn(L, H * D, device="cuda").half()
    out = torch.zeros(L, H * D, device="cuda")
    qout = torch.zeros(L, K.act_bytes(K.Q4_K, H * D, 1), dtype=torch.uint8, device="cuda")
    wsb = K.fa_workspace_bytes(16, H, n_ctx)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    pos = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    layouts = {"pos_major": (HKV * D, D), "head_major": (D, n_ctx * D)}
    ref = {}
    for n_past in npasts:
        pos.fill_(n_past)
        for lname, (ld, hs) in layouts.items():
            for var in [int(v) for v in os.environ.get('FA_VARIANTS', '0,3').split(',')]:
                if var == 0 and n_past + 1 > 16384:
                    continue

                def step():
                    sp = torch.cuda.current_stream().cuda_stream     # the capture stream inside torch.cuda.graph
                    for l in range(L):
                        lc = 0 if os.environ.get("FA_RESIDENT") else l     # one layer's K/V re-read: Infinity-Cache resident
                        K.call("kcpp_fa_decode_ex", q[l].data_ptr(), kc[lc].data_ptr(), vc[lc].data_ptr(), ld, hs,
                               out[l].data_ptr(), None, ws.data_ptr(), H, HKV, 0, pos.data_ptr(),
                               n_ctx, 1.0 / D ** 0.5, var, sp)
                step()
                torch.cuda.synchronize()
                key = (n_past, lname)
                if key not in ref:
                    ref[key] = out.clone()
                err = float((out - ref[key]).abs().max())
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    step()
                for _ in range(3):
                    g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(10):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 10 / L * 1e3
                kvb = 2 * HKV * D * 2 * (n_past + 1)
                print(json.dumps({"n_past": n_past, "layout": lname, "variant": var, "us_per_layer": round(us, 2),
                                  "GBps": round(kvb / us / 1e3, 1), "maxdiff_vs_v0": err}), flush=True)


def stamps():
    """phase stamps (s_memrealtime, 100 MHz) for the last of 32 graph-replayed layers: per phase min / median /
    max over workgroups, microseconds after the earliest workgroup entry.  FA_STAMP_VARIANTS: kcpp_fa_decode_ex
    variants (3: k_fa_dec4 (workgroups < 2048) + k_fa_comb4 (2048+))"""
    n_ctx = 4176
    L2 = 32
    kc = (torch.randn(L2, n_ctx * HKV * D, device="cuda") * 0.5).half()
    vc = torch.randn(L2, n_ctx * HKV * D, device="cuda").half()
    q = torch.randn(L2, H * D, device="cuda").half()
    out = torch.zeros(L2, H * D, device="cuda")
    qout = torch.zeros(L2, K.act_bytes(K.Q4_K, H * D, 1), dtype=torch.uint8, device="cuda")
    ws = torch.zeros(K.fa_workspace_bytes(16, H, n_ctx), dtype=torch.uint8, device="cuda")
    pos = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    variants = [int(v) for v in os.environ.get("FA_STAMP_VARIANTS", "3").split(",")]
    for n_past in (100, 3850):
        pos.fill_(n_past)
        for var in variants:
            lo, hi = HKV * D, D

            def step():
                sp = torch.cuda.current_stream().cuda_stream
                for l in range(L2):
                    K.raw().kcpp_fa_set_stamps(st.data_ptr() if l == L2 - 1 else None)
                    K.call("kcpp_fa_decode_ex", q[l].data_ptr(), kc[l].data_ptr(), vc[l].data_ptr(), lo, hi,
                           out[l].data_ptr(), None, ws.data_ptr(), H, HKV, 0, pos.data_ptr(),
                           n_ctx, 1.0 / D ** 0.5, var, sp)
                K.raw().kcpp_fa_set_stamps(None)
            st.zero_()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            for _ in range(4):
                g.replay()
            torch.cuda.synchronize()
            a = st.view(-1, 8).cpu().numpy()
            t0 = a[a[:, 0] > 0][:, 0].min()
            for name, rows in (("dec", a[:2048]), ("comb", a[2048:])):
                rows = rows[rows[:, 0] > 0]
                if not len(rows):
                    continue
                res = {}
                for ph in range(8):
                    col = rows[:, ph]
                    col = col[col > 0]
                    if len(col):
                        d = (col - t0) / 100.0
                        res[ph] = [round(float(d.min()), 2), round(float(np.median(d)), 2), round(float(d.max()), 2), len(col)]
                print(json.dumps({"n_past": n_past, "variant": var, "kernel": name, "phases_us_min_med_max_n": res}), flush=True)


if __name__ == "__main__":
    if os.environ.get("FA_STAMPS"):
        stamps()
    else:
        main()
