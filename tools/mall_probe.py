"""Infinity-Cache (MALL) prefetch probe (tools only): does streaming a decode kernel's weights through the
256 MiB Infinity Cache just before (or beside) the kernel shorten it?  HIP-event timed, graph-captured.
  cold      : GLU Q4_K mat-vec over weights rotated through > 600 MB (nothing resident)
  warm      : the same launch right after a prefetch kernel streamed exactly its weights (default policy)
  beside    : prefetch of the NEXT slot's weights on a second stream, concurrently with the mat-vec
usage: python tools/mall_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import stream_probe as SP  # noqa: E402


def main():
    import koboldcpp_amd.lib as K
    L = SP.lib()
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    sp0 = torch.cuda.current_stream().cuda_stream
    cases = [("glu", 12, 4096, 14336, 1, 1, 1), ("down_q4k", 12, 14336, 4096, 0, 2, 1), ("wo", 12, 4096, 4096, 0, 0, 1),
             ("qkv", 12, 4096, 6144, 0, 1, 2)]
    x = torch.randn(14336, device="cuda")
    nw = torch.ones(14336, device="cuda")
    y = torch.empty(2 * 14336, device="cuda")
    for name, t, Kd, N, mode, pro, rpw in cases:
        wb = K.row_bytes(t, Kd) * N
        nmat = 2 if mode == 1 else 1
        nslot = max(3, int(7e8 // (wb * nmat)) + 1)
        # one allocation per slot holding its gate|up back to back, so one prefetch covers a slot
        slots = [torch.empty(wb * nmat, dtype=torch.uint8, device="cuda") for _ in range(nslot)]
        for c, sl in enumerate(slots):
            for j in range(nmat):
                K.call("kcpp_weight_synth", t, 1, 100 + 2 * c + j, sl.data_ptr() + j * wb, Kd, N, sp0)
        act = torch.empty(K.act_bytes(t, Kd, 1), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", K.vec_dot_type(t), x.data_ptr(), Kd, act.data_ptr(), Kd, 1, sp0)
        args = []
        for sl in slots:
            d = K.DecArgs()
            d.K, d.x, d.nw, d.eps, d.act, d.nseg = Kd, x.data_ptr(), nw.data_ptr(), 1e-5, act.data_ptr(), 1
            d.W[0], d.N[0], d.Y[0] = sl.data_ptr(), N, y.data_ptr()
            if mode == 1:
                d.W2 = sl.data_ptr() + wb
            args.append(d)
        mv = lambda i, sp: K.gemv_dec(t, args[i % nslot], mode, pro, rpw, sp)
        pf = lambda i, sp, blocks=256: L.probe_stream(slots[i % nslot].data_ptr(), wb * nmat, blocks, 4, 0,
                                                       sink.data_ptr(), sp)
        cold = SP.timed(mv, 40)
        both = SP.timed(lambda i, sp: (pf(i, sp), mv(i, sp)), 40)
        pf_only = SP.timed(lambda i, sp: pf(i, sp), 40)
        # beside: prefetch slot i+1 on a forked stream while slot i's mat-vec runs; joined each step
        side = torch.cuda.Stream()
        evs = [(torch.cuda.Event(), torch.cuda.Event()) for _ in range(64)]

        def beside(i, sp):
            cur = torch.cuda.current_stream()
            e0, e1 = evs[i % 64]
            e0.record(cur)
            side.wait_event(e0)
            pf(i + 1, side.cuda_stream, 64)
            e1.record(side)
            mv(i, sp)
            cur.wait_event(e1)
        bes = SP.timed(beside, 40)
        rep = SP.timed(lambda i, sp: mv(i // 2, sp), 40)       # each slot twice in a row: cold, then warm
        r = {"case": name, "bytes": wb * nmat, "cold_us": round(cold, 2), "prefetch_us": round(pf_only, 2),
             "prefetch_then_mv_us": round(both, 2), "warm_mv_us_est": round(both - pf_only, 2),
             "mv_beside_next_prefetch_us": round(bes, 2), "warm_repeat_us": round(2 * rep - cold, 2)}
        print(json.dumps(r), flush=True)
        del slots, args
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
