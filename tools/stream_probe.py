"""Decode floor probe (tools only): HBM streaming-read time per launch at the decode mat-vec sizes,
the dependent-launch boundary, and the fused mat-vec kernels at the same sizes, all HIP-event
timed with inputs rotated through > 512 MB so nothing is Infinity-Cache resident.
usage: python tools/stream_probe.py [stream|dec|all]"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

SO = os.path.join(ROOT, "tools", "libstream_probe.so")


def lib():
    src = os.path.join(ROOT, "tools", "stream_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO, src])
    L = ctypes.CDLL(SO)
    P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.probe_stream.argtypes = [P, I64, I, I, I, P, P]
    L.probe_empty.argtypes = [I, P, P]
    L.probe_q4k.argtypes = [P, I, I, I, P, P]
    return L


def timed(fn, n, warm=4):
    """n launches captured into one graph (no host launch overhead), replayed and event-timed;
    fn(i, stream_ptr) launches one kernel"""
    sp0 = torch.cuda.current_stream().cuda_stream
    for i in range(warm):
        fn(i, sp0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sp = torch.cuda.current_stream().cuda_stream
        for i in range(n):
            fn(i, sp)
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3       # us per launch


def stream(L):
    pool = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    us = timed(lambda i, sp: L.probe_empty(1024, sink.data_ptr(), sp), 200)
    print(json.dumps({"probe": "empty-chain", "blocks": 1024, "us": round(us, 2)}))
    for size in (9437184, 33030144, 48168960, 66060288, 430940160):
        nslot = max(2, (1 << 30) // ((size + 4095) // 4096 * 4096))
        stride = (1 << 30) // nslot // 4096 * 4096
        best = None
        for blocks in (256, 512, 1024, 2048, 4096):
            for unroll in (2, 4, 8):
                for nt in (0, 1):
                    us = timed(lambda i, sp: L.probe_stream(pool.data_ptr() + (i % nslot) * stride, size, blocks, unroll, nt,
                                                         sink.data_ptr(), sp), 40 if size < 1e8 else 12)
                    r = {"probe": "stream", "bytes": size, "blocks": blocks, "unroll": unroll, "nt": nt,
                         "us": round(us, 2), "GBps": round(size / us / 1e3, 1)}
                    if best is None or us < best["us"]:
                        best = r
                    if os.environ.get("VERBOSE"):
                        print(json.dumps(r))
        print(json.dumps(dict(best, probe="stream-best")))


def q4k_pattern(L):
    pool = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    for nrows in (4096, 14336, 28672):
        size = nrows * 2304
        nslot = (1 << 30) // size
        for blocks in (256, 512, 1024, 2048):
            for unroll in (1, 2, 4, 8):
                us = timed(lambda i, sp: L.probe_q4k(pool.data_ptr() + (i % nslot) * size, nrows, blocks, unroll,
                                                     sink.data_ptr(), sp), 40)
                print(json.dumps({"probe": "q4k-pattern", "rows": nrows, "bytes": size, "blocks": blocks,
                                  "unroll": unroll, "us": round(us, 2), "GBps": round(size / us / 1e3, 1)}))


def dec():
    import koboldcpp_amd.lib as K
    sp = torch.cuda.current_stream().cuda_stream
    E, F = 4096, 14336
    cases = [  # name, type, K, N, mode, pro, rows_per_wave
        ("wo q4k pro0", 12, E, E, 0, 0, 1),
        ("qkv q4k pro1 rope", 12, E, E + 2048, 2, 1, 2),
        ("glu q4k pro1", 12, E, F, 1, 1, 1),
        ("down q4k pro2", 12, F, E, 0, 2, 1),
        ("down q6k pro2", 14, F, E, 0, 2, 1),
        ("down q4k pro0", 12, F, E, 0, 0, 1),
        ("down q6k pro0", 14, F, E, 0, 0, 1),
        ("head q6k pro1", 14, E, 128256, 0, 1, 4),
        ("glu q4k pro1 r2", 12, E, F, 1, 1, 2),
        ("glu q4k pro0", 12, E, F, 1, 0, 1),
        ("wo q4k pro0 r2", 12, E, E, 0, 0, 2),
        ("wo q4k pro0 r4", 12, E, E, 0, 0, 4),
        ("down q4k pro0 r2", 12, F, E, 0, 0, 2),
        ("rs wo q4k pro0", 112, E, E, 0, 0, 1),
        ("rs wo q4k pro2", 112, E, E, 0, 2, 1),
        ("rs qkv q4k pro1 rope", 112, E, E + 2048, 2, 1, 2),
        ("rs glu q4k pro1", 112, E, F, 1, 1, 1),
        ("rs down q4k pro2", 112, F, E, 0, 2, 1),
        ("rs down q6k pro2", 114, F, E, 0, 2, 1),
        ("rs v q6k pro1", 114, E, 1024, 0, 1, 1),
        ("rs head q6k pro1", 114, E, 128256, 0, 1, 1),
        ("rs glu q4k pro0", 112, E, F, 1, 0, 1),
        ("rs down q4k pro0", 112, F, E, 0, 0, 1),
        ("rs down q6k pro0", 114, F, E, 0, 0, 1),
        ("rs qkv q4k pro0 rope", 112, E, E + 2048, 2, 0, 2),
    ]
    if os.environ.get("PROBE_RS_ONLY"):
        cases = [c for c in cases if c[0].startswith("rs ")]
    x = torch.randn(F, device="cuda")
    nw = torch.ones(F, device="cuda")
    y = torch.empty(128256 * 2, device="cuda")
    q16 = torch.zeros(E, dtype=torch.int16, device="cuda")
    kc = torch.zeros(4096 * 1024, dtype=torch.int16, device="cuda")
    vc = torch.zeros(4096 * 1024, dtype=torch.int16, device="cuda")
    pos = torch.tensor([100], dtype=torch.int32, device="cuda")
    tab = torch.zeros(4096 * 64 * 2, device="cuda")
    only = os.environ.get("PROBE_CASE")
    for name, t, Kd, N, mode, pro, rpw in cases:
        if only and name != only:
            continue
        rb = K.row_bytes(t, Kd)
        wb = rb * N
        nmat = 2 if mode == 1 else 1
        ncopy = max(2, int(6e8 // (wb * nmat)) + 1)
        ws = []
        for c in range(ncopy):
            mats = [torch.empty(wb, dtype=torch.uint8, device="cuda") for _ in range(nmat)]
            for j, mt in enumerate(mats):
                K.call("kcpp_weight_synth", t, 1, 100 + 2 * c + j, mt.data_ptr(), Kd, N, sp)
            ws.append(mats)
        act = torch.empty(K.act_bytes(t, Kd, 1), dtype=torch.uint8, device="cuda")
        K.call("kcpp_quantize_act", K.vec_dot_type(t), x.data_ptr(), Kd, act.data_ptr(), Kd, 1, sp)
        args = []
        for mats in ws:
            d = K.DecArgs()
            d.K, d.x, d.nw, d.eps, d.act = Kd, x.data_ptr(), nw.data_ptr(), 1e-5, act.data_ptr()
            if mode == 2:
                d.nseg = 3
                for j, (n, role) in enumerate(((E, 0), (1024, 1), (1024, 2))):
                    d.W[j] = mats[0].data_ptr() + (0 if j == 0 else rb * (E + 1024 * (j - 1)))
                    d.N[j] = n
                    d.role[j] = role
                d.q16, d.kc, d.vc, d.ekv, d.D, d.pos, d.rope_tab = (q16.data_ptr(), kc.data_ptr(), vc.data_ptr(), 1024,
                                                                  128, pos.data_ptr(), tab.data_ptr())
            else:
                d.nseg, d.W[0], d.N[0], d.Y[0] = 1, mats[0].data_ptr(), N, y.data_ptr()
                if mode == 1:
                    d.W2 = mats[1].data_ptr()
            args.append(d)
        rc = K.gemv_dec(t, args[0], mode, pro, rpw, sp)
        if rc != 0:
            print(json.dumps({"probe": "dec", "case": name, "rc": rc}))
            continue
        us = timed(lambda i, sp: K.gemv_dec(t, args[i % len(args)], mode, pro, rpw, sp), 40)
        print(json.dumps({"probe": "dec", "case": name, "bytes": wb * nmat, "us": round(us, 2),
                          "GBps": round(wb * nmat / us / 1e3, 1)}))
        del ws, args
        torch.cuda.empty_cache()


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("stream", "all"):
        stream(lib())
    if what in ("pattern", "all"):
        q4k_pattern(lib())
    if what in ("dec", "all"):
        dec()
