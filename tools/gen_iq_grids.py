"""Generate koboldcpp_amd/csrc/iq_grids.h: the code books of the IQ1/IQ2/IQ3 weight formats.

The IQ2_XXS / IQ2_XS / IQ2_S / IQ3_XXS / IQ3_S / IQ1_S / IQ1_M blocks index fixed lattice code books (the reference
declares them in ggml-common.h).  They are part of the on-disk format, like a block layout, so this script recovers
them from the reference's BEHAVIOUR instead of from its text: it builds blocks that select every code-book entry
(unit scale, no sign flips) and runs the reference's own dequantize_row_iq* (oracle/_ref/libggml_ref.so, built by
`make -C oracle ref`), then reads the entries back from the dequantized floats.  The sign table is probed the same
way and checked against its closed form (7 sign bits + even parity).

Run in the build container (needs /root/reference for the library): python tools/gen_iq_grids.py
Test infrastructure for the generation step only; the product compiles the generated header.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
LIB = os.path.join(ROOT, "oracle", "_ref", "libggml_ref.so")
OUT = os.path.join(ROOT, "koboldcpp_amd", "csrc", "iq_grids.h")

ONE_F16 = 0x3C00


def deq(L, name, blocks, bsz):
    nb = len(blocks) // bsz
    y = np.zeros(nb * 256, np.float32)
    getattr(L, "dequantize_row_" + name)(blocks.ctypes.data_as(ctypes.c_void_p),
                                         y.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(nb * 256))
    return y.reshape(nb, 256)


def put16(b, off, v):
    b[off] = v & 0xFF
    b[off + 1] = (v >> 8) & 0xFF


def probe_iq2xxs(L):
    # block: d, qs[32] u16; sub-block ib: bytes 8ib..8ib+3 = 4 grid indices, 8ib+4..+7 = signs | scale << 28 (0)
    n = 256
    per = 32
    nb = n // per
    b = np.zeros(nb * 66, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        ib, l = divmod(k, 4)
        put16(b, blk * 66, ONE_F16)
        b[blk * 66 + 2 + 8 * ib + l] = i
    y = deq(L, "iq2_xxs", b, 66)                     # db = 0.125
    g = np.zeros((n, 8), np.int64)
    for i in range(n):
        blk, k = divmod(i, per)
        g[i] = np.rint(y[blk, 8 * k:8 * k + 8] * 8)
    return g


def probe_signs(L, g2xxs):
    # iq2_xxs, grid entry 0 everywhere, sign index s in sub-block lanes: negative positions = the sign byte
    n = 128
    per = 32
    nb = n // per
    b = np.zeros(nb * 66, np.uint8)
    for s in range(n):
        blk, k = divmod(s, per)
        ib, l = divmod(k, 4)
        put16(b, blk * 66, ONE_F16)
        o = blk * 66 + 2 + 8 * ib + 4
        w = int.from_bytes(bytes(b[o:o + 4]), "little") | (s << (7 * l))
        b[o:o + 4] = np.frombuffer(w.to_bytes(4, "little"), np.uint8)
    y = deq(L, "iq2_xxs", b, 66)
    signs = np.zeros(n, np.int64)
    for s in range(n):
        blk, k = divmod(s, per)
        v = y[blk, 8 * k:8 * k + 8]
        signs[s] = sum(1 << j for j in range(8) if v[j] < 0)
    return signs


def probe_iq2xs(L):
    n = 512
    per = 32
    nb = n // per
    b = np.zeros(nb * 74, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        put16(b, blk * 74, ONE_F16)
        put16(b, blk * 74 + 2 + 2 * k, i)            # 9-bit index, sign index 0
    y = deq(L, "iq2_xs", b, 74)                      # db = 0.125 (scales 0)
    return np.array([np.rint(y[i // per, 8 * (i % per):8 * (i % per) + 8] * 8) for i in range(n)], np.int64)


def probe_iq2s(L):
    n = 1024
    per = 32
    nb = n // per
    b = np.zeros(nb * 82, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        ib, l = divmod(k, 4)
        o = blk * 82
        put16(b, o, ONE_F16)
        b[o + 2 + k] = i & 0xFF                      # qs[4 ib + l]
        b[o + 2 + 64 + ib] |= ((i >> 8) & 3) << (2 * l)   # qh[ib]
    y = deq(L, "iq2_s", b, 82)
    return np.array([np.rint(y[i // per, 8 * (i % per):8 * (i % per) + 8] * 8) for i in range(n)], np.int64)


def probe_iq3xxs(L):
    # qs[64] = grid indices (4 values each), then 8 x u32 signs | scale << 28 (0): db = 0.25
    n = 256
    per = 64
    nb = n // per
    b = np.zeros(nb * 98, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        put16(b, blk * 98, ONE_F16)
        b[blk * 98 + 2 + k] = i
    y = deq(L, "iq3_xxs", b, 98)
    return np.array([np.rint(y[i // per, 4 * (i % per):4 * (i % per) + 4] * 4) for i in range(n)], np.int64)


def probe_iq3s(L):
    # qs[64] low 8 bits, qh[8] high bit per index, signs 0, scales 0: db = d (1 + 0) = 1
    n = 512
    per = 64
    nb = n // per
    b = np.zeros(nb * 110, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        o = blk * 110
        put16(b, o, ONE_F16)
        b[o + 2 + k] = i & 0xFF
        ib, t = divmod(k, 8)                         # qh[ib] bit t is the high bit of qs[8 ib + t]
        b[o + 2 + 64 + ib] |= ((i >> 8) & 1) << t
    y = deq(L, "iq3_s", b, 110)
    return np.array([np.rint(y[i // per, 4 * (i % per):4 * (i % per) + 4]) for i in range(n)], np.int64)


def probe_iq1s(L):
    # qs[32] low 8 bits, qh[8] u16: 3 high bits per index (l = 0..3), scale 0 (dl = d), delta + 1/8
    n = 2048
    per = 32
    nb = n // per
    b = np.zeros(nb * 50, np.uint8)
    for i in range(n):
        blk, k = divmod(i, per)
        ib, l = divmod(k, 4)
        o = blk * 50
        put16(b, o, ONE_F16)
        b[o + 2 + k] = i & 0xFF
        q = int(b[o + 34 + 2 * ib]) | (int(b[o + 35 + 2 * ib]) << 8)
        q |= ((i >> 8) & 7) << (3 * l)
        put16(b, o + 34 + 2 * ib, q)
    y = deq(L, "iq1_s", b, 50)
    return np.array([np.rint(y[i // per, 8 * (i % per):8 * (i % per) + 8] - 0.125) for i in range(n)], np.int64)


def main():
    if not os.path.exists(LIB):
        sys.exit("build the reference library first: make -C oracle ref")
    L = ctypes.CDLL(LIB)

    class InitParams(ctypes.Structure):           # struct ggml_init_params (ggml.h)
        _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", ctypes.c_void_p), ("no_alloc", ctypes.c_bool)]
    L.ggml_init.restype = ctypes.c_void_p
    ctx = L.ggml_init(InitParams(1 << 16, None, False))      # fills the f16 -> f32 table the dequantizers read
    g2xxs = probe_iq2xxs(L)
    signs = probe_signs(L, g2xxs)
    closed = np.array([s | ((bin(s).count("1") & 1) << 7) for s in range(128)])
    assert np.array_equal(signs, closed), "sign table: not the parity form"
    g2xs, g2s, g3xxs, g3s, g1s = probe_iq2xs(L), probe_iq2s(L), probe_iq3xxs(L), probe_iq3s(L), probe_iq1s(L)
    for g in (g2xxs, g2xs, g2s, g3xxs, g3s):
        assert g.min() > 0 and g.max() < 128
    assert set(np.unique(g1s)) <= {-1, 0, 1}

    def dwords_u8(g):            # rows of unsigned bytes -> little-endian dwords
        b = g.astype(np.uint8)
        return b.reshape(-1).view("<u4")

    def dwords_i8(g):
        b = g.astype(np.int8)
        return b.reshape(-1).view("<u4")

    tabs = [("kcpp_iq2xxs_grid", dwords_u8(g2xxs), "256 entries x 8 magnitudes (2 dwords each)"),
            ("kcpp_iq2xs_grid", dwords_u8(g2xs), "512 entries x 8 magnitudes"),
            ("kcpp_iq2s_grid", dwords_u8(g2s), "1024 entries x 8 magnitudes"),
            ("kcpp_iq3xxs_grid", dwords_u8(g3xxs), "256 entries x 4 magnitudes (1 dword each)"),
            ("kcpp_iq3s_grid", dwords_u8(g3s), "512 entries x 4 magnitudes"),
            ("kcpp_iq1s_grid", dwords_i8(g1s), "2048 entries x 8 values in {-1, 0, 1} (int8, 2 dwords each)")]
    with open(OUT, "w") as f:
        f.write("// iq_grids.h -- GENERATED by tools/gen_iq_grids.py (do not edit): the IQ1/IQ2/IQ3 lattice code books,\n")
        f.write("// recovered from the reference's own dequantize_row_iq* outputs (ggml-quants.c:3504-3739; the tables are\n")
        f.write("// declared in ggml-common.h).  Sign bytes are computed (kcpp_iq_signs: 7 bits + even parity).\n")
        f.write("// KCPP_IQ_TABLE decides the storage class: __constant__ in device code, static const on the host.\n")
        f.write("#pragma once\n#include <stdint.h>\n#ifndef KCPP_IQ_TABLE\n#define KCPP_IQ_TABLE(name, n) static const uint32_t name[n]\n#endif\n\n")
        for name, d, desc in tabs:
            f.write("// %s\nKCPP_IQ_TABLE(%s, %d) = {\n" % (desc, name, len(d)))
            for i in range(0, len(d), 8):
                f.write("    " + ", ".join("0x%08xu" % int(v) for v in d[i:i + 8]) + ",\n")
            f.write("};\n\n")
    L.ggml_free(ctypes.c_void_p(ctx))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
