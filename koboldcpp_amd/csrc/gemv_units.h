// gemv_units.h -- per-type weight "units" (64 or 32 elements, 16-B aligned slices of a block),
// activation units and their exact integer dot products (CPU vec_dot semantics,
// ggml-quants.c:3922,5519,7714,8282,8919).  Shared by the mat-vec kernels.
#pragma once
#include "kcpp_common.h"
#include "iq_grid.h"

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
// streamed-once weight loads: nontemporal (MI355X_MICROARCH.md "nt-weights")
__device__ __forceinline__ uint4 ld_nt(const void *p) {
    const v4u v = __builtin_nontemporal_load((const v4u *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int TYPE> struct Unit;

// ---- Q4_K: unit = (super-block sb, 64-elem chunk j): 32 B of nibbles + 16 B header
template <> struct Unit<KT_Q4_K> {
    static constexpr int ELEMS = 64;
    uint4 hdr, q0, q1;
    __device__ __forceinline__ void load(const uint8_t *row, int64_t nblk_total, int u) {
        const uint8_t *blk = row + (int64_t)(u >> 2) * 144;
        const int j = u & 3;
        hdr = ld_nt((const void *)blk);
        q0 = ld_nt((const void *)(blk + 16 + 32 * j));
        q1 = ld_nt((const void *)(blk + 32 + 32 * j));
    }
};
// ---- Q5_K: like Q4_K plus 32 B of high bits per super-block
template <> struct Unit<KT_Q5_K> {
    static constexpr int ELEMS = 64;
    uint4 hdr, q0, q1, h0, h1;
    __device__ __forceinline__ void load(const uint8_t *row, int64_t, int u) {
        const uint8_t *blk = row + (int64_t)(u >> 2) * 176;
        const int j = u & 3;
        hdr = ld_nt((const void *)blk);
        h0 = *(const uint4 *)(blk + 16);
        h1 = *(const uint4 *)(blk + 32);
        q0 = ld_nt((const void *)(blk + 48 + 32 * j));
        q1 = ld_nt((const void *)(blk + 64 + 32 * j));
    }
};
// ---- Q6_K (SoA): unit = (sb, half h, l-quarter lq): ql 2x16 B, qh 16 B, 16 B scales, d
template <> struct Unit<KT_Q6_K> {
    static constexpr int ELEMS = 64;
    uint4 qa, qb, qh, sc;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + (u >> 2);
        const int h = (u >> 1) & 1, lq = u & 1;
        const uint8_t *q = base + b * 192;
        qa = ld_nt((const void *)(q + 64 * h + 16 * lq));
        qb = ld_nt((const void *)(q + 64 * h + 32 + 16 * lq));
        qh = ld_nt((const void *)(q + 128 + 32 * h + 16 * lq));
        sc = *(const uint4 *)(base + nb * 192 + b * 16);
        d = *(const uint16_t *)(base + nb * 208 + b * 2);
    }
};
// ---- Q3_K (SoA planes, quant.hip kl_store_block): unit u = quarter qq = u & 3 of super-block u >> 2, i.e. the 64
// elements of half n = qq >> 1, shifts j0 = 2 (qq & 1) and j0 + 1 (dequantize_row_q3_K, ggml-quants.c:2328):
// qs bytes 32n..32n+31, all 32 hmask bytes (bits 4n + j), the scale word qq (scales 4qq..4qq+3), d
template <> struct Unit<KT_Q3_K> {
    static constexpr int ELEMS = 64;
    uint4 q0, q1, h0, h1;
    uint32_t s0, s1, s2;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + (u >> 2);
        const int n = (u >> 1) & 1;
        const uint8_t *q = base + nb * 32 + b * 64 + 32 * n;
        q0 = ld_nt((const void *)q);
        q1 = ld_nt((const void *)(q + 16));
        h0 = *(const uint4 *)(base + b * 32);
        h1 = *(const uint4 *)(base + b * 32 + 16);
        const uint32_t *sc = (const uint32_t *)(base + nb * 96 + b * 12);
        s0 = sc[0]; s1 = sc[1]; s2 = sc[2];
        d = *(const uint16_t *)(base + nb * 108 + b * 2);
    }
};
// ---- Q2_K (SoA planes, quant.hip kl_store_block): unit u = quarter qq = u & 3 of super-block u >> 2 (half
// n = qq >> 1, shifts j0 = 2 (qq & 1), j0 + 1, as Q3_K): qs bytes 32n..32n+31, scale dword qq (scales 4qq..4qq+3:
// low nibble scale, high nibble min), (d, dmin)
template <> struct Unit<KT_Q2_K> {
    static constexpr int ELEMS = 64;
    uint4 q0, q1;
    uint32_t sc, dd;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + (u >> 2);
        const int qq = u & 3;
        const uint8_t *q = base + nb * 16 + b * 64 + 32 * (qq >> 1);
        q0 = ld_nt((const void *)q);
        q1 = ld_nt((const void *)(q + 16));
        sc = *(const uint32_t *)(base + b * 16 + 4 * qq);
        dd = *(const uint32_t *)(base + nb * 80 + b * 4);
    }
};
// ---- Q4_0 (SoA): unit = one 32-elem block: 16 B nibbles + fp16 d
template <> struct Unit<KT_Q4_0> {
    static constexpr int ELEMS = 32;
    uint4 q;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q = ld_nt((const void *)(base + b * 16));
        d = *(const uint16_t *)(base + nb * 16 + b * 2);
    }
};
// ---- Q5_0 (SoA): unit = one 32-elem block: 16 B nibbles + 4 B high bits + fp16 d
template <> struct Unit<KT_Q5_0> {
    static constexpr int ELEMS = 32;
    uint4 q;
    uint32_t h;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q = ld_nt((const void *)(base + b * 16));
        h = *(const uint32_t *)(base + nb * 16 + b * 4);
        d = *(const uint16_t *)(base + nb * 20 + b * 2);
    }
};
// ---- Q4_1 / Q5_1 (SoA): unit = one 32-elem block: 16 B nibbles (+ 4 B high bits) + fp16 (d, m)
template <> struct Unit<KT_Q4_1> {
    static constexpr int ELEMS = 32;
    uint4 q;
    uint32_t dm;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q = ld_nt((const void *)(base + b * 16));
        dm = *(const uint32_t *)(base + nb * 16 + b * 4);
    }
};
template <> struct Unit<KT_Q5_1> {
    static constexpr int ELEMS = 32;
    uint4 q;
    uint32_t h, dm;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q = ld_nt((const void *)(base + b * 16));
        h = *(const uint32_t *)(base + nb * 16 + b * 4);
        dm = *(const uint32_t *)(base + nb * 20 + b * 4);
    }
};
// ---- IQ4_NL (SoA as Q4_0): unit = one 32-elem block: 16 B of code-book indices + fp16 d
template <> struct Unit<KT_IQ4_NL> {
    static constexpr int ELEMS = 32;
    uint4 q;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q = ld_nt((const void *)(base + b * 16));
        d = *(const uint16_t *)(base + nb * 16 + b * 2);
    }
};
// ---- IQ4_XS (SoA: qs [nb][128] ++ (d, scales_h, scales_l[4]) [nb][8]): unit u = sub-blocks 2j, 2j+1 (j = u & 3)
// of super-block u >> 2: qs bytes 32j .. 32j+31 and the 8-byte header
template <> struct Unit<KT_IQ4_XS> {
    static constexpr int ELEMS = 64;
    uint4 q0, q1;
    uint2 h;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + (u >> 2);
        const uint8_t *q = base + b * 128 + 32 * (u & 3);
        q0 = ld_nt((const void *)q);
        q1 = ld_nt((const void *)(q + 16));
        h = *(const uint2 *)(base + nb * 128 + b * 8);
    }
};
// ---- Q8_0 (SoA): unit = one 32-elem block: 32 B int8 + fp16 d
template <> struct Unit<KT_Q8_0> {
    static constexpr int ELEMS = 32;
    uint4 q0, q1;
    uint16_t d;
    __device__ __forceinline__ void load(const uint8_t *base, int64_t nb, int64_t b0, int u) {
        const int64_t b = b0 + u;
        q0 = ld_nt((const void *)(base + b * 32));
        q1 = ld_nt((const void *)(base + b * 32 + 16));
        d = *(const uint16_t *)(base + nb * 32 + b * 2);
    }
};

// ---- the grid types (iq_grid.h, ggml layout): unit u = sub-blocks 2j, 2j+1 (j = u & 3) of super-block u >> 2,
// decoded at load into signed int8 codes and integer group scales
template <int T> struct UnitIQ {
    static constexpr int ELEMS = 64;
    IqSub s[2];
    float dw;                                  // d_w * C
    __device__ __forceinline__ void load(const uint8_t *row, int64_t, int u) {
        const uint8_t *blk = row + (int64_t)(u >> 2) * ks_block_bytes(T);
        const int j = u & 3;
        iq_sub<T>(blk, 2 * j, s[0]);
        iq_sub<T>(blk, 2 * j + 1, s[1]);
        dw = iq_d<T>(blk) * iq_const<T>();     // (times a power of two: exact)
    }
};
#define KCPP_IQ_UNIT(T) template <> struct Unit<T> : UnitIQ<T> {};
KCPP_IQ_CASES(KCPP_IQ_UNIT)
#undef KCPP_IQ_UNIT

__device__ __forceinline__ int byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xFF; }
__device__ __forceinline__ uint32_t u4(const uint4 &v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w)); }

// scale/min of sub-block `is` from the 12 packed bytes (get_scale_min_k4, ggml-quants.c:1899)
__device__ __forceinline__ void k4_scale_min(const uint4 &hdr, int is, int &sc, int &m) {
    // bytes s[0..11] live in hdr.y (0-3), hdr.z (4-7), hdr.w (8-11)
    auto s = [&](int k) -> int { return k < 4 ? byte_of(hdr.y, k) : (k < 8 ? byte_of(hdr.z, k - 4) : byte_of(hdr.w, k - 8)); };
    if (is < 4) { sc = s(is) & 63; m = s(is + 4) & 63; }
    else {
        sc = (s(is + 4) & 0xF) | ((s(is - 4) >> 6) << 4);
        m = (s(is + 4) >> 4) | ((s(is) >> 6) << 4);
    }
}

// Activation unit for K-quants: 64 int8 + d + 4 bsums (sub-groups of 16)
struct ActK {
    int4 a[4];
    float d;
    int bs[4];
};
__device__ __forceinline__ void load_actk(const ActView &av, int u, ActK &x) {
    const int64_t e0 = (int64_t)u * 64;
    const int4 *p = (const int4 *)(av.qs + e0);
    x.a[0] = p[0]; x.a[1] = p[1]; x.a[2] = p[2]; x.a[3] = p[3];
    x.d = av.d[e0 >> 8];
    const int2 b = *(const int2 *)(av.bs + (e0 >> 4));
    x.bs[0] = (int16_t)(b.x & 0xFFFF); x.bs[1] = (int16_t)(b.x >> 16);
    x.bs[2] = (int16_t)(b.y & 0xFFFF); x.bs[3] = (int16_t)(b.y >> 16);
}
__device__ __forceinline__ int ai(const ActK &x, int i) {   // dword i (0..15) of the 64 int8
    const int4 &v = x.a[i >> 2];
    const int k = i & 3;
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}
// Activation unit for Q8_0-type: 32 int8 + d + asum
struct Act0 {
    int4 a[2];
    float d;
    int s;
};
__device__ __forceinline__ void load_act0(const ActView &av, int u, Act0 &x) {
    const int4 *p = (const int4 *)(av.qs + (int64_t)u * 32);
    x.a[0] = p[0]; x.a[1] = p[1];
    x.d = av.d[u];
    x.s = av.bs[u];
}

// Activation unit for Q8_1 (Q4_1 / Q5_1 weights): the Q8_0 unit plus block_q8_1.s
struct Act1 : Act0 {
    float sf;
};
__device__ __forceinline__ void load_act(const ActView &av, int u, Act1 &x) {
    load_act0(av, u, x);
    x.sf = av.s[u];
}

template <int TYPE> struct ActOf { typedef ActK T; };
template <> struct ActOf<KT_Q4_1> { typedef Act1 T; };
template <> struct ActOf<KT_Q5_1> { typedef Act1 T; };
template <> struct ActOf<KT_Q4_0> { typedef Act0 T; };
template <> struct ActOf<KT_Q5_0> { typedef Act0 T; };
template <> struct ActOf<KT_Q8_0> { typedef Act0 T; };
template <> struct ActOf<KT_IQ4_NL> { typedef Act0 T; };

__device__ __forceinline__ void load_act(const ActView &av, int u, ActK &x) { load_actk(av, u, x); }
__device__ __forceinline__ void load_act(const ActView &av, int u, Act0 &x) { load_act0(av, u, x); }

// ---------------------------------------------------------------- per-unit dot products
__device__ __forceinline__ float unit_dot(const Unit<KT_Q4_K> &w, int u, const ActK &x) {
    const int j = u & 3;
    int sc0, m0, sc1, m1;
    k4_scale_min(w.hdr, 2 * j, sc0, m0);
    k4_scale_min(w.hdr, 2 * j + 1, sc1, m1);
    int dlo = 0, dhi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t q = i < 4 ? u4(w.q0, i) : u4(w.q1, i - 4);
        dlo = sdot4((int)(q & 0x0F0F0F0Fu), ai(x, i), dlo);
        dhi = sdot4((int)((q >> 4) & 0x0F0F0F0Fu), ai(x, 8 + i), dhi);
    }
    const int sumi = sc0 * dlo + sc1 * dhi;
    const int summ = m0 * (x.bs[0] + x.bs[1]) + m1 * (x.bs[2] + x.bs[3]);
    const float d = __fmul_rn(x.d, h2f((uint16_t)(w.hdr.x & 0xFFFF)));
    const float dmin = __fmul_rn(x.d, h2f((uint16_t)(w.hdr.x >> 16)));
    return __fsub_rn(__fmul_rn(d, (float)sumi), __fmul_rn(dmin, (float)summ));
}

__device__ __forceinline__ float unit_dot(const Unit<KT_Q5_K> &w, int u, const ActK &x) {
    const int j = u & 3;
    int sc0, m0, sc1, m1;
    k4_scale_min(w.hdr, 2 * j, sc0, m0);
    k4_scale_min(w.hdr, 2 * j + 1, sc1, m1);
    int dlo = 0, dhi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t q = i < 4 ? u4(w.q0, i) : u4(w.q1, i - 4);
        const uint32_t h = i < 4 ? u4(w.h0, i) : u4(w.h1, i - 4);
        const uint32_t lo = (q & 0x0F0F0F0Fu) | (((h >> (2 * j)) & 0x01010101u) << 4);
        const uint32_t hi = ((q >> 4) & 0x0F0F0F0Fu) | (((h >> (2 * j + 1)) & 0x01010101u) << 4);
        dlo = sdot4((int)lo, ai(x, i), dlo);
        dhi = sdot4((int)hi, ai(x, 8 + i), dhi);
    }
    const int sumi = sc0 * dlo + sc1 * dhi;
    const int summ = m0 * (x.bs[0] + x.bs[1]) + m1 * (x.bs[2] + x.bs[3]);
    const float d = __fmul_rn(x.d, h2f((uint16_t)(w.hdr.x & 0xFFFF)));
    const float dmin = __fmul_rn(x.d, h2f((uint16_t)(w.hdr.x >> 16)));
    return __fsub_rn(__fmul_rn(d, (float)sumi), __fmul_rn(dmin, (float)summ));
}

// Q6_K activation unit is not contiguous: 4 planes of 16 elements at stride 32
struct Act6 {
    int4 a[4];
    float d;
    int bs[4];
};
__device__ __forceinline__ void load_act6(const ActView &av, int u, Act6 &x) {
    const int64_t sb = u >> 2;
    const int h = (u >> 1) & 1, lq = u & 1;
    const int64_t e0 = sb * 256 + 128 * h + 16 * lq;
#pragma unroll
    for (int p = 0; p < 4; ++p) x.a[p] = *(const int4 *)(av.qs + e0 + 32 * p);
    x.d = av.d[sb];
#pragma unroll
    for (int p = 0; p < 4; ++p) x.bs[p] = av.bs[(e0 + 32 * p) >> 4];
}
template <> struct ActOf<KT_Q6_K> { typedef Act6 T; };
__device__ __forceinline__ void load_act(const ActView &av, int u, Act6 &x) { load_act6(av, u, x); }

__device__ __forceinline__ float unit_dot(const Unit<KT_Q6_K> &w, int u, const Act6 &x) {
    const int h = (u >> 1) & 1, lq = u & 1;
    int dp[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t la = u4(w.qa, i), lb = u4(w.qb, i), hh = u4(w.qh, i);
        const uint32_t p0 = (la & 0x0F0F0F0Fu) | ((hh << 4) & 0x30303030u);
        const uint32_t p1 = (lb & 0x0F0F0F0Fu) | ((hh << 2) & 0x30303030u);
        const uint32_t p2 = ((la >> 4) & 0x0F0F0F0Fu) | (hh & 0x30303030u);
        const uint32_t p3 = ((lb >> 4) & 0x0F0F0F0Fu) | ((hh >> 2) & 0x30303030u);
        dp[0] = sdot4((int)p0, u4(*(const uint4 *)&x.a[0], i), dp[0]);
        dp[1] = sdot4((int)p1, u4(*(const uint4 *)&x.a[1], i), dp[1]);
        dp[2] = sdot4((int)p2, u4(*(const uint4 *)&x.a[2], i), dp[2]);
        dp[3] = sdot4((int)p3, u4(*(const uint4 *)&x.a[3], i), dp[3]);
    }
    // scales: is = lq + 2p + 8h  (dequantize_row_q6_K: sc[is + 0/2/4/6], ggml-quants.c:2997)
    int sumi = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int is = lq + 2 * p + 8 * h;
        const int s = (int8_t)byte_of(u4(w.sc, is >> 2), is & 3);
        sumi += s * (dp[p] - 32 * x.bs[p]);
    }
    return __fmul_rn(__fmul_rn(h2f(w.d), x.d), (float)sumi);
}

// Q3_K: v = low 2 bits | hmask bit << 2 (0..7) is the weight + 4, so each 16-group's dot is sum(v a) - 4 bsum;
// scale word qq of the unpacked 16 (aux shuffle, ggml-quants.c:2346-2351) holds this unit's 4 scales
__device__ __forceinline__ float unit_dot(const Unit<KT_Q3_K> &w, int u, const ActK &x) {
    const int qq = u & 3, n = qq >> 1, j0 = 2 * (qq & 1);
    const uint32_t k1 = 0x03030303u, k2 = 0x0f0f0f0fu;
    const uint32_t sw = qq == 0 ? (w.s0 & k2) | ((w.s2 & k1) << 4)
                      : qq == 1 ? (w.s1 & k2) | (((w.s2 >> 2) & k1) << 4)
                      : qq == 2 ? ((w.s0 >> 4) & k2) | (((w.s2 >> 4) & k1) << 4)
                                : ((w.s1 >> 4) & k2) | (((w.s2 >> 6) & k1) << 4);
    int sumi = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int j = j0 + (g >> 1);
        int dot = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int wi = 4 * (g & 1) + t;                  // qs / hmask dword: l = 4 wi .. 4 wi + 3
            const uint32_t qd = wi < 4 ? u4(w.q0, wi) : u4(w.q1, wi - 4);
            const uint32_t hd = wi < 4 ? u4(w.h0, wi) : u4(w.h1, wi - 4);
            const uint32_t v = ((qd >> (2 * j)) & 0x03030303u) | (((hd >> (4 * n + j)) & 0x01010101u) << 2);
            dot = sdot4((int)v, ai(x, 4 * g + t), dot);
        }
        sumi += ((int)((sw >> (8 * g)) & 0xFF) - 32) * (dot - 4 * x.bs[g]);
    }
    return __fmul_rn(__fmul_rn(h2f(w.d), x.d), (float)sumi);
}

// Q2_K: d x.d sum_g (sc_g & 15) dot_g - dmin x.d sum_g (sc_g >> 4) bsum_g  (ggml_vec_dot_q2_K_q8_K)
__device__ __forceinline__ float unit_dot(const Unit<KT_Q2_K> &w, int u, const ActK &x) {
    const int j0 = 2 * (u & 1);
    int sumi = 0, summ = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int j = j0 + (g >> 1);
        int dot = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int wi = 4 * (g & 1) + t;
            const uint32_t qd = wi < 4 ? u4(w.q0, wi) : u4(w.q1, wi - 4);
            dot = sdot4((int)((qd >> (2 * j)) & 0x03030303u), ai(x, 4 * g + t), dot);
        }
        const int s = (w.sc >> (8 * g)) & 0xFF;
        sumi += (s & 0xF) * dot;
        summ += (s >> 4) * x.bs[g];
    }
    const float dall = __fmul_rn(x.d, h2f((uint16_t)(w.dd & 0xFFFF))), dmin = __fmul_rn(x.d, h2f((uint16_t)(w.dd >> 16)));
    return __fsub_rn(__fmul_rn(dall, (float)sumi), __fmul_rn(dmin, (float)summ));
}

__device__ __forceinline__ float unit_dot(const Unit<KT_Q4_0> &w, int, const Act0 &x) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t q = u4(w.q, i);
        s = sdot4((int)(q & 0x0F0F0F0Fu), u4(*(const uint4 *)&x.a[0], i), s);
        s = sdot4((int)((q >> 4) & 0x0F0F0F0Fu), u4(*(const uint4 *)&x.a[1], i), s);
    }
    s -= 8 * x.s;
    return __fmul_rn((float)s, __fmul_rn(h2f(w.d), x.d));
}

// 4 high bits (bits 0..3 of v) -> bit 4 of 4 bytes: the multiply places bit i at bit 8i + i, masked to bit 8i
__device__ __forceinline__ uint32_t hbits4(uint32_t v) { return (((v & 0xFu) * 0x00204081u) & 0x01010101u) << 4; }

// ggml_vec_dot_q5_0_q8_0 (ggml-quants.c:4790): x = (q | h << 4) - 16, so sum x a = sum (q | h << 4) a - 16 sum a
__device__ __forceinline__ float unit_dot(const Unit<KT_Q5_0> &w, int, const Act0 &x) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t q = u4(w.q, i);
        s = sdot4((int)((q & 0x0F0F0F0Fu) | hbits4(w.h >> (4 * i))), u4(*(const uint4 *)&x.a[0], i), s);
        s = sdot4((int)(((q >> 4) & 0x0F0F0F0Fu) | hbits4(w.h >> (16 + 4 * i))), u4(*(const uint4 *)&x.a[1], i), s);
    }
    s -= 16 * x.s;
    return __fmul_rn((float)s, __fmul_rn(h2f(w.d), x.d));
}

// ggml_vec_dot_q4_1_q8_1 / _q5_1_q8_1 (ggml-quants.c:4503,5145): (d_w d_a) sum x a + m_w s_a, x = q (| h << 4)
__device__ __forceinline__ float dot_q41(uint4 q, uint32_t h, uint32_t dm, const Act1 &x) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t v = u4(q, i);
        s = sdot4((int)((v & 0x0F0F0F0Fu) | hbits4(h >> (4 * i))), u4(*(const uint4 *)&x.a[0], i), s);
        s = sdot4((int)(((v >> 4) & 0x0F0F0F0Fu) | hbits4(h >> (16 + 4 * i))), u4(*(const uint4 *)&x.a[1], i), s);
    }
    return __fadd_rn(__fmul_rn(__fmul_rn(h2f((uint16_t)(dm & 0xFFFF)), x.d), (float)s), __fmul_rn(h2f((uint16_t)(dm >> 16)), x.sf));
}
__device__ __forceinline__ float unit_dot(const Unit<KT_Q4_1> &w, int, const Act1 &x) { return dot_q41(w.q, 0u, w.dm, x); }
__device__ __forceinline__ float unit_dot(const Unit<KT_Q5_1> &w, int, const Act1 &x) { return dot_q41(w.q, w.h, w.dm, x); }

// ggml_vec_dot_iq4_nl_q8_0 (ggml-quants.c:12470; scalar :12660): (d_a d_w) sum kvalues[q] a over the block
__device__ __forceinline__ float unit_dot(const Unit<KT_IQ4_NL> &w, int, const Act0 &x) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t q = u4(w.q, i);
        s = sdot4((int)iq4nl_lut4(q & 0x0F0F0F0Fu), u4(*(const uint4 *)&x.a[0], i), s);
        s = sdot4((int)iq4nl_lut4((q >> 4) & 0x0F0F0F0Fu), u4(*(const uint4 *)&x.a[1], i), s);
    }
    return __fmul_rn((float)s, __fmul_rn(x.d, h2f(w.d)));
}

// ggml_vec_dot_iq4_xs_q8_K (ggml-quants.c:12672; AVX2 :12728): per 32-sub-block integer dot times (ls - 32), summed in
// int32, then (d_w d_a) once -- the AVX2 branch's order
__device__ __forceinline__ float unit_dot(const Unit<KT_IQ4_XS> &w, int u, const ActK &x) {
    const int j = u & 3;
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t qa = u4(w.q0, i), qb = u4(w.q1, i);
        s0 = sdot4((int)iq4nl_lut4(qa & 0x0F0F0F0Fu), ai(x, i), s0);
        s0 = sdot4((int)iq4nl_lut4((qa >> 4) & 0x0F0F0F0Fu), ai(x, 4 + i), s0);
        s1 = sdot4((int)iq4nl_lut4(qb & 0x0F0F0F0Fu), ai(x, 8 + i), s1);
        s1 = sdot4((int)iq4nl_lut4((qb >> 4) & 0x0F0F0F0Fu), ai(x, 12 + i), s1);
    }
    const uint32_t sh = w.h.x >> 16, sl = w.h.y;
    const int ib0 = 2 * j, ib1 = 2 * j + 1;
    const int ls0 = (int)(((sl >> (8 * (ib0 / 2))) & 0xF) | (((sh >> (2 * ib0)) & 3) << 4)) - 32;
    const int ls1 = (int)(((sl >> (8 * (ib1 / 2) + 4)) & 0xF) | (((sh >> (2 * ib1)) & 3) << 4)) - 32;
    return __fmul_rn(__fmul_rn(h2f((uint16_t)(w.h.x & 0xFFFF)), x.d), (float)(ls0 * s0 + ls1 * s1));
}

__device__ __forceinline__ float unit_dot(const Unit<KT_Q8_0> &w, int, const Act0 &x) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s = sdot4((int)u4(w.q0, i), u4(*(const uint4 *)&x.a[0], i), s);
        s = sdot4((int)u4(w.q1, i), u4(*(const uint4 *)&x.a[1], i), s);
    }
    return __fmul_rn((float)s, __fmul_rn(h2f(w.d), x.d));
}

// the grid types against Q8_K (ggml_vec_dot_iq*_q8_K generic branches, ggml-quants.c:9606-12468): per group of 8 the
// integer dot of codes and activation bytes, times the group's integer scale, summed in int32 over the unit, then
// (d_w C) d_a once
template <int T>
__device__ __forceinline__ float iq_unit_dot(const UnitIQ<T> &w, const ActK &x) {
    int tot = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            int p = sdot4((int)w.s[h].v[2 * l], ai(x, 8 * h + 2 * l), 0);
            p = sdot4((int)w.s[h].v[2 * l + 1], ai(x, 8 * h + 2 * l + 1), p);
            tot += w.s[h].ls[l] * p;
        }
    return __fmul_rn(__fmul_rn(w.dw, x.d), (float)tot);
}
#define KCPP_IQ_DOT(T) \
    __device__ __forceinline__ float unit_dot(const Unit<T> &w, int, const ActK &x) { return iq_unit_dot<T>(w, x); }
KCPP_IQ_CASES(KCPP_IQ_DOT)
#undef KCPP_IQ_DOT

// uniform unit loader: native-layout types index by row pointer, SoA types by block index
template <int TYPE>
__device__ __forceinline__ void load_unit(Unit<TYPE> &w, const uint8_t *W, int64_t nb, int64_t row, int64_t units_per_row, int u) {
    if constexpr (TYPE == KT_Q4_K) w.load(W + row * (units_per_row / 4) * 144, nb, u);
    else if constexpr (TYPE == KT_Q5_K) w.load(W + row * (units_per_row / 4) * 176, nb, u);
    else if constexpr (kIqGrid<TYPE>) w.load(W + row * (units_per_row / 4) * ks_block_bytes(TYPE), nb, u);
    else if constexpr (TYPE == KT_Q6_K || TYPE == KT_Q3_K || TYPE == KT_Q2_K || TYPE == KT_IQ4_XS)
        w.load(W, nb, row * (units_per_row / 4), u);
    else w.load(W, nb, row * units_per_row, u);
}

