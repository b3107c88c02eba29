// gemv_rs.h -- the row-major decode layouts KT_Q4_K_RS / KT_Q6_K_RS as seen by one lane of a single-token mat-vec:
// piece loads, the lane's Q8_K activation slices and the exact integer dot (gemv_rs.hip documents the layouts).
// Used by the stand-alone RS kernels (gemv_rs.hip).
#pragma once
#include "gemv_lean.h"

namespace rs {

// ---------------------------------------------------------------- Q4_K_RS
// piece c = l + 64 i of the nibble plane: super-block sb = c >> 3, pair j = (c >> 1) & 3, half hh = c & 1:
// low nibbles = elements 64 j + 16 hh + 0..15 (sub-block 2j), high nibbles = the same + 32 (sub-block 2j+1)
struct Q4Sel {
    bool hi;
    int sh, offh, shm;
};
__device__ __forceinline__ Q4Sel q4_sel(int j) {
    Q4Sel s;
    s.hi = j >= 2;
    s.sh = 16 * (j & 1);
    s.offh = s.hi ? 6 : 4;
    s.shm = s.hi ? s.sh + 4 : s.sh;
    return s;
}
// get_scale_min_k4 (ggml-quants.c:1899) for sub-blocks 2j, 2j+1 from header dwords y, z, w (scales[12])
__device__ __forceinline__ void q4_scales(const uint4 &h, const Q4Sel &s, int &sc0, int &m0, int &sc1, int &m1) {
    const uint32_t lo_sc = s.hi ? h.w : h.y, lo_m = s.hi ? h.w : h.z;
    sc0 = (int)(__builtin_amdgcn_ubfe(lo_sc, s.sh, 4) | (__builtin_amdgcn_ubfe(h.y, s.sh + s.offh, 2) << 4));
    sc1 = (int)(__builtin_amdgcn_ubfe(lo_sc, s.sh + 8, 4) | (__builtin_amdgcn_ubfe(h.y, s.sh + 8 + s.offh, 2) << 4));
    m0 = (int)(__builtin_amdgcn_ubfe(lo_m, s.shm, 4) | (__builtin_amdgcn_ubfe(h.z, s.sh + s.offh, 2) << 4));
    m1 = (int)(__builtin_amdgcn_ubfe(lo_m, s.shm + 8, 4) | (__builtin_amdgcn_ubfe(h.z, s.sh + 8 + s.offh, 2) << 4));
}

template <int TYPE> struct RS;

template <> struct RS<KT_Q4_K_RS> {
    static constexpr int BYTES = 144;
    static constexpr int PIECES_PER_SB = 8;
    struct Act { int4 lo, hi; float d; int bslo, bshi; };
    struct W { uint4 h, q; };
    struct Lane { Q4Sel s; int j, hh; };
    static __device__ __forceinline__ Lane lane_consts(int lane) {
        Lane c;
        c.j = (lane >> 1) & 3; c.hh = lane & 1; c.s = q4_sel(c.j);
        return c;
    }
    static __device__ __forceinline__ int sb_of(int lane, int i) { return (lane >> 3) + 8 * i; }
    static __device__ __forceinline__ void act(const uint8_t *lds, int K, int sb, const Lane &c, Act &x) {
        const int e0 = 256 * sb + 64 * c.j + 16 * c.hh;
        x.lo = *(const int4 *)(lds + e0);
        x.hi = *(const int4 *)(lds + e0 + 32);
        x.d = ((const float *)(lds + K))[sb];
        const int16_t *bs = (const int16_t *)(lds + K + (K / 256) * 4);
        x.bslo = bs[e0 >> 4];
        x.bshi = bs[(e0 >> 4) + 2];
    }
    // piece p (clamped to the row) of row `rp` with nsb super-blocks
    static __device__ __forceinline__ void load(const uint8_t *rp, int nsb, int p, W &w) {
        w.h = ld_nt(rp + 16 * (p >> 3));
        w.q = ld_nt(rp + 16 * nsb + 16 * p);
    }
    static __device__ __forceinline__ float dot(const W &w, const Act &x, const Lane &c) {
        int sc0, m0, sc1, m1;
        q4_scales(w.h, c.s, sc0, m0, sc1, m1);
        const uint32_t q[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
        const int al[4] = {x.lo.x, x.lo.y, x.lo.z, x.lo.w}, ah[4] = {x.hi.x, x.hi.y, x.hi.z, x.hi.w};
        int dlo = 0, dhi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            dlo = sdot4((int)(q[k] & 0x0F0F0F0Fu), al[k], dlo);
            dhi = sdot4((int)((q[k] >> 4) & 0x0F0F0F0Fu), ah[k], dhi);
        }
        const int sumi = __mul24(sc0, dlo) + __mul24(sc1, dhi);
        const int summ = __mul24(m0, x.bslo) + __mul24(m1, x.bshi);
        const float dw = h2f((uint16_t)(w.h.x & 0xFFFF)), dmw = h2f((uint16_t)(w.h.x >> 16));
        return x.d * fmaf(dw, (float)sumi, -dmw * (float)summ);
    }
};

// ---------------------------------------------------------------- Q5_K_RS
// Q4_K_RS's pieces plus the fifth bits: row = [nsb][16] headers ++ [nsb][128] nibbles ++ [nsb][32] qh (ggml's qh bytes
// of each super-block, dequantize_row_q5_K ggml-quants.c:2640: element 64 j + l (l < 32) takes bit 2 j of qh[l],
// element 64 j + 32 + l bit 2 j + 1).  Piece (sb, j, hh) reads qh[16 hh .. 16 hh + 15] (the four pieces of a half
// share those 16 B: one cache line, one HBM read); its bits are rotated onto bit 4 of each byte and or-ed onto the
// nibbles, so the sdot4 operands are the 5-bit values themselves.
template <> struct RS<KT_Q5_K_RS> {
    static constexpr int BYTES = 176;
    static constexpr int PIECES_PER_SB = 8;
    using Act = RS<KT_Q4_K_RS>::Act;
    struct W { uint4 h, q, qh; };
    struct Lane { Q4Sel s; int j, hh, rlo, rhi; };
    static __device__ __forceinline__ Lane lane_consts(int lane) {
        Lane c;
        c.j = (lane >> 1) & 3; c.hh = lane & 1; c.s = q4_sel(c.j);
        c.rlo = (2 * c.j - 4) & 31;          // rotate right: bit 2j of each byte -> bit 4
        c.rhi = (2 * c.j - 3) & 31;          //               bit 2j+1         -> bit 4
        return c;
    }
    static __device__ __forceinline__ int sb_of(int lane, int i) { return (lane >> 3) + 8 * i; }
    static __device__ __forceinline__ void act(const uint8_t *lds, int K, int sb, const Lane &c, Act &x) {
        const int e0 = 256 * sb + 64 * c.j + 16 * c.hh;
        x.lo = *(const int4 *)(lds + e0);
        x.hi = *(const int4 *)(lds + e0 + 32);
        x.d = ((const float *)(lds + K))[sb];
        const int16_t *bs = (const int16_t *)(lds + K + (K / 256) * 4);
        x.bslo = bs[e0 >> 4];
        x.bshi = bs[(e0 >> 4) + 2];
    }
    static __device__ __forceinline__ void load(const uint8_t *rp, int nsb, int p, W &w) {
        w.h = ld_nt(rp + 16 * (p >> 3));
        w.q = ld_nt(rp + 16 * nsb + 16 * p);
        w.qh = ld_nt(rp + 144 * nsb + 32 * (p >> 3) + 16 * (p & 1));
    }
    static __device__ __forceinline__ float dot(const W &w, const Act &x, const Lane &c) {
        int sc0, m0, sc1, m1;
        q4_scales(w.h, c.s, sc0, m0, sc1, m1);
        const uint32_t q[4] = {w.q.x, w.q.y, w.q.z, w.q.w}, h[4] = {w.qh.x, w.qh.y, w.qh.z, w.qh.w};
        const int al[4] = {x.lo.x, x.lo.y, x.lo.z, x.lo.w}, ah[4] = {x.hi.x, x.hi.y, x.hi.z, x.hi.w};
        int dlo = 0, dhi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t lo = (q[k] & 0x0F0F0F0Fu) | (__builtin_amdgcn_alignbit(h[k], h[k], c.rlo) & 0x10101010u);
            const uint32_t hi = ((q[k] >> 4) & 0x0F0F0F0Fu) | (__builtin_amdgcn_alignbit(h[k], h[k], c.rhi) & 0x10101010u);
            dlo = sdot4((int)lo, al[k], dlo);
            dhi = sdot4((int)hi, ah[k], dhi);
        }
        const int sumi = __mul24(sc0, dlo) + __mul24(sc1, dhi);
        const int summ = __mul24(m0, x.bslo) + __mul24(m1, x.bshi);
        const float dw = h2f((uint16_t)(w.h.x & 0xFFFF)), dmw = h2f((uint16_t)(w.h.x >> 16));
        return x.d * fmaf(dw, (float)sumi, -dmw * (float)summ);
    }
};

// ---------------------------------------------------------------- Q6_K_RS
// unit U = l + 64 i = 4 sb + u, u = (half h = u >> 1, 16-lane half lh = u & 1); its 64 elements are
// 256 sb + 128 h + 16 lh + 32 g + 0..15 for g = 0..3 (dequantize_row_q6_K, ggml-quants.c:2978):
//   g0: ql-lo & 15 | qh >> 0 & 3,  g1: ql-hi & 15 | qh >> 2 & 3,  g2: ql-lo >> 4 | qh >> 4 & 3,
//   g3: ql-hi >> 4 | qh >> 6 & 3;  scales sc[8 h + lh + 2 g] (one int8 per 16 elements).
template <> struct RS<KT_Q6_K_RS> {
    static constexpr int BYTES = 210;
    static constexpr int PIECES_PER_SB = 4;
    struct Act { int4 a[4]; float d; int bs[4]; };
    struct W { uint4 A, B, C; uint32_t sc; uint32_t d; };
    struct Lane { int h, lh; };
    static __device__ __forceinline__ Lane lane_consts(int lane) {
        Lane c;
        c.h = (lane >> 1) & 1; c.lh = lane & 1;
        return c;
    }
    static __device__ __forceinline__ int sb_of(int lane, int i) { return (lane >> 2) + 16 * i; }
    static __device__ __forceinline__ void act(const uint8_t *lds, int K, int sb, const Lane &c, Act &x) {
        const int e0 = 256 * sb + 128 * c.h + 16 * c.lh;
        const int16_t *bs = (const int16_t *)(lds + K + (K / 256) * 4);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            x.a[g] = *(const int4 *)(lds + e0 + 32 * g);
            x.bs[g] = bs[(e0 >> 4) + 2 * g];
        }
        x.d = ((const float *)(lds + K))[sb];
    }
    static __device__ __forceinline__ void load(const uint8_t *rp, int nsb, int p, W &w) {
        w.A = ld_nt(rp + 16 * p);
        w.B = ld_nt(rp + 64 * nsb + 16 * p);
        w.C = ld_nt(rp + 128 * nsb + 16 * p);
        w.sc = __builtin_nontemporal_load((const uint32_t *)(rp + 192 * nsb + 4 * p));
        w.d = __builtin_nontemporal_load((const uint16_t *)(rp + 208 * nsb + 2 * (p >> 2)));
    }
    static __device__ __forceinline__ float dot(const W &w, const Act &x, const Lane &) {
        const uint32_t A[4] = {w.A.x, w.A.y, w.A.z, w.A.w}, B[4] = {w.B.x, w.B.y, w.B.z, w.B.w};
        const uint32_t C[4] = {w.C.x, w.C.y, w.C.z, w.C.w};
        int dg[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q0 = (A[k] & 0x0F0F0F0Fu) | ((C[k] << 4) & 0x30303030u);
            const uint32_t q1 = (B[k] & 0x0F0F0F0Fu) | ((C[k] << 2) & 0x30303030u);
            const uint32_t q2 = ((A[k] >> 4) & 0x0F0F0F0Fu) | (C[k] & 0x30303030u);
            const uint32_t q3 = ((B[k] >> 4) & 0x0F0F0F0Fu) | ((C[k] >> 2) & 0x30303030u);
            const int av[4] = {k == 0 ? x.a[0].x : k == 1 ? x.a[0].y : k == 2 ? x.a[0].z : x.a[0].w,
                               k == 0 ? x.a[1].x : k == 1 ? x.a[1].y : k == 2 ? x.a[1].z : x.a[1].w,
                               k == 0 ? x.a[2].x : k == 1 ? x.a[2].y : k == 2 ? x.a[2].z : x.a[2].w,
                               k == 0 ? x.a[3].x : k == 1 ? x.a[3].y : k == 2 ? x.a[3].z : x.a[3].w};
            dg[0] = sdot4((int)q0, av[0], dg[0]);
            dg[1] = sdot4((int)q1, av[1], dg[1]);
            dg[2] = sdot4((int)q2, av[2], dg[2]);
            dg[3] = sdot4((int)q3, av[3], dg[3]);
        }
        int isum = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int sc = (int)(int8_t)((w.sc >> (8 * g)) & 0xFF);
            isum += sc * (dg[g] - 32 * x.bs[g]);
        }
        return x.d * (h2f((uint16_t)w.d) * (float)isum);
    }
};

}  // namespace rs
