// iq_grid.h -- the lattice-grid weight types IQ2_XXS / IQ2_XS / IQ2_S / IQ3_XXS / IQ3_S / IQ1_S / IQ1_M on the device.
//
// Blocks stay in the ggml layout (ggml-common.h:340-405; every field at an even byte offset, so the reads here are
// 16-bit).  One 32-element sub-block decodes to IqSub: its 32 weights as signed int8 codes (four groups of 8, two
// dwords each) and an integer scale per group, so that
//     weight = d_sb * C * ls[group] * code          (C = iq_const<TYPE>(), a power of two)
// which is the integer structure of the reference's ggml_vec_dot_iq*_q8_K generic branches
// (ggml-quants.c:9606,9917,10502,10980,11303,11848,12179): the per-sub-block integer dots times ls, summed, times
// (d_w d_a) and the type's constant.  IQ1_S / IQ1_M carry their +-1/8 delta inside the code (code = 8 grid +- 1, C =
// 1/8: 8 (grid sum) +- (q8 sum) is exactly 8 (sumi + delta sumi1) of the reference).  The codes are what the
// mat-vec feeds v_dot4 and what the MFMA GEMM turns into exact f16 fragments.
//
// Dequantization (kcpp_dequantize / get_rows) follows dequantize_row_iq* (ggml-quants.c:3504-3739) float op by
// float op, so it is bit-exact; see iq_deq_sub.
#pragma once
#include "kcpp_common.h"

#define KCPP_IQ_TABLE(name, n) static __constant__ uint32_t name[n]
#include "iq_grids.h"
#undef KCPP_IQ_TABLE

struct IqSub {
    uint32_t v[8];    // 32 signed int8 codes, element order
    int ls[4];        // integer scale of each group of 8
};

__device__ __forceinline__ bool is_iq_grid(int t) {
    return t == KT_IQ2_XXS || t == KT_IQ2_XS || t == KT_IQ2_S || t == KT_IQ3_XXS || t == KT_IQ3_S || t == KT_IQ1_S ||
           t == KT_IQ1_M;
}
template <int T> constexpr float iq_const() {
    return (T == KT_IQ3_XXS) ? 0.25f : (T == KT_IQ3_S ? 1.0f : 0.125f);
}

__device__ __forceinline__ uint32_t iq_ld16(const uint8_t *p, int off) { return *(const uint16_t *)(p + off); }
__device__ __forceinline__ uint32_t iq_ld32(const uint8_t *p, int off) { return iq_ld16(p, off) | (iq_ld16(p, off + 2) << 16); }
__device__ __forceinline__ uint32_t iq_byte(const uint8_t *p, int off) { return p[off]; }

// ksigns_iq2xs: 7 sign bits plus the even-parity 8th
__device__ __forceinline__ uint32_t iq_sign8(uint32_t s7) { return s7 | ((__builtin_popcount(s7) & 1u) << 7); }
// four unsigned magnitudes (bytes of g, each >= 1) negated where the matching bit of s4 is set
__device__ __forceinline__ uint32_t iq_apply_signs(uint32_t g, uint32_t s4) {
    const uint32_t m = (((s4 & 0xFu) * 0x00204081u) & 0x01010101u) * 0xFFu;
    return (g ^ m) + (m & 0x01010101u);           // per-byte two's complement, no carry (g bytes >= 1)
}
// four IQ1 grid bytes (-1 / 0 / +1) -> 8 grid + delta (delta = +1 or -1) through one v_perm byte lookup
__device__ __forceinline__ uint32_t iq1_codes(uint32_t g, bool neg) {
    // selector = byte & 3: 0 (grid 0), 1 (grid +1), 3 (grid -1)
    const uint32_t tab = neg ? 0xF70007FFu : 0xF9000901u;     // bytes: [0] g=0, [1] g=+1, [3] g=-1
    return __builtin_amdgcn_perm(0u, tab, g & 0x03030303u);
}

// the f16 super-block scale d of a block
template <int T>
__device__ __forceinline__ float iq_d(const uint8_t *blk) {
    if constexpr (T == KT_IQ1_M) {
        const uint32_t s01 = iq_ld32(blk, 48), s23 = iq_ld32(blk, 52);
        const uint32_t sc0 = s01 & 0xFFFF, sc1 = s01 >> 16, sc2 = s23 & 0xFFFF, sc3 = s23 >> 16;
        return h2f((uint16_t)((sc0 >> 12) | ((sc1 >> 8) & 0x00f0) | ((sc2 >> 4) & 0x0f00) | (sc3 & 0xf000)));
    } else {
        return h2f((uint16_t)iq_ld16(blk, 0));
    }
}

// sub-block ib (0..7) of the block at blk
template <int T>
__device__ __forceinline__ void iq_sub(const uint8_t *blk, int ib, IqSub &s) {
    if constexpr (T == KT_IQ2_XXS) {          // qs: per sub-block 4 grid bytes ++ (signs 4 x 7 | scale << 28)
        const uint32_t a0 = iq_ld32(blk, 2 + 8 * ib), a1 = iq_ld32(blk, 6 + 8 * ib);
        const int ls = 2 * (int)(a1 >> 28) + 1;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t gi = (a0 >> (8 * l)) & 0xFF, sg = iq_sign8((a1 >> (7 * l)) & 127);
            s.v[2 * l] = iq_apply_signs(kcpp_iq2xxs_grid[2 * gi], sg & 15);
            s.v[2 * l + 1] = iq_apply_signs(kcpp_iq2xxs_grid[2 * gi + 1], sg >> 4);
            s.ls[l] = ls;
        }
    } else if constexpr (T == KT_IQ2_XS) {    // qs u16: 9-bit grid index | 7-bit sign index; scales[8]: two nibbles
        const uint32_t sc = iq_byte(blk, 66 + ib);
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t q = iq_ld16(blk, 2 + 8 * ib + 2 * l);
            const uint32_t gi = q & 511, sg = iq_sign8(q >> 9);
            s.v[2 * l] = iq_apply_signs(kcpp_iq2xs_grid[2 * gi], sg & 15);
            s.v[2 * l + 1] = iq_apply_signs(kcpp_iq2xs_grid[2 * gi + 1], sg >> 4);
            s.ls[l] = 2 * (int)(l < 2 ? sc & 15 : sc >> 4) + 1;
        }
    } else if constexpr (T == KT_IQ2_S) {     // qs[64]: grid low bytes ++ sign bytes; qh[8]: 2 high bits per index
        const uint32_t qh = iq_byte(blk, 66 + ib), sc = iq_byte(blk, 74 + ib);
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t gi = iq_byte(blk, 2 + 4 * ib + l) | ((qh << (8 - 2 * l)) & 0x300);
            const uint32_t sg = iq_byte(blk, 34 + 4 * ib + l);
            s.v[2 * l] = iq_apply_signs(kcpp_iq2s_grid[2 * gi], sg & 15);
            s.v[2 * l + 1] = iq_apply_signs(kcpp_iq2s_grid[2 * gi + 1], sg >> 4);
            s.ls[l] = 2 * (int)(l < 2 ? sc & 15 : sc >> 4) + 1;
        }
    } else if constexpr (T == KT_IQ3_XXS) {   // qs[64] grid bytes (4 values each) ++ 8 x (signs 4 x 7 | scale << 28)
        const uint32_t a = iq_ld32(blk, 66 + 4 * ib);
        const uint32_t q01 = iq_ld32(blk, 2 + 8 * ib), q23 = iq_ld32(blk, 6 + 8 * ib);
        const int ls = 2 * (int)(a >> 28) + 1;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t qq = l < 2 ? q01 : q23;
            const uint32_t g1 = (qq >> (16 * (l & 1))) & 0xFF, g2 = (qq >> (16 * (l & 1) + 8)) & 0xFF;
            const uint32_t sg = iq_sign8((a >> (7 * l)) & 127);
            s.v[2 * l] = iq_apply_signs(kcpp_iq3xxs_grid[g1], sg & 15);
            s.v[2 * l + 1] = iq_apply_signs(kcpp_iq3xxs_grid[g2], sg >> 4);
            s.ls[l] = ls;
        }
    } else if constexpr (T == KT_IQ3_S) {     // qs[64] low bytes, qh[8] high bits, signs[32], scales[4] nibbles
        const uint32_t qh = iq_byte(blk, 66 + ib);
        const uint32_t scb = iq_byte(blk, 106 + ib / 2);
        const int ls = 2 * (int)((ib & 1) ? scb >> 4 : scb & 15) + 1;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t i1 = iq_byte(blk, 2 + 8 * ib + 2 * l) | ((qh << (8 - 2 * l)) & 256);
            const uint32_t i2 = iq_byte(blk, 3 + 8 * ib + 2 * l) | ((qh << (7 - 2 * l)) & 256);
            const uint32_t sg = iq_byte(blk, 74 + 4 * ib + l);
            s.v[2 * l] = iq_apply_signs(kcpp_iq3s_grid[i1], sg & 15);
            s.v[2 * l + 1] = iq_apply_signs(kcpp_iq3s_grid[i2], sg >> 4);
            s.ls[l] = ls;
        }
    } else if constexpr (T == KT_IQ1_S) {     // qs[32] low bytes, qh u16 [8]: 3 x 3 high bits | scale << 12 | sign 15
        const uint32_t qh = iq_ld16(blk, 34 + 2 * ib);
        const int ls = 2 * (int)((qh >> 12) & 7) + 1;
        const bool neg = (qh & 0x8000) != 0;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t gi = iq_byte(blk, 2 + 4 * ib + l) | (((qh >> (3 * l)) & 7) << 8);
            s.v[2 * l] = iq1_codes(kcpp_iq1s_grid[2 * gi], neg);
            s.v[2 * l + 1] = iq1_codes(kcpp_iq1s_grid[2 * gi + 1], neg);
            s.ls[l] = ls;
        }
    } else {                                  // IQ1_M: qs[32], qh[16] (2 x (3 high bits | delta sign) per byte), scales
        const uint32_t qh0 = iq_byte(blk, 32 + 2 * ib), qh1 = iq_byte(blk, 33 + 2 * ib);
        const uint32_t sc = iq_ld16(blk, 48 + 2 * (ib / 2));
        const int ls1 = 2 * (int)((sc >> (6 * (ib % 2))) & 7) + 1, ls2 = 2 * (int)((sc >> (6 * (ib % 2) + 3)) & 7) + 1;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const uint32_t qh = l < 2 ? qh0 : qh1;
            const uint32_t gi = iq_byte(blk, 4 * ib + l) | ((qh << (8 - 4 * (l % 2))) & 0x700);
            const bool neg = (qh & (0x08u << (4 * (l % 2)))) != 0;
            s.v[2 * l] = iq1_codes(kcpp_iq1s_grid[2 * gi], neg);
            s.v[2 * l + 1] = iq1_codes(kcpp_iq1s_grid[2 * gi + 1], neg);
            s.ls[l] = l < 2 ? ls1 : ls2;
        }
    }
}

// dequantize_row_iq* of sub-block ib into o[0..32): the reference's float expressions, op by op
template <int T>
__device__ __forceinline__ void iq_deq_sub(const uint8_t *blk, int ib, float *o) {
    const float d = iq_d<T>(blk);
    if constexpr (T == KT_IQ1_S || T == KT_IQ1_M) {
        // dl (grid + delta): grid + delta in f32 (exact), one rounding for the product
        IqSub s;
        iq_sub<T>(blk, ib, s);
        float dl[2];
        if constexpr (T == KT_IQ1_S) {
            const uint32_t qh = iq_ld16(blk, 34 + 2 * ib);
            dl[0] = dl[1] = __fmul_rn(d, (float)(2 * (int)((qh >> 12) & 7) + 1));
        } else {
            dl[0] = __fmul_rn(d, (float)s.ls[0]);
            dl[1] = __fmul_rn(d, (float)s.ls[2]);
        }
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            const int code = (int)(int8_t)((s.v[e >> 2] >> (8 * (e & 3))) & 0xFF);   // 8 grid + delta
            o[e] = __fmul_rn(dl[e >> 4], (float)code * 0.125f);                        // grid + delta, exact
        }
    } else {
        // db = d (0.5 + ls) 0.25 / d (0.5 + ls) 0.5 / d (1 + 2 ls); weight = (db grid) with the sign flipped
        IqSub s;
        iq_sub<T>(blk, ib, s);
        float db[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const int raw = (s.ls[l] - 1) / 2;                // the stored 4-bit scale
            if constexpr (T == KT_IQ3_S) db[l] = __fmul_rn(d, (float)(1 + 2 * raw));
            else if constexpr (T == KT_IQ3_XXS) db[l] = __fmul_rn(__fmul_rn(d, 0.5f + (float)raw), 0.5f);
            else db[l] = __fmul_rn(__fmul_rn(d, 0.5f + (float)raw), 0.25f);
        }
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            const int code = (int)(int8_t)((s.v[e >> 2] >> (8 * (e & 3))) & 0xFF);
            const float m = __fmul_rn(db[e >> 3], (float)(code < 0 ? -code : code));
            o[e] = code < 0 ? -m : m;
        }
    }
}

// switch over the grid types: KCPP_IQ_CASES(X) expands X(type) for each
#define KCPP_IQ_CASES(X) X(KT_IQ2_XXS) X(KT_IQ2_XS) X(KT_IQ2_S) X(KT_IQ3_XXS) X(KT_IQ3_S) X(KT_IQ1_S) X(KT_IQ1_M)
template <int T> constexpr bool kIqGrid = T == KT_IQ2_XXS || T == KT_IQ2_XS || T == KT_IQ2_S || T == KT_IQ3_XXS ||
                                          T == KT_IQ3_S || T == KT_IQ1_S || T == KT_IQ1_M;

// dequantize block b (ggml layout, 2-B aligned) into o[0..256)
template <int T>
__device__ __forceinline__ void iq_deq_block(const uint8_t *blk, float *o) {
#pragma unroll 1
    for (int ib = 0; ib < 8; ++ib) iq_deq_sub<T>(blk, ib, o + 32 * ib);
}
