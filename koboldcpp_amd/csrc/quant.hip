// quant.hip -- weight layout (repack / synth / dequant) and activation quantization kernels.
//
// Activation quantization mirrors the CPU vec_dot_type conversion bit-for-bit:
//   Q8_K: quantize_row_q8_K_ref   (reference ggml/src/ggml-quants.c:3786-3823)
//   Q8_0: quantize_row_q8_0 AVX2  (reference ggml/src/ggml-quants.c:940-1000)
// Dequantization mirrors dequantize_row_* (ggml-quants.c:1523,1617,2556,2764,2978).
#include "kcpp_common.h"
#include "kcpp_internal.h"
#include "iq_grid.h"

// ---------------------------------------------------------------- weight layout
// place one ggml-layout block (src) into the kcpp GPU layout at block index b (bpr blocks per row)
__device__ __forceinline__ void kl_store_block(int type, const uint8_t *src, uint8_t *dst, int64_t b, int64_t nb,
                                               int64_t bpr) {
    switch (type) {
    case KT_Q2_K: {   // SoA planes: scales [nb][16] ++ qs [nb][64] ++ (d, dmin) [nb][4]
        uint8_t *sc = dst + b * 16, *q = dst + nb * 16 + b * 64, *dd = dst + nb * 80 + b * 4;
        for (int i = 0; i < 16; ++i) sc[i] = src[i];
        for (int i = 0; i < 64; ++i) q[i] = src[16 + i];
        for (int i = 0; i < 4; ++i) dd[i] = src[80 + i];
    } break;
    case KT_Q3_K: {   // SoA planes: hmask [nb][32] ++ qs [nb][64] ++ scales [nb][12] ++ d [nb][2] (16-B aligned loads)
        uint8_t *hm = dst + b * 32, *q = dst + nb * 32 + b * 64, *sc = dst + nb * 96 + b * 12, *d = dst + nb * 108 + b * 2;
        for (int i = 0; i < 32; ++i) hm[i] = src[i];
        for (int i = 0; i < 64; ++i) q[i] = src[32 + i];
        for (int i = 0; i < 12; ++i) sc[i] = src[96 + i];
        d[0] = src[108]; d[1] = src[109];
    } break;
    case KT_Q6_K: {
        uint8_t *q = dst + b * 192, *sc = dst + nb * 192 + b * 16, *d = dst + nb * 208 + b * 2;
        for (int i = 0; i < 192; ++i) q[i] = src[i];
        for (int i = 0; i < 16; ++i) sc[i] = src[192 + i];
        d[0] = src[208]; d[1] = src[209];
    } break;
    case KT_Q4_0: {
        uint8_t *q = dst + b * 16, *d = dst + nb * 16 + b * 2;
        d[0] = src[0]; d[1] = src[1];
        for (int i = 0; i < 16; ++i) q[i] = src[2 + i];
    } break;
    case KT_IQ4_NL: { // SoA planes as Q4_0: qs [nb][16] ++ d [nb][2]  (block_iq4_nl: d, qs[16])
        uint8_t *q = dst + b * 16, *d = dst + nb * 16 + b * 2;
        d[0] = src[0]; d[1] = src[1];
        for (int i = 0; i < 16; ++i) q[i] = src[2 + i];
    } break;
    case KT_IQ4_XS: { // SoA planes: qs [nb][128] ++ (d, scales_h, scales_l[4]) [nb][8]  (block_iq4_xs: d, sh, sl[4], qs[128])
        uint8_t *q = dst + b * 128, *h = dst + nb * 128 + b * 8;
        for (int i = 0; i < 8; ++i) h[i] = src[i];
        for (int i = 0; i < 128; ++i) q[i] = src[8 + i];
    } break;
    case KT_Q4_1: {   // SoA planes: qs [nb][16] ++ (d, m) [nb][4]  (block_q4_1: d, m, qs[16])
        uint8_t *q = dst + b * 16, *dm = dst + nb * 16 + b * 4;
        for (int i = 0; i < 4; ++i) dm[i] = src[i];
        for (int i = 0; i < 16; ++i) q[i] = src[4 + i];
    } break;
    case KT_Q5_1: {   // SoA planes: qs [nb][16] ++ qh [nb][4] ++ (d, m) [nb][4]  (block_q5_1: d, m, qh[4], qs[16])
        uint8_t *q = dst + b * 16, *h = dst + nb * 16 + b * 4, *dm = dst + nb * 20 + b * 4;
        for (int i = 0; i < 4; ++i) { dm[i] = src[i]; h[i] = src[4 + i]; }
        for (int i = 0; i < 16; ++i) q[i] = src[8 + i];
    } break;
    case KT_Q5_0: {   // SoA planes: qs [nb][16] ++ qh [nb][4] ++ d [nb][2]  (block_q5_0: d, qh[4], qs[16])
        uint8_t *q = dst + b * 16, *h = dst + nb * 16 + b * 4, *d = dst + nb * 20 + b * 2;
        d[0] = src[0]; d[1] = src[1];
        for (int i = 0; i < 4; ++i) h[i] = src[2 + i];
        for (int i = 0; i < 16; ++i) q[i] = src[6 + i];
    } break;
    case KT_Q8_0: {
        uint8_t *q = dst + b * 32, *d = dst + nb * 32 + b * 2;
        d[0] = src[0]; d[1] = src[1];
        for (int i = 0; i < 32; ++i) q[i] = src[2 + i];
    } break;
    case KT_Q8_0_T: {   // kcpp_common.h: 32-row tiles of [half][row][16 B] per block, d plane in groups of 4 blocks
        const int64_t n = b / bpr, blk = b % bpr, t = n >> 5, r = n & 31;
        uint8_t *q = dst + (t * bpr + blk) * 1024 + r * 16;
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i) q[512 * h + i] = src[2 + 16 * h + i];
        uint8_t *d = dst + nb * 32 + (t * (bpr / 4) + blk / 4) * 256 + r * 8 + (blk % 4) * 2;
        d[0] = src[0]; d[1] = src[1];
    } break;
    case KT_Q4_K_RS: {
        const int64_t n = b / bpr, sb = b % bpr;
        uint8_t *row = dst + n * 144 * bpr;
        for (int i = 0; i < 16; ++i) row[16 * sb + i] = src[i];
        for (int i = 0; i < 128; ++i) row[16 * bpr + 128 * sb + i] = src[16 + i];
    } break;
    case KT_Q5_K_RS: {   // row: [nsb][16] headers (d, dmin, scales) ++ [nsb][128] nibbles ++ [nsb][32] qh
        const int64_t n = b / bpr, sb = b % bpr;
        uint8_t *row = dst + n * 176 * bpr;
        for (int i = 0; i < 16; ++i) row[16 * sb + i] = src[i];
        for (int i = 0; i < 128; ++i) row[16 * bpr + 128 * sb + i] = src[48 + i];
        for (int i = 0; i < 32; ++i) row[144 * bpr + 32 * sb + i] = src[16 + i];
    } break;
    case KT_Q6_K_RS: {
        const int64_t n = b / bpr, sb = b % bpr;
        uint8_t *row = dst + n * 210 * bpr;
        for (int u = 0; u < 4; ++u) {
            const int h = u >> 1, lh = u & 1;
            const int64_t U = 4 * sb + u;
            for (int i = 0; i < 16; ++i) {
                row[16 * U + i] = src[64 * h + 16 * lh + i];
                row[64 * bpr + 16 * U + i] = src[64 * h + 32 + 16 * lh + i];
                row[128 * bpr + 16 * U + i] = src[128 + 32 * h + 16 * lh + i];
            }
            for (int g = 0; g < 4; ++g) row[192 * bpr + 4 * U + g] = src[192 + 8 * h + lh + 2 * g];
        }
        row[208 * bpr + 2 * sb] = src[208]; row[208 * bpr + 2 * sb + 1] = src[209];
    } break;
    default: {
        const int bb = ks_block_bytes(type);
        for (int i = 0; i < bb; ++i) dst[b * bb + i] = src[i];
    }
    }
}
__device__ __forceinline__ void kl_load_block(int type, const uint8_t *src, uint8_t *blk, int64_t b, int64_t nb,
                                              int64_t bpr) {
    switch (type) {
    case KT_Q2_K: {
        const uint8_t *sc = src + b * 16, *q = src + nb * 16 + b * 64, *dd = src + nb * 80 + b * 4;
        for (int i = 0; i < 16; ++i) blk[i] = sc[i];
        for (int i = 0; i < 64; ++i) blk[16 + i] = q[i];
        for (int i = 0; i < 4; ++i) blk[80 + i] = dd[i];
    } break;
    case KT_Q3_K: {
        const uint8_t *hm = src + b * 32, *q = src + nb * 32 + b * 64, *sc = src + nb * 96 + b * 12, *d = src + nb * 108 + b * 2;
        for (int i = 0; i < 32; ++i) blk[i] = hm[i];
        for (int i = 0; i < 64; ++i) blk[32 + i] = q[i];
        for (int i = 0; i < 12; ++i) blk[96 + i] = sc[i];
        blk[108] = d[0]; blk[109] = d[1];
    } break;
    case KT_Q6_K: {
        const uint8_t *q = src + b * 192, *sc = src + nb * 192 + b * 16, *d = src + nb * 208 + b * 2;
        for (int i = 0; i < 192; ++i) blk[i] = q[i];
        for (int i = 0; i < 16; ++i) blk[192 + i] = sc[i];
        blk[208] = d[0]; blk[209] = d[1];
    } break;
    case KT_Q4_0: {
        const uint8_t *q = src + b * 16, *d = src + nb * 16 + b * 2;
        blk[0] = d[0]; blk[1] = d[1];
        for (int i = 0; i < 16; ++i) blk[2 + i] = q[i];
    } break;
    case KT_IQ4_NL: {
        const uint8_t *q = src + b * 16, *d = src + nb * 16 + b * 2;
        blk[0] = d[0]; blk[1] = d[1];
        for (int i = 0; i < 16; ++i) blk[2 + i] = q[i];
    } break;
    case KT_IQ4_XS: {
        const uint8_t *q = src + b * 128, *h = src + nb * 128 + b * 8;
        for (int i = 0; i < 8; ++i) blk[i] = h[i];
        for (int i = 0; i < 128; ++i) blk[8 + i] = q[i];
    } break;
    case KT_Q4_1: {
        const uint8_t *q = src + b * 16, *dm = src + nb * 16 + b * 4;
        for (int i = 0; i < 4; ++i) blk[i] = dm[i];
        for (int i = 0; i < 16; ++i) blk[4 + i] = q[i];
    } break;
    case KT_Q5_1: {
        const uint8_t *q = src + b * 16, *h = src + nb * 16 + b * 4, *dm = src + nb * 20 + b * 4;
        for (int i = 0; i < 4; ++i) { blk[i] = dm[i]; blk[4 + i] = h[i]; }
        for (int i = 0; i < 16; ++i) blk[8 + i] = q[i];
    } break;
    case KT_Q5_0: {
        const uint8_t *q = src + b * 16, *h = src + nb * 16 + b * 4, *d = src + nb * 20 + b * 2;
        blk[0] = d[0]; blk[1] = d[1];
        for (int i = 0; i < 4; ++i) blk[2 + i] = h[i];
        for (int i = 0; i < 16; ++i) blk[6 + i] = q[i];
    } break;
    case KT_Q8_0: {
        const uint8_t *q = src + b * 32, *d = src + nb * 32 + b * 2;
        blk[0] = d[0]; blk[1] = d[1];
        for (int i = 0; i < 32; ++i) blk[2 + i] = q[i];
    } break;
    case KT_Q8_0_T: {
        const int64_t n = b / bpr, bi = b % bpr, t = n >> 5, r = n & 31;
        const uint8_t *q = src + (t * bpr + bi) * 1024 + r * 16;
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i) blk[2 + 16 * h + i] = q[512 * h + i];
        const uint8_t *d = src + nb * 32 + (t * (bpr / 4) + bi / 4) * 256 + r * 8 + (bi % 4) * 2;
        blk[0] = d[0]; blk[1] = d[1];
    } break;
    case KT_Q4_K_RS: {
        const int64_t n = b / bpr, sb = b % bpr;
        const uint8_t *row = src + n * 144 * bpr;
        for (int i = 0; i < 16; ++i) blk[i] = row[16 * sb + i];
        for (int i = 0; i < 128; ++i) blk[16 + i] = row[16 * bpr + 128 * sb + i];
    } break;
    case KT_Q5_K_RS: {
        const int64_t n = b / bpr, sb = b % bpr;
        const uint8_t *row = src + n * 176 * bpr;
        for (int i = 0; i < 16; ++i) blk[i] = row[16 * sb + i];
        for (int i = 0; i < 128; ++i) blk[48 + i] = row[16 * bpr + 128 * sb + i];
        for (int i = 0; i < 32; ++i) blk[16 + i] = row[144 * bpr + 32 * sb + i];
    } break;
    case KT_Q6_K_RS: {
        const int64_t n = b / bpr, sb = b % bpr;
        const uint8_t *row = src + n * 210 * bpr;
        for (int u = 0; u < 4; ++u) {
            const int h = u >> 1, lh = u & 1;
            const int64_t U = 4 * sb + u;
            for (int i = 0; i < 16; ++i) {
                blk[64 * h + 16 * lh + i] = row[16 * U + i];
                blk[64 * h + 32 + 16 * lh + i] = row[64 * bpr + 16 * U + i];
                blk[128 + 32 * h + 16 * lh + i] = row[128 * bpr + 16 * U + i];
            }
            for (int g = 0; g < 4; ++g) blk[192 + 8 * h + lh + 2 * g] = row[192 * bpr + 4 * U + g];
        }
        blk[208] = row[208 * bpr + 2 * sb]; blk[209] = row[208 * bpr + 2 * sb + 1];
    } break;
    default: {
        const int bb = ks_block_bytes(type);
        for (int i = 0; i < bb; ++i) blk[i] = src[b * bb + i];
    }
    }
}

__global__ void k_repack(int type, const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, int64_t nb, int64_t bpr,
                         int dir) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint8_t blk[256];
    const int bb = ks_block_bytes(type);
    if (dir == 0) {                    // ggml -> kcpp
        for (int i = 0; i < bb; ++i) blk[i] = src[b * bb + i];
        kl_store_block(type, blk, dst, b, nb, bpr);
    } else {                           // kcpp -> ggml
        kl_load_block(type, src, blk, b, nb, bpr);
        for (int i = 0; i < bb; ++i) dst[b * bb + i] = blk[i];
    }
}

// block b of the tensor gets the content of block b + boff of the synthetic stream (boff != 0: a row slice)
__global__ void k_synth(int type, uint64_t seed, uint64_t tid, uint8_t *__restrict__ dst, int64_t nb, int64_t bpr,
                        int64_t boff) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint8_t blk[256];
    ks_fill_block(type, seed, tid, (uint64_t)(b + boff), blk);
    kl_store_block(type, blk, dst, b, nb, bpr);
}

__device__ __forceinline__ void scale_min_k4(int j, const uint8_t *q, int &d, int &m) {
    if (j < 4) { d = q[j] & 63; m = q[j + 4] & 63; }
    else {
        d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

// the 16 biased 6-bit Q3_K scales from the 12 packed bytes (dequantize_row_q3_K, ggml-quants.c:2346-2351)
__device__ __forceinline__ void q3k_scales(const uint8_t *s12, int8_t *sc) {
    uint32_t a0 = s12[0] | (s12[1] << 8) | (s12[2] << 16) | ((uint32_t)s12[3] << 24);
    uint32_t a1 = s12[4] | (s12[5] << 8) | (s12[6] << 16) | ((uint32_t)s12[7] << 24);
    const uint32_t tmp = s12[8] | (s12[9] << 8) | (s12[10] << 16) | ((uint32_t)s12[11] << 24);
    const uint32_t k1 = 0x03030303u, k2 = 0x0f0f0f0fu;
    const uint32_t a2 = ((a0 >> 4) & k2) | (((tmp >> 4) & k1) << 4), a3 = ((a1 >> 4) & k2) | (((tmp >> 6) & k1) << 4);
    a0 = (a0 & k2) | (((tmp >> 0) & k1) << 4);
    a1 = (a1 & k2) | (((tmp >> 2) & k1) << 4);
    const uint32_t a[4] = {a0, a1, a2, a3};
    for (int i = 0; i < 16; ++i) sc[i] = (int8_t)((a[i >> 2] >> (8 * (i & 3))) & 0xFF);
}

// dequantize block b of a kcpp-layout tensor (nb blocks total) into o[0..block_elems)
__device__ void deq_block(int type, const uint8_t *src, int64_t nb, int64_t bpr, int64_t b, float *o) {
    uint8_t blk[256];
    kl_load_block(type, src, blk, b, nb, bpr);
    switch (ks_base_type(type)) {
    case KT_F32: o[0] = *(const float *)blk; break;
    case KT_F16: o[0] = h2f(*(const uint16_t *)blk); break;
    case KT_Q4_0: {
        float d = h2f(blk[0] | (blk[1] << 8));
        for (int j = 0; j < 16; ++j) {
            o[j] = ((blk[2 + j] & 0x0F) - 8) * d;
            o[j + 16] = ((blk[2 + j] >> 4) - 8) * d;
        }
    } break;
    case KT_Q4_1: case KT_Q5_1: {   // dequantize_row_q4_1 / _q5_1, ggml-quants.c:1543-1616 (x d + m, two roundings)
        const float d = h2f(blk[0] | (blk[1] << 8)), m = h2f(blk[2] | (blk[3] << 8));
        const bool five = type == KT_Q5_1;
        const uint32_t qh = five ? (blk[4] | (blk[5] << 8) | (blk[6] << 16) | ((uint32_t)blk[7] << 24)) : 0u;
        const uint8_t *qs = blk + (five ? 8 : 4);
        for (int j = 0; j < 16; ++j) {
            const int x0 = (qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10), x1 = (qs[j] >> 4) | ((qh >> (j + 12)) & 0x10);
            o[j] = __fadd_rn(__fmul_rn((float)x0, d), m);
            o[j + 16] = __fadd_rn(__fmul_rn((float)x1, d), m);
        }
    } break;
    case KT_Q5_0: {   // dequantize_row_q5_0, ggml-quants.c:1564-1588
        const float d = h2f(blk[0] | (blk[1] << 8));
        const uint32_t qh = blk[2] | (blk[3] << 8) | (blk[4] << 16) | ((uint32_t)blk[5] << 24);
        for (int j = 0; j < 16; ++j) {
            o[j] = (float)((int)((blk[6 + j] & 0x0F) | (((qh >> j) << 4) & 0x10)) - 16) * d;
            o[j + 16] = (float)((int)((blk[6 + j] >> 4) | ((qh >> (j + 12)) & 0x10)) - 16) * d;
        }
    } break;
    case KT_Q8_0: {
        float d = h2f(blk[0] | (blk[1] << 8));
        for (int j = 0; j < 32; ++j) o[j] = (int8_t)blk[2 + j] * d;
    } break;
    case KT_IQ4_NL: {   // dequantize_row_iq4_nl, ggml-quants.c:3743-3759: d * kvalues[q] (one rounding)
        const float d = h2f(blk[0] | (blk[1] << 8));
        for (int j = 0; j < 16; ++j) {
            o[j] = __fmul_rn(d, (float)kv_iq4nl(blk[2 + j] & 0xF));
            o[j + 16] = __fmul_rn(d, (float)kv_iq4nl(blk[2 + j] >> 4));
        }
    } break;
    case KT_IQ4_XS: {   // dequantize_row_iq4_xs, ggml-quants.c:3761-3782: (d (ls - 32)) * kvalues[q]
        const float d = h2f(blk[0] | (blk[1] << 8));
        const int sh = blk[2] | (blk[3] << 8);
        for (int ib = 0; ib < 8; ++ib) {
            const int ls = ((blk[4 + ib / 2] >> 4 * (ib % 2)) & 0xF) | (((sh >> 2 * ib) & 3) << 4);
            const float dl = __fmul_rn(d, (float)(ls - 32));
            const uint8_t *qs = blk + 8 + 16 * ib;
            for (int j = 0; j < 16; ++j) {
                o[32 * ib + j] = __fmul_rn(dl, (float)kv_iq4nl(qs[j] & 0xF));
                o[32 * ib + j + 16] = __fmul_rn(dl, (float)kv_iq4nl(qs[j] >> 4));
            }
        }
    } break;
    case KT_Q4_K: case KT_Q5_K: {
        const bool five = ks_base_type(type) == KT_Q5_K;
        const float d = h2f(blk[0] | (blk[1] << 8)), mn = h2f(blk[2] | (blk[3] << 8));
        const uint8_t *sc = blk + 4, *qh = blk + 16, *q = blk + (five ? 48 : 16);
        for (int c = 0; c < 4; ++c) {
            int s1, m1, s2, m2;
            scale_min_k4(2 * c, sc, s1, m1);
            scale_min_k4(2 * c + 1, sc, s2, m2);
            const float d1 = d * s1, mm1 = mn * m1, d2 = d * s2, mm2 = mn * m2;
            for (int l = 0; l < 32; ++l) {
                int lo = q[32 * c + l] & 0xF, hi = q[32 * c + l] >> 4;
                if (five) { lo += ((qh[l] >> (2 * c)) & 1) << 4; hi += ((qh[l] >> (2 * c + 1)) & 1) << 4; }
                o[64 * c + l] = __fsub_rn(__fmul_rn(d1, (float)lo), mm1);
                o[64 * c + 32 + l] = __fsub_rn(__fmul_rn(d2, (float)hi), mm2);
            }
        }
    } break;
    case KT_Q2_K: {                                   // ggml-quants.c:2251-2282: (d (sc & 15)) q - dmin (sc >> 4)
        const float d = h2f(blk[80] | (blk[81] << 8)), mn = h2f(blk[82] | (blk[83] << 8));
        for (int e = 0; e < 256; ++e) {
            const int n = e >> 7, j = (e >> 5) & 3, l = e & 31;
            const int sc = blk[e >> 4], q = (blk[16 + 32 * n + l] >> (2 * j)) & 3;
            o[e] = __fsub_rn(__fmul_rn(__fmul_rn(d, (float)(sc & 0xF)), (float)q), __fmul_rn(mn, (float)(sc >> 4)));
        }
    } break;
    case KT_Q3_K: {                                   // ggml-quants.c:2328-2376 (exact: d (sc - 32) q3)
        const float d = h2f(blk[108] | (blk[109] << 8));
        int8_t sc[16];
        q3k_scales(blk + 96, sc);
        const uint8_t *hm = blk, *q = blk + 32;
        for (int e = 0; e < 256; ++e) {
            const int n = e >> 7, j = (e >> 5) & 3, l = e & 31;
            const int v = ((q[32 * n + l] >> (2 * j)) & 3) - ((hm[l] >> (4 * n + j)) & 1 ? 0 : 4);
            o[e] = __fmul_rn(__fmul_rn(d, (float)(sc[8 * n + 2 * j + (l >> 4)] - 32)), (float)v);
        }
    } break;
    case KT_Q6_K: {
        const float d = h2f(blk[208] | (blk[209] << 8));
        const uint8_t *ql = blk, *qh = blk + 128;
        const int8_t *sc = (const int8_t *)(blk + 192);
        for (int n = 0; n < 2; ++n) {
            for (int l = 0; l < 32; ++l) {
                int is = l / 16;
                int q1 = ((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                int q2 = ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                int q3 = ((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                int q4 = ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                o[l + 0] = __fmul_rn(__fmul_rn(d, (float)sc[is + 0]), (float)q1);
                o[l + 32] = __fmul_rn(__fmul_rn(d, (float)sc[is + 2]), (float)q2);
                o[l + 64] = __fmul_rn(__fmul_rn(d, (float)sc[is + 4]), (float)q3);
                o[l + 96] = __fmul_rn(__fmul_rn(d, (float)sc[is + 6]), (float)q4);
            }
            o += 128; ql += 64; qh += 32; sc += 8;
        }
    } break;
    }
}

// one thread per block: dequantize into y (row-major [N][K])
__global__ void k_dequant(int type, const uint8_t *__restrict__ src, float *__restrict__ y, int64_t nb, int64_t bpr) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    deq_block(type, src, nb, bpr, b, y + b * ks_block_elems(type));
}
// the grid types (ggml layout): one thread per 32-element sub-block
template <int T>
__global__ void k_dequant_iq(const uint8_t *__restrict__ src, float *__restrict__ y, int64_t nsub) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsub) return;
    iq_deq_sub<T>(src + (i >> 3) * ks_block_bytes(T), (int)(i & 7), y + 32 * i);
}
// get_rows of a grid type: one thread per sub-block of the selected row
template <int T>
__global__ void k_get_rows_iq(const uint8_t *__restrict__ src, int64_t K, int64_t N, const int32_t *__restrict__ ids,
                              float *__restrict__ y, int64_t ldy) {
    const int64_t t = blockIdx.y;
    const int64_t r = min(max((int64_t)ids[t], (int64_t)0), N - 1);
    const int64_t nsub = K / 32;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsub; i += (int64_t)gridDim.x * blockDim.x)
        iq_deq_sub<T>(src + (r * (K / 256) + (i >> 3)) * ks_block_bytes(T), (int)(i & 7), y + t * ldy + 32 * i);
}

// get_rows: one workgroup per token; thread i dequantizes element chunks of 8 of the selected row.
// K-quant element e of super-block sb uses the same formulas as deq_block (ggml-quants.c:2556-3006).
__device__ __forceinline__ float deq_elem(int type, const uint8_t *src, int64_t nb, int64_t b, int e) {
    switch (type) {
    case KT_F32: return ((const float *)src)[b];
    case KT_F16: return h2f(((const uint16_t *)src)[b]);
    case KT_Q4_0: {
        const float d = h2f(*(const uint16_t *)(src + nb * 16 + b * 2));
        const uint8_t q = src[b * 16 + (e & 15)];
        return ((e < 16 ? (q & 0xF) : (q >> 4)) - 8) * d;
    }
    case KT_Q4_1: case KT_Q5_1: {
        const bool five = type == KT_Q5_1;
        const uint32_t dm = *(const uint32_t *)(src + nb * (five ? 20 : 16) + b * 4);
        const uint8_t q = src[b * 16 + (e & 15)];
        const uint32_t qh = five ? *(const uint32_t *)(src + nb * 16 + b * 4) : 0u;
        const int x = (int)((e < 16 ? (q & 0xF) : (q >> 4)) | (((qh >> e) & 1) << 4));
        return __fadd_rn(__fmul_rn((float)x, h2f((uint16_t)(dm & 0xFFFF))), h2f((uint16_t)(dm >> 16)));
    }
    case KT_Q5_0: {
        const float d = h2f(*(const uint16_t *)(src + nb * 20 + b * 2));
        const uint8_t q = src[b * 16 + (e & 15)];
        const uint32_t qh = *(const uint32_t *)(src + nb * 16 + b * 4);
        return (float)((int)((e < 16 ? (q & 0xF) : (q >> 4)) | (((qh >> e) & 1) << 4)) - 16) * d;
    }
    case KT_Q8_0: return (int8_t)src[b * 32 + e] * h2f(*(const uint16_t *)(src + nb * 32 + b * 2));
    case KT_IQ4_NL: {
        const float d = h2f(*(const uint16_t *)(src + nb * 16 + b * 2));
        const uint8_t q = src[b * 16 + (e & 15)];
        return __fmul_rn(d, (float)kv_iq4nl(e < 16 ? (q & 0xF) : (q >> 4)));
    }
    case KT_IQ4_XS: {
        const uint8_t *h = src + nb * 128 + b * 8;
        const int ib = e >> 5, j = e & 31;
        const int ls = ((h[4 + ib / 2] >> 4 * (ib % 2)) & 0xF) | ((((h[2] | (h[3] << 8)) >> 2 * ib) & 3) << 4);
        const uint8_t q = src[b * 128 + 16 * ib + (j & 15)];
        return __fmul_rn(__fmul_rn(h2f(h[0] | (h[1] << 8)), (float)(ls - 32)), (float)kv_iq4nl(j < 16 ? (q & 0xF) : (q >> 4)));
    }
    case KT_Q4_K: case KT_Q5_K: {
        const bool five = type == KT_Q5_K;
        const uint8_t *blk = src + b * (five ? 176 : 144);
        const float d = h2f(blk[0] | (blk[1] << 8)), mn = h2f(blk[2] | (blk[3] << 8));
        const int c = e >> 6, l = e & 31, hi = (e >> 5) & 1;
        int sc, m;
        scale_min_k4(2 * c + hi, blk + 4, sc, m);
        const uint8_t qb = blk[(five ? 48 : 16) + 32 * c + l];
        int q = hi ? (qb >> 4) : (qb & 0xF);
        if (five) q += ((blk[16 + l] >> (2 * c + hi)) & 1) << 4;
        return __fsub_rn(__fmul_rn(d * sc, (float)q), mn * m);
    }
    case KT_Q4_K_RS: case KT_Q5_K_RS: case KT_Q6_K_RS: case KT_Q8_0_T: return 0.0f;   // row gathers of decode layouts: unused
    case KT_Q2_K: {
        const float d = h2f(*(const uint16_t *)(src + nb * 80 + b * 4)), mn = h2f(*(const uint16_t *)(src + nb * 80 + b * 4 + 2));
        const int n = e >> 7, j = (e >> 5) & 3, l = e & 31;
        const int sc = src[b * 16 + (e >> 4)], q = (src[nb * 16 + b * 64 + 32 * n + l] >> (2 * j)) & 3;
        return __fsub_rn(__fmul_rn(__fmul_rn(d, (float)(sc & 0xF)), (float)q), __fmul_rn(mn, (float)(sc >> 4)));
    }
    case KT_Q3_K: {
        const float d = h2f(*(const uint16_t *)(src + nb * 108 + b * 2));
        int8_t sc[16];
        q3k_scales(src + nb * 96 + b * 12, sc);
        const int n = e >> 7, j = (e >> 5) & 3, l = e & 31;
        const int v = ((src[nb * 32 + b * 64 + 32 * n + l] >> (2 * j)) & 3) - ((src[b * 32 + l] >> (4 * n + j)) & 1 ? 0 : 4);
        return __fmul_rn(__fmul_rn(d, (float)(sc[8 * n + 2 * j + (l >> 4)] - 32)), (float)v);
    }
    case KT_Q6_K: {
        const uint8_t *q6 = src + b * 192;
        const int8_t *scp = (const int8_t *)(src + nb * 192 + b * 16);
        const float d = h2f(*(const uint16_t *)(src + nb * 208 + b * 2));
        const int n = e >> 7, r = e & 127, p = r >> 5, l = r & 31;
        const uint8_t ql = q6[64 * n + l + 32 * (p & 1)], qh = q6[128 + 32 * n + l];
        const int q = (((p >> 1) ? (ql >> 4) : (ql & 0xF)) | (((qh >> (2 * p)) & 3) << 4)) - 32;
        return __fmul_rn(__fmul_rn(d, (float)scp[8 * n + l / 16 + 2 * p]), (float)q);
    }
    }
    return 0.0f;
}

__global__ void k_get_rows(int type, const uint8_t *__restrict__ src, int64_t K, int64_t N,
                           const int32_t *__restrict__ ids, float *__restrict__ y, int64_t ldy) {
    const int64_t t = blockIdx.y;
    // out-of-range ids (ggml asserts on the host) are clamped so a bad id cannot fault the device
    const int64_t r = min(max((int64_t)ids[t], (int64_t)0), N - 1);
    const int be = ks_block_elems(type);
    const int64_t bpr = K / be, nb = bpr * N;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += (int64_t)gridDim.x * blockDim.x)
        y[t * ldy + k] = deq_elem(type, src, nb, r * bpr + k / be, (int)(k % be));
}

// ---------------------------------------------------------------- activation quantization
// one aligned 16-lane group per super-block, 16 elements per lane
// GLU: the input element is silu(x[i]) * x[i + uoff] (gate | up halves of one fused GEMM output row),
// the same expression as k_silu_mul, so quantize(silu(g)*u) is bit-identical to the unfused pair.
template <bool GLU>
__global__ void __launch_bounds__(256) k_quant_q8k(const float *__restrict__ x, int64_t ldx, uint8_t *__restrict__ out,
                                                   int64_t K, int64_t M, int64_t uoff) {
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nsb = K / 256;
    const int64_t g = gt >> 4;                        // global super-block
    const int l16 = threadIdx.x & 15;
    const bool valid = g < nsb * M;
    const int64_t m = valid ? g / nsb : 0, sb = valid ? g % nsb : 0;
    float v[16];
    const float4 *src = (const float4 *)(x + m * ldx + sb * 256 + 16 * l16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 f = valid ? src[k] : make_float4(0, 0, 0, 0);
        v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
    }
    if constexpr (GLU) {
        const float4 *usrc = (const float4 *)(x + m * ldx + uoff + sb * 256 + 16 * l16);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 f = valid ? usrc[k] : make_float4(0, 0, 0, 0);
            const float u4v[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) { const float g = v[4 * k + e]; v[4 * k + e] = (g / (1.0f + expf(-g))) * u4v[e]; }
        }
    }
    int8_t *qs = (int8_t *)out + m * K + sb * 256;
    float *d = (float *)(out + M * K) + m * nsb + sb;
    int16_t *bs = (int16_t *)(out + M * K + M * nsb * 4) + m * (K / 16) + sb * 16;
    if (valid) q8k_quant16(v, l16, qs, d, bs);
}

// Q8_0 (AVX2 semantics): 8 lanes per 32-block, 4 elements per lane.
// S1: Q8_1 (quantize_row_q8_1's AVX2 branch, ggml-quants.c:1280-1330): the same qs / d plus s = f16(d * sum qs)
// TA: the KT_Q8_0_TA layout of the same values (the activation of KT_Q8_0_T weights)
template <bool S1, bool TA = false>
__global__ void k_quant_q80(const float *__restrict__ x, int64_t ldx, uint8_t *__restrict__ out, int64_t K, int64_t M) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nb = K / 32;
    const int64_t blk = t >> 3;
    const int sub = t & 7;
    const bool valid = blk < nb * M;
    const int64_t m = valid ? blk / nb : 0, ib = valid ? blk % nb : 0;
    float4 v = valid ? *(const float4 *)(x + m * ldx + ib * 32 + sub * 4) : make_float4(0, 0, 0, 0);
    float am = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    am = fmaxf(am, __shfl_xor(am, 4, 64));
    const float d = am / 127.f;
    const float id = (am != 0.0f) ? 127.f / am : 0.0f;
    float xs[4] = {v.x, v.y, v.z, v.w};
    int q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        float r = rintf(__fmul_rn(xs[e], id));
        int iv = (int)r;
        q[e] = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
    }
    int s = q[0] + q[1] + q[2] + q[3];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (!valid) return;
    if (TA) {          // KT_Q8_0_TA (kcpp_common.h): lane sub holds bytes 4 sub .. + 3 of the block = half sub / 4
        const int64_t g = m >> 5, tok = m & 31, ng = (M + 31) / 32;
        const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
        *(int *)((int8_t *)out + (g * nb + ib) * 1024 + (sub >> 2) * 512 + tok * 16 + 4 * (sub & 3)) = packed;
        if (sub == 0) ((float *)(out + ng * 32 * K))[(g * nb + ib) * 32 + tok] = h2f(f2h(d));
        return;
    }
    const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    ((int *)((int8_t *)out + m * K + ib * 32))[sub] = packed;
    if (sub == 0) {
        ((float *)(out + M * K))[m * nb + ib] = h2f(f2h(d));        // the dot uses GGML_FP16_TO_FP32(y.d)
        ((int16_t *)(out + M * K + M * nb * 4))[m * nb + ib] = (int16_t)s;
        if constexpr (S1) {
            // the f32 product, rounded, THEN f16: without the barrier the compiler folds mul + cvt into one
            // v_fma_mix (a single rounding of the exact product), which differs from the CPU on f16 ties
            float p = __fmul_rn(d, (float)s);
            asm volatile("" : "+v"(p));
            ((float *)(out + M * K + M * nb * 4 + ((M * nb * 2 + 3) & ~(int64_t)3)))[m * nb + ib] = h2f(f2h(p));
        }
    }
}

// ---------------------------------------------------------------- host launchers
extern "C" {

int kcpp_weight_repack(int type, const void *src_ggml, void *dst_kcpp, int64_t K, int64_t N, int to_ggml, void *stream) {
    const int64_t nb = kl_nblocks(type, K, N);
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(k_repack, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, (hipStream_t)stream, type,
                       (const uint8_t *)src_ggml, (uint8_t *)dst_kcpp, nb, K / ks_block_elems(type), to_ggml);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_weight_synth_rows(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, int64_t row0,
                           void *stream) {
    const int64_t nb = kl_nblocks(type, K, N);
    if (nb <= 0) return 0;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, (hipStream_t)stream, type, seed, tid,
                       (uint8_t *)dst, nb, K / ks_block_elems(type), row0 * (K / ks_block_elems(type)));
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_weight_synth(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, void *stream) {
    return kcpp_weight_synth_rows(type, seed, tid, dst, K, N, 0, stream);
}

int kcpp_dequantize(int type, const void *w, float *y, int64_t K, int64_t N, void *stream) {
    const int64_t nb = kl_nblocks(type, K, N);
    switch (type) {
#define KCPP_IQ_DEQ(T)                                                                                             \
    case T:                                                                                                        \
        hipLaunchKernelGGL(k_dequant_iq<T>, dim3((unsigned)((8 * nb + 127) / 128)), dim3(128), 0, (hipStream_t)stream, \
                           (const uint8_t *)w, y, 8 * nb);                                                         \
        KCPP_CHECK(hipGetLastError());                                                                             \
        return 0;
        KCPP_IQ_CASES(KCPP_IQ_DEQ)
#undef KCPP_IQ_DEQ
    default: break;
    }
    hipLaunchKernelGGL(k_dequant, dim3((unsigned)((nb + 127) / 128)), dim3(128), 0, (hipStream_t)stream, type,
                       (const uint8_t *)w, y, nb, K / ks_block_elems(type));
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_quantize_act(int vtype, const float *x, int64_t ldx, void *out, int64_t K, int64_t M, void *stream) {
    if (vtype == KT_Q8_K) {
        if (K % 256) return -1;
        const int64_t nthr = K / 16 * M;
        hipLaunchKernelGGL(k_quant_q8k<false>, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                           ldx, (uint8_t *)out, K, M, (int64_t)0);
    } else if (vtype == KT_Q8_0) {
        if (K % 32) return -1;
        const int64_t nthreads = K / 32 * M * 8;
        hipLaunchKernelGGL(k_quant_q80<false>, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                           ldx, (uint8_t *)out, K, M);
    } else if (vtype == KT_Q8_0_TA) {
        if (K % 32) return -1;
        const int64_t nthreads = K / 32 * M * 8;
        hipLaunchKernelGGL((k_quant_q80<false, true>), dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, x, ldx, (uint8_t *)out, K, M);
    } else if (vtype == KT_Q8_1) {
        if (K % 32) return -1;
        const int64_t nthreads = K / 32 * M * 8;
        hipLaunchKernelGGL(k_quant_q80<true>, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                           ldx, (uint8_t *)out, K, M);
    } else {
        return -2;
    }
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_quantize_act_glu(const float *x, int64_t ldx, int64_t uoff, void *out, int64_t K, int64_t M, void *stream) {
    if (K % 256) return -1;
    const int64_t nthr = K / 16 * M;
    hipLaunchKernelGGL(k_quant_q8k<true>, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                       (uint8_t *)out, K, M, uoff);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_get_rows(int type, const void *w, int64_t K, int64_t N, const int32_t *ids, int64_t T, float *y, int64_t ldy,
                  void *stream) {
    if (type == KT_Q4_K_RS || type == KT_Q5_K_RS || type == KT_Q6_K_RS || type == KT_Q8_0_T) return -2;
    switch (type) {
#define KCPP_IQ_ROWS(TT)                                                                                            \
    case TT:                                                                                                        \
        if (K % 256) return -1;                                                                                    \
        hipLaunchKernelGGL(k_get_rows_iq<TT>, dim3((unsigned)((K / 32 + 127) / 128), (unsigned)T), dim3(128), 0,    \
                           (hipStream_t)stream, (const uint8_t *)w, K, N, ids, y, ldy);                            \
        KCPP_CHECK(hipGetLastError());                                                                             \
        return 0;
        KCPP_IQ_CASES(KCPP_IQ_ROWS)
#undef KCPP_IQ_ROWS
    default: break;
    }
    hipLaunchKernelGGL(k_get_rows, dim3((unsigned)((K + 255) / 256), (unsigned)T), dim3(256), 0, (hipStream_t)stream, type,
                       (const uint8_t *)w, K, N, ids, y, ldy);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int64_t kcpp_act_bytes(int wtype, int64_t K, int64_t M) { return act_bytes(vec_dot_type(wtype), K, M); }
int kcpp_vec_dot_type(int wtype) { return vec_dot_type(wtype); }

}  // extern "C"
