/*
 * ggml_oracle.c -- TEST INFRASTRUCTURE ONLY (see ggml_oracle.h).
 *
 * Plain-C restatement of the reference CPU ggml semantics on the Llama
 * token-generation path.  Each function cites the reference file:line it follows.
 * Never linked into the product library; imported only by tests/, smoke() and the
 * cpu_baseline leg of bench.py.
 */
#include "ggml_oracle.h"
#include "../include/kcpp_synth.h"

#include <immintrin.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define QK_K 256

typedef struct { uint16_t d; uint8_t qs[16]; } blk_q4_0;                  /* ggml-common.h:144 */
typedef struct { uint16_t d; uint8_t qh[4]; uint8_t qs[16]; } blk_q5_0;   /* ggml-common.h:161 */
typedef struct { uint16_t d, m; uint8_t qs[16]; } blk_q4_1;               /* ggml-common.h:149 */
typedef struct { uint16_t d, m; uint8_t qh[4]; uint8_t qs[16]; } blk_q5_1; /* ggml-common.h:168 */
typedef struct { uint16_t d, s; int8_t qs[32]; } blk_q8_1;                 /* ggml-common.h:193 */
typedef struct { uint16_t d; int8_t qs[32]; } blk_q8_0;                   /* ggml-common.h:186 */
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } blk_q4_K;   /* :286 */
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; } blk_q5_K; /* :303 */
typedef struct { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; } blk_q6_K;       /* :321 */
typedef struct { uint8_t hmask[32]; uint8_t qs[64]; uint8_t scales[12]; uint16_t d; } blk_q3_K;    /* :267 */
typedef struct { uint8_t scales[16]; uint8_t qs[64]; uint16_t d, dmin; } blk_q2_K;                 /* :250 */
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } blk_q8_K;  /* :330 */
typedef struct { uint16_t d; uint8_t qs[16]; } blk_iq4_nl;                                            /* :407 */
typedef struct { uint16_t d; uint16_t scales_h; uint8_t scales_l[4]; uint8_t qs[128]; } blk_iq4_xs;  /* :413 */

/* the IQ1/IQ2/IQ3 grid formats (ggml-common.h:340-405) */
typedef struct { uint16_t d; uint16_t qs[32]; } blk_iq2_xxs;
typedef struct { uint16_t d; uint16_t qs[32]; uint8_t scales[8]; } blk_iq2_xs;
typedef struct { uint16_t d; uint8_t qs[64]; uint8_t qh[8]; uint8_t scales[8]; } blk_iq2_s;
typedef struct { uint16_t d; uint8_t qs[96]; } blk_iq3_xxs;
typedef struct { uint16_t d; uint8_t qs[64]; uint8_t qh[8]; uint8_t signs[32]; uint8_t scales[4]; } blk_iq3_s;
typedef struct { uint16_t d; uint8_t qs[32]; uint16_t qh[8]; } blk_iq1_s;
typedef struct { uint8_t qs[32]; uint8_t qh[16]; uint8_t scales[8]; } blk_iq1_m;
_Static_assert(sizeof(blk_iq2_xxs) == 66 && sizeof(blk_iq2_xs) == 74 && sizeof(blk_iq2_s) == 82, "iq2");
_Static_assert(sizeof(blk_iq3_xxs) == 98 && sizeof(blk_iq3_s) == 110, "iq3");
_Static_assert(sizeof(blk_iq1_s) == 50 && sizeof(blk_iq1_m) == 56, "iq1");
/* the code books, recovered from the reference's dequantization by tools/gen_iq_grids.py */
#include "../koboldcpp_amd/csrc/iq_grids.h"
#define G2XXS(i) ((const uint8_t *)(kcpp_iq2xxs_grid + 2 * (i)))
#define G2XS(i) ((const uint8_t *)(kcpp_iq2xs_grid + 2 * (i)))
#define G2S(i) ((const uint8_t *)(kcpp_iq2s_grid + 2 * (i)))
#define G3XXS(i) ((const uint8_t *)(kcpp_iq3xxs_grid + (i)))
#define G3S(i) ((const uint8_t *)(kcpp_iq3s_grid + (i)))
#define G1S(i) ((const int8_t *)(kcpp_iq1s_grid + 2 * (i)))
/* ksigns_iq2xs (ggml-common.h): 7 sign bits plus the even-parity 8th */
static inline int ksign(int i) { return i | ((__builtin_popcount(i) & 1) << 7); }
#define IQ1_DELTA 0.125f         /* IQ1S_DELTA / IQ1M_DELTA, ggml-common.h */

/* the IQ4_NL / IQ4_XS non-linear code book, ggml-quants.c:3741 */
static const int8_t kvalues_iq4nl[16] = {-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113};

_Static_assert(sizeof(blk_q4_0) == 18, "q4_0");
_Static_assert(sizeof(blk_q5_0) == 22, "q5_0");
_Static_assert(sizeof(blk_q4_1) == 20 && sizeof(blk_q5_1) == 24 && sizeof(blk_q8_1) == 36, "q4_1 / q5_1 / q8_1");
_Static_assert(sizeof(blk_q8_0) == 34, "q8_0");
_Static_assert(sizeof(blk_q4_K) == 144, "q4_K");
_Static_assert(sizeof(blk_q5_K) == 176, "q5_K");
_Static_assert(sizeof(blk_q6_K) == 210, "q6_K");
_Static_assert(sizeof(blk_q3_K) == 110, "q3_K");
_Static_assert(sizeof(blk_q2_K) == 84, "q2_K");
_Static_assert(sizeof(blk_q8_K) == 292, "q8_K");
_Static_assert(sizeof(blk_iq4_nl) == 18 && sizeof(blk_iq4_xs) == 136, "iq4_nl / iq4_xs");

float orc_fp16_to_fp32(uint16_t h) { return _cvtsh_ss(h); }
uint16_t orc_fp32_to_fp16(float f) { return _cvtss_sh(f, 0); }
#define H2F orc_fp16_to_fp32
#define F2H orc_fp32_to_fp16

/* get_scale_min_k4, ggml-quants.c:1899-1906 */
static inline void scale_min_k4(int j, const uint8_t *q, uint8_t *d, uint8_t *m) {
    if (j < 4) { *d = q[j] & 63; *m = q[j + 4] & 63; }
    else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

int64_t orc_row_bytes(int type, int64_t k) {
    return k / ks_block_elems(type) * ks_block_bytes(type);
}

/* the 16 6-bit Q3_K scales (unsigned, biased by 32) from the 12 packed bytes (dequantize_row_q3_K's aux shuffle,
 * ggml-quants.c:2346-2351) */
static void q3k_scales(const uint8_t *s12, int8_t *sc) {
    uint32_t aux[4];
    memcpy(aux, s12, 12);
    const uint32_t kmask1 = 0x03030303u, kmask2 = 0x0f0f0f0fu, tmp = aux[2];
    aux[2] = ((aux[0] >> 4) & kmask2) | (((tmp >> 4) & kmask1) << 4);
    aux[3] = ((aux[1] >> 4) & kmask2) | (((tmp >> 6) & kmask1) << 4);
    aux[0] = (aux[0] & kmask2) | (((tmp >> 0) & kmask1) << 4);
    aux[1] = (aux[1] & kmask2) | (((tmp >> 2) & kmask1) << 4);
    memcpy(sc, aux, 16);
}

void orc_dequantize_row(int type, const void *vx, float *y, int64_t k) {
    switch (type) {
    case KT_F32: memcpy(y, vx, k * 4); return;
    case KT_F16: { const uint16_t *x = vx; for (int64_t i = 0; i < k; ++i) y[i] = H2F(x[i]); } return;
    case KT_Q4_0: {                                   /* ggml-quants.c:1523-1540 */
        const blk_q4_0 *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d);
            for (int j = 0; j < 16; ++j) {
                y[i * 32 + j] = ((x[i].qs[j] & 0x0F) - 8) * d;
                y[i * 32 + j + 16] = ((x[i].qs[j] >> 4) - 8) * d;
            }
        }
    } return;
    case KT_Q4_1: {                                   /* ggml-quants.c:1543-1562 */
        const blk_q4_1 *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d), m = H2F(x[i].m);
            for (int j = 0; j < 16; ++j) {
                y[i * 32 + j] = (x[i].qs[j] & 0x0F) * d + m;
                y[i * 32 + j + 16] = (x[i].qs[j] >> 4) * d + m;
            }
        }
    } return;
    case KT_Q5_1: {                                   /* ggml-quants.c:1590-1616 */
        const blk_q5_1 *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d), m = H2F(x[i].m);
            uint32_t qh;
            memcpy(&qh, x[i].qh, 4);
            for (int j = 0; j < 16; ++j) {
                y[i * 32 + j] = ((x[i].qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10)) * d + m;
                y[i * 32 + j + 16] = ((x[i].qs[j] >> 4) | ((qh >> (j + 12)) & 0x10)) * d + m;
            }
        }
    } return;
    case KT_Q5_0: {                                   /* ggml-quants.c:1564-1588 */
        const blk_q5_0 *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d);
            uint32_t qh;
            memcpy(&qh, x[i].qh, 4);
            for (int j = 0; j < 16; ++j) {
                const int x0 = ((x[i].qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10)) - 16;
                const int x1 = ((x[i].qs[j] >> 4) | ((qh >> (j + 12)) & 0x10)) - 16;
                y[i * 32 + j] = x0 * d;
                y[i * 32 + j + 16] = x1 * d;
            }
        }
    } return;
    case KT_IQ4_NL: {                                 /* dequantize_row_iq4_nl, ggml-quants.c:3743-3759 */
        const blk_iq4_nl *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d);
            for (int j = 0; j < 16; ++j) {
                y[i * 32 + j] = d * kvalues_iq4nl[x[i].qs[j] & 0xf];
                y[i * 32 + j + 16] = d * kvalues_iq4nl[x[i].qs[j] >> 4];
            }
        }
    } return;
    case KT_IQ4_XS: {                                 /* dequantize_row_iq4_xs, ggml-quants.c:3761-3782 */
        const blk_iq4_xs *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            const uint8_t *qs = x[i].qs;
            for (int ib = 0; ib < QK_K / 32; ++ib) {
                const int ls = ((x[i].scales_l[ib / 2] >> 4 * (ib % 2)) & 0xf) | (((x[i].scales_h >> 2 * ib) & 3) << 4);
                const float dl = d * (ls - 32);
                for (int j = 0; j < 16; ++j) {
                    y[i * QK_K + 32 * ib + j] = dl * kvalues_iq4nl[qs[j] & 0xf];
                    y[i * QK_K + 32 * ib + j + 16] = dl * kvalues_iq4nl[qs[j] >> 4];
                }
                qs += 16;
            }
        }
    } return;
    case KT_IQ2_XXS: {                                /* dequantize_row_iq2_xxs, ggml-quants.c:3504-3528 */
        const blk_iq2_xxs *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                uint32_t a[2];
                memcpy(a, x[i].qs + 4 * ib, 8);
                const float db = d * (0.5f + (a[1] >> 28)) * 0.25f;
                for (int l = 0; l < 4; ++l) {
                    const uint8_t *g = G2XXS(((const uint8_t *)a)[l]);
                    const int sg = ksign((a[1] >> 7 * l) & 127);
                    for (int j = 0; j < 8; ++j) *y++ = db * g[j] * (sg & (1 << j) ? -1.f : 1.f);
                }
            }
        }
    } return;
    case KT_IQ2_XS: {                                 /* dequantize_row_iq2_xs, ggml-quants.c:3532-3555 */
        const blk_iq2_xs *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                const float db[2] = {d * (0.5f + (x[i].scales[ib] & 0xf)) * 0.25f, d * (0.5f + (x[i].scales[ib] >> 4)) * 0.25f};
                for (int l = 0; l < 4; ++l) {
                    const uint16_t q = x[i].qs[4 * ib + l];
                    const uint8_t *g = G2XS(q & 511);
                    const int sg = ksign(q >> 9);
                    for (int j = 0; j < 8; ++j) *y++ = db[l / 2] * g[j] * (sg & (1 << j) ? -1.f : 1.f);
                }
            }
        }
    } return;
    case KT_IQ2_S: {                                  /* dequantize_row_iq2_s, ggml-quants.c:3559-3587 */
        const blk_iq2_s *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                const float db[2] = {d * (0.5f + (x[i].scales[ib] & 0xf)) * 0.25f, d * (0.5f + (x[i].scales[ib] >> 4)) * 0.25f};
                for (int l = 0; l < 4; ++l) {
                    const uint8_t *g = G2S(x[i].qs[4 * ib + l] | ((x[i].qh[ib] << (8 - 2 * l)) & 0x300));
                    const int sg = x[i].qs[32 + 4 * ib + l];
                    for (int j = 0; j < 8; ++j) *y++ = db[l / 2] * g[j] * (sg & (1 << j) ? -1.f : 1.f);
                }
            }
        }
    } return;
    case KT_IQ3_XXS: {                                /* dequantize_row_iq3_xxs, ggml-quants.c:3591-3619 */
        const blk_iq3_xxs *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                uint32_t a;
                memcpy(&a, x[i].qs + 64 + 4 * ib, 4);
                const float db = d * (0.5f + (a >> 28)) * 0.5f;
                for (int l = 0; l < 4; ++l) {
                    const int sg = ksign((a >> 7 * l) & 127);
                    const uint8_t *g1 = G3XXS(x[i].qs[8 * ib + 2 * l]), *g2 = G3XXS(x[i].qs[8 * ib + 2 * l + 1]);
                    for (int j = 0; j < 4; ++j) {
                        y[j] = db * g1[j] * (sg & (1 << j) ? -1.f : 1.f);
                        y[j + 4] = db * g2[j] * (sg & (1 << (j + 4)) ? -1.f : 1.f);
                    }
                    y += 8;
                }
            }
        }
    } return;
    case KT_IQ3_S: {                                  /* dequantize_row_iq3_s, ggml-quants.c:3623-3662 */
        const blk_iq3_s *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                const int sc = ib & 1 ? x[i].scales[ib / 2] >> 4 : x[i].scales[ib / 2] & 0xf;
                const float db = d * (1 + 2 * sc);
                const uint8_t *qs = x[i].qs + 8 * ib, *sg = x[i].signs + 4 * ib;
                const int qh = x[i].qh[ib];
                for (int l = 0; l < 4; ++l) {
                    const uint8_t *g1 = G3S(qs[2 * l] | ((qh << (8 - 2 * l)) & 256));
                    const uint8_t *g2 = G3S(qs[2 * l + 1] | ((qh << (7 - 2 * l)) & 256));
                    for (int j = 0; j < 4; ++j) {
                        y[j] = db * g1[j] * (sg[l] & (1 << j) ? -1.f : 1.f);
                        y[j + 4] = db * g2[j] * (sg[l] & (1 << (j + 4)) ? -1.f : 1.f);
                    }
                    y += 8;
                }
            }
        }
    } return;
    case KT_IQ1_S: {                                  /* dequantize_row_iq1_s, ggml-quants.c:3666-3689 */
        const blk_iq1_s *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            for (int ib = 0; ib < 8; ++ib) {
                const int qh = x[i].qh[ib];
                const float dl = d * (2 * ((qh >> 12) & 7) + 1);
                const float delta = qh & 0x8000 ? -IQ1_DELTA : IQ1_DELTA;
                for (int l = 0; l < 4; ++l) {
                    const int8_t *g = G1S(x[i].qs[4 * ib + l] | (((qh >> 3 * l) & 7) << 8));
                    for (int j = 0; j < 8; ++j) *y++ = dl * (g[j] + delta);
                }
            }
        }
    } return;
    case KT_IQ1_M: {                                  /* dequantize_row_iq1_m, ggml-quants.c:3691-3739 */
        const blk_iq1_m *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            uint16_t sc[4];
            memcpy(sc, x[i].scales, 8);
            const float d = H2F((uint16_t)((sc[0] >> 12) | ((sc[1] >> 8) & 0x00f0) | ((sc[2] >> 4) & 0x0f00) | (sc[3] & 0xf000)));
            for (int ib = 0; ib < 8; ++ib) {
                const uint8_t *qs = x[i].qs + 4 * ib, *qh = x[i].qh + 2 * ib;
                const float dl1 = d * (2 * ((sc[ib / 2] >> (6 * (ib % 2) + 0)) & 7) + 1);
                const float dl2 = d * (2 * ((sc[ib / 2] >> (6 * (ib % 2) + 3)) & 7) + 1);
                const int idx[4] = {qs[0] | ((qh[0] << 8) & 0x700), qs[1] | ((qh[0] << 4) & 0x700),
                                    qs[2] | ((qh[1] << 8) & 0x700), qs[3] | ((qh[1] << 4) & 0x700)};
                const float delta[4] = {qh[0] & 0x08 ? -IQ1_DELTA : IQ1_DELTA, qh[0] & 0x80 ? -IQ1_DELTA : IQ1_DELTA,
                                        qh[1] & 0x08 ? -IQ1_DELTA : IQ1_DELTA, qh[1] & 0x80 ? -IQ1_DELTA : IQ1_DELTA};
                for (int l = 0; l < 4; ++l) {
                    const int8_t *g = G1S(idx[l]);
                    for (int j = 0; j < 8; ++j) *y++ = (l < 2 ? dl1 : dl2) * (g[j] + delta[l]);
                }
            }
        }
    } return;
    case KT_Q8_0: {                                   /* ggml-quants.c:1617-1631 */
        const blk_q8_0 *x = vx;
        for (int64_t i = 0; i < k / 32; ++i) {
            const float d = H2F(x[i].d);
            for (int j = 0; j < 32; ++j) y[i * 32 + j] = x[i].qs[j] * d;
        }
    } return;
    case KT_Q4_K: {                                   /* ggml-quants.c:2556-2578 */
        const blk_q4_K *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const uint8_t *q = x[i].qs;
            const float d = H2F(x[i].d), min = H2F(x[i].dmin);
            int is = 0; uint8_t sc, m;
            for (int j = 0; j < QK_K; j += 64) {
                scale_min_k4(is + 0, x[i].scales, &sc, &m);
                const float d1 = d * sc, m1 = min * m;
                scale_min_k4(is + 1, x[i].scales, &sc, &m);
                const float d2 = d * sc, m2 = min * m;
                for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
                q += 32; is += 2;
            }
        }
    } return;
    case KT_Q5_K: {                                   /* ggml-quants.c:2764-2790 */
        const blk_q5_K *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const uint8_t *ql = x[i].qs, *qh = x[i].qh;
            const float d = H2F(x[i].d), min = H2F(x[i].dmin);
            int is = 0; uint8_t sc, m, u1 = 1, u2 = 2;
            for (int j = 0; j < QK_K; j += 64) {
                scale_min_k4(is + 0, x[i].scales, &sc, &m);
                const float d1 = d * sc, m1 = min * m;
                scale_min_k4(is + 1, x[i].scales, &sc, &m);
                const float d2 = d * sc, m2 = min * m;
                for (int l = 0; l < 32; ++l) *y++ = d1 * ((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * ((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)) - m2;
                ql += 32; is += 2; u1 <<= 2; u2 <<= 2;
            }
        }
    } return;
    case KT_Q2_K: {                                   /* ggml-quants.c:2251-2282 */
        const blk_q2_K *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d), min = H2F(x[i].dmin);
            const uint8_t *q = x[i].qs;
            int is = 0;
            for (int n = 0; n < QK_K; n += 128) {
                int shift = 0;
                for (int j = 0; j < 4; ++j) {
                    uint8_t sc = x[i].scales[is++];
                    float dl = d * (sc & 0xF), ml = min * (sc >> 4);
                    for (int l = 0; l < 16; ++l) *y++ = dl * ((int8_t)((q[l] >> shift) & 3)) - ml;
                    sc = x[i].scales[is++];
                    dl = d * (sc & 0xF); ml = min * (sc >> 4);
                    for (int l = 0; l < 16; ++l) *y++ = dl * ((int8_t)((q[l + 16] >> shift) & 3)) - ml;
                    shift += 2;
                }
                q += 32;
            }
        }
    } return;
    case KT_Q3_K: {                                   /* ggml-quants.c:2328-2376 */
        const blk_q3_K *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d_all = H2F(x[i].d);
            int8_t sc[16];
            q3k_scales(x[i].scales, sc);
            const uint8_t *q = x[i].qs, *hm = x[i].hmask;
            uint8_t m = 1;
            int is = 0;
            for (int n = 0; n < QK_K; n += 128) {
                int shift = 0;
                for (int j = 0; j < 4; ++j) {
                    float dl = d_all * (sc[is++] - 32);
                    for (int l = 0; l < 16; ++l) *y++ = dl * ((int8_t)((q[l] >> shift) & 3) - ((hm[l] & m) ? 0 : 4));
                    dl = d_all * (sc[is++] - 32);
                    for (int l = 0; l < 16; ++l) *y++ = dl * ((int8_t)((q[l + 16] >> shift) & 3) - ((hm[l + 16] & m) ? 0 : 4));
                    shift += 2;
                    m <<= 1;
                }
                q += 32;
            }
        }
    } return;
    case KT_Q6_K: {                                   /* ggml-quants.c:2978-3006 */
        const blk_q6_K *x = vx;
        for (int64_t i = 0; i < k / QK_K; ++i) {
            const float d = H2F(x[i].d);
            const uint8_t *ql = x[i].ql, *qh = x[i].qh;
            const int8_t *sc = x[i].scales;
            for (int n = 0; n < QK_K; n += 128) {
                for (int l = 0; l < 32; ++l) {
                    int is = l / 16;
                    const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    y[l + 0] = d * sc[is + 0] * q1;
                    y[l + 32] = d * sc[is + 2] * q2;
                    y[l + 64] = d * sc[is + 4] * q3;
                    y[l + 96] = d * sc[is + 6] * q4;
                }
                y += 128; ql += 64; qh += 32; sc += 8;
            }
        }
    } return;
    default: abort();
    }
}

/* type_traits[..].vec_dot_type, ggml.c:793-959 */
int orc_vec_dot_type(int wtype) {
    switch (wtype) {
        case KT_Q4_0: case KT_Q5_0: case KT_Q8_0: case KT_IQ4_NL: return KT_Q8_0;   /* ggml.c:1053 */
        case KT_IQ4_XS: return KT_Q8_K;                                             /* ggml.c:1065 */
        case KT_IQ2_XXS: case KT_IQ2_XS: case KT_IQ2_S: case KT_IQ3_XXS: case KT_IQ3_S:
        case KT_IQ1_S: case KT_IQ1_M: return KT_Q8_K;                               /* ggml.c:985-1076 */
        case KT_Q4_1: case KT_Q5_1: return KT_Q8_1;
        case KT_Q2_K: case KT_Q3_K: case KT_Q4_K: case KT_Q5_K: case KT_Q6_K: return KT_Q8_K;
        case KT_F16: return KT_F16;
        default: return KT_F32;
    }
}

/* nearest_int, ggml-quants.c:1640-1645 */
static inline int nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i; memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

/* quantize_row_q8_K_ref, ggml-quants.c:3786-3823 */
void orc_quantize_row_q8_K(const float *x, void *vy, int64_t k) {
    blk_q8_K *y = vy;
    for (int64_t i = 0; i < k / QK_K; ++i) {
        float max = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; max = x[j]; }
        }
        if (!amax) {
            y[i].d = 0; memset(y[i].qs, 0, QK_K); memset(y[i].bsums, 0, sizeof(y[i].bsums));
            x += QK_K; continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            int v = nearest_int(iscale * x[j]);
            y[i].qs[j] = v < 127 ? v : 127;
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = sum;
        }
        y[i].d = 1 / iscale;
        x += QK_K;
    }
}

/* quantize_row_q8_0, AVX2 branch ggml-quants.c:940-1000 */
void orc_quantize_row_q8_0(const float *x, void *vy, int64_t k) {
    blk_q8_0 *y = vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0;
        for (int j = 0; j < 32; ++j) { float a = fabsf(x[i * 32 + j]); amax = a > amax ? a : amax; }
        const float d = amax / 127.f;
        y[i].d = F2H(d);
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        for (int j = 0; j < 32; ++j) {
            float v = nearbyintf(x[i * 32 + j] * id);   /* _MM_ROUND_NEAREST: half-to-even */
            int iv = (int)v;
            y[i].qs[j] = (int8_t)(iv > 127 ? 127 : (iv < -128 ? -128 : iv));
        }
    }
}

/* quantize_row_q8_1 (AVX2 branch, ggml-quants.c:1280-1330): the Q8_0 quantization plus s = f16(d * sum qs), d unrounded */
void orc_quantize_row_q8_1(const float *x, void *vy, int64_t k) {
    blk_q8_1 *y = vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        blk_q8_0 b;
        orc_quantize_row_q8_0(x + i * 32, &b, 32);
        float amax = 0;
        for (int j = 0; j < 32; ++j) { float a = fabsf(x[i * 32 + j]); amax = a > amax ? a : amax; }
        const float d = amax / 127.f;
        int sum = 0;
        for (int j = 0; j < 32; ++j) { y[i].qs[j] = b.qs[j]; sum += b.qs[j]; }
        y[i].d = b.d;
        y[i].s = F2H(d * (float)sum);
    }
}

/* quantize_row_q4_0_ref, ggml-quants.c:669-704 (quantize_row_q4_0 calls it, :707) */
void orc_quantize_row_q4_0(const float *x, void *vy, int64_t k) {
    blk_q4_0 *y = vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < 32; ++j) {
            const float v = x[i * 32 + j];
            if (amax < fabsf(v)) { amax = fabsf(v); max = v; }
        }
        const float d = max / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = F2H(d);
        for (int j = 0; j < 16; ++j) {
            const float x0 = x[i * 32 + j] * id, x1 = x[i * 32 + 16 + j] * id;
            const int8_t a = (int8_t)(x0 + 8.5f), b = (int8_t)(x1 + 8.5f);
            const uint8_t xi0 = a < 15 ? a : 15, xi1 = b < 15 ? b : 15;
            y[i].qs[j] = xi0 | (uint8_t)(xi1 << 4);
        }
    }
}

void orc_quantize_row(int vtype, const float *x, void *y, int64_t k) {
    switch (vtype) {
        case KT_Q4_0: orc_quantize_row_q4_0(x, y, k); break;
        case KT_Q8_K: orc_quantize_row_q8_K(x, y, k); break;
        case KT_Q8_0: orc_quantize_row_q8_0(x, y, k); break;
        case KT_Q8_1: orc_quantize_row_q8_1(x, y, k); break;
        case KT_F16: { uint16_t *h = y; for (int64_t i = 0; i < k; ++i) h[i] = F2H(x[i]); } break;
        case KT_F32: memcpy(y, x, k * 4); break;
        default: abort();
    }
}

/* ---------------- dot products (scalar restatement of ggml-quants.c) ---------------- */

static float dot_q4_K(int n, const blk_q4_K *x, const blk_q8_K *y) {       /* :7714, scalar :8223 */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        int sumi = 0, summ = 0;
        for (int j = 0; j < 8; ++j) {
            uint8_t sc, m;
            scale_min_k4(j, x[i].scales, &sc, &m);
            const uint8_t *q4 = x[i].qs + 32 * (j / 2);
            const int8_t *q8 = y[i].qs + 32 * j;
            int dot = 0;
            for (int l = 0; l < 32; ++l) dot += ((j & 1) ? (q4[l] >> 4) : (q4[l] & 0xF)) * q8[l];
            sumi += sc * dot;
            summ += m * (y[i].bsums[2 * j] + y[i].bsums[2 * j + 1]);
        }
        const float d = y[i].d * H2F(x[i].d);
        const float dmin = y[i].d * H2F(x[i].dmin);
        sumf += d * (float)sumi;
        sumf -= dmin * (float)summ;
    }
    return sumf;
}

static float dot_q5_K(int n, const blk_q5_K *x, const blk_q8_K *y) {       /* :8282 */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        int sumi = 0, summ = 0;
        for (int j = 0; j < 8; ++j) {
            uint8_t sc, m;
            scale_min_k4(j, x[i].scales, &sc, &m);
            const uint8_t *q4 = x[i].qs + 32 * (j / 2);
            const int8_t *q8 = y[i].qs + 32 * j;
            int dot = 0;
            for (int l = 0; l < 32; ++l) {
                int v = ((j & 1) ? (q4[l] >> 4) : (q4[l] & 0xF)) + ((x[i].qh[l] >> j) & 1) * 16;
                dot += v * q8[l];
            }
            sumi += sc * dot;
            summ += m * (y[i].bsums[2 * j] + y[i].bsums[2 * j + 1]);
        }
        const float d = y[i].d * H2F(x[i].d);
        const float dmin = y[i].d * H2F(x[i].dmin);
        sumf += d * (float)sumi;
        sumf -= dmin * (float)summ;
    }
    return sumf;
}

static float dot_q6_K(int n, const blk_q6_K *x, const blk_q8_K *y) {       /* :8919, scalar ~:9530 */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        int8_t a[QK_K];
        const uint8_t *q4 = x[i].ql, *qh = x[i].qh;
        int8_t *pa = a;
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                pa[l + 0] = (int8_t)((q4[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                pa[l + 32] = (int8_t)((q4[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                pa[l + 64] = (int8_t)((q4[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                pa[l + 96] = (int8_t)((q4[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
            pa += 128; q4 += 64; qh += 32;
        }
        int sumi = 0;
        for (int g = 0; g < 16; ++g) {
            int dot = 0;
            for (int l = 0; l < 16; ++l) dot += a[g * 16 + l] * y[i].qs[g * 16 + l];
            sumi += x[i].scales[g] * dot;
        }
        sumf += H2F(x[i].d) * y[i].d * (float)sumi;
    }
    return sumf;
}

static float dot_q2_K(int n, const blk_q2_K *x, const blk_q8_K *y) {       /* :6448, scalar branch */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const uint8_t *q2 = x[i].qs, *sc = x[i].scales;
        const int8_t *q8 = y[i].qs;
        int summs = 0;
        for (int j = 0; j < 16; ++j) summs += y[i].bsums[j] * (sc[j] >> 4);
        const float dall = y[i].d * H2F(x[i].d), dmin = y[i].d * H2F(x[i].dmin);
        int isum = 0, is = 0;
        for (int k = 0; k < QK_K / 128; ++k) {
            for (int shift = 0; shift < 8; shift += 2) {
                int d = sc[is++] & 0xF, isuml = 0;
                for (int l = 0; l < 16; ++l) isuml += q8[l] * ((q2[l] >> shift) & 3);
                isum += d * isuml;
                d = sc[is++] & 0xF;
                isuml = 0;
                for (int l = 16; l < 32; ++l) isuml += q8[l] * ((q2[l] >> shift) & 3);
                isum += d * isuml;
                q8 += 32;
            }
            q2 += 32;
        }
        sumf += dall * isum - dmin * summs;
    }
    return sumf;
}

static float dot_q3_K(int n, const blk_q3_K *x, const blk_q8_K *y) {       /* :6933, scalar branch */
    float sums[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n / QK_K; ++i) {
        int8_t a[QK_K], *pa = a;
        const uint8_t *q3 = x[i].qs, *hm = x[i].hmask;
        uint8_t m = 1;
        for (int j = 0; j < QK_K; j += 128) {
            for (int sh = 0; sh < 8; sh += 2) {
                for (int l = 0; l < 32; ++l) pa[l] = (int8_t)(((q3[l] >> sh) & 3) - ((hm[l] & m) ? 0 : 4));
                pa += 32;
                m <<= 1;
            }
            q3 += 32;
        }
        int8_t sc[16];
        q3k_scales(x[i].scales, sc);
        int32_t aux32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int8_t *q8 = y[i].qs;
        pa = a;
        for (int j = 0; j < QK_K / 16; ++j)
            for (int h = 0; h < 2; ++h) {
                for (int l = 0; l < 8; ++l) aux32[l] += (sc[j] - 32) * (int16_t)(q8[l] * pa[l]);
                q8 += 8; pa += 8;
            }
        const float d = H2F(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
    }
    float sumf = 0;
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
}

static float dot_q4_0(int n, const blk_q4_0 *x, const blk_q8_0 *y) {       /* :3922, scalar tail */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        int s0 = 0, s1 = 0;
        for (int j = 0; j < 16; ++j) {
            s0 += ((x[ib].qs[j] & 0x0F) - 8) * y[ib].qs[j];
            s1 += ((x[ib].qs[j] >> 4) - 8) * y[ib].qs[j + 16];
        }
        sumf += (s0 + s1) * (H2F(x[ib].d) * H2F(y[ib].d));
    }
    return sumf;
}

static float dot_q5_0(int n, const blk_q5_0 *x, const blk_q8_0 *y) {       /* :4790, scalar tail */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        uint32_t qh;
        memcpy(&qh, x[ib].qh, 4);
        int s0 = 0, s1 = 0;
        for (int j = 0; j < 16; ++j) {
            const int x0 = ((x[ib].qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10)) - 16;
            const int x1 = ((x[ib].qs[j] >> 4) | ((qh >> (j + 12)) & 0x10)) - 16;
            s0 += x0 * y[ib].qs[j];
            s1 += x1 * y[ib].qs[j + 16];
        }
        sumf += (H2F(x[ib].d) * H2F(y[ib].d)) * (s0 + s1);
    }
    return sumf;
}

static float dot_q4_1(int n, const blk_q4_1 *x, const blk_q8_1 *y) {       /* :4503, scalar tail */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        int s0 = 0, s1 = 0;
        for (int j = 0; j < 16; ++j) {
            s0 += (x[ib].qs[j] & 0x0F) * y[ib].qs[j];
            s1 += (x[ib].qs[j] >> 4) * y[ib].qs[j + 16];
        }
        sumf += (H2F(x[ib].d) * H2F(y[ib].d)) * (s0 + s1) + H2F(x[ib].m) * H2F(y[ib].s);
    }
    return sumf;
}

static float dot_q5_1(int n, const blk_q5_1 *x, const blk_q8_1 *y) {       /* :5145, scalar tail */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        uint32_t qh;
        memcpy(&qh, x[ib].qh, 4);
        int s0 = 0, s1 = 0;
        for (int j = 0; j < 16; ++j) {
            s0 += ((x[ib].qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10)) * y[ib].qs[j];
            s1 += ((x[ib].qs[j] >> 4) | ((qh >> (j + 12)) & 0x10)) * y[ib].qs[j + 16];
        }
        sumf += (H2F(x[ib].d) * H2F(y[ib].d)) * (s0 + s1) + H2F(x[ib].m) * H2F(y[ib].s);
    }
    return sumf;
}

static float dot_q8_0(int n, const blk_q8_0 *x, const blk_q8_0 *y) {       /* :5519, scalar tail */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        int s = 0;
        for (int j = 0; j < 32; ++j) s += x[ib].qs[j] * y[ib].qs[j];
        sumf += s * (H2F(x[ib].d) * H2F(y[ib].d));
    }
    return sumf;
}

static float dot_iq4_nl(int n, const blk_iq4_nl *x, const blk_q8_0 *y) {   /* :12470, scalar tail :12660-12668 */
    float sumf = 0;
    for (int ib = 0; ib < n / 32; ++ib) {
        const float d = H2F(y[ib].d) * H2F(x[ib].d);
        int sumi1 = 0, sumi2 = 0;
        for (int j = 0; j < 16; ++j) {
            sumi1 += y[ib].qs[j] * kvalues_iq4nl[x[ib].qs[j] & 0xf];
            sumi2 += y[ib].qs[j + 16] * kvalues_iq4nl[x[ib].qs[j] >> 4];
        }
        sumf += d * (sumi1 + sumi2);
    }
    return sumf;
}

static float dot_iq4_xs(int n, const blk_iq4_xs *x, const blk_q8_K *y) {   /* :12672, scalar branch :12974-13006 */
    float sumf = 0;
    for (int ibl = 0; ibl < n / QK_K; ++ibl) {
        const float d4d8 = H2F(x[ibl].d) * y[ibl].d;
        uint16_t h = x[ibl].scales_h;
        const uint8_t *qs = x[ibl].qs;
        const int8_t *q8 = y[ibl].qs;
        for (int ib = 0; ib < QK_K / 32; ib += 2) {
            const uint8_t ls1 = (x[ibl].scales_l[ib / 2] & 0xf) | ((h << 4) & 0x30);
            const uint8_t ls2 = (x[ibl].scales_l[ib / 2] >> 4) | ((h << 2) & 0x30);
            h >>= 4;
            const float d1 = d4d8 * (ls1 - 32), d2 = d4d8 * (ls2 - 32);
            int sumi1 = 0, sumi2 = 0;
            for (int j = 0; j < 16; ++j) {
                sumi1 += q8[j] * kvalues_iq4nl[qs[j] & 0xf];
                sumi2 += q8[j + 16] * kvalues_iq4nl[qs[j] >> 4];
            }
            sumf += d1 * (sumi1 + sumi2);
            qs += 16; q8 += 32;
            sumi1 = sumi2 = 0;
            for (int j = 0; j < 16; ++j) {
                sumi1 += q8[j] * kvalues_iq4nl[qs[j] & 0xf];
                sumi2 += q8[j + 16] * kvalues_iq4nl[qs[j] >> 4];
            }
            sumf += d2 * (sumi1 + sumi2);
            qs += 16; q8 += 32;
        }
    }
    return sumf;
}

/* the grid types against Q8_K: the reference's generic branches (integer sub-block dots times the sub-block scale,
 * summed in int32 per super-block, then (d_w d_a) once per super-block, then the format's constant) */
static float dot_iq2_xxs(int n, const blk_iq2_xxs *x, const blk_q8_K *y) {  /* ggml-quants.c:9606, generic :9886-9914 */
    float sumf = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = H2F(x[i].d) * y[i].d;
        const int8_t *q8 = y[i].qs;
        int32_t bsum = 0;
        for (int ib = 0; ib < 8; ++ib) {
            uint32_t a[2];
            memcpy(a, x[i].qs + 4 * ib, 8);
            const int ls = 2 * (a[1] >> 28) + 1;
            int32_t sumi = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const uint8_t *g = G2XXS(((const uint8_t *)a)[l]);
                const int sg = ksign((a[1] >> 7 * l) & 127);
                for (int j = 0; j < 8; ++j) sumi += g[j] * q8[j] * (sg & (1 << j) ? -1 : 1);
            }
            bsum += sumi * ls;
        }
        sumf += d * bsum;
    }
    return 0.125f * sumf;
}
static float dot_iq2_xs(int n, const blk_iq2_xs *x, const blk_q8_K *y) {    /* :9917, generic branch */
    float sumf = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = H2F(x[i].d) * y[i].d;
        const int8_t *q8 = y[i].qs;
        int32_t bsum = 0;
        for (int ib = 0; ib < 8; ++ib) {
            const int ls1 = 2 * (x[i].scales[ib] & 0xf) + 1, ls2 = 2 * (x[i].scales[ib] >> 4) + 1;
            int32_t s1 = 0, s2 = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const uint16_t q = x[i].qs[4 * ib + l];
                const uint8_t *g = G2XS(q & 511);
                const int sg = ksign(q >> 9);
                int32_t t = 0;
                for (int j = 0; j < 8; ++j) t += g[j] * q8[j] * (sg & (1 << j) ? -1 : 1);
                if (l < 2) s1 += t; else s2 += t;
            }
            bsum += s1 * ls1 + s2 * ls2;
        }
        sumf += d * bsum;
    }
    return 0.125f * sumf;
}
static float dot_iq2_s(int n, const blk_iq2_s *x, const blk_q8_K *y) {      /* :10502, generic branch */
    float sumf = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = H2F(x[i].d) * y[i].d;
        const int8_t *q8 = y[i].qs;
        int32_t bsum = 0;
        for (int ib = 0; ib < 8; ++ib) {
            const int ls1 = 1 + 2 * (x[i].scales[ib] & 0xf), ls2 = 1 + 2 * (x[i].scales[ib] >> 4);
            int32_t s1 = 0, s2 = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const uint8_t *g = G2S(x[i].qs[4 * ib + l] | ((x[i].qh[ib] << (8 - 2 * l)) & 0x300));
                const int sg = x[i].qs[32 + 4 * ib + l];
                int32_t t = 0;
                for (int j = 0; j < 8; ++j) t += q8[j] * g[j] * (sg & (1 << j) ? -1 : 1);
                if (l < 2) s1 += t; else s2 += t;
            }
            bsum += ls1 * s1 + ls2 * s2;
        }
        sumf += d * bsum;
    }
    return 0.125f * sumf;
}
static float dot_iq3_xxs(int n, const blk_iq3_xxs *x, const blk_q8_K *y) { /* :10980, generic branch */
    float sumf = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = H2F(x[i].d) * y[i].d;
        const int8_t *q8 = y[i].qs;
        int32_t bsum = 0;
        for (int ib = 0; ib < 8; ++ib) {
            uint32_t a;
            memcpy(&a, x[i].qs + 64 + 4 * ib, 4);
            const int ls = 2 * (a >> 28) + 1;
            int32_t sumi = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const uint8_t *g1 = G3XXS(x[i].qs[8 * ib + 2 * l]), *g2 = G3XXS(x[i].qs[8 * ib + 2 * l + 1]);
                const int sg = ksign((a >> 7 * l) & 127);
                for (int j = 0; j < 4; ++j) {
                    sumi += g1[j] * q8[j] * (sg & (1 << j) ? -1 : 1);
                    sumi += g2[j] * q8[j + 4] * (sg & (1 << (j + 4)) ? -1 : 1);
                }
            }
            bsum += sumi * ls;
        }
        sumf += d * bsum;
    }
    return 0.25f * sumf;
}
static float dot_iq3_s(int n, const blk_iq3_s *x, const blk_q8_K *y) {     /* :11303, generic branch */
    float sumf = 0.f;
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = H2F(x[i].d) * y[i].d;
        const int8_t *q8 = y[i].qs;
        int32_t bsum = 0;
        for (int ib = 0; ib < 8; ++ib) {
            const int ls = 2 * (ib & 1 ? x[i].scales[ib / 2] >> 4 : x[i].scales[ib / 2] & 0xf) + 1;
            const uint8_t *qs = x[i].qs + 8 * ib, *sg = x[i].signs + 4 * ib;
            const int qh = x[i].qh[ib];
            int32_t sumi = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const uint8_t *g1 = G3S(qs[2 * l] | ((qh << (8 - 2 * l)) & 256));
                const uint8_t *g2 = G3S(qs[2 * l + 1] | ((qh << (7 - 2 * l)) & 256));
                for (int j = 0; j < 4; ++j) {
                    sumi += g1[j] * q8[j] * (sg[l] & (1 << j) ? -1 : 1);
                    sumi += g2[j] * q8[j + 4] * (sg[l] & (1 << (j + 4)) ? -1 : 1);
                }
            }
            bsum += sumi * ls;
        }
        sumf += d * bsum;
    }
    return sumf;
}
static float dot_iq1_s(int n, const blk_iq1_s *x, const blk_q8_K *y) {     /* :11848, generic branch */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const int8_t *q8 = y[i].qs;
        int sumi = 0, sumi1 = 0;
        for (int ib = 0; ib < 8; ++ib) {
            const int qh = x[i].qh[ib];
            const int ls = 2 * ((qh >> 12) & 7) + 1, delta = qh & 0x8000 ? -1 : 1;
            int lsum = 0;
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const int8_t *g = G1S(x[i].qs[4 * ib + l] | (((qh >> 3 * l) & 7) << 8));
                for (int j = 0; j < 8; ++j) lsum += q8[j] * g[j];
            }
            sumi += ls * lsum;
            sumi1 += ls * delta * (y[i].bsums[2 * ib] + y[i].bsums[2 * ib + 1]);
        }
        sumf += H2F(x[i].d) * y[i].d * (sumi + IQ1_DELTA * sumi1);
    }
    return sumf;
}
static float dot_iq1_m(int n, const blk_iq1_m *x, const blk_q8_K *y) {     /* :12179, generic branch */
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        const int8_t *q8 = y[i].qs;
        uint16_t sc[4];
        memcpy(sc, x[i].scales, 8);
        const float d = H2F((uint16_t)((sc[0] >> 12) | ((sc[1] >> 8) & 0x00f0) | ((sc[2] >> 4) & 0x0f00) | (sc[3] & 0xf000)));
        int sumi1 = 0, sumi2 = 0;
        for (int ib = 0; ib < 8; ++ib) {
            const uint8_t *qs = x[i].qs + 4 * ib, *qh = x[i].qh + 2 * ib;
            int s1[2] = {0, 0}, s2[2] = {0, 0};
            for (int l = 0; l < 4; ++l, q8 += 8) {
                const int8_t *g = G1S(qs[l] | (((uint16_t)qh[l / 2] << (8 - 4 * (l % 2))) & 0x700));
                const int delta = qh[l / 2] & (0x08 << 4 * (l % 2)) ? -1 : 1;
                int a = 0, b = 0;
                for (int j = 0; j < 8; ++j) { a += q8[j] * g[j]; b += q8[j]; }
                s1[l / 2] += a;
                s2[l / 2] += b * delta;
            }
            const int ls1 = 2 * ((sc[ib / 2] >> (6 * (ib % 2) + 0)) & 7) + 1;
            const int ls2 = 2 * ((sc[ib / 2] >> (6 * (ib % 2) + 3)) & 7) + 1;
            sumi1 += s1[0] * ls1 + s1[1] * ls2;
            sumi2 += s2[0] * ls1 + s2[1] * ls2;
        }
        sumf += d * y[i].d * (sumi1 + IQ1_DELTA * sumi2);
    }
    return sumf;
}

static float dot_f16(int n, const uint16_t *x, const uint16_t *y) {        /* ggml.c:2258 */
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)(H2F(x[i]) * H2F(y[i]));
    return (float)s;
}

float orc_vec_dot(int wtype, int n, const void *w, const void *a) {
    switch (wtype) {
        case KT_Q4_K: return dot_q4_K(n, w, a);
        case KT_Q5_K: return dot_q5_K(n, w, a);
        case KT_Q6_K: return dot_q6_K(n, w, a);
        case KT_Q3_K: return dot_q3_K(n, w, a);
        case KT_Q2_K: return dot_q2_K(n, w, a);
        case KT_Q4_0: return dot_q4_0(n, w, a);
        case KT_Q5_0: return dot_q5_0(n, w, a);
        case KT_Q4_1: return dot_q4_1(n, w, a);
        case KT_Q5_1: return dot_q5_1(n, w, a);
        case KT_Q8_0: return dot_q8_0(n, w, a);
        case KT_IQ4_NL: return dot_iq4_nl(n, w, a);
        case KT_IQ4_XS: return dot_iq4_xs(n, w, a);
        case KT_IQ2_XXS: return dot_iq2_xxs(n, w, a);
        case KT_IQ2_XS: return dot_iq2_xs(n, w, a);
        case KT_IQ2_S: return dot_iq2_s(n, w, a);
        case KT_IQ3_XXS: return dot_iq3_xxs(n, w, a);
        case KT_IQ3_S: return dot_iq3_s(n, w, a);
        case KT_IQ1_S: return dot_iq1_s(n, w, a);
        case KT_IQ1_M: return dot_iq1_m(n, w, a);
        case KT_F16: return dot_f16(n, w, a);
        case KT_F32: { const float *x = w, *y = a; double s = 0; for (int i = 0; i < n; ++i) s += x[i] * y[i]; return (float)s; }
        default: abort();
    }
}

/* ggml_compute_forward_mul_mat, ggml.c:12486-12707: src1 rows -> vec_dot_type, then row dots */
void orc_mul_mat(int wtype, const void *W, int64_t K, int64_t N, const float *X, int64_t M,
                 float *dst, int nthreads) {
    const int vt = orc_vec_dot_type(wtype);
    const int64_t abytes = orc_row_bytes(vt, K), wbytes = orc_row_bytes(wtype, K);
    uint8_t *qa = malloc(abytes * M);
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    #pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t m = 0; m < M; ++m) orc_quantize_row(vt, X + m * K, qa + m * abytes, K);
    const int64_t NB = 16;
    #pragma omp parallel for num_threads(nthreads) schedule(dynamic, 4) collapse(2)
    for (int64_t nb = 0; nb < (N + NB - 1) / NB; ++nb)
        for (int64_t m = 0; m < M; ++m)
            for (int64_t n = nb * NB; n < (nb + 1) * NB && n < N; ++n)
                dst[m * N + n] = orc_vec_dot(wtype, (int)K, (const uint8_t *)W + n * wbytes, qa + m * abytes);
    free(qa);
}

/* ggml_compute_forward_rms_norm_f32 (ggml.c:12059-12103) then ggml_mul by w */
void orc_rms_norm(const float *x, const float *w, float *y, int64_t ne0, int64_t nrows, float eps) {
    for (int64_t r = 0; r < nrows; ++r) {
        const float *xr = x + r * ne0;
        float *yr = y + r * ne0;
        double sum = 0.0;
        for (int64_t i = 0; i < ne0; ++i) sum += (double)(xr[i] * xr[i]);
        const float mean = (float)(sum / ne0);
        const float scale = 1.0f / sqrtf(mean + eps);
        for (int64_t i = 0; i < ne0; ++i) yr[i] = xr[i] * scale;
        if (w) for (int64_t i = 0; i < ne0; ++i) yr[i] = yr[i] * w[i];
    }
}

/* rope helpers, ggml.c:14216-14270 */
static float rope_yarn_ramp(const float low, const float high, const int i0) {
    const float y = (i0 / 2 - low) / fmaxf(0.001f, high - low);
    return 1 - fminf(1, fmaxf(0, y));
}
static float rope_corr_dim(int n_dims, int n_ctx_orig, float n_rot, float base) {
    return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float)M_PI)) / (2 * logf(base));
}

void orc_rope(const float *x, float *y, int64_t head_dim, int64_t n_heads, int64_t n_tokens,
              const int32_t *pos, int n_dims, float freq_base, float freq_scale,
              const float *freq_factors, float ext_factor, float attn_factor,
              float beta_fast, float beta_slow, int n_ctx_orig) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    float corr[2];
    {
        float start = floorf(rope_corr_dim(n_dims, n_ctx_orig, beta_fast, freq_base));
        float end = ceilf(rope_corr_dim(n_dims, n_ctx_orig, beta_slow, freq_base));
        corr[0] = fmaxf(0, start); corr[1] = fminf(n_dims - 1, end);
    }
    float *cache = malloc(sizeof(float) * head_dim);
    for (int64_t t = 0; t < n_tokens; ++t) {
        float theta = (float)pos[t];
        for (int64_t i0 = 0; i0 < head_dim; i0 += 2) {           /* ggml_rope_cache_init */
            const float ff = freq_factors ? freq_factors[i0 / 2] : 1.0f;
            float theta_extrap = theta / ff;
            float theta_interp = freq_scale * theta_extrap;
            float th = theta_interp, mscale = attn_factor;
            if (ext_factor != 0.0f) {
                float ramp_mix = rope_yarn_ramp(corr[0], corr[1], (int)i0) * ext_factor;
                th = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
                mscale *= 1.0f + 0.1f * logf(1.0f / freq_scale);
            }
            cache[i0] = cosf(th) * mscale;
            cache[i0 + 1] = sinf(th) * mscale;
            theta *= theta_scale;
        }
        for (int64_t h = 0; h < n_heads; ++h) {
            const float *src = x + (t * n_heads + h) * head_dim;
            float *dst = y + (t * n_heads + h) * head_dim;
            for (int64_t i0 = 0; i0 < n_dims; i0 += 2) {
                const float c = cache[i0], s = cache[i0 + 1];
                const float x0 = src[i0], x1 = src[i0 + 1];
                dst[i0] = x0 * c - x1 * s;
                dst[i0 + 1] = x0 * s + x1 * c;
            }
            for (int64_t i0 = n_dims; i0 < head_dim; ++i0) dst[i0] = src[i0];
        }
    }
    free(cache);
}

/* Diagnostic switch (not reference behaviour): accumulate V in f32 instead of the reference's
 * f16 VKQ16 accumulator, to separate f16-accumulation noise from real discrepancies. */
static int g_fa_f32_accum = 0;
void orc_set_fa_f32_accum(int on) { g_fa_f32_accum = on; }

/* ggml_compute_forward_flash_attn_ext_f16, F16 K/V branch (ggml.c:15667-15875) */
void orc_flash_attn_ext(const float *q, const uint16_t *k, const uint16_t *v, int64_t kv_stride,
                        const uint16_t *mask, float *out, int D, int n_q, int n_head,
                        int n_kv, int n_head_kv, float scale, int nthreads) {
    const int rk = n_head / n_head_kv;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    #pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
    for (int ir = 0; ir < n_q * n_head; ++ir) {
        const int iq1 = ir / n_head, h = ir % n_head;   /* row order irrelevant */
        const int hk = h / rk;
        uint16_t qh[512];
        uint16_t vkq16[512];
        float vkq32[512];
        const float *pq = q + ((int64_t)iq1 * n_head + h) * D;
        for (int d = 0; d < D; ++d) { qh[d] = F2H(pq[d]); vkq16[d] = 0; vkq32[d] = 0.0f; }
        float S = 0.0f, M = -INFINITY;
        for (int ic = 0; ic < n_kv; ++ic) {
            const float mv = mask ? H2F(mask[(int64_t)iq1 * n_kv + ic]) : 0.0f;
            if (mv == -INFINITY) continue;
            const uint16_t *kr = k + (int64_t)ic * kv_stride + (int64_t)hk * D;
            float s = dot_f16(D, kr, qh);
            s = s * scale;
            s += mv;
            const float Mold = M;
            float ms = 1.0f, vs = 1.0f;
            const uint16_t *vr = v + (int64_t)ic * kv_stride + (int64_t)hk * D;
            if (s > M) {
                M = s;
                ms = expf(Mold - M);
                if (g_fa_f32_accum) for (int d = 0; d < D; ++d) vkq32[d] *= ms;
                else for (int d = 0; d < D; ++d) vkq16[d] = F2H(H2F(vkq16[d]) * ms);   /* ggml_vec_scale_f16 */
            } else {
                vs = expf(s - M);
            }
            if (g_fa_f32_accum) for (int d = 0; d < D; ++d) vkq32[d] = fmaf(H2F(vr[d]), vs, vkq32[d]);
            else for (int d = 0; d < D; ++d) vkq16[d] = F2H(fmaf(H2F(vr[d]), vs, H2F(vkq16[d])));  /* ggml_vec_mad_f16 */
            S = S * ms + vs;
        }
        if (!g_fa_f32_accum) for (int d = 0; d < D; ++d) vkq32[d] = H2F(vkq16[d]);
        const float S_inv = 1.0f / S;
        float *po = out + ((int64_t)iq1 * n_head + h) * D;
        for (int d = 0; d < D; ++d) po[d] = vkq32[d] * S_inv;
    }
}

/* ggml_compute_forward_flash_attn_ext_f16 with a QUANTIZED K and V (ggml.c:15748-15851): Q is converted to K's
 * vec_dot_type (Q8_0) by its from_float, s = vec_dot(K row, Q_q), V rows dequantized (to_float) and accumulated in
 * f32 (ggml_vec_scale_f32 / ggml_vec_mad_f32).  k / v: ggml block rows, position p of kv head hk at
 * base + p*row_bytes + hk*orc_row_bytes(type, D). */
void orc_flash_attn_ext_q(const float *q, const void *k, const void *v, int64_t k_row_bytes, int64_t v_row_bytes,
                          int ktype, int vtype, const uint16_t *mask, float *out, int D, int n_q, int n_head,
                          int n_kv, int n_head_kv, float scale, int nthreads) {
    const int rk = n_head / n_head_kv;
    const int64_t kh = orc_row_bytes(ktype, D), vh = orc_row_bytes(vtype, D);
    const int qt = orc_vec_dot_type(ktype);
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    #pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
    for (int ir = 0; ir < n_q * n_head; ++ir) {
        const int iq1 = ir / n_head, h = ir % n_head;
        const int hk = h / rk;
        uint8_t qq[1024];
        float vkq32[512], v32[512];
        orc_quantize_row(qt, q + ((int64_t)iq1 * n_head + h) * D, qq, D);
        for (int d = 0; d < D; ++d) vkq32[d] = 0.0f;
        float S = 0.0f, M = -INFINITY;
        for (int ic = 0; ic < n_kv; ++ic) {
            const float mv = mask ? H2F(mask[(int64_t)iq1 * n_kv + ic]) : 0.0f;
            if (mv == -INFINITY) continue;
            float s = orc_vec_dot(ktype, D, (const uint8_t *)k + ic * k_row_bytes + hk * kh, qq);
            s = s * scale;
            s += mv;
            const float Mold = M;
            float ms = 1.0f, vs = 1.0f;
            if (s > M) {
                M = s;
                ms = expf(Mold - M);
                for (int d = 0; d < D; ++d) vkq32[d] *= ms;
            } else {
                vs = expf(s - M);
            }
            orc_dequantize_row(vtype, (const uint8_t *)v + ic * v_row_bytes + hk * vh, v32, D);
            for (int d = 0; d < D; ++d) vkq32[d] = fmaf(v32[d], vs, vkq32[d]);
            S = S * ms + vs;
        }
        const float S_inv = 1.0f / S;
        float *po = out + ((int64_t)iq1 * n_head + h) * D;
        for (int d = 0; d < D; ++d) po[d] = vkq32[d] * S_inv;
    }
}

/* ======================= Llama forward (build_llama) ======================= */
struct orc_llama {
    orc_hparams hp;
    const void *const *w;
    const int *t;
    int nthreads;
    uint16_t *kc, *vc;     /* [n_layer][n_ctx][n_head_kv*D] f16, or ggml block rows of type tk / tv */
    int tk, tv;            /* cache types (llama_context_params type_k / type_v): KT_F16, KT_Q8_0, KT_Q4_0 */
    float *last_hidden;
};

int orc_llama_set_kv_types(orc_llama *m, int tk, int tv) {
    if ((tk != KT_F16 && tk != KT_Q8_0 && tk != KT_Q4_0) || (tv != KT_F16 && tv != KT_Q8_0 && tv != KT_Q4_0)) return -1;
    if ((tk == KT_F16) != (tv == KT_F16)) return -1;    /* mixed F16 / quantized: not restated */
    m->tk = tk; m->tv = tv;
    return 0;
}

orc_llama *orc_llama_create(const orc_hparams *hp, const void *const *data, const int *types, int nthreads) {
    orc_llama *m = calloc(1, sizeof(*m));
    m->hp = *hp;
    int nw = 3 + (hp->n_expert ? 10 : 9) * hp->n_layer;
    void **w = malloc(sizeof(void *) * nw);
    int *t = malloc(sizeof(int) * nw);
    memcpy(w, data, sizeof(void *) * nw);
    memcpy(t, types, sizeof(int) * nw);
    m->w = (const void *const *)w; m->t = t;
    m->nthreads = nthreads > 0 ? nthreads : omp_get_max_threads();
    const int64_t D = hp->n_embd / hp->n_head;
    const int64_t kvsz = (int64_t)hp->n_layer * hp->n_ctx * hp->n_head_kv * D;
    m->kc = calloc(kvsz, 2);     /* f16 size bounds the quantized rows too (Q8_0 34/32, Q4_0 18/32 B per element) */
    m->vc = calloc(kvsz, 2);
    m->tk = m->tv = KT_F16;
    m->last_hidden = calloc(hp->n_embd, 4);
    return m;
}

void orc_llama_free(orc_llama *m) {
    if (!m) return;
    free((void *)m->w); free((void *)m->t); free(m->kc); free(m->vc); free(m->last_hidden); free(m);
}

void orc_llama_last_hidden(orc_llama *m, float *out) { memcpy(out, m->last_hidden, 4 * m->hp.n_embd); }

static void add_inplace(float *a, const float *b, int64_t n) { for (int64_t i = 0; i < n; ++i) a[i] += b[i]; }

/* llm_build_moe_ffn (src/llama.cpp:9416-9520) for the llama architecture: router mul_mat, soft_max
 * (ggml.c:13909, ggml_float sum), top_k = argsort descending (the exchange sort of
 * ggml_compute_forward_argsort_f32), normalized weights (sum_rows + div), per selected expert
 * up / silu(gate) mul_mat_id, down mul_mat_id, weighted, summed in top-k order.  Writes moe[T][E]. */
static void moe_ffn(const orc_hparams *hp, const void *const *lw, const int *lt, const float *cur, int T, float *moe, int NT) {
    const int E = hp->n_embd, F = hp->n_ff, NE = hp->n_expert, NU = hp->n_expert_used;
    float *lg = malloc(sizeof(float) * T * NE);
    orc_mul_mat(lt[9], lw[9], E, NE, cur, T, lg, NT);
    const int64_t rg = orc_row_bytes(lt[6], E) * F, ru = orc_row_bytes(lt[7], E) * F, rd = orc_row_bytes(lt[8], F) * E;
    float *g = malloc(sizeof(float) * F), *u = malloc(sizeof(float) * F), *o = malloc(sizeof(float) * E);
    for (int t = 0; t < T; ++t) {
        float *p = lg + (int64_t)t * NE;
        float mx = -INFINITY;
        for (int e = 0; e < NE; ++e) mx = fmaxf(mx, p[e]);
        double sum = 0.0;
        for (int e = 0; e < NE; ++e) { const float v = expf(p[e] - mx); sum += (double)v; p[e] = v; }
        const float inv = (float)(1.0 / sum);
        for (int e = 0; e < NE; ++e) p[e] *= inv;
        int idx[64];
        for (int e = 0; e < NE; ++e) idx[e] = e;
        for (int j = 0; j < NE; ++j)
            for (int k = j + 1; k < NE; ++k)
                if (p[idx[j]] < p[idx[k]]) { const int tmp = idx[j]; idx[j] = idx[k]; idx[k] = tmp; }
        double ws = 0.0;
        for (int j = 0; j < NU; ++j) ws += (double)p[idx[j]];
        const float wsum = (float)ws;
        float *mo = moe + (int64_t)t * E;
        for (int j = 0; j < NU; ++j) {
            const int e = idx[j];
            const float w = p[e] / wsum;
            const float *ct = cur + (int64_t)t * E;
            orc_mul_mat(lt[6], (const uint8_t *)lw[6] + e * rg, E, F, ct, 1, g, 1);
            orc_mul_mat(lt[7], (const uint8_t *)lw[7] + e * ru, E, F, ct, 1, u, 1);
            for (int i = 0; i < F; ++i) g[i] = u[i] * (g[i] / (1.0f + expf(-g[i])));   /* up * silu(gate) */
            orc_mul_mat(lt[8], (const uint8_t *)lw[8] + e * rd, F, E, g, 1, o, 1);
            for (int i = 0; i < E; ++i) {
                const float v = o[i] * w;
                mo[i] = j == 0 ? v : mo[i] + v;
            }
        }
    }
    free(lg); free(g); free(u); free(o);
}

int orc_llama_eval(orc_llama *m, const int32_t *tokens, int T, int n_past, float *logits) {
    const orc_hparams *hp = &m->hp;
    const int E = hp->n_embd, H = hp->n_head, HKV = hp->n_head_kv, D = E / H, F = hp->n_ff;
    const int EKV = HKV * D;
    const int NT = m->nthreads;
    if (n_past + T > hp->n_ctx) return -1;
    float *x = malloc(sizeof(float) * T * E), *cur = malloc(sizeof(float) * T * E);
    float *q = malloc(sizeof(float) * T * E), *kk = malloc(sizeof(float) * T * EKV), *vv = malloc(sizeof(float) * T * EKV);
    float *attn = malloc(sizeof(float) * T * E), *tmp = malloc(sizeof(float) * T * E);
    float *g = malloc(sizeof(float) * T * F), *u = malloc(sizeof(float) * T * F);
    int32_t *pos = malloc(sizeof(int32_t) * T);
    for (int t = 0; t < T; ++t) pos[t] = n_past + t;
    /* token embeddings: get_rows (dequantize one row) */
    const int64_t erow = orc_row_bytes(m->t[0], E);
    for (int t = 0; t < T; ++t) orc_dequantize_row(m->t[0], (const uint8_t *)m->w[0] + (int64_t)tokens[t] * erow, x + (int64_t)t * E, E);
    const int n_kv = n_past + T;
    uint16_t *mask = malloc(sizeof(uint16_t) * (int64_t)T * n_kv);
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < n_kv; ++j)
            mask[(int64_t)t * n_kv + j] = (j <= n_past + t) ? 0 : 0xFC00; /* -inf */
    const float kq_scale = 1.0f / sqrtf((float)D);
    const int LW = hp->n_expert ? 10 : 9;
    for (int il = 0; il < hp->n_layer; ++il) {
        const void *const *lw = m->w + 3 + LW * il;
        const int *lt = m->t + 3 + LW * il;
        orc_rms_norm(x, (const float *)lw[0], cur, E, T, hp->eps);
        orc_mul_mat(lt[1], lw[1], E, E, cur, T, q, NT);
        orc_mul_mat(lt[2], lw[2], E, EKV, cur, T, kk, NT);
        orc_mul_mat(lt[3], lw[3], E, EKV, cur, T, vv, NT);
        orc_rope(q, q, D, H, T, pos, D, hp->rope_base, hp->rope_freq_scale, NULL, 0.0f, 1.0f, 32.0f, 1.0f, hp->n_ctx);
        orc_rope(kk, kk, D, HKV, T, pos, D, hp->rope_base, hp->rope_freq_scale, NULL, 0.0f, 1.0f, 32.0f, 1.0f, hp->n_ctx);
        uint16_t *kl = m->kc + (int64_t)il * hp->n_ctx * EKV, *vl = m->vc + (int64_t)il * hp->n_ctx * EKV;
        if (m->tk != KT_F16) {                           /* ggml_cpy f32 -> Q8_0 / Q4_0 (from_float) into the cache */
            const int64_t kb = orc_row_bytes(m->tk, EKV), vb = orc_row_bytes(m->tv, EKV);
            for (int t = 0; t < T; ++t) {
                orc_quantize_row(m->tk, kk + (int64_t)t * EKV, (uint8_t *)kl + (n_past + t) * kb, EKV);
                orc_quantize_row(m->tv, vv + (int64_t)t * EKV, (uint8_t *)vl + (n_past + t) * vb, EKV);
            }
            orc_flash_attn_ext_q(q, kl, vl, kb, vb, m->tk, m->tv, mask, attn, D, T, H, n_kv, HKV, kq_scale, NT);
        } else {
        for (int t = 0; t < T; ++t)
            for (int i = 0; i < EKV; ++i) {           /* ggml_cpy f32 -> f16 into the cache */
                kl[(int64_t)(n_past + t) * EKV + i] = F2H(kk[(int64_t)t * EKV + i]);
                vl[(int64_t)(n_past + t) * EKV + i] = F2H(vv[(int64_t)t * EKV + i]);
            }
        orc_flash_attn_ext(q, kl, vl, EKV, mask, attn, D, T, H, n_kv, HKV, kq_scale, NT);
        }
        orc_mul_mat(lt[4], lw[4], E, E, attn, T, tmp, NT);
        add_inplace(tmp, x, (int64_t)T * E);             /* ffn_inp = attn_out + inpSA */
        memcpy(x, tmp, sizeof(float) * T * E);
        orc_rms_norm(x, (const float *)lw[5], cur, E, T, hp->eps);
        if (hp->n_expert) {
            moe_ffn(hp, lw, lt, cur, T, tmp, NT);
            for (int64_t i = 0; i < (int64_t)T * E; ++i) x[i] = tmp[i] + x[i];   /* ggml_add(moe_out, ffn_inp) */
            continue;
        }
        orc_mul_mat(lt[6], lw[6], E, F, cur, T, g, NT);
        orc_mul_mat(lt[7], lw[7], E, F, cur, T, u, NT);
        for (int64_t i = 0; i < (int64_t)T * F; ++i) g[i] = (g[i] / (1.0f + expf(-g[i]))) * u[i];  /* silu(gate)*up */
        orc_mul_mat(lt[8], lw[8], F, E, g, T, tmp, NT);
        add_inplace(x, tmp, (int64_t)T * E);             /* l_out = ffn_out + ffn_inp */
    }
    memcpy(m->last_hidden, x + (int64_t)(T - 1) * E, sizeof(float) * E);
    orc_rms_norm(x + (int64_t)(T - 1) * E, (const float *)m->w[1], cur, E, 1, hp->eps);
    orc_mul_mat(m->t[2], m->w[2], E, hp->n_vocab, cur, 1, logits, NT);
    free(x); free(cur); free(q); free(kk); free(vv); free(attn); free(tmp); free(g); free(u); free(pos); free(mask);
    return 0;
}

/* deterministic synthetic tensors (same generator as the product; used by tests) */
void orc_synth_fill(int type, uint64_t seed, uint64_t tid, int64_t nblocks, void *dst) {
    const int bb = ks_block_bytes(type);
    #pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblocks; ++b) ks_fill_block(type, seed, tid, (uint64_t)b, (uint8_t *)dst + b * bb);
}
