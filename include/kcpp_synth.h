/*
 * kcpp_synth.h -- deterministic synthetic GGUF-format weights (host + device).
 *
 * There are no real Llama checkpoints on the build/GPU machines, so benchmarks and
 * parity tests use random-init weights *in the exact on-disk block formats* of
 * ggml (ggml/src/ggml-common.h:144-335 of the reference: block_q4_0, block_q8_0,
 * block_q2_K, block_q3_K, block_q4_K, block_q5_K, block_q6_K).  Every byte is a pure function of
 * (seed, tensor id, block index), so the GPU runtime, the CPU oracle and the
 * reference-ggml harness all see bit-identical tensors without shipping files.
 *
 * Scales are chosen so dequantized weights have std ~0.02 (N(0,0.02^2) in
 * SURVEY.md §8d config 2) and norm weights are 1 +- 0.01.
 *
 * Plain C99, usable from gcc (oracle), g++ (runtime) and hipcc (device code).
 */
#ifndef KCPP_SYNTH_H
#define KCPP_SYNTH_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define KS_FN static inline __host__ __device__
#else
#define KS_FN static inline
#endif

/* ggml_type ids (ggml/include/ggml.h:364-399 of the reference) */
enum kcpp_type {
    KT_F32 = 0, KT_F16 = 1, KT_Q4_0 = 2, KT_Q4_1 = 3, KT_Q5_0 = 6, KT_Q5_1 = 7,
    KT_Q8_0 = 8, KT_Q8_1 = 9, KT_Q2_K = 10, KT_Q3_K = 11, KT_Q4_K = 12,
    KT_Q5_K = 13, KT_Q6_K = 14, KT_Q8_K = 15, KT_IQ2_XXS = 16, KT_IQ2_XS = 17, KT_IQ3_XXS = 18, KT_IQ1_S = 19,
    KT_IQ4_NL = 20, KT_IQ3_S = 21, KT_IQ2_S = 22, KT_IQ4_XS = 23, KT_IQ1_M = 29, KT_BF16 = 30,
    /* GPU-internal row-major decode layouts of Q4_K / Q5_K / Q6_K (same bytes per row, re-arranged inside
       each row so the single-token mat-vec reads 1 KiB-contiguous wave loads; csrc/kcpp_common.h).
       Not ggml ids: they never leave the device library. */
    KT_Q4_K_RS = 112, KT_Q5_K_RS = 113, KT_Q6_K_RS = 114,
    /* GPU-internal tile layout of Q8_0 (32-row tiles, each block's 32 rows x 32 B one contiguous 1 KiB MFMA operand,
       csrc/gemm_q80t.hip) and its activation layout (32-token groups in the same fragment order) */
    KT_Q8_0_T = 115, KT_Q8_0_TA = 116
};

/* the lattice-grid types (IQ1 / IQ2 / IQ3): ggml layout on the device, decoded through the code books */
KS_FN int is_iq_grid_type(int t) {
    return t == KT_IQ2_XXS || t == KT_IQ2_XS || t == KT_IQ2_S || t == KT_IQ3_XXS || t == KT_IQ3_S || t == KT_IQ1_S ||
           t == KT_IQ1_M;
}

/* the ggml type whose blocks a layout holds */
KS_FN int ks_base_type(int type) {
    return type == KT_Q4_K_RS ? KT_Q4_K : (type == KT_Q5_K_RS ? KT_Q5_K : (type == KT_Q6_K_RS ? KT_Q6_K :
           (type == KT_Q8_0_T ? KT_Q8_0 : type)));
}

KS_FN uint64_t ks_mix(uint64_t z) {          /* splitmix64 finalizer */
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* round-to-nearest-even f32 -> f16 bits (matches F16C _cvtss_sh(x,0) for finite x) */
KS_FN uint16_t ks_f32_to_f16(float f) {
    uint32_t x; memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return (uint16_t)(sign | (ax > 0x7F800000u ? 0x7E00u : 0x7C00u));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);            /* overflow -> inf */
    if (ax < 0x38800000u) {                                              /* subnormal / zero */
        if (ax < 0x33000000u) return (uint16_t)sign;
        uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;
        int shift = 126 - (int)(ax >> 23);                               /* 14..24 */
        uint32_t r = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (r & 1u))) r++;
        return (uint16_t)(sign | r);
    }
    uint32_t r = ((ax >> 13) - (112u << 10));
    uint32_t rem = ax & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) r++;
    return (uint16_t)(sign | r);
}

KS_FN float ks_unit(uint64_t h) {            /* [0,1) */
    return (float)((h >> 40) & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

/* bytes per block and elements per block for the supported types */
KS_FN int ks_block_elems(int type) {
    switch (type) {
        case KT_F32: case KT_F16: return 1;
        case KT_Q4_0: case KT_Q4_1: case KT_Q5_0: case KT_Q5_1: case KT_Q8_0: case KT_Q8_1: case KT_IQ4_NL: case KT_Q8_0_T: return 32;
        default: return 256;
    }
}
KS_FN int ks_block_bytes(int type) {
    switch (type) {
        case KT_F32: return 4;
        case KT_F16: return 2;
        case KT_Q4_0: case KT_IQ4_NL: return 18;
        case KT_Q4_1: return 20;
        case KT_IQ4_XS: return 136;
        case KT_Q5_0: return 22;
        case KT_Q5_1: return 24;
        case KT_Q8_1: return 36;
        case KT_Q8_0: case KT_Q8_0_T: return 34;
        case KT_Q2_K: return 84;
        case KT_Q3_K: return 110;
        case KT_Q4_K: case KT_Q4_K_RS: return 144;
        case KT_Q5_K: case KT_Q5_K_RS: return 176;
        case KT_Q6_K: case KT_Q6_K_RS: return 210;
        case KT_Q8_K: return 292;
        case KT_IQ2_XXS: return 66;      /* block_iq2_xxs .. block_iq1_m, ggml-common.h:340-405 */
        case KT_IQ2_XS: return 74;
        case KT_IQ2_S: return 82;
        case KT_IQ3_XXS: return 98;
        case KT_IQ3_S: return 110;
        case KT_IQ1_S: return 50;
        case KT_IQ1_M: return 56;
        default: return 0;
    }
}

/* Fill one block (ggml on-disk layout) of tensor `tid` at block index `b`. */
KS_FN void ks_fill_block(int type, uint64_t seed, uint64_t tid, uint64_t b, uint8_t *dst) {
    type = ks_base_type(type);
    uint64_t base = ks_mix(seed ^ (tid * 0xD1B54A32D192ED03ull)) ^ (b * 0x9E3779B97F4A7C15ull);
    int nb = ks_block_bytes(type);
    /* random payload, 8 bytes per hash */
    for (int i = 0; i < nb; i += 8) {
        uint64_t h = ks_mix(base + (uint64_t)i);
        for (int j = 0; j < 8 && i + j < nb; ++j) dst[i + j] = (uint8_t)(h >> (8 * j));
    }
    uint64_t hs = ks_mix(base ^ 0xA5A5A5A5A5A5A5A5ull);
    float u0 = ks_unit(hs), u1 = ks_unit(ks_mix(hs));
    uint16_t h0, h1;
    switch (type) {
        case KT_F32: {
            float v = 1.0f + (u0 - 0.5f) * 0.02f;       /* norm weights */
            memcpy(dst, &v, 4);
        } break;
        case KT_F16: {
            uint16_t v = ks_f32_to_f16((u0 - 0.5f) * 0.07f);
            memcpy(dst, &v, 2);
        } break;
        case KT_Q4_0:
            h0 = ks_f32_to_f16(0.0043f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_Q4_1: case KT_Q5_1: {   /* w = d q + m, q in 0..15 (0..31): mean -m/d-centred */
            const float d = type == KT_Q4_1 ? 0.0043f : 0.00215f;
            h0 = ks_f32_to_f16(d * (0.75f + 0.5f * u0));
            h1 = ks_f32_to_f16(-(type == KT_Q4_1 ? 7.5f : 15.5f) * d * (0.9f + 0.2f * u1));
            memcpy(dst, &h0, 2); memcpy(dst + 2, &h1, 2);
        } break;
        case KT_Q5_0:       /* w = d ((q | h << 4) - 16), std ~9.2 d */
            h0 = ks_f32_to_f16(0.00215f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_Q8_0:
            h0 = ks_f32_to_f16(0.00027f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ4_NL:     /* w = d kvalues_iq4nl[q], std(kvalues) ~70 */
            h0 = ks_f32_to_f16(2.8e-4f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ4_XS:     /* w = d (ls - 32) kvalues_iq4nl[q], ls 6-bit: std(ls - 32) ~18.5 */
            h0 = ks_f32_to_f16(1.6e-5f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        /* the grid types (every index / sign / scale bit pattern is a valid code): d scaled for std ~0.02 */
        case KT_IQ2_XXS: case KT_IQ2_XS: case KT_IQ2_S:   /* w = d (0.5 + ls) / 4 grid, grid in {8, 25, 43} */
            h0 = ks_f32_to_f16(3.0e-4f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ3_XXS:    /* w = d (0.5 + ls) / 2 grid, grid 4..62 */
            h0 = ks_f32_to_f16(1.4e-4f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ3_S:      /* w = d (1 + 2 ls) grid, grid 1..15 */
            h0 = ks_f32_to_f16(1.3e-4f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ1_S:      /* w = d (2 ls + 1) (grid +- 1/8), grid in {-1, 0, 1} */
            h0 = ks_f32_to_f16(2.7e-3f * (0.75f + 0.5f * u0));
            memcpy(dst, &h0, 2);
            break;
        case KT_IQ1_M: {    /* as IQ1_S; the f16 scale lives in the top nibbles of the four scale words */
            h0 = ks_f32_to_f16(2.7e-3f * (0.75f + 0.5f * u0));
            uint8_t *sc = dst + 48;
            for (int j = 0; j < 4; ++j) sc[2 * j + 1] = (uint8_t)((sc[2 * j + 1] & 0x0F) | (((h0 >> (4 * j)) & 0xF) << 4));
        } break;
        case KT_Q4_K: case KT_Q5_K: {
            float d = (type == KT_Q4_K ? 1.35e-4f : 6.7e-5f) * (0.75f + 0.5f * u0);
            float dm = (type == KT_Q4_K ? 1.0e-3f : 1.0e-3f) * (0.75f + 0.5f * u1);
            h0 = ks_f32_to_f16(d); h1 = ks_f32_to_f16(dm);
            memcpy(dst, &h0, 2); memcpy(dst + 2, &h1, 2);
            /* scales[12]: keep the 6-bit scales/mins in [16,63] by forcing bit 4/5 patterns */
            uint8_t *s = dst + 4;
            for (int j = 0; j < 4; ++j) { s[j] |= 0x10; s[j + 4] |= 0x10; }
            for (int j = 0; j < 4; ++j) { s[j + 8] = (uint8_t)(s[j + 8] | 0x11); }
        } break;
        case KT_Q2_K: {     /* w = d (sc & 15) q - dmin (sc >> 4), q in 0..3: std(sc q) ~12.7 */
            h0 = ks_f32_to_f16(1.6e-3f * (0.75f + 0.5f * u0)); h1 = ks_f32_to_f16(2.4e-3f * (0.75f + 0.5f * u1));
            memcpy(dst + 80, &h0, 2); memcpy(dst + 82, &h1, 2);
        } break;
        case KT_Q3_K: {     /* w = d (sc - 32) q3, sc 6-bit, q3 in -4..3: std(sc - 32) ~18.5, std(q3) ~2.3 */
            h0 = ks_f32_to_f16(4.6e-4f * (0.75f + 0.5f * u0));
            memcpy(dst + 108, &h0, 2);
        } break;
        case KT_Q6_K: {
            h0 = ks_f32_to_f16(7.0e-5f * (0.75f + 0.5f * u0));
            memcpy(dst + 208, &h0, 2);
            int8_t *sc = (int8_t *)(dst + 192);
            for (int j = 0; j < 16; ++j) sc[j] = (int8_t)(8 + ((uint8_t)sc[j] % 16));
        } break;
        default: break;
    }
}

#endif /* KCPP_SYNTH_H */
