// gemm.hip -- batched (prefill / ubatch) quantized mat-mul on CDNA4 matrix cores.
//
// Replaces the reference's batched paths -- mul_mat_q (ggml/src/ggml-cuda/mmq.cuh:2572-2905, DP4A
// on AMD, no MFMA) and the default ROCm "dequantize the whole weight to F16 + hipblasGemmEx with
// FP16 compute" path (ggml-cuda.cu:1186-1284) -- while computing exactly what the CPU vec_dot does
// (ggml-quants.c:3922,5519,7714,8282,8919): weights x CPU-quantized activations (Q8_K / Q8_0) as
// exact integer block dots, scaled per super-block (or per 32-block) in fp32.
//
// How the integer dot stays exact on f16 MFMA (v_mfma_f32_32x32x16_f16, fp32 accumulate):
//   * activations are int8 values -> exact in f16;
//   * the weight operand is the *integer* sub-block product sc*q (Q4_K <= 945, Q5_K <= 1953:
//     exact in f16), or for Q6_K sc*(q-32) split as 8*(sc>>3)*(q-32) + (sc&7)*(q-32), both
//     exact, accumulated into the same fp32 accumulator by two MFMAs;
//   * products are exact and partial sums stay < 2^24, so the fp32 accumulator holds the same
//     integer as the CPU's int32 `sumi`; Q4_K/Q5_K mins use a 16-deep MFMA over the Q8_K bsums.
// Dequantization to those f16 integers costs 2 VALU ops per pair of weights (v_perm_b32 builds
// 1024+q halves, v_pk_fma_f16 scales and removes the 1024 bias exactly).
//
// Tiling: workgroup = 4 waves = 128 tokens x 64 weight rows, K step 256.  The 64x256 weight tile
// is dequantized once per workgroup into LDS in MFMA-fragment order (ds_read_b128 per lane,
// conflict-free); each wave owns 32 tokens x 64 rows (two 32x32 MFMA tiles).
#include "kcpp_common.h"
#include "kcpp_internal.h"
#include "iq_grid.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16acc __attribute__((ext_vector_type(16)));

#define GB_M 128
#define GB_N 64
#define GB_K 256

// ---------------------------------------------------------------- activation -> f16 operand
// a16 [Mp][K] f16 (int8 values), dy [Mp][K/G] f32 (copied), bs16 [Mp][K/16] f16 (Q8_K bsums)
__global__ void k_act_to_f16(const uint8_t *__restrict__ act, int vt, int64_t K, int64_t M, int64_t Mp,
                             _Float16 *__restrict__ a16, float *__restrict__ dy, _Float16 *__restrict__ bs16) {
    const int64_t m = blockIdx.y;
    const int64_t G = vt == KT_Q8_K ? 256 : 32;
    const bool valid = m < M;
    const int8_t *qs = (const int8_t *)act + m * K;
    for (int64_t i = (int64_t)threadIdx.x * 4 + (int64_t)blockIdx.x * 1024; i < K && i < ((int64_t)blockIdx.x + 1) * 1024;
         i += (int64_t)blockDim.x * 4) {
        const int v = valid ? *(const int *)(qs + i) : 0;
        a16[m * K + i + 0] = (_Float16)(int8_t)(v & 0xFF);
        a16[m * K + i + 1] = (_Float16)(int8_t)((v >> 8) & 0xFF);
        a16[m * K + i + 2] = (_Float16)(int8_t)((v >> 16) & 0xFF);
        a16[m * K + i + 3] = (_Float16)(int8_t)((v >> 24) & 0xFF);
    }
    if (blockIdx.x == 0) {
        const float *d = (const float *)(act + M * K) + m * (K / G);
        for (int64_t i = threadIdx.x; i < K / G; i += blockDim.x) dy[m * (K / G) + i] = valid ? d[i] : 0.0f;
        if (vt == KT_Q8_K) {
            const int16_t *bs = (const int16_t *)(act + M * K + M * (K / 256) * 4) + m * (K / 16);
            for (int64_t i = threadIdx.x; i < K / 16; i += blockDim.x) bs16[m * (K / 16) + i] = valid ? (_Float16)bs[i] : (_Float16)0;
        }
    }
}

// ---------------------------------------------------------------- dequant helpers
// v_perm_b32 byte selects: 4..7 = bytes of src0 (t), 0..3 = bytes of src1 (0x64 each):
// bytes (b0,0x64,b1,0x64) are the f16 halves 1024+b0, 1024+b1 (exact for b < 1024)
__device__ __forceinline__ h2v bias_lo(uint32_t t) { return __builtin_bit_cast(h2v, __builtin_amdgcn_perm(t, 0x64646464u, 0x00050004u)); }
__device__ __forceinline__ h2v bias_hi(uint32_t t) { return __builtin_bit_cast(h2v, __builtin_amdgcn_perm(t, 0x64646464u, 0x00070006u)); }

// (1024 + q) * s - (1024 + off) * s  ==  (q - off) * s   exactly (single rounding of an exact value)
__device__ __forceinline__ h2v scale2(h2v x, _Float16 s, _Float16 bias) {
    const h2v sv = {s, s};
    const h2v bv = {bias, bias};
    return __builtin_elementwise_fma(x, sv, bv);
}
// 8 weights (two dwords of bytes) -> fragment of 8 halves, (byte - off) * s
__device__ __forceinline__ h8v frag8(uint32_t t0, uint32_t t1, float s, float off) {
    const _Float16 sh = (_Float16)s;
    const _Float16 bh = (_Float16)(-(1024.0f + off) * s);
    const h2v a = scale2(bias_lo(t0), sh, bh), b = scale2(bias_hi(t0), sh, bh);
    const h2v c = scale2(bias_lo(t1), sh, bh), d = scale2(bias_hi(t1), sh, bh);
    h8v r;
    r[0] = a[0]; r[1] = a[1]; r[2] = b[0]; r[3] = b[1]; r[4] = c[0]; r[5] = c[1]; r[6] = d[0]; r[7] = d[1];
    return r;
}

// Q6_K variant: (byte - off) exactly first (small ints), then * s (exact: |8*(sc>>3)*(q-32)| <= 4096,
// a multiple of 8; |(sc&7)*(q-32)| <= 224).  A single fma would need a bias beyond the f16 range.
__device__ __forceinline__ h8v frag8_sub(uint32_t t0, uint32_t t1, float s, float off) {
    const h2v sv = {(_Float16)s, (_Float16)s};
    const h2v bv = {(_Float16)(-(1024.0f + off)), (_Float16)(-(1024.0f + off))};
    const h2v a = (bias_lo(t0) + bv) * sv, b = (bias_hi(t0) + bv) * sv;
    const h2v c = (bias_lo(t1) + bv) * sv, d = (bias_hi(t1) + bv) * sv;
    h8v r;
    r[0] = a[0]; r[1] = a[1]; r[2] = b[0]; r[3] = b[1]; r[4] = c[0]; r[5] = c[1]; r[6] = d[0]; r[7] = d[1];
    return r;
}

// get_scale_min_k4 (ggml-quants.c:1899) on the 12 scale bytes held in hdr.y/z/w (registers only)
__device__ __forceinline__ void k4_sm(const uint4 &hdr, int j, int &d, int &m) {
    auto b = [&](int k) -> int {
        const uint32_t w = k < 4 ? hdr.y : (k < 8 ? hdr.z : hdr.w);
        return (w >> (8 * (k & 3))) & 0xFF;
    };
    if (j < 4) { d = b(j) & 63; m = b(j + 4) & 63; }
    else { d = (b(j + 4) & 0xF) | ((b(j - 4) >> 6) << 4); m = (b(j + 4) >> 4) | ((b(j) >> 6) << 4); }
}

// get_scale_min_k4 for all 8 sub-blocks at once, four 6-bit values per dword: byte j of sc_lo / m_lo is
// sub-block j, byte j of sc_hi / m_hi sub-block 4 + j (scales bytes 0-3 = hdr.y, 4-7 = hdr.z, 8-11 = hdr.w)
__device__ __forceinline__ void k4_all(const uint4 &h, uint32_t &sc_lo, uint32_t &sc_hi, uint32_t &m_lo, uint32_t &m_hi) {
    sc_lo = h.y & 0x3F3F3F3Fu;
    m_lo = h.z & 0x3F3F3F3Fu;
    sc_hi = (h.w & 0x0F0F0F0Fu) | ((h.y >> 2) & 0x30303030u);
    m_hi = ((h.w >> 4) & 0x0F0F0F0Fu) | ((h.z >> 2) & 0x30303030u);
}

// fragment slot for element k (0..255) of weight row nl (0..63): (tile, step, lane); 16 B per slot
__device__ __forceinline__ int bslot(int nl, int k) {
    const int tile = nl >> 5, s = k >> 4, h = (k >> 3) & 1;
    return ((tile * 16 + s) * 64 + h * 32 + (nl & 31));
}

template <int TYPE> struct GemmTraits {
    static constexpr int NB = 1;            // B fragment planes (Q6_K: 2)
    static constexpr bool MINS = false;     // Q8_K bsum x mins term
    static constexpr bool SB = true;        // per-256 scaling (K-quants) vs per-32 (Q4_0/Q8_0)
};
template <> struct GemmTraits<KT_Q4_K> { static constexpr int NB = 1; static constexpr bool MINS = true; static constexpr bool SB = true; };
template <> struct GemmTraits<KT_Q5_K> { static constexpr int NB = 1; static constexpr bool MINS = true; static constexpr bool SB = true; };
template <> struct GemmTraits<KT_Q6_K> { static constexpr int NB = 2; static constexpr bool MINS = false; static constexpr bool SB = true; };
template <> struct GemmTraits<KT_Q3_K> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = true; };
template <> struct GemmTraits<KT_Q2_K> { static constexpr int NB = 1; static constexpr bool MINS = true; static constexpr bool SB = true; };
template <> struct GemmTraits<KT_Q4_0> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_Q5_0> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_Q8_0> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_Q4_1> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_Q5_1> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_IQ4_NL> { static constexpr int NB = 1; static constexpr bool MINS = false; static constexpr bool SB = false; };
template <> struct GemmTraits<KT_IQ4_XS> { static constexpr int NB = 2; static constexpr bool MINS = false; static constexpr bool SB = true; };
// Q8_1-activation types: the per-block m_w * s_a term (block_q8_1.s)
template <int TYPE> constexpr bool kGemmM1 = TYPE == KT_Q4_1 || TYPE == KT_Q5_1;

template <int NB> struct GemmSmem {
    h8v bf[NB][2 * 16 * 64];      // [plane][tile*16*64 + step*64 + lane]
    h8v bm[2 * 64];               // mins fragment [tile*64 + lane]
    float wd[GB_N][8];            // K-quants: [0]=d, [1]=dmin ; Q4_0/Q8_0: d per 32-block
    float dy[GB_M][8];            // K-quants: [0]=dy of this super-block ; Q4_0/Q8_0: per 32-block
    float wm[GB_N][8];            // Q4_1 / Q5_1: m per 32-block
    float sy[GB_M][8];            // Q4_1 / Q5_1: block_q8_1.s per 32-block
};

// dequantize the 64 x 256 weight tile of super-block `sb` into LDS (thread t: row t>>2, chunk t&3)
template <int TYPE, typename SM>
__device__ __forceinline__ void stage_weights(SM &S, const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                              int64_t n0, int64_t sb) {
    const int t = threadIdx.x, nl = t >> 2, c = t & 3;
    const int64_t n = min(n0 + nl, N - 1);
    const int64_t bpr = K / ks_block_elems(TYPE);
    const int64_t nbt = bpr * N;
    if constexpr (TYPE == KT_Q4_K || TYPE == KT_Q5_K) {
        const int BB = TYPE == KT_Q4_K ? 144 : 176;
        const uint8_t *blk = W + (n * bpr + sb) * BB;
        const uint4 hdr = *(const uint4 *)blk;
        const uint4 q0 = *(const uint4 *)(blk + (TYPE == KT_Q4_K ? 16 : 48) + 32 * c);
        const uint4 q1 = *(const uint4 *)(blk + (TYPE == KT_Q4_K ? 32 : 64) + 32 * c);
        uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0;
        if constexpr (TYPE == KT_Q5_K) { h0 = *(const uint4 *)(blk + 16); h1 = *(const uint4 *)(blk + 32); }
        int s0, m0, s1, m1;
        k4_sm(hdr, 2 * c, s0, m0);
        k4_sm(hdr, 2 * c + 1, s1, m1);
        const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const uint32_t hd[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t lo0 = qd[2 * i] & 0x0F0F0F0Fu, lo1 = qd[2 * i + 1] & 0x0F0F0F0Fu;
            uint32_t hi0 = (qd[2 * i] >> 4) & 0x0F0F0F0Fu, hi1 = (qd[2 * i + 1] >> 4) & 0x0F0F0F0Fu;
            if constexpr (TYPE == KT_Q5_K) {
                lo0 |= ((hd[2 * i] >> (2 * c)) & 0x01010101u) << 4;
                lo1 |= ((hd[2 * i + 1] >> (2 * c)) & 0x01010101u) << 4;
                hi0 |= ((hd[2 * i] >> (2 * c + 1)) & 0x01010101u) << 4;
                hi1 |= ((hd[2 * i + 1] >> (2 * c + 1)) & 0x01010101u) << 4;
            }
            S.bf[0][bslot(nl, 64 * c + 8 * i)] = frag8(lo0, lo1, (float)s0, 0.0f);
            S.bf[0][bslot(nl, 64 * c + 32 + 8 * i)] = frag8(hi0, hi1, (float)s1, 0.0f);
        }
        // mins fragment: k = g (0..15) holds m_{g/2}; this thread owns g = 4c..4c+3
        _Float16 *bm = (_Float16 *)&S.bm[(nl >> 5) * 64 + (c >> 1) * 32 + (nl & 31)] + 4 * (c & 1);
        bm[0] = (_Float16)m0; bm[1] = (_Float16)m0; bm[2] = (_Float16)m1; bm[3] = (_Float16)m1;
        if (c == 0) {
            S.wd[nl][0] = h2f((uint16_t)(hdr.x & 0xFFFF));
            S.wd[nl][1] = h2f((uint16_t)(hdr.x >> 16));
        }
    } else if constexpr (TYPE == KT_Q6_K) {
        const int64_t b = n * bpr + sb;
        const uint8_t *q = W + b * 192;
        const int8_t *scp = (const int8_t *)(W + nbt * 192 + b * 16);
        const int hh = c >> 1;                   // 128-element half
        const int pb = 2 * (c & 1);              // planes pb, pb+1
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const int p = pb + pp;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2 ql = *(const uint2 *)(q + 64 * hh + 32 * (p & 1) + 8 * i);
                const uint2 qh = *(const uint2 *)(q + 128 + 32 * hh + 8 * i);
                const int sh4 = 4 * (p >> 1);
                const uint32_t v0 = ((ql.x >> sh4) & 0x0F0F0F0Fu) | (((qh.x >> (2 * p)) & 0x03030303u) << 4);
                const uint32_t v1 = ((ql.y >> sh4) & 0x0F0F0F0Fu) | (((qh.y >> (2 * p)) & 0x03030303u) << 4);
                const int scv = scp[8 * hh + (i >> 1) + 2 * p];
                const int shi = scv >> 3, slo = scv & 7;
                const int k = 128 * hh + 32 * p + 8 * i;
                S.bf[0][bslot(nl, k)] = frag8_sub(v0, v1, (float)(8 * shi), 32.0f);
                S.bf[1][bslot(nl, k)] = frag8_sub(v0, v1, (float)slo, 32.0f);
            }
        }
        if (c == 0) S.wd[nl][0] = h2f(*(const uint16_t *)(W + nbt * 208 + b * 2));
    } else if constexpr (TYPE == KT_Q2_K) {
        // chunk c = quarter c (half n = c >> 1, shifts 2 (c & 1), +1); weights (sc & 15) q exact (<= 45); mins
        // (sc >> 4) per 16-group straight into the bsum fragment; SoA planes: scales [nb][16], qs [nb][64], d/dmin
        const int64_t b = n * bpr + sb;
        const int hn = c >> 1, j0 = 2 * (c & 1);
        const uint8_t *qp = W + nbt * 16 + b * 64 + 32 * hn;
        const uint4 q0 = *(const uint4 *)qp, q1 = *(const uint4 *)(qp + 16);
        const uint32_t sw = *(const uint32_t *)(W + b * 16 + 4 * c);
        const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = j0 + (i >> 2), w0 = 2 * (i & 3);
            const int sc = (int)((sw >> (8 * (2 * (i >> 2) + ((i & 3) >> 1)))) & 0xF);
            S.bf[0][bslot(nl, 64 * c + 8 * i)] = frag8((qd[w0] >> (2 * j)) & 0x03030303u, (qd[w0 + 1] >> (2 * j)) & 0x03030303u,
                                                       (float)sc, 0.0f);
        }
        _Float16 *bm = (_Float16 *)&S.bm[(nl >> 5) * 64 + (c >> 1) * 32 + (nl & 31)] + 4 * (c & 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) bm[t] = (_Float16)(float)((sw >> (8 * t + 4)) & 0xF);
        if (c == 0) {
            const uint32_t dd = *(const uint32_t *)(W + nbt * 80 + b * 4);
            S.wd[nl][0] = h2f((uint16_t)(dd & 0xFFFF));
            S.wd[nl][1] = h2f((uint16_t)(dd >> 16));
        }
    } else if constexpr (TYPE == KT_Q3_K) {
        // chunk c = quarter c of the super-block (half n = c >> 1, shifts j0 = 2 (c & 1), j0 + 1); weights
        // (sc - 32) (v - 4) with v = 2 low bits | hmask bit << 2 -- exact f16 integers (|.| <= 128); SoA planes
        // (quant.hip kl_store_block): hmask [nb][32], qs [nb][64], scales [nb][12], d [nb][2]
        const int64_t b = n * bpr + sb;
        const int hn = c >> 1, j0 = 2 * (c & 1);
        const uint4 h0 = *(const uint4 *)(W + b * 32), h1 = *(const uint4 *)(W + b * 32 + 16);
        const uint8_t *qp = W + nbt * 32 + b * 64 + 32 * hn;
        const uint4 q0 = *(const uint4 *)qp, q1 = *(const uint4 *)(qp + 16);
        const uint32_t *scp = (const uint32_t *)(W + nbt * 96 + b * 12);
        const uint32_t a0 = scp[0], a1 = scp[1], a2 = scp[2];
        const uint32_t k1 = 0x03030303u, k2 = 0x0f0f0f0fu;
        const uint32_t sw = c == 0 ? (a0 & k2) | ((a2 & k1) << 4)
                          : c == 1 ? (a1 & k2) | (((a2 >> 2) & k1) << 4)
                          : c == 2 ? ((a0 >> 4) & k2) | (((a2 >> 4) & k1) << 4)
                                   : ((a1 >> 4) & k2) | (((a2 >> 6) & k1) << 4);
        const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const uint32_t hd[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = j0 + (i >> 2), w0 = 2 * (i & 3);            // elements l = 8 (i & 3) .. + 7
            const uint32_t v0 = ((qd[w0] >> (2 * j)) & 0x03030303u) | (((hd[w0] >> (4 * hn + j)) & 0x01010101u) << 2);
            const uint32_t v1 = ((qd[w0 + 1] >> (2 * j)) & 0x03030303u) | (((hd[w0 + 1] >> (4 * hn + j)) & 0x01010101u) << 2);
            const int sc = (int)((sw >> (8 * (2 * (i >> 2) + ((i & 3) >> 1)))) & 0xFF) - 32;
            S.bf[0][bslot(nl, 64 * c + 8 * i)] = frag8_sub(v0, v1, (float)sc, 4.0f);
        }
        if (c == 0) S.wd[nl][0] = h2f(*(const uint16_t *)(W + nbt * 108 + b * 2));
    } else if constexpr (TYPE == KT_Q4_0) {
        // this thread: 32-blocks 2c, 2c+1 of the 8 in the super-step
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int jb = 2 * c + bb;
            const int64_t b = n * bpr + sb * 8 + jb;
            const uint4 qv = *(const uint4 *)(W + b * 16);
            const uint32_t qd[4] = {qv.x, qv.y, qv.z, qv.w};
            S.bf[0][bslot(nl, 32 * jb + 0)] = frag8(qd[0] & 0x0F0F0F0Fu, qd[1] & 0x0F0F0F0Fu, 1.0f, 8.0f);
            S.bf[0][bslot(nl, 32 * jb + 8)] = frag8(qd[2] & 0x0F0F0F0Fu, qd[3] & 0x0F0F0F0Fu, 1.0f, 8.0f);
            S.bf[0][bslot(nl, 32 * jb + 16)] = frag8((qd[0] >> 4) & 0x0F0F0F0Fu, (qd[1] >> 4) & 0x0F0F0F0Fu, 1.0f, 8.0f);
            S.bf[0][bslot(nl, 32 * jb + 24)] = frag8((qd[2] >> 4) & 0x0F0F0F0Fu, (qd[3] >> 4) & 0x0F0F0F0Fu, 1.0f, 8.0f);
            S.wd[nl][jb] = h2f(*(const uint16_t *)(W + nbt * 16 + b * 2));
        }
    } else if constexpr (TYPE == KT_Q5_0) {
        // as Q4_0 with the fifth bit: (q | h << 4) - 16 in [-16, 15], exact in f16
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int jb = 2 * c + bb;
            const int64_t b = n * bpr + sb * 8 + jb;
            const uint4 qv = *(const uint4 *)(W + b * 16);
            const uint32_t h = *(const uint32_t *)(W + nbt * 16 + b * 4);
            const uint32_t qd[4] = {qv.x, qv.y, qv.z, qv.w};
            auto hb = [&](int sh) { return (((h >> sh) & 0xFu) * 0x00204081u & 0x01010101u) << 4; };
            S.bf[0][bslot(nl, 32 * jb + 0)] = frag8((qd[0] & 0x0F0F0F0Fu) | hb(0), (qd[1] & 0x0F0F0F0Fu) | hb(4), 1.0f, 16.0f);
            S.bf[0][bslot(nl, 32 * jb + 8)] = frag8((qd[2] & 0x0F0F0F0Fu) | hb(8), (qd[3] & 0x0F0F0F0Fu) | hb(12), 1.0f, 16.0f);
            S.bf[0][bslot(nl, 32 * jb + 16)] = frag8(((qd[0] >> 4) & 0x0F0F0F0Fu) | hb(16), ((qd[1] >> 4) & 0x0F0F0F0Fu) | hb(20),
                                                     1.0f, 16.0f);
            S.bf[0][bslot(nl, 32 * jb + 24)] = frag8(((qd[2] >> 4) & 0x0F0F0F0Fu) | hb(24), ((qd[3] >> 4) & 0x0F0F0F0Fu) | hb(28),
                                                     1.0f, 16.0f);
            S.wd[nl][jb] = h2f(*(const uint16_t *)(W + nbt * 20 + b * 2));
        }
    } else if constexpr (TYPE == KT_Q4_1 || TYPE == KT_Q5_1) {
        // q (| h << 4) in [0, 31] as is (s = 1, off = 0); d and m per block (SoA: qs [nb][16] (++ qh [nb][4]) ++ dm [nb][4])
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int jb = 2 * c + bb;
            const int64_t b = n * bpr + sb * 8 + jb;
            const uint4 qv = *(const uint4 *)(W + b * 16);
            const uint32_t qd[4] = {qv.x, qv.y, qv.z, qv.w};
            uint32_t h = 0;
            if constexpr (TYPE == KT_Q5_1) h = *(const uint32_t *)(W + nbt * 16 + b * 4);
            auto hb = [&](int sh) { return (((h >> sh) & 0xFu) * 0x00204081u & 0x01010101u) << 4; };
            S.bf[0][bslot(nl, 32 * jb + 0)] = frag8((qd[0] & 0x0F0F0F0Fu) | hb(0), (qd[1] & 0x0F0F0F0Fu) | hb(4), 1.0f, 0.0f);
            S.bf[0][bslot(nl, 32 * jb + 8)] = frag8((qd[2] & 0x0F0F0F0Fu) | hb(8), (qd[3] & 0x0F0F0F0Fu) | hb(12), 1.0f, 0.0f);
            S.bf[0][bslot(nl, 32 * jb + 16)] = frag8(((qd[0] >> 4) & 0x0F0F0F0Fu) | hb(16), ((qd[1] >> 4) & 0x0F0F0F0Fu) | hb(20),
                                                     1.0f, 0.0f);
            S.bf[0][bslot(nl, 32 * jb + 24)] = frag8(((qd[2] >> 4) & 0x0F0F0F0Fu) | hb(24), ((qd[3] >> 4) & 0x0F0F0F0Fu) | hb(28),
                                                     1.0f, 0.0f);
            const uint32_t dm = *(const uint32_t *)(W + nbt * (TYPE == KT_Q5_1 ? 20 : 16) + b * 4);
            S.wd[nl][jb] = h2f((uint16_t)(dm & 0xFFFF));
            S.wm[nl][jb] = h2f((uint16_t)(dm >> 16));
        }
    } else if constexpr (TYPE == KT_IQ4_NL) {
        // code-book values kvalues_iq4nl[q] in [-127, 113] through v_perm (iq4nl_lut4), as Q8_0's biased bytes
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int jb = 2 * c + bb;
            const int64_t b = n * bpr + sb * 8 + jb;
            const uint4 qv = *(const uint4 *)(W + b * 16);
            const uint32_t qd[4] = {qv.x, qv.y, qv.z, qv.w};
            auto lv = [&](uint32_t x) { return iq4nl_lut4(x & 0x0F0F0F0Fu) ^ 0x80808080u; };
            S.bf[0][bslot(nl, 32 * jb + 0)] = frag8(lv(qd[0]), lv(qd[1]), 1.0f, 128.0f);
            S.bf[0][bslot(nl, 32 * jb + 8)] = frag8(lv(qd[2]), lv(qd[3]), 1.0f, 128.0f);
            S.bf[0][bslot(nl, 32 * jb + 16)] = frag8(lv(qd[0] >> 4), lv(qd[1] >> 4), 1.0f, 128.0f);
            S.bf[0][bslot(nl, 32 * jb + 24)] = frag8(lv(qd[2] >> 4), lv(qd[3] >> 4), 1.0f, 128.0f);
            S.wd[nl][jb] = h2f(*(const uint16_t *)(W + nbt * 16 + b * 2));
        }
    } else if constexpr (TYPE == KT_IQ4_XS) {
        // sub-blocks 2c, 2c+1: (ls - 32) kv split as 8 (sc >> 3) kv + (sc & 7) kv over two planes (as Q6_K), both exact
        // f16 integers; SoA: qs [nb][128] ++ (d, scales_h, scales_l[4]) [nb][8]
        const int64_t b = n * bpr + sb;
        const uint2 hv = *(const uint2 *)(W + nbt * 128 + b * 8);
        const uint32_t shv = hv.x >> 16, slv = hv.y;
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int ib = 2 * c + bb;
            const uint4 qv = *(const uint4 *)(W + b * 128 + 16 * ib);
            const uint32_t qd[4] = {qv.x, qv.y, qv.z, qv.w};
            const int sc = (int)(((slv >> (8 * (ib >> 1) + 4 * (ib & 1))) & 0xF) | (((shv >> (2 * ib)) & 3) << 4)) - 32;
            const float shi = (float)(8 * (sc >> 3)), slo = (float)(sc & 7);
            auto lv = [&](uint32_t x) { return iq4nl_lut4(x & 0x0F0F0F0Fu) ^ 0x80808080u; };
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int sh = i < 2 ? 0 : 4, w0 = 2 * (i & 1);
                const uint32_t t0 = lv(qd[w0] >> sh), t1 = lv(qd[w0 + 1] >> sh);
                S.bf[0][bslot(nl, 32 * ib + 8 * i)] = frag8_sub(t0, t1, shi, 128.0f);
                S.bf[1][bslot(nl, 32 * ib + 8 * i)] = frag8_sub(t0, t1, slo, 128.0f);
            }
        }
        if (c == 0) S.wd[nl][0] = h2f((uint16_t)(hv.x & 0xFFFF));
    } else if constexpr (kIqGrid<TYPE>) {
        // the grid types (iq_grid.h, ggml layout): sub-blocks 2c, 2c+1; codes biased to bytes (+128), times the group's
        // integer scale: exact f16 integers (|code ls| <= 62 x 31); d C per super-block
        const uint8_t *blk = W + (n * bpr + sb) * ks_block_bytes(TYPE);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int ib = 2 * c + bb;
            IqSub q;
            iq_sub<TYPE>(blk, ib, q);
#pragma unroll
            for (int l = 0; l < 4; ++l)
                S.bf[0][bslot(nl, 32 * ib + 8 * l)] = frag8(q.v[2 * l] ^ 0x80808080u, q.v[2 * l + 1] ^ 0x80808080u,
                                                           (float)q.ls[l], 128.0f);
        }
        if (c == 0) S.wd[nl][0] = iq_d<TYPE>(blk) * iq_const<TYPE>();
    } else {   // Q8_0: int8 -> (q ^ 0x80) = q + 128 as a byte
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int jb = 2 * c + bb;
            const int64_t b = n * bpr + sb * 8 + jb;
            const uint4 q0 = *(const uint4 *)(W + b * 32), q1 = *(const uint4 *)(W + b * 32 + 16);
            const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
                S.bf[0][bslot(nl, 32 * jb + 8 * i)] = frag8(qd[2 * i] ^ 0x80808080u, qd[2 * i + 1] ^ 0x80808080u, 1.0f, 128.0f);
            S.wd[nl][jb] = h2f(*(const uint16_t *)(W + nbt * 32 + b * 2));
        }
    }
}

template <int TYPE>
__global__ void __launch_bounds__(256, 2) k_gemm(const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                              const _Float16 *__restrict__ a16, const float *__restrict__ dyg,
                                              const _Float16 *__restrict__ bs16, int64_t M, float *__restrict__ Y,
                                              int64_t ldy, const float *res, int64_t ldr, const float *__restrict__ sg,
                                              float *__restrict__ part, int64_t Mp) {
    using T = GemmTraits<TYPE>;
    __shared__ GemmSmem<T::NB> S;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n0 = (int64_t)blockIdx.x * GB_N, m0 = (int64_t)blockIdx.y * GB_M;
    // split-K (gridDim.z > 1): this workgroup's super-block range; partials to part [z][Mp][N], summed in order by
    // k_splitk_reduce
    const int64_t nsb_all = K / GB_K, nsb_z = nsb_all / gridDim.z;
    const int64_t sb0 = (int64_t)blockIdx.z * nsb_z, nsb = sb0 + nsb_z;
    const int64_t G = T::SB ? 256 : 32;
    const int lr = lane & 31, lh = lane >> 5;
    const int64_t arow = m0 + 32 * wave + lr;                  // token row this lane feeds into A
    const _Float16 *ap = a16 + arow * K + 8 * lh;
    f16acc tot[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) { tot[0][i] = 0.0f; tot[1][i] = 0.0f; }

    for (int64_t sb = sb0; sb < nsb; ++sb) {
        __syncthreads();                                        // previous step done with LDS
        stage_weights<TYPE>(S, W, K, N, n0, sb);
        // K-quants: the super-block's 16 A fragments, issued behind the weight loads (one latency per step, not one
        // per MFMA pair); per-32 types load theirs per half super-block below (register pressure of 8 epilogues)
        h8v av[16];
        if constexpr (T::SB) {
#pragma unroll
            for (int s = 0; s < 16; ++s) av[s] = *(const h8v *)(ap + sb * GB_K + 16 * s);
        }
        if (threadIdx.x < GB_M) {
            if constexpr (T::SB) S.dy[threadIdx.x][0] = dyg[(m0 + threadIdx.x) * (K / 256) + sb];
            else {
#pragma unroll
                for (int j = 0; j < 8; ++j) S.dy[threadIdx.x][j] = dyg[(m0 + threadIdx.x) * (K / 32) + sb * 8 + j];
                if constexpr (kGemmM1<TYPE>) {
                    const bool ok = m0 + threadIdx.x < M;
#pragma unroll
                    for (int j = 0; j < 8; ++j) S.sy[threadIdx.x][j] = ok ? sg[(m0 + threadIdx.x) * (K / 32) + sb * 8 + j] : 0.0f;
                }
            }
        }
        __syncthreads();
        if constexpr (T::SB) {
            f16acc acc[2], accm[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) { acc[0][i] = acc[1][i] = 0.0f; accm[0][i] = accm[1][i] = 0.0f; }
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const h8v a = av[s];
#pragma unroll
                for (int tl = 0; tl < 2; ++tl) {
                    acc[tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, S.bf[0][(tl * 16 + s) * 64 + lane], acc[tl], 0, 0, 0);
                    if constexpr (T::NB == 2)
                        acc[tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, S.bf[T::NB - 1][(tl * 16 + s) * 64 + lane], acc[tl], 0, 0, 0);
                }
            }
            if constexpr (T::MINS) {
                const h8v am = *(const h8v *)(bs16 + arow * (K / 16) + sb * 16 + 8 * lh);
#pragma unroll
                for (int tl = 0; tl < 2; ++tl)
                    accm[tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(am, S.bm[tl * 64 + lane], accm[tl], 0, 0, 0);
            }
            // epilogue: tot += dy*d*sumi - dy*dmin*summ  (ggml_vec_dot_q4_K_q8_K, ggml-quants.c:7796-7859)
#pragma unroll
            for (int tl = 0; tl < 2; ++tl) {
                const float dw = S.wd[tl * 32 + lr][0];
                const float dm = T::MINS ? S.wd[tl * 32 + lr][1] : 0.0f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int tk = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float dy = S.dy[tk][0];
                    float v = __fmul_rn(__fmul_rn(dy, dw), acc[tl][r]);
                    if constexpr (T::MINS) v = __fsub_rn(v, __fmul_rn(__fmul_rn(dy, dm), accm[tl][r]));
                    tot[tl][r] = __fadd_rn(tot[tl][r], v);
                }
            }
        } else {
            // Q4_1 / Q5_1: + sum_j m_w[j] s_a[j] over the 8 blocks, an fp32 product of the [tokens x 8] s and
            // [8 x rows] m tiles on the matrix cores (ggml_vec_dot_q4_1_q8_1 / _q5_1_q8_1, ggml-quants.c:4503,5145)
            if constexpr (kGemmM1<TYPE>) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const float a = S.sy[32 * wave + lr][2 * kk + lh];
#pragma unroll
                    for (int tl = 0; tl < 2; ++tl)
                        tot[tl] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, S.wm[tl * 32 + lr][2 * kk + lh], tot[tl], 0, 0, 0);
                }
            }
#pragma unroll 1
            for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
            for (int s = 0; s < 8; ++s) av[s] = *(const h8v *)(ap + sb * GB_K + 128 * hb + 16 * s);
#pragma unroll
            for (int jq = 0; jq < 4; ++jq) {
                const int jb = 4 * hb + jq;
                f16acc acc[2];
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[0][i] = acc[1][i] = 0.0f;
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int s = 2 * jb + ss;
                    const h8v a = av[2 * jq + ss];
#pragma unroll
                    for (int tl = 0; tl < 2; ++tl)
                        acc[tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, S.bf[0][(tl * 16 + s) * 64 + lane], acc[tl], 0, 0, 0);
                }
                // tot += sumi * (d_w * d_a)   (ggml_vec_dot_q8_0_q8_0 scalar tail, ggml-quants.c:5519)
#pragma unroll
                for (int tl = 0; tl < 2; ++tl) {
                    const float dw = S.wd[tl * 32 + lr][jb];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int tk = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * lh;
                        tot[tl][r] = __fadd_rn(tot[tl][r], __fmul_rn(acc[tl][r], __fmul_rn(dw, S.dy[tk][jb])));
                    }
                }
            }
            }
        }
    }
    // store (+ residual)
#pragma unroll
    for (int tl = 0; tl < 2; ++tl) {
        const int64_t n = n0 + tl * 32 + lr;
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t t = m0 + 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (gridDim.z > 1) { if (t < M) part[((int64_t)blockIdx.z * Mp + t) * N + n] = tot[tl][r]; }
            else if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[tl][r], res[t * ldr + n]) : tot[tl][r];
        }
    }
}


__device__ __forceinline__ uint4 ldg16(const void *p) { return *(const uint4 *)p; }

// ================================================================ K-quant GEMM v2 (Q4_K / Q5_K / Q6_K)
// Same exact-integer MFMA formulation as k_gemm, restructured for throughput:
//   * the activation operand is converted once into MFMA fragment order (k_act_frag): every wave-load
//     of A is one contiguous 1 KiB (16 B per lane), read straight from L2 into registers, two half
//     super-blocks in flight (the next one issued while the current one is multiplied);
//   * the dequantized weight tile (64 rows x 256, f16 sc*q integers) is double-buffered in LDS: the
//     raw bytes of super-block sb+1 are loaded into registers before the MFMAs of sb are issued and
//     dequantized into the other buffer after them -- one barrier per super-block;
//   * XCD-aware tile order: the workgroups of one token tile sit on the same XCD (blockIdx % 8 under
//     round-robin dispatch; speed only), so each XCD's L2 holds one activation slice instead of all.
// Epilogue per super-block: tot += dy * (d * S - dmin * Mn)  (S, Mn exact integers; CPU:
// ggml_vec_dot_q4_K_q8_K, ggml-quants.c:7796-7859 -- same value, fp32 combination order differs).

// A fragment order: af[(mt*(K/16) + s16)*64 + lane] = 8 halves of token 32mt + (lane&31),
// k = 16 s16 + 8 (lane>>5) .. +7.  bsf[(mt*(K/256) + sb)*64 + lane] = Q8_K bsums g = 8 (lane>>5)..+7.
__global__ void k_act_frag(const uint8_t *__restrict__ act, int64_t K, int64_t M, int64_t Mp, h8v *__restrict__ af,
                           float *__restrict__ dy, h8v *__restrict__ bsf) {
    const int64_t nA = Mp * K / 8, nS = (Mp / 32) * (K / 256) * 64, nD = Mp * (K / 256);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int8_t *qs = (const int8_t *)act;
    const float *d = (const float *)(act + M * K);
    const int16_t *bs = (const int16_t *)(act + M * K + M * (K / 256) * 4);
    if (i < nA) {
        const int lane = (int)(i & 63);
        const int64_t s16 = (i >> 6) % (K / 16), mt = (i >> 6) / (K / 16);
        const int64_t m = 32 * mt + (lane & 31), k0 = 16 * s16 + 8 * (lane >> 5);
        uint2 v = make_uint2(0, 0);
        if (m < M) v = *(const uint2 *)(qs + m * K + k0);
        const uint32_t w[2] = {v.x, v.y};
        h8v r;
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = (_Float16)(int8_t)((w[e >> 2] >> (8 * (e & 3))) & 0xFF);
        af[i] = r;
    } else if (i < nA + nS) {
        const int64_t j = i - nA;
        const int lane = (int)(j & 63);
        const int64_t sb = (j >> 6) % (K / 256), mt = (j >> 6) / (K / 256);
        const int64_t m = 32 * mt + (lane & 31);
        h8v r;
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = m < M ? (_Float16)bs[m * (K / 16) + sb * 16 + 8 * (lane >> 5) + e] : (_Float16)0;
        bsf[j] = r;
    } else if (i < nA + nS + nD) {
        const int64_t j = i - nA - nS;
        const int64_t m = j / (K / 256);
        dy[j] = m < M ? d[j] : 0.0f;
    }
}

template <int TYPE> struct KqRaw;
template <> struct KqRaw<KT_Q4_K> { uint4 h, q0, q1; };
template <> struct KqRaw<KT_Q5_K> { uint4 h, q0, q1, qh0, qh1; };
template <> struct KqRaw<KT_Q6_K> { uint4 ql[4], qh[2]; uint32_t sc; uint32_t d; };

// raw bytes of unit (row n, chunk c) of super-block sb; LAY 0: the kcpp layout, 1: the row-major decode
// layouts KT_Q4_K_RS / KT_Q5_K_RS / KT_Q6_K_RS (kcpp_common.h; same raw unit, gathered from the row's planes)
template <int TYPE, int LAY>
__device__ __forceinline__ void kq_load(KqRaw<TYPE> &r, const uint8_t *__restrict__ W, int64_t bpr, int64_t nbt,
                                        int64_t n, int c, int64_t sb) {
    const int64_t b = n * bpr + sb;
    if constexpr (LAY == 1 && TYPE == KT_Q4_K) {
        const uint8_t *row = W + n * 144 * bpr;
        r.h = ldg16(row + 16 * sb);
        r.q0 = ldg16(row + 16 * bpr + 128 * sb + 32 * c);
        r.q1 = ldg16(row + 16 * bpr + 128 * sb + 32 * c + 16);
    } else if constexpr (LAY == 1 && TYPE == KT_Q5_K) {
        const uint8_t *row = W + n * 176 * bpr;
        r.h = ldg16(row + 16 * sb);
        r.qh0 = ldg16(row + 144 * bpr + 32 * sb);
        r.qh1 = ldg16(row + 144 * bpr + 32 * sb + 16);
        r.q0 = ldg16(row + 16 * bpr + 128 * sb + 32 * c);
        r.q1 = ldg16(row + 16 * bpr + 128 * sb + 32 * c + 16);
    } else if constexpr (LAY == 1 && TYPE == KT_Q6_K) {
        const int hh = c >> 1, pb = 2 * (c & 1);
        const uint8_t *row = W + n * 210 * bpr;
        const int64_t U0 = 4 * sb + 2 * hh;                     // units (hh, lh = 0) and (hh, lh = 1)
        r.ql[0] = ldg16(row + 16 * U0);
        r.ql[1] = ldg16(row + 16 * U0 + 16);
        r.ql[2] = ldg16(row + 64 * bpr + 16 * U0);
        r.ql[3] = ldg16(row + 64 * bpr + 16 * U0 + 16);
        r.qh[0] = ldg16(row + 128 * bpr + 16 * U0);
        r.qh[1] = ldg16(row + 128 * bpr + 16 * U0 + 16);
        // unit (hh, lh) holds sc[8 hh + lh + 2 g], g = 0..3; the stage wants sc[8 hh + pb + 0..3]
        const uint32_t s0 = *(const uint32_t *)(row + 192 * bpr + 4 * U0), s1 = *(const uint32_t *)(row + 192 * bpr + 4 * U0 + 4);
        const int k0 = pb / 2 * 2;
        r.sc = ((s0 >> (8 * k0)) & 0xFF) | (((s1 >> (8 * k0)) & 0xFF) << 8) | (((s0 >> (8 * k0 + 8)) & 0xFF) << 16) |
               (((s1 >> (8 * k0 + 8)) & 0xFF) << 24);
        r.d = *(const uint16_t *)(row + 208 * bpr + 2 * sb);
    } else if constexpr (TYPE == KT_Q4_K) {
        const uint8_t *blk = W + b * 144;
        r.h = ldg16(blk);
        r.q0 = ldg16(blk + 16 + 32 * c);
        r.q1 = ldg16(blk + 32 + 32 * c);
    } else if constexpr (TYPE == KT_Q5_K) {
        const uint8_t *blk = W + b * 176;
        r.h = ldg16(blk);
        r.qh0 = ldg16(blk + 16);
        r.qh1 = ldg16(blk + 32);
        r.q0 = ldg16(blk + 48 + 32 * c);
        r.q1 = ldg16(blk + 64 + 32 * c);
    } else {
        const int hh = c >> 1, pb = 2 * (c & 1);
        const uint8_t *q = W + b * 192;
#pragma unroll
        for (int i = 0; i < 4; ++i) r.ql[i] = ldg16(q + 64 * hh + 16 * i);
        r.qh[0] = ldg16(q + 128 + 32 * hh);
        r.qh[1] = ldg16(q + 128 + 32 * hh + 16);
        r.sc = *(const uint32_t *)(W + nbt * 192 + b * 16 + 8 * hh + 2 * pb);
        r.d = *(const uint16_t *)(W + nbt * 208 + b * 2);
    }
}

template <int NB> struct KqSmem {
    h8v bf[2][NB][2 * 16 * 64];   // [buf][plane][tile*16*64 + step*64 + lane]
    h8v bm[2][2 * 64];            // mins fragment [buf][tile*64 + lane]
    float wd[2][GB_N][2];         // d, dmin per row
};

// dequantize the raw unit into LDS buffer `buf` (fragment order; thread: row nl, chunk c)
template <int TYPE, typename SM>
__device__ __forceinline__ void kq_stage(SM &S, int buf, const KqRaw<TYPE> &r, int nl, int c) {
    if constexpr (TYPE == KT_Q4_K || TYPE == KT_Q5_K) {
        int s0, m0, s1, m1;
        k4_sm(r.h, 2 * c, s0, m0);
        k4_sm(r.h, 2 * c + 1, s1, m1);
        const uint32_t qd[8] = {r.q0.x, r.q0.y, r.q0.z, r.q0.w, r.q1.x, r.q1.y, r.q1.z, r.q1.w};
        uint32_t hd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (TYPE == KT_Q5_K) {
            hd[0] = r.qh0.x; hd[1] = r.qh0.y; hd[2] = r.qh0.z; hd[3] = r.qh0.w;
            hd[4] = r.qh1.x; hd[5] = r.qh1.y; hd[6] = r.qh1.z; hd[7] = r.qh1.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t lo0 = qd[2 * i] & 0x0F0F0F0Fu, lo1 = qd[2 * i + 1] & 0x0F0F0F0Fu;
            uint32_t hi0 = (qd[2 * i] >> 4) & 0x0F0F0F0Fu, hi1 = (qd[2 * i + 1] >> 4) & 0x0F0F0F0Fu;
            if constexpr (TYPE == KT_Q5_K) {
                lo0 |= ((hd[2 * i] >> (2 * c)) & 0x01010101u) << 4;
                lo1 |= ((hd[2 * i + 1] >> (2 * c)) & 0x01010101u) << 4;
                hi0 |= ((hd[2 * i] >> (2 * c + 1)) & 0x01010101u) << 4;
                hi1 |= ((hd[2 * i + 1] >> (2 * c + 1)) & 0x01010101u) << 4;
            }
            S.bf[buf][0][bslot(nl, 64 * c + 8 * i)] = frag8(lo0, lo1, (float)s0, 0.0f);
            S.bf[buf][0][bslot(nl, 64 * c + 32 + 8 * i)] = frag8(hi0, hi1, (float)s1, 0.0f);
        }
        _Float16 *bm = (_Float16 *)&S.bm[buf][(nl >> 5) * 64 + (c >> 1) * 32 + (nl & 31)] + 4 * (c & 1);
        bm[0] = (_Float16)m0; bm[1] = (_Float16)m0; bm[2] = (_Float16)m1; bm[3] = (_Float16)m1;
        if (c == 0) {
            S.wd[buf][nl][0] = h2f((uint16_t)(r.h.x & 0xFFFF));
            S.wd[buf][nl][1] = h2f((uint16_t)(r.h.x >> 16));
        }
    } else {
        const int hh = c >> 1, pb = 2 * (c & 1);
        const uint32_t qlw[16] = {r.ql[0].x, r.ql[0].y, r.ql[0].z, r.ql[0].w, r.ql[1].x, r.ql[1].y, r.ql[1].z, r.ql[1].w,
                                  r.ql[2].x, r.ql[2].y, r.ql[2].z, r.ql[2].w, r.ql[3].x, r.ql[3].y, r.ql[3].z, r.ql[3].w};
        const uint32_t qhw[8] = {r.qh[0].x, r.qh[0].y, r.qh[0].z, r.qh[0].w, r.qh[1].x, r.qh[1].y, r.qh[1].z, r.qh[1].w};
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const int p = pb + pp;
            const int sh4 = 4 * (p >> 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // ql bytes 32*(p&1) + 8i .. +7 ; qh bytes 8i .. +7
                const uint32_t l0 = qlw[8 * (p & 1) + 2 * i], l1 = qlw[8 * (p & 1) + 2 * i + 1];
                const uint32_t h0 = qhw[2 * i], h1 = qhw[2 * i + 1];
                const uint32_t v0 = ((l0 >> sh4) & 0x0F0F0F0Fu) | (((h0 >> (2 * p)) & 0x03030303u) << 4);
                const uint32_t v1 = ((l1 >> sh4) & 0x0F0F0F0Fu) | (((h1 >> (2 * p)) & 0x03030303u) << 4);
                const int scv = (int)(int8_t)((r.sc >> (8 * ((i >> 1) + 2 * pp))) & 0xFF);
                const int shi = scv >> 3, slo = scv & 7;
                const int k = 128 * hh + 32 * p + 8 * i;
                S.bf[buf][0][bslot(nl, k)] = frag8_sub(v0, v1, (float)(8 * shi), 32.0f);
                S.bf[buf][1][bslot(nl, k)] = frag8_sub(v0, v1, (float)slo, 32.0f);
            }
        }
        if (c == 0) S.wd[buf][nl][0] = h2f((uint16_t)r.d);
    }
}

// grid: (Mp / (128 TM)) * ceil(N / 64) workgroups, 256 threads; wave w: tokens [32 TM w, 32 TM (w+1)) of the
// tile x 64 rows (TM x 2 MFMA tiles; every LDS weight fragment feeds TM MFMAs)
template <int TYPE, int TM, int LAY>
__global__ void __launch_bounds__(256, TM == 1 ? 2 : 1) k_gemm_kq(const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                                    const h8v *__restrict__ af, const float *__restrict__ dyg,
                                                    const h8v *__restrict__ bsf, int64_t M, int MT, float *__restrict__ Y,
                                                    int64_t ldy, const float *res, int64_t ldr) {
    constexpr int NB = TYPE == KT_Q6_K ? 2 : 1;
    constexpr bool MINS = TYPE != KT_Q6_K;
    constexpr int BM = GB_M * TM;
    __shared__ KqSmem<NB> S;
    __shared__ float sdy[2][BM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    // XCD-aware tile order: workgroup id -> (token tile, row tile) so that ids with equal id % 8 (one XCD
    // under round-robin dispatch) share a token tile whenever MT divides 8
    const int64_t id = blockIdx.x, nwg = gridDim.x;
    int64_t mt, nt;
    if (8 % MT == 0 && nwg % 8 == 0) {
        const int64_t x = id & 7, j = id >> 3;
        mt = x % MT;
        nt = j * (8 / MT) + x / MT;
    } else {
        mt = id % MT;
        nt = id / MT;
    }
    const int64_t n0 = nt * GB_N;
    const int64_t m0 = mt * BM;
    const int64_t nsb = K / 256, bpr = K / 256, nbt = bpr * N;
    const int nl = tid >> 2, c = tid & 3;
    const int64_t nrow = min(n0 + nl, N - 1);
    const int64_t wt0 = (m0 >> 5) + TM * wave;                 // this wave's first 32-token tile
    const h8v *ap = af + wt0 * (K / 16) * 64 + lane;           // token tile j: + j * (K/16) * 64
    const h8v *bp = bsf + wt0 * nsb * 64 + lane;               // token tile j: + j * nsb * 64
    const int64_t tstride = (K / 16) * 64;

    f16acc tot[TM][2];
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) { tot[j][0][i] = 0.0f; tot[j][1][i] = 0.0f; }

    KqRaw<TYPE> raw;
    kq_load<TYPE, LAY>(raw, W, bpr, nbt, nrow, c, 0);
    float dyn[TM];
#pragma unroll
    for (int j = 0; j < TM; ++j) dyn[j] = dyg[(m0 + j * 128 + (tid & 127)) * nsb];
    h8v a0[TM][8], a1[TM][8];
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int s = 0; s < 8; ++s) a0[j][s] = ap[j * tstride + s * 64];
    kq_stage<TYPE>(S, 0, raw, nl, c);
    if (tid < 128) {
#pragma unroll
        for (int j = 0; j < TM; ++j) sdy[0][j * 128 + tid] = dyn[j];
    }
    __syncthreads();

    for (int64_t sb = 0; sb < nsb; ++sb) {
        const int buf = (int)(sb & 1);
        const bool more = sb + 1 < nsb;
        if (more) {
            kq_load<TYPE, LAY>(raw, W, bpr, nbt, nrow, c, sb + 1);
#pragma unroll
            for (int j = 0; j < TM; ++j) dyn[j] = dyg[(m0 + j * 128 + (tid & 127)) * nsb + sb + 1];
        }
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int s = 0; s < 8; ++s) a1[j][s] = ap[j * tstride + (sb * 16 + 8 + s) * 64];
        // per-token dy of this super-block for the accumulator rows of every token tile
        float dyv[TM][16];
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)&sdy[buf][32 * (TM * wave + j) + 8 * q + 4 * lh];
                dyv[j][4 * q] = v.x; dyv[j][4 * q + 1] = v.y; dyv[j][4 * q + 2] = v.z; dyv[j][4 * q + 3] = v.w;
            }
        // mins term first (tot -= dy * dmin * sum_j m_j bsum_j), so its accumulators are free before the main loop
        if constexpr (MINS) {
#pragma unroll
            for (int j = 0; j < TM; ++j) {
                const h8v am = bp[j * nsb * 64 + sb * 64];
#pragma unroll
                for (int tl = 0; tl < 2; ++tl) {
                    f16acc accm;
#pragma unroll
                    for (int i = 0; i < 16; ++i) accm[i] = 0.0f;
                    accm = __builtin_amdgcn_mfma_f32_32x32x16_f16(am, S.bm[buf][tl * 64 + lane], accm, 0, 0, 0);
                    const float dm = S.wd[buf][tl * 32 + lr][1];
#pragma unroll
                    for (int r = 0; r < 16; ++r) tot[j][tl][r] = fmaf(-__fmul_rn(dyv[j][r], dm), accm[r], tot[j][tl][r]);
                }
            }
        }
        f16acc acc[TM][2];
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) { acc[j][0][i] = 0.0f; acc[j][1][i] = 0.0f; }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
            for (int tl = 0; tl < 2; ++tl) {
                const h8v b0 = S.bf[buf][0][(tl * 16 + s) * 64 + lane];
#pragma unroll
                for (int j = 0; j < TM; ++j) acc[j][tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[j][s], b0, acc[j][tl], 0, 0, 0);
                if constexpr (NB == 2) {
                    const h8v b1 = S.bf[buf][1][(tl * 16 + s) * 64 + lane];
#pragma unroll
                    for (int j = 0; j < TM; ++j) acc[j][tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[j][s], b1, acc[j][tl], 0, 0, 0);
                }
            }
        }
        if (more) {
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int s = 0; s < 8; ++s) a0[j][s] = ap[j * tstride + ((sb + 1) * 16 + s) * 64];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
            for (int tl = 0; tl < 2; ++tl) {
                const h8v b0 = S.bf[buf][0][(tl * 16 + 8 + s) * 64 + lane];
#pragma unroll
                for (int j = 0; j < TM; ++j) acc[j][tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[j][s], b0, acc[j][tl], 0, 0, 0);
                if constexpr (NB == 2) {
                    const h8v b1 = S.bf[buf][1][(tl * 16 + 8 + s) * 64 + lane];
#pragma unroll
                    for (int j = 0; j < TM; ++j) acc[j][tl] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[j][s], b1, acc[j][tl], 0, 0, 0);
                }
            }
        }
        // tot += dy * d * S
#pragma unroll
        for (int tl = 0; tl < 2; ++tl) {
            const float dw = S.wd[buf][tl * 32 + lr][0];
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) tot[j][tl][r] = fmaf(dyv[j][r], __fmul_rn(dw, acc[j][tl][r]), tot[j][tl][r]);
        }
        if (more) {
            kq_stage<TYPE>(S, buf ^ 1, raw, nl, c);
            if (tid < 128) {
#pragma unroll
                for (int j = 0; j < TM; ++j) sdy[buf ^ 1][j * 128 + tid] = dyn[j];
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int tl = 0; tl < 2; ++tl) {
        const int64_t n = n0 + tl * 32 + lr;
        if (n >= N) continue;
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t t = m0 + 32 * (TM * wave + j) + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[j][tl][r], res[t * ldr + n]) : tot[j][tl][r];
            }
    }
}

// ================================================================ Q4_K GEMM v3
// Same exact-integer formulation and per-super-block epilogue as k_gemm_kq (bit-identical results: every
// integer partial sum is exact in fp32), re-tiled so the activation is read from L2 once per 128 weight
// rows instead of once per 64 and the weights never pass through LDS:
//   * workgroup = 128 tokens x 128 weight rows; wave w = rows [32w, 32w+32) x all 128 tokens (4 MFMA
//     32x32x16 tiles);
//   * A (activation, f16 integers) staged in LDS by global_load_lds (16 B per lane; the fragment images
//     are lane-linear, so the LDS-DMA writes them as they are read), two buffers: super-block sb+1's copy
//     is in flight while sb is multiplied, one barrier per super-block;
//   * B: each lane dequantizes its own weight row straight into MFMA fragments from raw Q4_K bytes
//     loaded one super-block ahead.  The k order inside a sub-block pair is permuted so that a lane's 8
//     k-values are the low and high nibbles of 4 consecutive qs bytes (one dword -> one fragment):
//       MFMA step s = 4p + st (p = sub-block pair, st = 0..3), lane half kg = lane >> 5, half e:
//       e < 4 : k = 64p + 16kg + 4st + e        (sub-block 2p, low nibble of qs byte 32p + 16kg + 4st + e)
//       e >= 4: k = 64p + 32 + 16kg + 4st + e-4 (sub-block 2p+1, high nibble of the same byte)
//     and k_act_frag3 writes A in the same order.
// k_act_frag3: af as k_act_frag with the permuted k order; dyT[sb][Mp] (transposed, so one super-block's
// 128 token scales are one contiguous 512 B LDS-DMA); bsf as k_act_frag.
__global__ void k_act_frag3(const uint8_t *__restrict__ act, int64_t K, int64_t M, int64_t Mp, h8v *__restrict__ af,
                            float *__restrict__ dyT, h8v *__restrict__ bsf) {
    const int64_t nA = Mp * K / 8, nS = (Mp / 32) * (K / 256) * 64, nD = Mp * (K / 256);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int8_t *qs = (const int8_t *)act;
    const float *d = (const float *)(act + M * K);
    const int16_t *bs = (const int16_t *)(act + M * K + M * (K / 256) * 4);
    if (i < nA) {
        const int lane = (int)(i & 63), kg = lane >> 5;
        const int64_t s16 = (i >> 6) % (K / 16), mt = (i >> 6) / (K / 16);
        const int64_t m = 32 * mt + (lane & 31);
        const int p = (int)((s16 >> 2) & 3), st = (int)(s16 & 3);
        const int64_t k0 = 256 * (s16 >> 4) + 64 * p + 16 * kg + 4 * st;
        uint32_t lo = 0, hi = 0;
        if (m < M) {
            lo = *(const uint32_t *)(qs + m * K + k0);
            hi = *(const uint32_t *)(qs + m * K + k0 + 32);
        }
        h8v r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            r[e] = (_Float16)(int8_t)((lo >> (8 * e)) & 0xFF);
            r[4 + e] = (_Float16)(int8_t)((hi >> (8 * e)) & 0xFF);
        }
        af[i] = r;
    } else if (i < nA + nS) {
        const int64_t j = i - nA;
        const int lane = (int)(j & 63);
        const int64_t sb = (j >> 6) % (K / 256), mt = (j >> 6) / (K / 256);
        const int64_t m = 32 * mt + (lane & 31);
        h8v r;
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = m < M ? (_Float16)bs[m * (K / 16) + sb * 16 + 8 * (lane >> 5) + e] : (_Float16)0;
        bsf[j] = r;
    } else if (i < nA + nS + nD) {
        const int64_t j = i - nA - nS;
        const int64_t sb = j / Mp, m = j % Mp;
        dyT[j] = m < M ? d[m * (K / 256) + sb] : 0.0f;
    }
}

#ifndef V3_PRIO_DEF
#define V3_PRIO_DEF 1
#endif
#ifndef KCPP_GEMM_PROBE
#define KCPP_GEMM_PROBE 0       // timing probes only (tools/gemm_ab.py with a PROBE_DEFS build): 1 no loads in the
#endif                          // super-block loop, 2 no main-loop MFMAs, 3 no barrier, 4 no A staging, 5 no weight loads
constexpr bool V3_PRIO = V3_PRIO_DEF;

template <int BMT> struct Q4v3Smem {
    h8v a[2][BMT][16 * 64];   // activation fragments [buf][token tile][step * 64 + lane]   (16 KiB per tile)
    h8v bs[2][BMT][64];       // Q8_K bsum fragments  [buf][token tile][lane]
    float dy[2][32 * BMT];    // activation scale of the super-block per token [buf][token]
};

// 16 B global -> LDS per lane (LDS address = wave-uniform base + 16 * lane)
// LDS-DMA issued from inline asm: the compiler does not track these writes, so it inserts no vmcnt(0) in front of
// the LDS reads that follow (it cannot tell the ring stage being filled from the one being read, and a compiler-
// visible DMA would drain every prefetch at the first read); the kernel orders them itself (s_waitcnt + barrier).
// lds_base: wave-uniform LDS byte address; lane l writes lds_base + size * l.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void dma16(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_base))) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_base))) : "memory", "m0");
}


// one qs dword (4 bytes of a sub-block pair) -> fragment: 4 low nibbles * s0, 4 high nibbles * s1 (exact)
__device__ __forceinline__ h8v frag_q4v3(uint32_t w, float s0, float s1) {
    const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
    const _Float16 a = (_Float16)s0, ab = (_Float16)(-1024.0f * s0);
    const _Float16 b = (_Float16)s1, bb = (_Float16)(-1024.0f * s1);
    const h2v x0 = scale2(bias_lo(lo), a, ab), x1 = scale2(bias_hi(lo), a, ab);
    const h2v x2 = scale2(bias_lo(hi), b, bb), x3 = scale2(bias_hi(hi), b, bb);
    h8v r;
    r[0] = x0[0]; r[1] = x0[1]; r[2] = x1[0]; r[3] = x1[1]; r[4] = x2[0]; r[5] = x2[1]; r[6] = x3[0]; r[7] = x3[1];
    return r;
}

__device__ __forceinline__ uint32_t u4c(const uint4 &v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w)); }

// grid: MT * ceil(N / 128) workgroups (MT = Mp / (32 BMT)), 64 NW threads, one workgroup per CU.
// Workgroup = 32 BMT tokens x 128 weight rows.  Wave w owns weight rows [32 (w % 4), +32) against the
// TPW = 4 BMT / NW token tiles [TPW (w / 4), +TPW): NW = 4 dequantizes every B fragment once per workgroup and
// feeds it to TPW MFMAs; NW = 8 (two waves per SIMD, so one wave's LDS reads and dequantization hide under the
// other's MFMAs) dequantizes each row twice.  BMT = 2 doubles the grid of small-N shapes (wo, q|k|v, down).
// XCD-aware tile order: blocks b and b + 8 share an XCD (dealt round-robin).  XCD x serves token tiles
// [G set, +G) (set = x % (MT / G)) against the row tiles of class x / (MT / G): the G token-tile workgroups of one
// row tile run back to back on one XCD, so its weights come from HBM once and from that XCD's L2 G - 1 times,
// while the XCD's L2 holds G token tiles of activations.  Falls back to plain order when the grid does not divide.
__device__ __forceinline__ void xcd_tile(int64_t id, int64_t nwg, int MT, int64_t ntn, int G, int64_t &mt, int64_t &nt) {
    const int nset = G > 0 && MT % G == 0 ? MT / G : 0;
    const int xper = nset > 0 && 8 % nset == 0 ? 8 / nset : 0;
    if (xper > 0 && nwg % 8 == 0 && ntn % xper == 0) {
        const int64_t x = id & 7, j = id >> 3;
        mt = (x % nset) * G + j % G;
        nt = (j / G) * xper + x / nset;
    } else {
        mt = id % MT;
        nt = id / MT;
    }
}

template <int LAY, int NW, int BMT, int PF>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) k_gemm_q4v3(const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                                         const h8v *__restrict__ af, const float *__restrict__ dyT,
                                                         const h8v *__restrict__ bsf, int64_t M, int64_t Mp, int MT,
                                                         float *__restrict__ Y, int64_t ldy, const float *res, int64_t ldr,
                                                         int KS, float *__restrict__ part, int XG) {
    constexpr int TPW = 4 * BMT / NW;         // token tiles per wave
    constexpr int SPW = 16 * BMT / NW;        // A staging: LDS-DMA steps per wave and super-block
    static_assert(TPW >= 1 && SPW >= 1, "tile shape");
    __shared__ Q4v3Smem<BMT> S;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave & 3, wt = wave >> 2;
    const int lr = lane & 31, kg = lane >> 5;
    // XCD-aware tile order (as k_gemm_kq): ids with equal id % 8 share a token tile when MT divides 8
    // KS > 1: split-K -- the grid is KS copies of the tile grid, copy `split` covers super-blocks
    // [split nsb / KS, (split + 1) nsb / KS) and writes its fp32 partial tile to part [KS][Mp][N]
    const int64_t nwg = gridDim.x / KS, id = blockIdx.x % nwg;
    const int split = (int)(blockIdx.x / nwg);
    int64_t mt, nt;
    xcd_tile(id, nwg, MT, (N + 127) / 128, XG, mt, nt);
    const int64_t m0 = mt * 32 * BMT, n0 = nt * 128;
    const int64_t nsb = K / 256, bpr = nsb;
    // this lane's weight row; clamped at N (its results are not stored)
    const int64_t nrow = min(n0 + 32 * wr + lr, N - 1);
    const uint8_t *hp, *qp;
    if constexpr (LAY == 1) {
        hp = W + nrow * 144 * bpr;
        qp = hp + 16 * bpr + 16 * kg;
    } else {
        hp = W + nrow * bpr * 144;
        qp = hp + 16 + 16 * kg;
    }
    constexpr int64_t HS = LAY == 1 ? 16 : 144, QS = LAY == 1 ? 128 : 144;   // bytes per super-block
    // LDS-DMA: wave w copies steps [SPW (w / BMT), +SPW) of token tile w % BMT (16 KiB per tile and
    // super-block); waves < BMT the bsum fragments of tile w; wave 0: dy (128 BMT bytes)
    const int stt = wave % BMT, st0 = SPW * (wave / BMT);
    const h8v *asrc = af + (m0 / 32 + stt) * (K / 16) * 64 + lane;
    const h8v *bsrc = bsf + (m0 / 32 + stt) * nsb * 64 + lane;
    const float *dsrc = dyT + m0 + 4 * lane;
    auto stage = [&](int buf, int64_t sb) {
#pragma unroll
        for (int st = 0; st < SPW; ++st) dma16(asrc + (16 * sb + st0 + st) * 64, &S.a[buf][stt][(st0 + st) * 64]);
        if (wave < BMT) dma16(bsrc + sb * 64, &S.bs[buf][stt][0]);
        if (wave == 0 && lane < 8 * BMT) dma16(dsrc + sb * Mp, &S.dy[buf][0]);
    };
    // raw weight super-blocks are loaded PF ahead into register sets X / Y (PF = 2: ping-pong, the loop unrolled
    // by two so each set stays in fixed registers); sb's set is copied out before it is refilled with sb + PF
    uint4 hX, qX[4], hY, qY[4];
    auto load_raw = [&](int64_t sb, uint4 &h, uint4 (&q)[4]) {
        h = ldg16(hp + HS * sb);
#pragma unroll
        for (int p = 0; p < 4; ++p) q[p] = ldg16(qp + QS * sb + 32 * p);
    };

    const int64_t sbb = nsb * split / KS, sbe = nsb * (split + 1) / KS;
    f16acc tot[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) tot[j][i] = 0.0f;
    stage(0, sbb);
    load_raw(sbb, hX, qX);
    if (PF == 2 && sbb + 1 < sbe) load_raw(sbb + 1, hY, qY);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    auto body = [&](int64_t sb, int buf, uint4 &hs, uint4 (&qs)[4]) {
        const uint4 hc = hs;
        uint32_t sc_lo, sc_hi, m_lo, m_hi;
        k4_all(hc, sc_lo, sc_hi, m_lo, m_hi);
        uint4 qc[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) qc[p] = qs[p];
#if KCPP_GEMM_PROBE != 1 && KCPP_GEMM_PROBE != 4
        if (sb + 1 < sbe) stage(buf ^ 1, sb + 1);
#endif
#if KCPP_GEMM_PROBE != 1 && KCPP_GEMM_PROBE != 5
        if (sb + PF < sbe) load_raw(sb + PF, hs, qs);
#endif
        f16acc acc[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.0f;
        // 16 MFMA steps; the A fragments of step s+1 are read from LDS before step s's MFMAs are issued
        const h8v *abase = &S.a[buf][TPW * wt][lane];
        h8v an[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j) an[j] = abase[j * 1024];
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            h8v ac[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j) ac[j] = an[j];
            if (s + 1 < 16) {
#pragma unroll
                for (int j = 0; j < TPW; ++j) an[j] = abase[j * 1024 + (s + 1) * 64];
            }
            const int p = s >> 2, st = s & 3;
            if (st == 0) {                        // sub-blocks 2p, 2p+1: bytes 2(p&1), +1 of the low / high dword
                const uint32_t sdw = p < 2 ? sc_lo : sc_hi;
                s0 = (int)((sdw >> (16 * (p & 1))) & 0xFF);
                s1 = (int)((sdw >> (16 * (p & 1) + 8)) & 0xFF);
            }
            const h8v b = frag_q4v3(u4c(qc[p], st), (float)s0, (float)s1);
            if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(1);
#if KCPP_GEMM_PROBE == 2
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc[j][0] += (float)ac[j][0] * (float)b[0];
#else
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac[j], b, acc[j], 0, 0, 0);
#endif
            if constexpr (V3_PRIO) __builtin_amdgcn_s_setprio(0);
        }
        // epilogue: tot -= dy * dmin * (sum_j m_j bsum_j), then tot += dy * (d * S)  (k_gemm_kq's order)
        h8v bm;                                   // mins of sub-blocks 4kg .. 4kg+3, each for its two 16-groups
        const uint32_t mdw = kg ? m_hi : m_lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const _Float16 mn = (_Float16)(float)((mdw >> (8 * e)) & 0xFF);
            bm[2 * e] = mn;
            bm[2 * e + 1] = mn;
        }
        const float dw = h2f((uint16_t)(hc.x & 0xFFFF)), dm = h2f((uint16_t)(hc.x >> 16));
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int tt = TPW * wt + j;
            float dyv[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)&S.dy[buf][32 * tt + 8 * q + 4 * kg];
                dyv[4 * q] = v.x; dyv[4 * q + 1] = v.y; dyv[4 * q + 2] = v.z; dyv[4 * q + 3] = v.w;
            }
            f16acc accm;
#pragma unroll
            for (int i = 0; i < 16; ++i) accm[i] = 0.0f;
            accm = __builtin_amdgcn_mfma_f32_32x32x16_f16(S.bs[buf][tt][lane], bm, accm, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) tot[j][r] = fmaf(-__fmul_rn(dyv[r], dm), accm[r], tot[j][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) tot[j][r] = fmaf(dyv[r], __fmul_rn(dw, acc[j][r]), tot[j][r]);
        }
        // the next super-block's A copy (and, PF = 2, its raw weights) must have landed; sb + 2's raw loads, issued
        // last, may stay in flight (loads retire in order)
        if (PF == 2 && sb + 2 < sbe) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if KCPP_GEMM_PROBE != 3
        __syncthreads();
#endif
    };
    if constexpr (PF == 2) {
        int64_t sb = sbb;
        for (; sb + 1 < sbe; sb += 2) {
            body(sb, 0, hX, qX);
            __builtin_amdgcn_sched_barrier(0);
            body(sb + 1, 1, hY, qY);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (sb < sbe) body(sb, 0, hX, qX);
    } else {
        for (int64_t sb = sbb; sb < sbe; ++sb) body(sb, (int)((sb - sbb) & 1), hX, qX);
    }
    const int64_t n = n0 + 32 * wr + lr;
    if (n >= N) return;
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t t = m0 + 32 * (TPW * wt + j) + (r & 3) + 8 * (r >> 2) + 4 * kg;
            if (KS > 1) part[((int64_t)split * Mp + t) * N + n] = tot[j][r];
            else if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[j][r], res[t * ldr + n]) : tot[j][r];
        }
}

// split-K partials [KS][Mp][N] summed in split order, then the residual (the unsplit kernel's tot + res)
__global__ void k_splitk_reduce(const float *__restrict__ part, int KS, int64_t M, int64_t Mp, int64_t N,
                                float *__restrict__ Y, int64_t ldy, const float *res, int64_t ldr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int64_t t = i / N, n = i % N;
    float g = part[t * N + n];
    for (int k = 1; k < KS; ++k) g = __fadd_rn(g, part[((int64_t)k * Mp + t) * N + n]);
    Y[t * ldy + n] = res ? __fadd_rn(g, res[t * ldr + n]) : g;
}

// kcpp_gemm_rms_norm / kcpp_gemm_q6p_rms_norm: the residual GEMM's split-K reduce also forms the next rms_norm's
// Q8_K activation (ops.hip k_rms_norm with partials; bit for bit the reduce followed by kcpp_rms_norm)
struct NormHook { const float *w; void *qout; float eps; bool used; };
static thread_local NormHook *g_norm_hook = nullptr;
static void splitk_finish(const float *part, int KS, int64_t M, int64_t Mp, int64_t N, float *y, int64_t ly,
                          const float *r, int64_t lr, hipStream_t s) {
    if (g_norm_hook && !g_norm_hook->used && ly == N &&
        kcpp_reduce_rms_norm(part, KS, Mp, r, lr, y, ly, g_norm_hook->w, g_norm_hook->qout, N, M, g_norm_hook->eps, s) == 0) {
        g_norm_hook->used = true;
        return;
    }
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((M * N + 255) / 256)), dim3(256), 0, s, part, KS, M, Mp, N, y, ly,
                       r, lr);
}

// ================================================================ Q6_K GEMM v3 (row-major decode layout Q6_K_RS)
// k_gemm_q4v3's structure for Q6_K: activation by LDS-DMA, each wave dequantizes its own 32 rows into MFMA
// fragments, exact integer weights sc*(q-32) split as 8*(sc>>3)*(q-32) + (sc&7)*(q-32) into two MFMAs (as v2).
// k order: MFMA step s = 4u + g (u = RS unit (h = u >> 1, lh = u & 1), g = 0..3), lane half kg, half e:
//   k = 128 h + 16 lh + 32 g + 8 kg + e    -- one 16-element sub-block per fragment (one scale), the lane's
// bytes 8kg..8kg+7 of the unit's ql-lo / ql-hi / qh planes (dequantize_row_q6_K, ggml-quants.c:2978).
// grouped layouts (MoE prefill): group e's gcnt[e] real rows sit at virtual rows [P_e, P_e + 128 ceil(n_e / 128)),
// P_e = the padded sizes before it; vrow -> (group, its virtual base, its real first row, its count)
__device__ __forceinline__ int grp_find(const int32_t *gcnt, int gne, int64_t v, int64_t &P, int64_t &r0, int64_t &n) {
    P = 0;
    r0 = 0;
    for (int e = 0; e < gne; ++e) {
        const int64_t c = gcnt[e], pe = (c + 127) / 128 * 128;
        if (v < P + pe) { n = c; return e; }
        P += pe;
        r0 += c;
    }
    n = 0;
    return -1;
}

// gcnt set: the image has Mp virtual rows of the grouped layout (grp_find), real rows from the M-row Q8_K act
__global__ void k_act_frag6(const uint8_t *__restrict__ act, int64_t K, int64_t M, int64_t Mp, h8v *__restrict__ af,
                            float *__restrict__ dyT, const int32_t *gcnt, int gne) {
    const int64_t nA = Mp * K / 8, nD = Mp * (K / 256);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int8_t *qs = (const int8_t *)act;
    const float *d = (const float *)(act + M * K);
    auto real = [&](int64_t vm) -> int64_t {          // virtual row -> real row, or -1
        if (!gcnt) return vm < M ? vm : -1;
        int64_t P, r0, n;
        if (grp_find(gcnt, gne, vm, P, r0, n) < 0) return -1;
        return vm - P < n ? r0 + (vm - P) : -1;
    };
    if (i < nA) {
        const int lane = (int)(i & 63), kg = lane >> 5;
        const int64_t s16 = (i >> 6) % (K / 16), mt = (i >> 6) / (K / 16);
        const int64_t m = real(32 * mt + (lane & 31));
        const int u = (int)((s16 >> 2) & 3), g = (int)(s16 & 3);
        const int64_t k0 = 256 * (s16 >> 4) + 128 * (u >> 1) + 16 * (u & 1) + 32 * g + 8 * kg;
        uint2 v = make_uint2(0, 0);
        if (m >= 0) v = *(const uint2 *)(qs + m * K + k0);
        h8v r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            r[e] = (_Float16)(int8_t)((v.x >> (8 * e)) & 0xFF);
            r[4 + e] = (_Float16)(int8_t)((v.y >> (8 * e)) & 0xFF);
        }
        af[i] = r;
    } else if (i < nA + nD) {
        const int64_t j = i - nA;
        const int64_t sb = j / Mp, m = real(j % Mp);
        dyT[j] = m >= 0 ? d[m * (K / 256) + sb] : 0.0f;
    }
}

template <int BMT> struct Q6v3Smem {
    h8v a[2][BMT][16 * 64];
    float dy[2][32 * BMT];
};

template <int NW, int BMT>
__global__ void __launch_bounds__(64 * NW, 1) k_gemm_q6v3(const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                                         const h8v *__restrict__ af, const float *__restrict__ dyT,
                                                         int64_t M, int64_t Mp, int MT, float *__restrict__ Y, int64_t ldy,
                                                         const float *res, int64_t ldr, int KS, float *__restrict__ part,
                                                         const int32_t *gcnt, int gne, int64_t wstride) {
    constexpr int TPW = 4 * BMT / NW;
    constexpr int SPW = 16 * BMT / NW;
    static_assert(TPW >= 1 && SPW >= 1, "tile shape");
    __shared__ Q6v3Smem<BMT> S;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave & 3, wt = wave >> 2;
    const int lr = lane & 31, kg = lane >> 5;
    // KS > 1: split-K -- the grid is KS copies of the tile grid, copy `split` covers super-blocks
    // [split nsb / KS, (split + 1) nsb / KS) and writes its fp32 partial tile to part [KS][Mp][N]
    const int64_t nwg = gridDim.x / KS, id = blockIdx.x % nwg;
    const int split = (int)(blockIdx.x / nwg);
    int64_t mt, nt;
    if (8 % MT == 0 && nwg % 8 == 0) {
        const int64_t x = id & 7, j = id >> 3;
        mt = x % MT;
        nt = j * (8 / MT) + x / MT;
    } else {
        mt = id % MT;
        nt = id / MT;
    }
    const int64_t m0 = mt * 32 * BMT, n0 = nt * 128;
    const int64_t nsb = K / 256, bpr = nsb;
    // grouped (KS = 1, 32 BMT divides 128): the tile's group -> its weights; rows stored back at real positions
    int64_t gP = 0, gr0 = 0, gn = 0;
    if (gcnt) {
        const int e = grp_find(gcnt, gne, m0, gP, gr0, gn);
        if (e < 0) return;
        W += e * wstride;
    }
    const int64_t nrow = min(n0 + 32 * wr + lr, N - 1);
    const uint8_t *row = W + nrow * 210 * bpr;
    const uint8_t *plo = row + 8 * kg, *phi = row + 64 * bpr + 8 * kg, *pqh = row + 128 * bpr + 8 * kg;
    const uint8_t *psc = row + 192 * bpr;
    const uint16_t *pd = (const uint16_t *)(row + 208 * bpr);
    const int stt = wave % BMT, st0 = SPW * (wave / BMT);
    const h8v *asrc = af + (m0 / 32 + stt) * (K / 16) * 64 + lane;
    const float *dsrc = dyT + m0 + 4 * lane;
    auto stage = [&](int buf, int64_t sb) {
#pragma unroll
        for (int st = 0; st < SPW; ++st) dma16(asrc + (16 * sb + st0 + st) * 64, &S.a[buf][stt][(st0 + st) * 64]);
        if (wave == 0 && lane < 8 * BMT) dma16(dsrc + sb * Mp, &S.dy[buf][0]);
    };
    uint2 nlo[4], nhi[4], nqh[4];
    uint4 nsc;
    uint16_t nd;
    auto load_raw = [&](int64_t sb) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t U = 4 * sb + u;
            nlo[u] = *(const uint2 *)(plo + 16 * U);
            nhi[u] = *(const uint2 *)(phi + 16 * U);
            nqh[u] = *(const uint2 *)(pqh + 16 * U);
        }
        nsc = ldg16(psc + 16 * sb);
        nd = pd[sb];
    };

    const int64_t sbb = nsb * split / KS, sbe = nsb * (split + 1) / KS;
    f16acc tot[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) tot[j][i] = 0.0f;
    stage(0, sbb);
    load_raw(sbb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int64_t sb = sbb; sb < sbe; ++sb) {
        const int buf = (int)((sb - sbb) & 1);
        uint2 clo[4], chi[4], cqh[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { clo[u] = nlo[u]; chi[u] = nhi[u]; cqh[u] = nqh[u]; }
        const uint4 csc = nsc;
        const uint16_t cd = nd;
        if (sb + 1 < sbe) {
            stage(buf ^ 1, sb + 1);
            load_raw(sb + 1);
        }
        f16acc acc[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.0f;
        const h8v *abase = &S.a[buf][TPW * wt][lane];
        h8v an[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j) an[j] = abase[j * 1024];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            h8v ac[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j) ac[j] = an[j];
            if (s + 1 < 16) {
#pragma unroll
                for (int j = 0; j < TPW; ++j) an[j] = abase[j * 1024 + (s + 1) * 64];
            }
            const int u = s >> 2, g = s & 3;
            const uint2 P = (g & 1) ? chi[u] : clo[u];
            const uint2 Hq = cqh[u];
            const uint32_t v0 = ((P.x >> (4 * (g >> 1))) & 0x0F0F0F0Fu) | (((Hq.x >> (2 * g)) & 0x03030303u) << 4);
            const uint32_t v1 = ((P.y >> (4 * (g >> 1))) & 0x0F0F0F0Fu) | (((Hq.y >> (2 * g)) & 0x03030303u) << 4);
            const int scv = (int)(int8_t)((u4c(csc, u) >> (8 * g)) & 0xFF);
            const h8v bh = frag8_sub(v0, v1, (float)(8 * (scv >> 3)), 32.0f);
            const h8v bl = frag8_sub(v0, v1, (float)(scv & 7), 32.0f);
#pragma unroll
            for (int j = 0; j < TPW; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac[j], bh, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac[j], bl, acc[j], 0, 0, 0);
            }
        }
        const float dw = h2f(cd);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int tt = TPW * wt + j;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)&S.dy[buf][32 * tt + 8 * q + 4 * kg];
                const float dv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    tot[j][4 * q + e] = fmaf(dv[e], __fmul_rn(dw, acc[j][4 * q + e]), tot[j][4 * q + e]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const int64_t n = n0 + 32 * wr + lr;
    if (n >= N) return;
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t t = m0 + 32 * (TPW * wt + j) + (r & 3) + 8 * (r >> 2) + 4 * kg;
            if (gcnt) {
                if (t - gP < gn) Y[(gr0 + t - gP) * ldy + n] = tot[j][r];
            } else if (KS > 1) part[((int64_t)split * Mp + t) * N + n] = tot[j][r];
            else if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[j][r], res[t * ldr + n]) : tot[j][r];
        }
}

// ================================================================ Q8_0 small-batch GEMM (M <= 32)
// BASELINE config 3 (Llama-3-8B Q8_0, ubatch 32) is HBM-bound: the weights must stream at full bandwidth while
// only 32 tokens use them.  One v_mfma_i32_32x32x32_i8 per 32-block computes the exact integer block dot of
// ggml_vec_dot_q8_0_q8_0 (ggml-quants.c:5519) straight from the raw int8 weight and activation bytes (no
// dequantization, no LDS operand staging); the block result is scaled sumi * (d_w * d_x) in fp32 as the
// scalar CPU path does.  Workgroup = 128 weight rows (wave: 32 rows x the 32 tokens) x one K range; S K ranges
// per row tile give >= ~384 workgroups, their fp32 partials [S][32][N] are summed in split order by
// k_q80s_reduce (deterministic), which also applies the residual or silu(g) * u.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
#define Q80S_UNROLL 8

static int q80s_splits(int64_t K, int64_t N) {
    const int64_t nt = (N + 127) / 128, nb = K / 32;
    int64_t S = (384 + nt - 1) / nt;
    S = std::min<int64_t>(S, std::max<int64_t>(1, nb / (2 * Q80S_UNROLL)));
    S = std::max<int64_t>(S, (nb + 47) / 48);          // <= 48 blocks per split: <= 54 KiB of dynamic LDS
    return (int)std::max<int64_t>(S, 1);
}

// up to 3 weight segments back to back in the output columns (q|k|v); segment boundaries multiples of 128
struct Q80Segs {
    const uint8_t *W[3];
    int64_t N[3];
    int nseg;
};

// The small-batch Q8_0 GEMM: the weight tile streams through LDS in row-contiguous pieces (a first version's direct
// fragment loads touched 32 rows x 32 B per wave instruction, 32 cache lines for 1 KiB; removed); every LDS-DMA wave
// instruction reads 64 / (2 CH) rows x 32 CH bytes (CH blocks of each row) into an XOR-swizzled [row][32 CH B] image
// (16-B piece c of row n at slot c ^ (n % 2CH)), double-buffered by CH-block chunks with the activation chunk beside
// it; CH = 4 (40 KiB of LDS: three workgroups per CU keep more weight bytes in flight than CH = 8 at one).  Same block math and
// split-K partials.
// CH blocks per chunk (4: 40 KiB of LDS, three workgroups per CU)
#ifndef Q80_CH
#define Q80_CH 4
#endif
#ifndef Q80_ST
#define Q80_ST 2        // ring depth; 3 measured slower on config 3 (6.51k vs 6.71k tok/s: 2 instead of 3 workgroups per CU)
#endif
struct Q80s2Smem {
    uint8_t w[Q80_ST][128 * 32 * Q80_CH];  // weight chunk [stage][row][32 CH B] (swizzled 16-B pieces)
    i32x4 a[Q80_ST][Q80_CH][64];           // activation fragments [stage][block][lane]
    float dx[48 * 32];                     // token scales of the split's blocks [block][token] (q80s_splits: <= 48 blocks)
};

__global__ void __launch_bounds__(256) k_gemm_q80s2(const Q80Segs sg, int64_t K, int64_t N,
                                                   const uint8_t *__restrict__ act, int64_t M, float *__restrict__ part) {
    __shared__ Q80s2Smem S;
    float *sdx = S.dx;        // static LDS: the compiler can tell it from the DMA targets (a dynamic array made it
                              // wait for every outstanding LDS-DMA before each read of a token scale)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, kg = lane >> 5;
    const int64_t nb = K / 32, S_ = gridDim.y;
    const int64_t bps = (nb + S_ - 1) / S_, b0 = (int64_t)blockIdx.y * bps, b1 = std::min<int64_t>(nb, b0 + bps);
    const int64_t nt0 = (int64_t)blockIdx.x * 128;
    const int seg = (sg.nseg > 1 && nt0 >= sg.N[0]) ? ((sg.nseg > 2 && nt0 >= sg.N[0] + sg.N[1]) ? 2 : 1) : 0;
    const int64_t soff = seg == 0 ? 0 : (seg == 1 ? sg.N[0] : sg.N[0] + sg.N[1]);
    const int64_t Ns = seg == 0 ? sg.N[0] : (seg == 1 ? sg.N[1] : sg.N[2]);
    const uint8_t *W = seg == 0 ? sg.W[0] : (seg == 1 ? sg.W[1] : sg.W[2]);
    const uint16_t *dwp = (const uint16_t *)(W + Ns * nb * 32);
    const int64_t trow = std::min<int64_t>(lr, M - 1);
    const int8_t *qx = (const int8_t *)act + trow * K + 16 * kg;
    const float *dx = (const float *)(act + M * K);
    // weight LDS-DMA: a wave instruction covers RPI rows of 2 CH pieces (16 B per lane); lane -> (row, slot)
    constexpr int PPR = 2 * Q80_CH, RPI = 64 / PPR, IPW = 128 / RPI / 4;   // pieces per row, rows / instr, instr / wave
    const int wsub = lane / PPR, wslot = lane % PPR;
    auto stage = [&](int buf, int64_t cb) {                      // chunk = blocks [cb, cb + CH)
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int rl = RPI * (IPW * wave + i) + wsub;        // local row 0..127
            const int64_t row = std::min<int64_t>(nt0 - soff + rl, Ns - 1);
            const int piece = wslot ^ (rl % PPR);                // the 16-B piece this LDS slot holds
            const int64_t blk = std::min<int64_t>(cb + (piece >> 1), b1 - 1);
            dma16(W + (row * nb + blk) * 32 + 16 * (piece & 1), &S.w[buf][(IPW * wave + i) * 1024]);
        }
        if (wave < Q80_CH) dma16(qx + std::min<int64_t>(cb + wave, b1 - 1) * 32, &S.a[buf][wave][0]);
    };
    for (int64_t i = tid; i < (b1 - b0) * 32; i += 256) {
        const int64_t b = i >> 5, t = i & 31;
        sdx[i] = t < M ? dx[t * nb + b0 + b] : 0.0f;
    }
    float tot[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) tot[r] = 0.0f;
    const int nl = 32 * wave + lr;                               // this lane's B row within the tile
    const int64_t nrow = std::min<int64_t>(nt0 - soff + nl, Ns - 1);
    // Q80_ST-stage ring: chunk i in stage i % Q80_ST, issued Q80_ST - 1 chunks ahead
#pragma unroll
    for (int q = 0; q < Q80_ST - 1; ++q)
        if (b0 + q * Q80_CH < b1) stage(q, b0 + q * Q80_CH);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int64_t cb = b0; cb < b1; cb += Q80_CH) {
        const int ci = (int)((cb - b0) / Q80_CH);
        const int buf = ci % Q80_ST;
        const bool ahead = cb + (Q80_ST - 1) * Q80_CH < b1;
        // the weight block scales (plain global loads) are taken -- and waited for -- BEFORE the next chunk's LDS-DMA
        // goes out: the compiler does not see the DMA, so the vmcnt it places in front of the first use of a scale
        // would otherwise also wait for the whole prefetch and expose its latency every chunk
        float dwv[Q80_CH];
#pragma unroll
        for (int u = 0; u < Q80_CH; ++u) dwv[u] = h2f(dwp[nrow * nb + std::min<int64_t>(cb + u, b1 - 1)]);
#pragma unroll
        for (int u = 0; u < Q80_CH; ++u) asm volatile("" ::"v"(dwv[u]));
        if (ahead) stage((ci + Q80_ST - 1) % Q80_ST, cb + (Q80_ST - 1) * Q80_CH);
#pragma unroll
        for (int u = 0; u < Q80_CH; ++u) {
            if (cb + u >= b1) break;
            const int piece = 2 * u + kg;
            const i32x4 wv = *(const i32x4 *)&S.w[buf][nl * 32 * Q80_CH + ((piece ^ (nl % PPR)) * 16)];
            i32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0;
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(S.a[buf][u][lane], wv, acc, 0, 0, 0);
            const float *sd = sdx + (cb + u - b0) * 32;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 d4 = *(const float4 *)(sd + 8 * q + 4 * kg);
                const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    tot[4 * q + e] = __fadd_rn(tot[4 * q + e], __fmul_rn((float)acc[4 * q + e], __fmul_rn(dwv[u], dv[e])));
            }
        }
        // chunk ci + 1 must have landed; with three stages chunk ci + 2 (issued this iteration, last) may stay in flight
        if (Q80_ST == 3 && ahead) {
            static_assert(Q80_ST != 3 || (128 / (64 / (2 * Q80_CH)) / 4 == 4 && Q80_CH == 4), "vmcnt below: 4 + 1 per stage");
            asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    const int64_t n = nt0 + nl;
    if (n >= N) return;
    float *pp = part + (int64_t)blockIdx.y * 32 * N + n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int t = (r & 3) + 8 * (r >> 2) + 4 * kg;
        pp[(int64_t)t * N] = tot[r];
    }
}

// Y[t][n] = sum_s part[s][t][n] (+ res), or silu(sum_s g) * (sum_s u) with u partials in part2
__global__ void k_q80s_reduce(const float *__restrict__ part, const float *__restrict__ part2, int S, int64_t M,
                              int64_t N, float *__restrict__ Y, int64_t ldy, const float *res, int64_t ldr,
                              uint8_t *__restrict__ qout = nullptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;                            // N % 32 == 0 with qout: whole 32-lane blocks retire together
    const int64_t t = i / N, n = i % N;
    float g = part[t * N + n];
    for (int s = 1; s < S; ++s) g = __fadd_rn(g, part[((int64_t)s * 32 + t) * N + n]);
    if (part2) {
        float u = part2[t * N + n];
        for (int s = 1; s < S; ++s) u = __fadd_rn(u, part2[((int64_t)s * 32 + t) * N + n]);
        const float h = (g / (1.0f + expf(-g))) * u;
        if (!qout) {
            Y[t * ldy + n] = h;
            return;
        }
        // h quantized to Q8_0 for the down projection, as k_quant_q80: one 32-lane group per block
        float am = fabsf(h);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 32));
        const float id = (am != 0.0f) ? 127.f / am : 0.0f;
        int q = (int)rintf(__fmul_rn(h, id));
        q = q > 127 ? 127 : (q < -128 ? -128 : q);
        int sq = q;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sq += __shfl_xor(sq, o, 32);
        const int64_t nb = N / 32, b = t * nb + n / 32;
        ((int8_t *)qout)[t * N + n] = (int8_t)q;
        if ((n & 31) == 0) {
            ((float *)(qout + M * N))[b] = h2f(f2h(am / 127.f));
            ((int16_t *)(qout + M * N + M * nb * 4))[b] = (int16_t)sq;
        }
    } else {
        Y[t * ldy + n] = res ? __fadd_rn(g, res[t * ldr + n]) : g;
    }
}

__global__ void k_silu_mul_strided(float *__restrict__ y, int64_t ldy, const float *__restrict__ u, int64_t N, int64_t M) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * M) return;
    const int64_t m = i / N, n = i % N;
    const float g = y[m * ldy + n];
    y[m * ldy + n] = (g / (1.0f + expf(-g))) * u[i];
}

// v1 split-K factor, from the weight shape alone: on grids under 512 workgroups (two per CU) at a 512-token ubatch the
// K range is split (2 .. 8 ways; partials summed in split order by k_splitk_reduce).  Chosen without M so that a
// prompt gives the same bits however it is cut into ubatches (the f32 partial order depends only on the weight).
static int ks1_of(int64_t K, int64_t N) {
    const int64_t nwg = (N + GB_N - 1) / GB_N * (512 / GB_M);
    int ks = 1;
    while (ks < 8 && nwg * ks * 2 <= 1024 && (K / GB_K) % (ks * 2) == 0) ks *= 2;
    return ks;
}

static int64_t ws_layout(int type, int64_t K, int64_t N, int64_t M, int64_t &o_a16, int64_t &o_dy, int64_t &o_bs, int64_t &o_up) {
    const int64_t Mp = (M + GB_M - 1) / GB_M * GB_M;
    const int64_t G = (type == KT_Q4_0 || type == KT_Q5_0 || type == KT_Q8_0 || type == KT_Q4_1 || type == KT_Q5_1 ||
                       type == KT_IQ4_NL) ? 32 : 256;
    int64_t off = 0;
    o_a16 = off; off += (Mp * K * 2 + 255) & ~255LL;
    o_dy = off; off += (Mp * (K / G) * 4 + 255) & ~255LL;
    o_bs = off; off += (Mp * (K / 16) * 2 + 255) & ~255LL;
    o_up = off; off += (M * N * 4 + 255) & ~255LL;
    if (type == KT_Q8_0) off += 2 * (int64_t)q80s_splits(K, N) * 32 * N * 4;   // small-M split-K partials (g, u)
    if (type == KT_Q4_K || type == KT_Q4_K_RS || type == KT_Q6_K_RS) off += 2 * Mp * N * 4;   // v3 split-K partials
    else if (type == KT_Q5_K || type == KT_Q5_K_RS) off += (int64_t)std::max(2, ks1_of(K, N)) * Mp * N * 4;   // v4 / v1
    else off += (int64_t)ks1_of(K, N) * Mp * N * 4;                                             // v1 split-K partials
    return off;
}


// ================================================================ Q4_K GEMM v4 (int8 matrix cores)
// v3 is bound by moving operands, not by the matrix cores (probes at M = 512, gate|up 4096 x 28672: 266 us, 142 us
// with the in-loop loads removed, 216 us with the MFMAs removed): its f16 activation image is twice the Q8_K bytes
// and every weight row is loaded by two waves one super-block ahead.  v4 multiplies the Q8_K bytes themselves on
// v_mfma_i32_32x32x32_i8, one MFMA per 32-element sub-block and token tile, with an exact int32 accumulator:
//   sum_k q*sc*a = 8 * sum_k (q*(sc>>3))*a + sum_k (q*(sc&7))*a,  q*(sc>>3), q*(sc&7) <= 105 (int8),
// so each sub-block takes two MFMAs into acc_h / acc_l and isum = 8 acc_h + acc_l is the CPU's int32 sumi exactly
// (v3 holds the same integer in fp32); the per-super-block epilogue is v3's, so the results are bit-identical.
// Operands are staged with LDS-DMA straight from the Q8_K buffer (no fragment-image kernel): per super-block the
// workgroup's 128 token rows x 256 B of int8, their bsums and scales, and its 128 weight rows' 144 B, the weights
// in a 3-stage ring two super-blocks ahead (HBM latency), the activations double-buffered one ahead (L2 hits).
// Workgroup = 128 tokens x 128 weight rows, 8 waves; wave w: weight rows 32 (w & 3) .. +32 x token tiles
// 2 (w >> 2), +1.  Fragment k order: lane half g of token / weight row r holds bytes 16g .. 16g+15 of the
// sub-block (any order common to both operands is exact); the Q4_K byte j of pair p holds element j of sub-block
// 2p (low nibble) and 2p+1 (high nibble).
// Swizzled LDS images: one LDS-DMA instruction (64 lanes x 16 B, lane-linear in LDS) fetches 8 rows x 8 chunks of
// 16 B -- one 128-B line per row (a fragment-ordered fetch touches 32 lines per instruction) -- lane j: row
// 8k + (j & 7), chunk 8h + (j >> 3), at slot 72 (4h + k) + j (72: rows 8 apart start 8 slots apart mod 16, so the
// 16-lane groups of a fragment read hit 16 distinct bank quads: conflict-free).  Chunk c of row m of a 32-row tile:
// slot 72 (4 (c >> 3) + (m >> 3)) + (m & 7) + 8 (c & 7).
__device__ __forceinline__ int swz(int m, int c) { return 72 * (4 * (c >> 3) + (m >> 3)) + (m & 7) + 8 * (c & 7); }

// TPW = 2 (v4): 4 row tiles (128 rows) x 2 token halves, 3 weight stages; TPW = 4 (v5): 8 row tiles (256 rows), every
// wave against all 4 token tiles, so each dequantized weight fragment feeds twice the MFMAs; 2 weight stages (LDS).
// Slot counts: the highest swizzled slot + 1 (activations 16 chunks: 568, weights 8 chunks: 280).
template <int WR, int NST> struct Q4v4Smem {
    i32x4 a[2][4][568];      // [buf][token tile][swz(row, chunk)]: 16 activation bytes, chunks 0..15 of the 256
    i32x4 bs[2][4][64];      // [buf][token tile][lane]: 8 bsums (int16) of the lane half's 128 elements
    float dy[2][128];        // [buf][token]: Q8_K scale of the super-block
    uint4 wh[NST][WR][32];   // [stage][row tile][row]: Q4_K header (d, dmin, 12 B scales / mins)
    i32x4 wq[NST][WR][280];  // [stage][row tile][swz(row, chunk)]: qs chunks 0..7 (pair p, half g: chunk 2p + g)
};
// Q5_K adds the fifth bits: qh bytes 16 g .. 16 g + 15 of row r (bit j = sub-block j) at slot 32 g + r
template <int WR, int NST> struct Q5v4Smem : Q4v4Smem<WR, NST> {
    i32x4 wqh[NST][WR][64];  // [stage][row tile][32 g + row]
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// bytes of x (each <= 15) times s (<= 7), per byte: two 16-bit lanes, no carry out of a byte (v_pk_mul_lo_u16;
// the scalar factor is taken for both halves by op_sel)
__device__ __forceinline__ int mulb(uint32_t x, uint32_t s) {
    const u16x2 f = {(unsigned short)s, (unsigned short)s};
    return (int)__builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, x) * f);
}

// Q5_K (TYPE = KT_Q5_K, TPW = 2 only -- the qh stages do not fit v5's LDS): q = lo + 16 hb, lo <= 15, hb <= 1, so
//   sum_k q*sc*a = 8 (sum_k (lo*(sc>>3))*a + sum_k (hb*2sc)*a) + sum_k (lo*(sc&7))*a,  hb*2sc <= 126,
// a third MFMA per sub-block, into acc_h; isum = 8 acc_h + acc_l is again the CPU's exact int32 sumi
// (ggml_vec_dot_q5_K_q8_K, ggml-quants.c), and the epilogue is unchanged.
template <int TYPE, int LAY, int TPW>
// GLU: W2 / Y2 set -- the grid's second half computes the up matrix into Y2 (one launch for both: twice the
// workgroups on the small expert grids, no second ramp; every tile's arithmetic unchanged).
// Grouped (MoE prefill, gcnt set, KS = 1): act holds gne groups of token rows back to back (Q8_K planes of M rows in
// all), group e = gcnt[e] rows against weight matrix W + e wstride; the grid is every group's tile grid in order,
// each group's outputs at its first row of Y (and Y2).
__global__ void __launch_bounds__(512, 1) k_gemm_q4v4(const uint8_t *__restrict__ W, int64_t K, int64_t N,
                                                     const uint8_t *__restrict__ act, int64_t M, int64_t Mp, int MT,
                                                     float *__restrict__ Y, int64_t ldy, const float *res, int64_t ldr,
                                                     int KS, float *__restrict__ part, int XG, const uint8_t *W2,
                                                     float *Y2, int64_t ldy2, const int32_t *gcnt, int gne,
                                                     int64_t wstride) {
    constexpr int WT = 4 / TPW, WR = 8 / WT, NR = 32 * WR, NST = TPW == 2 ? 3 : 2, NI = WR / 2;
    constexpr bool Q5 = TYPE == KT_Q5_K;
    static_assert(TYPE == KT_Q4_K || (Q5 && TPW == 2), "v4 int8 GEMM: Q4_K (TPW 2 / 4) or Q5_K (TPW 2)");
    __shared__ std::conditional_t<Q5, Q5v4Smem<WR, NST>, Q4v4Smem<WR, NST>> S;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave % WR, wt = wave / WR;
    const int lr = lane & 31, kg = lane >> 5;
    const int64_t per = W2 ? gridDim.x / 2 : gridDim.x;       // workgroups per matrix
    const bool second = blockIdx.x >= per;
    int64_t bid = second ? blockIdx.x - per : blockIdx.x;
    if (second) { W = W2; Y = Y2; ldy = ldy2; res = nullptr; }
    const int64_t nsb = K / 256, bpr = nsb;
    const int8_t *qs = (const int8_t *)act;
    const float *dq = (const float *)(act + M * K);
    const int16_t *bsq = (const int16_t *)(act + M * K + M * nsb * 4);
    int64_t nwg = per / KS;
    if (gcnt) {                 // uniform scan for this workgroup's group (<= 64 groups)
        const int64_t ntn = (N + NR - 1) / NR;
        int64_t t0 = 0, r0 = 0;
        int e = 0;
        for (; e < gne; ++e) {
            const int64_t te = (gcnt[e] + 127) / 128 * ntn;
            if (bid < t0 + te) break;
            t0 += te;
            r0 += gcnt[e];
        }
        if (e >= gne) return;
        bid -= t0;
        W += e * wstride;
        Y += r0 * ldy;
        qs += r0 * K;
        dq += r0 * nsb;
        bsq += r0 * (K / 16);
        M = gcnt[e];
        MT = (int)((M + 127) / 128);
        nwg = MT * ntn;
    }
    const int64_t id = bid % nwg;
    const int split = (int)(bid / nwg);
    int64_t mt, nt;
    xcd_tile(id, nwg, MT, (N + NR - 1) / NR, XG, mt, nt);
    const int64_t m0 = mt * 128, n0 = nt * NR;
    // DMA assignments (per super-block): A: token tile wave & 3, sub-blocks 4 (wave >> 2) .. +4; bsums: waves 0-3
    // (tile = wave); dy: waves 4, 5 (tokens 64 (wave - 4) .. +64); weights: NI groups of 8 rows, group i = 8u + wave
    // (row tile i >> 2, rows 8 (i & 3) ..); headers: waves 0 .. NI - 1 (row tiles 2 wave + (lane >> 5))
    // A: token tile wave & 3, chunk half wave >> 2, row groups 0..3; lane: row 8k + (lane & 7), chunk 8h + (lane >> 3)
    const int att = wave & 3, ah8 = wave >> 2;
    const int8_t *arow = qs + min(m0 + 32 * att + (lane & 7), M - 1) * K + 16 * (8 * ah8 + (lane >> 3));
    const int16_t *bsrow = bsq + min(m0 + 32 * wave + lr, M - 1) * (K / 16) + 8 * kg;
    const float *dyrow = dq + min(m0 + 64 * max(wave - 4, 0) + lane, M - 1) * nsb;
    // bytes per super-block and row: Q4_K 144 (header 16, qs 128), Q5_K 176 (header 16, qh 32, qs 128); LAY 1 keeps
    // each row's headers, qs and (Q5_K) qh as planes: [nsb][16] ++ [nsb][128] ++ [nsb][32]
    constexpr int64_t BPB = Q5 ? 176 : 144;
    constexpr int64_t HS = LAY == 1 ? 16 : BPB, QS = LAY == 1 ? 128 : BPB, QHS = LAY == 1 ? 32 : BPB;
    const int64_t qoff = LAY == 1 ? 16 * bpr : (Q5 ? 48 : 16), qhoff = LAY == 1 ? 144 * bpr : 16;
    const uint8_t *wq0[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        const int i = 8 * u + wave;
        const int64_t row = min(n0 + 32 * (i >> 2) + 8 * (i & 3) + (lane & 7), N - 1);
        wq0[u] = W + row * BPB * bpr + qoff + 16 * (lane >> 3);
    }
    const int hrt = 2 * wave + kg;
    const int64_t hrow = min(n0 + 32 * hrt + lr, N - 1);
    const uint8_t *wh0 = W + hrow * BPB * bpr;
    // qh (Q5_K): waves 4 .. 7, row tile wave - 4, lane = 32 g + row
    const uint8_t *wqh0 = W + min(n0 + 32 * max(wave - 4, 0) + lr, N - 1) * BPB * bpr + qhoff + 16 * kg;
    auto stage_a = [&](int buf, int64_t sb) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dma16(arow + (int64_t)min(8 * k, (int)max<int64_t>(M - 1 - (m0 + 32 * att + (lane & 7)), 0)) * K + sb * 256,
                  &S.a[buf][att][72 * (4 * ah8 + k)]);
        if (wave < 4) dma16(bsrow + sb * 16, &S.bs[buf][wave][0]);
        else if (wave < 6) dma4(dyrow + sb, &S.dy[buf][64 * (wave - 4)]);
    };
    auto stage_w = [&](int st, int64_t sb) {
#pragma unroll
        for (int u = 0; u < NI; ++u) {
            const int i = 8 * u + wave;
            dma16(wq0[u] + QS * sb, &S.wq[st][i >> 2][72 * (i & 3)]);
        }
        if (wave < NI) dma16(wh0 + HS * sb, &S.wh[st][2 * wave][0]);
        if constexpr (Q5)
            if (wave >= 4) dma16(wqh0 + QHS * sb, &S.wqh[st][wave - 4][0]);
    };

    const int64_t sbb = nsb * split / KS, sbe = nsb * (split + 1) / KS;
    f16acc tot[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) tot[j][i] = 0.0f;
    stage_a(0, sbb);
#pragma unroll
    for (int q = 0; q < NST - 1; ++q)
        if (sbb + q < sbe) stage_w(q, sbb + q);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    int st = 0;
    // waves 4-7 (the later-dispatched half, each sharing a SIMD with one of waves 0-3 running the same program) at
    // static priority 1: the arbitration loser otherwise (MI355X_MICROARCH.md, two waves per SIMD, item 4); bitwise
    // the same results.  tools/gemm_ab.py: q|k|v 53.3 -> 50.5 us, bench prefill 34.16k -> 34.56k tok/s
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    for (int64_t sb = sbb; sb < sbe; ++sb) {
        const int buf = (int)((sb - sbb) & 1);
        const bool wn = sb + NST - 1 < sbe && KCPP_GEMM_PROBE != 1 && KCPP_GEMM_PROBE != 5;
#if KCPP_GEMM_PROBE != 1 && KCPP_GEMM_PROBE != 4
        if (sb + 1 < sbe) stage_a(buf ^ 1, sb + 1);
#endif
        if (wn) stage_w(st == 0 ? NST - 1 : st - 1, sb + NST - 1);
        const uint4 hc = S.wh[st][wr][lr];
        uint32_t sc_lo, sc_hi, m_lo, m_hi;
        k4_all(hc, sc_lo, sc_hi, m_lo, m_hi);
        // the super-block's weight fragments dequantized once (bw[p]: q*(sc>>3), q*(sc&7) of sub-blocks 2p, 2p+1),
        // then per token tile its 16 MFMAs and right behind them its epilogue (v3's: tot -= dy * dmin * (sum_j m_j
        // bsum_j), then tot += dy * (d * isum)), so only one tile's integer accumulators are live
        i32x4 bw[4][4];
        i32x4 qhv;
        if constexpr (Q5) qhv = S.wqh[st][wr][32 * kg + lr];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const i32x4 w4 = S.wq[st][wr][swz(lr, 2 * p + kg)];
            const uint32_t sdw = p < 2 ? sc_lo : sc_hi;
            const uint32_t s0 = (sdw >> (16 * (p & 1))) & 0xFF, s1 = (sdw >> (16 * (p & 1) + 8)) & 0xFF;
            const uint32_t h0 = s0 >> 3, l0 = s0 & 7, h1 = s1 >> 3, l1 = s1 & 7;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t x = (uint32_t)w4[e];
                const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
                bw[p][0][e] = mulb(lo, h0);
                bw[p][1][e] = mulb(lo, l0);
                bw[p][2][e] = mulb(hi, h1);
                bw[p][3][e] = mulb(hi, l1);
            }
        }
        h8v bm;
        const uint32_t mdw = kg ? m_hi : m_lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const _Float16 mn = (_Float16)(float)((mdw >> (8 * e)) & 0xFF);
            bm[2 * e] = mn;
            bm[2 * e + 1] = mn;
        }
        const float dw = h2f((uint16_t)(hc.x & 0xFFFF)), dm = h2f((uint16_t)(hc.x >> 16));
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int tt = TPW * wt + j;
            i32x16 ah, al;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const i32x4 a0 = S.a[buf][tt][swz(lr, 4 * p + kg)], a1 = S.a[buf][tt][swz(lr, 4 * p + 2 + kg)];
                // Q5_K: hb*sc of sub-blocks 2p, 2p+1, made per token tile (held for all four pairs they spill)
                i32x4 bh0, bh1;
                if constexpr (Q5) {
                    const uint32_t sdw = p < 2 ? sc_lo : sc_hi;
                    const uint32_t s0 = (sdw >> (16 * (p & 1))) & 0xFF, s1 = (sdw >> (16 * (p & 1) + 8)) & 0xFF;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {     // hb * 2sc
                        const uint32_t hx = (uint32_t)qhv[e];
                        bh0[e] = mulb((hx >> (2 * p)) & 0x01010101u, 2 * s0);
                        bh1[e] = mulb((hx >> (2 * p + 1)) & 0x01010101u, 2 * s1);
                    }
                }
#if KCPP_GEMM_PROBE == 2
                ah[0] += a0[0] * bw[p][0][0] + a1[1] * bw[p][3][1];
                al[0] += a0[1] * bw[p][1][0] + a1[0] * bw[p][2][1];
                continue;
#endif
                if (p == 0) {
                    i32x16 z;
#pragma unroll
                    for (int i = 0; i < 16; ++i) z[i] = 0;
                    ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bw[p][0], z, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bw[p][1], z, 0, 0, 0);
                    if constexpr (Q5) ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bh0, ah, 0, 0, 0);
                } else {
                    ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bw[p][0], ah, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bw[p][1], al, 0, 0, 0);
                    if constexpr (Q5) ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bh0, ah, 0, 0, 0);
                }
                ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bw[p][2], ah, 0, 0, 0);
                al = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bw[p][3], al, 0, 0, 0);
                if constexpr (Q5) ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bh1, ah, 0, 0, 0);
            }
            float dyv[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)&S.dy[buf][32 * tt + 8 * q + 4 * kg];
                dyv[4 * q] = v.x; dyv[4 * q + 1] = v.y; dyv[4 * q + 2] = v.z; dyv[4 * q + 3] = v.w;
            }
            const i32x4 bsv = S.bs[buf][tt][lane];
            h8v ab;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                ab[2 * e] = (_Float16)(int16_t)(bsv[e] & 0xFFFF);
                ab[2 * e + 1] = (_Float16)(int16_t)((uint32_t)bsv[e] >> 16);
            }
            f16acc accm;
#pragma unroll
            for (int i = 0; i < 16; ++i) accm[i] = 0.0f;
            accm = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab, bm, accm, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) tot[j][r] = fmaf(-__fmul_rn(dyv[r], dm), accm[r], tot[j][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float is = (float)(ah[r] * 8 + al[r]);
                tot[j][r] = fmaf(dyv[r], __fmul_rn(dw, is), tot[j][r]);
            }
        }
        // A (sb + 1) and W (sb + 1) must have landed; with three stages W (sb + 2), issued last, may stay in flight
        // (in-order retire)
        if (NST == 3 && wn) {
            static_assert(NST != 3 || NI == 2, "vmcnt counts below assume two weight groups per wave");
            if (wave < NI || (Q5 && wave >= 4)) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // 3 weight DMAs
            else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        st = st == NST - 1 ? 0 : st + 1;
    }
    const int64_t n = n0 + 32 * wr + lr;
    if (n >= N) return;
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t t = m0 + 32 * (TPW * wt + j) + (r & 3) + 8 * (r >> 2) + 4 * kg;
            if (KS > 1) part[((int64_t)split * Mp + t) * N + n] = tot[j][r];
            else if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[j][r], res[t * ldr + n]) : tot[j][r];
        }
}

// ================================================================ Q6_K GEMM on int8 matrix cores (prefill image)
// q6v3 spends two f16 MFMAs per 16 k (sc*(q-32) needs 13 bits) plus the dequantization VALU of every fragment.  The
// prefill image keeps each weight's exact integer v = sc*(q-32) in [-4096, 4064] as two int8 planes,
//   v = 64 A + C,  A = floor((v + 32) / 64) in [-64, 64],  C = v - 64 A in [-32, 31],
// so one super-block row is 2 x 256 bytes and the sub-block scales are already inside: per 32 k two
// v_mfma_i32_32x32x32_i8 (int32 accumulators acc_A, acc_C) and no dequantization at all; isum = 64 acc_A + acc_C is
// the CPU's int32 sumi of the super-block (ggml_vec_dot_q6_K_q8_K, ggml-quants.c:8919) exactly, and the epilogue is
// q6v3's (tot = fma(dy, d * isum, tot)), so the results are q6v3's bit for bit wherever q6v3's fp32 accumulator holds
// its integer exactly (|sumi| < 2^24), and the CPU's exact integer always.
// Image: per 32-row tile rt and super-block sb, 16 blocks of 1 KiB (k-block kb = 0..7, plane p = 0 (A) / 1 (C)) at
// ((rt nsb + sb) 16 + 2 kb + p) KiB; lane l of a block = row 32 rt + (l & 31), k = 256 sb + 32 kb + 16 (l >> 5) + e,
// e = 0..15 -- exactly one v_mfma B operand, one contiguous 1 KiB wave load.  The row scale d stays in the Q6_K_RS
// weights (read beside the image).  Prefill only: decode keeps the 0.82 B / weight RS layout.
__device__ __forceinline__ int64_t q6p_off(int64_t n, int64_t k, int64_t nsb, int p) {
    const int64_t rt = n >> 5, sb = k >> 8;
    const int kk = (int)(k & 255), kb = kk >> 5, kg = (kk >> 4) & 1, e = kk & 15;
    return ((rt * nsb + sb) * 16 + 2 * kb + p) * 1024 + 16 * ((int)(n & 31) + 32 * kg) + e;
}

// one thread = (row n, super-block sb, RS unit u, byte j): the four elements g = 0..3 of that byte position
// (q6v3's unit decoding: k = 128 h + 16 lh + 32 g + j, sub-block 8 h + lh + 2 g, scale byte 4 u + g)
__global__ void k_q6p_build(const uint8_t *__restrict__ W, int64_t K, int64_t N, int64_t Np, uint8_t *__restrict__ img) {
    const int64_t nsb = K / 256;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Np * nsb * 64) return;
    const int j = (int)(i & 15), u = (int)((i >> 4) & 3);
    const int64_t sb = (i >> 6) % nsb, n = (i >> 6) / nsb;
    const int h = u >> 1, lh = u & 1;
    int8_t A[4], C[4];
    if (n < N) {
        const uint8_t *row = W + n * 210 * nsb;
        const int64_t U = 4 * sb + u;
        const uint8_t lo = row[16 * U + j], hi = row[64 * nsb + 16 * U + j], qh = row[128 * nsb + 16 * U + j];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int ql = ((g & 1) ? hi : lo) >> (4 * (g >> 1)) & 0xF;
            const int q = ql | (((qh >> (2 * g)) & 3) << 4);
            const int sc = (int8_t)row[192 * nsb + 4 * U + g];
            const int v = sc * (q - 32);
            const int a = (v + 32) >> 6;            // arithmetic shift: floor
            A[g] = (int8_t)a;
            C[g] = (int8_t)(v - 64 * a);
        }
    } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) A[g] = C[g] = 0;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int64_t k = 256 * sb + 128 * h + 16 * lh + 32 * g + j;
        img[q6p_off(n, k, nsb, 0)] = (uint8_t)A[g];
        img[q6p_off(n, k, nsb, 1)] = (uint8_t)C[g];
    }
}

struct Q6pSmem {
    i32x4 a[2][4][568];      // [buf][token tile][swz(row, chunk)]: 16 activation bytes, chunks 0..15 of the 256
    float dy[2][128];        // [buf][token]: Q8_K scale of the super-block
};

// grid: MT * (N / 128) * KS workgroups (KS copies of the tile grid along K, as q6v3), 256 threads, one workgroup per
// CU.  Workgroup = 128 tokens x 128 weight rows; wave w owns rows [32 w, +32) against all four 32-token tiles (every
// B fragment feeds four MFMAs).  B fragments go global -> registers one super-block ahead (two register sets, the
// loop unrolled by two so no set is copied while its loads are in flight); A (Q8_K bytes) and dy by LDS-DMA, double
// buffered, in q4v4's swizzled image.  XG = token tiles per XCD group (xcd_tile): MT keeps a row tile's four token
// tiles on one XCD, so its image comes from HBM once and from that XCD's L2 three times.
template <int NW>
__global__ void __launch_bounds__(64 * NW, 1) k_gemm_q6p(const i32x4 *__restrict__ img, const uint8_t *__restrict__ Wrs,
                                                    int64_t K, int64_t N, const uint8_t *__restrict__ act, int64_t M,
                                                    int64_t Mp, int MT, float *__restrict__ Y, int64_t ldy,
                                                    const float *res, int64_t ldr, int KS, float *__restrict__ part,
                                                    int XG) {
    constexpr int TPW = 16 / NW;                     // token tiles per wave: 4 (4 waves) or 2 (8 waves)
    __shared__ Q6pSmem S;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, kg = lane >> 5;
    const int64_t nsb = K / 256;
    const int8_t *qs = (const int8_t *)act;
    const float *dq = (const float *)(act + M * K);
    const int64_t ntn = N / 128, nwg = (int64_t)gridDim.x / KS;
    const int64_t id = blockIdx.x % nwg;
    const int split = (int)(blockIdx.x / nwg);
    int64_t mt, nt;
    xcd_tile(id, nwg, MT, ntn, XG, mt, nt);
    // wave w: rows [32 (w & 3), +32) of the tile against token tiles TPW (w >> 2) .. + TPW
    const int wr = wave & 3, jt0 = TPW * (wave >> 2);
    const int64_t m0 = mt * 128, rt = nt * 4 + wr;
    // A: token tile (wave & 3), chunk halves h (all, or wave >> 2 with 8 waves), row groups 0..3; lane: row
    // 8k + (lane & 7), chunk 8h + (lane >> 3).  dy: waves 0, 1 (tokens 64 wave + lane)
    const int att = wave & 3;
    const int64_t arow0 = m0 + 32 * att + (lane & 7);
    const int8_t *arow = qs + min(arow0, M - 1) * K + 16 * (lane >> 3);
    const float *dyrow = dq + min(m0 + 64 * min(wave, 1) + lane, M - 1) * nsb;
    auto stage_a = [&](int buf, int64_t sb) {
#pragma unroll
        for (int hh = 0; hh < 8 / NW; ++hh) {
            const int h = NW == 8 ? (wave >> 2) : hh;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                dma16(arow + (int64_t)min(8 * k, (int)max<int64_t>(M - 1 - arow0, 0)) * K + 128 * h + sb * 256,
                      &S.a[buf][att][72 * (4 * h + k)]);
        }
        if (wave < 2) dma4(dyrow + sb, &S.dy[buf][64 * wave]);
    };
    const i32x4 *wsrc = img + rt * nsb * 16 * 64 + lane;
    const uint16_t *pd = (const uint16_t *)(Wrs + (32 * rt + lr) * 210 * nsb + 208 * nsb);

    const int64_t sbb = nsb * split / KS, sbe = nsb * (split + 1) / KS;
    f16acc tot[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) tot[j][i] = 0.0f;

    // one register set: fragment pair kb of super-block sb + 1 is loaded into the registers of pair kb of sb right
    // after their last MFMA, so every load has one super-block of MFMAs to land in
    i32x4 b[16];
    stage_a(0, sbb);
#pragma unroll
    for (int q = 0; q < 16; ++q) b[q] = wsrc[(sbb * 16 + q) * 64];
    uint16_t d = pd[sbb];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);      // as k_gemm_q4v4 (q6p down 114.1 -> 113.1 us)
    for (int64_t sb = sbb; sb < sbe; ++sb) {
        const int buf = (int)((sb - sbb) & 1);
        const bool nx = sb + 1 < sbe;
        if (nx) stage_a(buf ^ 1, sb + 1);
        const float dw = h2f(d);
        if (nx) d = pd[sb + 1];
        // k-block outer, token tile inner: eight independent accumulators, one A fragment live at a time
        i32x16 aa[TPW], ac[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) aa[j][i] = ac[j][i] = 0;
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
#pragma unroll
            for (int j = 0; j < TPW; ++j) {
                const i32x4 a = S.a[buf][jt0 + j][swz(lr, 2 * kb + kg)];
                aa[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[2 * kb], aa[j], 0, 0, 0);
                ac[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[2 * kb + 1], ac[j], 0, 0, 0);
            }
            if (nx) {
                b[2 * kb] = wsrc[((sb + 1) * 16 + 2 * kb) * 64];
                b[2 * kb + 1] = wsrc[((sb + 1) * 16 + 2 * kb + 1) * 64];
            }
        }
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *(const float4 *)&S.dy[buf][32 * (jt0 + j) + 8 * q + 4 * kg];
                const float dv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * q + e;
                    tot[j][r] = fmaf(dv[e], __fmul_rn(dw, (float)(aa[j][r] * 64 + ac[j][r])), tot[j][r]);
                }
            }
        }
        // A (sb + 1) landed (the d and 16 B loads issued after it may stay in flight); everyone is done with buf
        if (nx) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        __syncthreads();
    }
    const int64_t n = 32 * rt + lr;
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t t = m0 + 32 * (jt0 + j) + (r & 3) + 8 * (r >> 2) + 4 * kg;
            if (KS > 1) part[((int64_t)split * Mp + t) * N + n] = tot[j][r];
            else if (t < M) Y[t * ldy + n] = res ? __fadd_rn(tot[j][r], res[t * ldr + n]) : tot[j][r];
        }
}

static int g_gemm_variant = -1;
static int gemm_variant() {
    if (g_gemm_variant < 0) g_gemm_variant = 0;
    return g_gemm_variant;
}

// BASELINE config 3's small-batch Q8_0 path: split-K int8-MFMA partials, then the ordered reduce (plain, + residual,
// silu(g) * u, or silu(g) * u quantized straight to Q8_0 into qout for the next GEMM)
static int gemm_q80_small(const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
                          int64_t ldy, const float *res, int64_t ldr, int mode, uint8_t *qout, uint8_t *wsp, hipStream_t s) {
    const int S = q80s_splits(K, N);
    float *part = (float *)wsp;
    float *part2 = part + (int64_t)S * 32 * N;
    const int64_t nb = K / 32, bps = (nb + S - 1) / S;
    const dim3 grid((unsigned)((N + 127) / 128), (unsigned)S);
    Q80Segs sg = {{(const uint8_t *)W, nullptr, nullptr}, {N, 0, 0}, 1};
    auto q80 = [&](float *pt) {
        hipLaunchKernelGGL(k_gemm_q80s2, grid, dim3(256), 0, s, sg, K, N, (const uint8_t *)act, M, pt);
    };
    q80(part);
    KCPP_CHECK(hipGetLastError());
    if (mode == 1) {
        sg.W[0] = (const uint8_t *)W2;
        q80(part2);
        KCPP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_q80s_reduce, dim3((unsigned)((M * N + 255) / 256)), dim3(256), 0, s, part, mode == 1 ? part2 : nullptr,
                       S, M, N, Y, ldy, mode == 1 ? nullptr : res, ldr, qout);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

extern "C" {

int kcpp_gemm_set_variant(int v) {
    const int old = gemm_variant();
    g_gemm_variant = v;
    return old;
}

// q|k|v style: nseg <= 3 Q8_0 weights [K][N_i] whose outputs sit back to back in Y's columns, M <= 32,
// every N_i a multiple of 128; ws from kcpp_gemm_workspace_bytes(KT_Q8_0, K, sum N_i, M)
int kcpp_gemm_q80_segs(const void *const *W, const int64_t *N, int nseg, int64_t K, const void *act, int64_t M, float *Y,
                       int64_t ldy, void *ws, void *stream) {
    if (nseg < 1 || nseg > 3 || M < 1 || M > 32 || K % 32 || !ws) return -1;
    Q80Segs sg = {{nullptr, nullptr, nullptr}, {0, 0, 0}, nseg};
    int64_t Ntot = 0;
    for (int i = 0; i < nseg; ++i) {
        if (N[i] <= 0 || (N[i] % 128 && i + 1 < nseg)) return -1;
        sg.W[i] = (const uint8_t *)W[i];
        sg.N[i] = N[i];
        Ntot += N[i];
    }
    int64_t o_a16, o_dy, o_bs, o_up;
    ws_layout(KT_Q8_0, K, Ntot, M, o_a16, o_dy, o_bs, o_up);
    float *part = (float *)((uint8_t *)ws + o_up + ((M * Ntot * 4 + 255) & ~255LL));
    const int S = q80s_splits(K, Ntot);
    const int64_t nb = K / 32, bps = (nb + S - 1) / S;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_gemm_q80s2, dim3((unsigned)((Ntot + 127) / 128), (unsigned)S), dim3(256), 0, s, sg,
                       K, Ntot, (const uint8_t *)act, M, part);
    KCPP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_q80s_reduce, dim3((unsigned)((M * Ntot + 255) / 256)), dim3(256), 0, s, part, nullptr, S, M, Ntot, Y, ldy,
                       nullptr, 0);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// Q6_K prefill image (k_q6p_build / k_gemm_q6p): N % 128 == 0, K % 256 == 0
int64_t kcpp_q6p_image_bytes(int64_t K, int64_t N) {
    if (K <= 0 || N <= 0 || K % 256 || N % 128) return 0;
    return N * K * 2;
}

int kcpp_q6p_build(const void *W, int64_t K, int64_t N, void *img, void *stream) {
    if (!W || !img || !kcpp_q6p_image_bytes(K, N)) return -1;
    const int64_t nth = N * (K / 256) * 64;
    hipLaunchKernelGGL(k_q6p_build, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, (hipStream_t)stream, (const uint8_t *)W,
                       K, N, N, (uint8_t *)img);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// kcpp_gemm(KT_Q6_K_RS, ...) with the prefill image(s) beside the RS weights: the same results bit for bit (same
// K split rule, same epilogue order), int8 matrix cores.  M > 32; mode 0 (res optional) or 1 (silu(g) * u, W2 / img2);
// ws from kcpp_gemm_workspace_bytes(KT_Q6_K_RS, K, N, M).  Returns -3 for shapes the image does not cover.
int kcpp_gemm_q6p(const void *img, const void *W, const void *img2, const void *W2, int64_t K, int64_t N, const void *act,
                  int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, void *stream) {
    if (!img || !W || !act || !Y || !ws || M < 1 || (mode == 1 && (!img2 || !W2)) || mode < 0 || mode > 1) return -1;
    if (!kcpp_q6p_image_bytes(K, N)) return -3;
    hipStream_t s = (hipStream_t)stream;
    int64_t o_a16, o_dy, o_bs, o_up;
    ws_layout(KT_Q6_K_RS, K, N, M, o_a16, o_dy, o_bs, o_up);
    uint8_t *w8 = (uint8_t *)ws;
    float *up = (float *)(w8 + o_up);
    float *part = (float *)(w8 + o_up + ((M * N * 4 + 255) & ~255LL));
    const int64_t Mp = (M + 127) / 128 * 128, nsb = K / 256, nt = N / 128;
    const int MT = (int)(Mp / 128);
    // q6v3's split rule (kcpp_gemm, variant 0), so the f32 summation order -- and every bit -- is the same
    const bool big = Mp / 128 * nt >= 384;
    const int KS = (mode == 0 && nsb % 2 == 0 && !big && (nt < 16 || nsb >= 32)) ? 2 : 1;
    const int XG = 8 % MT == 0 ? MT : 1;
    static const int NWq = [] { const char *e = getenv("KCPP_Q6P_NW"); return e && atoi(e) == 4 ? 4 : 8; }();
    const unsigned nwg = (unsigned)(MT * nt * KS);
    auto launch = [&](const void *im, const void *w, float *y, int64_t ly, const float *r, int64_t lr) -> int {
        if (NWq == 8)
            hipLaunchKernelGGL(k_gemm_q6p<8>, dim3(nwg), dim3(512), 0, s, (const i32x4 *)im, (const uint8_t *)w, K, N,
                               (const uint8_t *)act, M, Mp, MT, y, ly, r, lr, KS, part, XG);
        else
            hipLaunchKernelGGL(k_gemm_q6p<4>, dim3(nwg), dim3(256), 0, s, (const i32x4 *)im, (const uint8_t *)w, K, N,
                               (const uint8_t *)act, M, Mp, MT, y, ly, r, lr, KS, part, XG);
        KCPP_CHECK(hipGetLastError());
        if (KS > 1) {
            splitk_finish(part, KS, M, Mp, N, y, ly, r, lr, s);
            KCPP_CHECK(hipGetLastError());
        }
        return 0;
    };
    int rc = launch(img, W, Y, ldy, mode == 1 ? nullptr : res, ldr);
    if (rc || mode != 1) return rc;
    if ((rc = launch(img2, W2, up, N, nullptr, 0))) return rc;
    hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// kcpp_gemm / kcpp_gemm_q6p (mode 0) followed by kcpp_rms_norm(Y, ldy, norm_w, -> q8k_out): when the GEMM splits K, its
// reduce forms the norm's Q8_K activation in the same launch; the results are those of the two calls bit for bit
static int gemm_then_norm(int rc_gemm_call(void *), void *ctx, float *Y, int64_t ldy, int64_t N, int64_t M,
                          const float *norm_w, float eps, void *q8k_out, void *stream) {
    NormHook h{norm_w, q8k_out, eps, false};
    g_norm_hook = &h;
    const int rc = rc_gemm_call(ctx);
    g_norm_hook = nullptr;
    if (rc) return rc;
    if (h.used) return 0;
    return kcpp_rms_norm(Y, ldy, norm_w, nullptr, 0, q8k_out, N, M, eps, stream);
}

int kcpp_gemm_rms_norm(int type, const void *W, int64_t K, int64_t N, const void *act, int64_t M, float *Y, int64_t ldy,
                       const float *res, int64_t ldr, void *ws, void *stream, const float *norm_w, float eps, void *q8k_out) {
    if (!norm_w || !q8k_out) return -1;
    struct C { int type; const void *W; int64_t K, N; const void *act; int64_t M; float *Y; int64_t ldy; const float *res;
               int64_t ldr; void *ws, *stream; } c{type, W, K, N, act, M, Y, ldy, res, ldr, ws, stream};
    return gemm_then_norm([](void *p) {
        const C &c = *(const C *)p;
        return kcpp_gemm(c.type, c.W, nullptr, c.K, c.N, c.act, c.M, c.Y, c.ldy, c.res, c.ldr, 0, c.ws, c.stream);
    }, &c, Y, ldy, N, M, norm_w, eps, q8k_out, stream);
}

int kcpp_gemm_q6p_rms_norm(const void *img, const void *W, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
                           int64_t ldy, const float *res, int64_t ldr, void *ws, void *stream, const float *norm_w, float eps,
                           void *q8k_out) {
    if (!norm_w || !q8k_out) return -1;
    struct C { const void *img, *W; int64_t K, N; const void *act; int64_t M; float *Y; int64_t ldy; const float *res;
               int64_t ldr; void *ws, *stream; } c{img, W, K, N, act, M, Y, ldy, res, ldr, ws, stream};
    return gemm_then_norm([](void *p) {
        const C &c = *(const C *)p;
        return kcpp_gemm_q6p(c.img, c.W, nullptr, nullptr, c.K, c.N, c.act, c.M, c.Y, c.ldy, c.res, c.ldr, 0, c.ws, c.stream);
    }, &c, Y, ldy, N, M, norm_w, eps, q8k_out, stream);
}

int64_t kcpp_gemm_workspace_bytes(int type, int64_t K, int64_t N, int64_t M) {
    if (type == KT_Q8_0_T) return kcpp_q80t_ws_bytes(K, N, M);
    int64_t a, b, c, d;
    return ws_layout(type, K, N, M, a, b, c, d);
}

int kcpp_gemm_q80_glu_q80(const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, void *qout,
                          void *ws, void *stream) {
    if (M < 1 || M > 32 || K % 32 || N % 32 || !ws || !qout) return -1;
    int64_t o_a16, o_dy, o_bs, o_up;
    ws_layout(KT_Q8_0, K, N, M, o_a16, o_dy, o_bs, o_up);
    return gemm_q80_small(W, W2, K, N, act, M, nullptr, 0, nullptr, 0, 1, (uint8_t *)qout,
                          (uint8_t *)ws + o_up + ((M * N * 4 + 255) & ~255LL), (hipStream_t)stream);
}

// grouped expert GEMM (MoE prefill): ng groups of cnt_host[e] token rows (act: Q8_K of all M = sum rows, grouped
// back to back), group e against W + e wstride (and W2 + e wstride); mode 0: Y = X W^T, mode 1: Y = silu(X W^T) *
// (X W2^T) with up [M][N] as scratch.  cnt_dev: the same counts on the device (read by the kernel); Q4_K / Q5_K
// (+ RS) only, K a multiple of 256.  One launch per mode (+ the GLU product); every row's arithmetic is v4's unsplit
// (bitwise the single-expert kcpp_gemm result wherever that runs unsplit)
int64_t kcpp_gemm_grouped_ws_bytes(int type, int64_t K, int64_t M, int ng) {
    if (type != KT_Q6_K_RS) return 0;
    const int64_t Pv = M + 128LL * ng;                  // >= the padded virtual rows
    return ((Pv * K * 2 + 255) & ~255LL) + Pv * (K / 256) * 4;
}

int kcpp_gemm_grouped(int type, const void *W, const void *W2, int64_t wstride, int64_t K, int64_t N, const void *act,
                      int64_t M, const int32_t *cnt_host, const int32_t *cnt_dev, int ng, float *Y, float *up, int mode,
                      void *ws, void *stream) {
    if (type != KT_Q4_K && type != KT_Q4_K_RS && type != KT_Q5_K && type != KT_Q5_K_RS && type != KT_Q6_K_RS) return -1;
    if (K % 256 || ng < 1 || ng > 64 || !cnt_dev || !cnt_host || (mode == 1 && (!W2 || !up)) || mode < 0 || mode > 1)
        return -1;
    if (type == KT_Q6_K_RS) {
        // Q6_K (RS layout): k_gemm_q6v3 over a 128-row-padded virtual layout (the f16 fragment image of every
        // group, padding rows zero), 128 x 128 tiles, 8 waves, unsplit; plain mode only
        if (mode != 0 || !ws) return -1;
        int64_t Pv = 0, rows = 0;
        for (int e = 0; e < ng; ++e) {
            if (cnt_host[e] < 0) return -1;
            Pv += (cnt_host[e] + 127) / 128 * 128;
            rows += cnt_host[e];
        }
        if (rows != M) return -1;
        if (!Pv) return 0;
        hipStream_t s = (hipStream_t)stream;
        h8v *a16 = (h8v *)ws;
        float *dyT = (float *)((uint8_t *)ws + ((Pv * K * 2 + 255) & ~255LL));
        const int64_t nth = Pv * K / 8 + Pv * (K / 256);
        hipLaunchKernelGGL(k_act_frag6, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, s, (const uint8_t *)act, K, M, Pv,
                           a16, dyT, cnt_dev, ng);
        KCPP_CHECK(hipGetLastError());
        // tile shape (never changes a bit): 128 x 128, 8 waves; variants 15 / 17 force (BMT, NW) = (4, 4) / (2, 8)
        const int gv = gemm_variant();
        const int BMT = gv == 17 ? 2 : 4, NWv = gv == 15 ? 4 : 8;
        const int MT = (int)(Pv / (32 * BMT));
        const unsigned nwg = (unsigned)(MT * ((N + 127) / 128));
#define KCPP_G6(NW_, B_)                                                                                                   \
    hipLaunchKernelGGL((k_gemm_q6v3<NW_, B_>), dim3(nwg), dim3(64 * NW_), 0, s, (const uint8_t *)W, K, N, (const h8v *)a16, \
                       dyT, Pv, Pv, MT, Y, N, (const float *)nullptr, (int64_t)0, 1, (float *)nullptr, cnt_dev, ng, wstride)
        if (BMT == 2) KCPP_G6(8, 2);
        else if (NWv == 4) KCPP_G6(4, 4);
        else KCPP_G6(8, 4);
#undef KCPP_G6
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (((uintptr_t)((const uint8_t *)act + M * K + M * (K / 256) * 4) & 15) != 0) return -3;
    int64_t tiles = 0, rows = 0;
    const int64_t ntn = (N + 127) / 128;
    for (int e = 0; e < ng; ++e) {
        if (cnt_host[e] < 0) return -1;
        tiles += (cnt_host[e] + 127) / 128 * ntn;
        rows += cnt_host[e];
    }
    if (rows != M) return -1;
    if (!tiles) return 0;
    hipStream_t s = (hipStream_t)stream;
    auto kern = type == KT_Q5_K_RS ? k_gemm_q4v4<KT_Q5_K, 1, 2>
                : type == KT_Q5_K  ? k_gemm_q4v4<KT_Q5_K, 0, 2>
                : type == KT_Q4_K_RS ? k_gemm_q4v4<KT_Q4_K, 1, 2> : k_gemm_q4v4<KT_Q4_K, 0, 2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)(tiles * (mode == 1 ? 2 : 1))), dim3(512), 0, s, (const uint8_t *)W, K, N,
                       (const uint8_t *)act, M, M, 1, Y, N, (const float *)nullptr, (int64_t)0, 1, (float *)nullptr, 1,
                       (const uint8_t *)(mode == 1 ? W2 : nullptr), up, N, cnt_dev, ng, wstride);
    KCPP_CHECK(hipGetLastError());
    if (mode == 1) {
        hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, N, up, N, M);
        KCPP_CHECK(hipGetLastError());
    }
    return 0;
}

int kcpp_gemm(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
              int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, void *stream) {
    if (type == KT_Q8_0_T) {          // the tile layout (gemm_q80t.hip): every M, activation KT_Q8_0_TA
        const void *Ws[1] = {W};
        const int64_t Ns[1] = {N};
        return kcpp_gemm_q80t(Ws, Ns, 1, W2, K, act, M, Y, ldy, res, ldr, mode, nullptr, ws, stream);
    }
    hipStream_t s = (hipStream_t)stream;
    if (K % GB_K) return -1;
    if (!ws) return -2;
    int64_t o_a16, o_dy, o_bs, o_up;
    ws_layout(type, K, N, M, o_a16, o_dy, o_bs, o_up);
    const int64_t Mp = (M + GB_M - 1) / GB_M * GB_M;
    uint8_t *w8 = (uint8_t *)ws;
    _Float16 *a16 = (_Float16 *)(w8 + o_a16);
    float *dy = (float *)(w8 + o_dy);
    _Float16 *bs16 = (_Float16 *)(w8 + o_bs);
    float *up = (float *)(w8 + o_up);
    const int vt = vec_dot_type(type);
    const int gv = gemm_variant();
    const bool iqg = type == KT_IQ2_XXS || type == KT_IQ2_XS || type == KT_IQ2_S || type == KT_IQ3_XXS ||
                     type == KT_IQ3_S || type == KT_IQ1_S || type == KT_IQ1_M;
    if ((type == KT_Q4_1 || type == KT_Q5_1 || type == KT_IQ4_NL || type == KT_IQ4_XS || iqg) && (M <= 16 || gv == 20)) {
        // the legacy Q8_1-activation types (Q4_1 / Q5_1 files) and the code-book types (IQ4_NL / IQ4_XS) at small
        // batch: the exact mat-vec over groups of 8 columns (one pass over the weights each); past 16 columns the
        // MFMA GEMM below is faster (tools/gemm_lowbit_ab.py: Q4_1 4096 x 14336 at 16 / 37 / 512 tokens: mat-vec
        // 52 / 125 / 1592 us, GEMM 67 / 72 / 229 us)
        for (int64_t c0 = 0; c0 < M; c0 += 8) {
            const int rc = gemv_cols(type, W, W2, K, N, act, std::min<int64_t>(8, M - c0), M, c0, Y, ldy, res, ldr, mode,
                                     stream);
            if (rc) return rc;
        }
        return 0;
    }
    if (type == KT_Q8_0 && M <= 32 && K % 32 == 0) return gemm_q80_small(W, W2, K, N, act, M, Y, ldy, res, ldr, mode, nullptr,
                                                                        w8 + o_up + ((M * N * 4 + 255) & ~255LL), s);
    // v3: 128 tokens x 128 rows per workgroup when that gives >= 384 workgroups, else 64 x 128 (BMT = 2); on those
    // small grids the K range is split in two (KS = 2: twice the workgroups, two per CU, partials summed in order by
    // k_splitk_reduce) when the grid is tiny (< 128 workgroups) or K long (>= 32 super-blocks): measured at M = 512
    // (tools/gemm_ab.py) down 14336 x 4096 122.9 -> 112.3 us, attn_v 4096 x 1024 (Q6_K) 56.7 -> 33.9 us, wo 4096 x 4096
    // 43.3 -> 45.6 us (not split), gate|up (big grid) 236.8 -> 273.0 us (not split).
    // kcpp_gemm_set_variant: 2 forces v2, 3 v3 without the split, 4 v3 with the split wherever the mode allows
    const bool v3 = gv == 0 || (gv >= 3 && gv <= 13) || (gv >= 15 && gv <= 17);
    float *part = (float *)(w8 + o_up + ((M * N * 4 + 255) & ~255LL));
    // (the rule reads the weight shape only -- "< 128 tiles" as counted at the 512-token ubatch, 64 x 128 tiles --
    // so a prompt's bits do not depend on how it is cut into ubatches)
    auto splitk = [&](bool big, int64_t) {
        if (mode != 0 || (K / 256) % 2) return 1;
        return (gv == 4 || ((gv == 0 || (gv >= 15 && gv <= 17)) && !big && ((N + 127) / 128 < 16 || K / 256 >= 32))) ? 2 : 1;
    };
    const bool bs_aligned = ((uintptr_t)((const uint8_t *)act + M * K + M * (K / 256) * 4) & 15) == 0;
    // v4 for every Q4_K shape past the small-batch range (tools/gemm_ab.py, M = 512, v3 -> v4): gate|up 28672 rows
    // 249 -> 216 us, down 14336 -> 4096 122 -> 101, q|k|v 6144 rows 59.4 -> 52.1 (unsplit), wo 4096 rows 43.1 -> 38.5
    // (split-K); its tile grid is split in two along K when it has <= 128 tiles.  Variant 11 forces v4 (split rule),
    // 13 v4 unsplit, 3 / 4 force v3.
    const bool v4_pick = gv == 0;
    // Q5_K: v4 with the fifth-bit MFMA (TPW 2 only) for the plain / residual projections it splits along K (<= 32
    // row tiles; tools/gemm_ab.py, v2 -> v4: Mixtral expert down 14336 -> 4096 M = 128 134.3 -> 96.3 us, M = 512
    // 151.4 -> 124.6; wo 4096^2 42.6 -> 34.6 / 49.1 -> 45.4) -- a weight-shape rule, as the split changes bits -- and
    // for GLU (gate + up in one launch) up to 256 tokens: 4096 -> 2 x 14336 M = 128 93.9 -> 73.1.  Unsplit shapes
    // stay on v2 (`profiles/r05_q5k_v4_gemm_ab.jsonl`: GLU M = 512 ~270 vs ~305; dense gate|up 4096 -> 28672 M = 512
    // ~240 vs ~271; q|k|v 6144 rows M = 128 43.6 vs 55.7); unsplit v4 and v2 are bitwise equal
    // (test_gemm_v4_int8_matches_v2_bitwise), so the GLU token-count rule does not change a bit.  Variants 11 / 13
    // force v4.
    const bool q5split = mode == 0 && (K / 256) % 2 == 0 && (N + 127) / 128 <= 32;
    const bool q5 = (type == KT_Q5_K || type == KT_Q5_K_RS) && (gv != 0 || q5split || (mode == 1 && Mp <= 256));
    if ((type == KT_Q4_K || type == KT_Q4_K_RS || q5) && (gv == 11 || gv == 12 || gv == 13 || gv == 14 || v4_pick) && bs_aligned &&
        M > 32) {
        // v4: int8 MFMA straight from the Q8_K buffer (no fragment image); 128 x 128 tiles, split-K when the tile
        // grid is small
        const int64_t nt = (N + 127) / 128;
        const int MT = (int)(Mp / 128);
        // the split is chosen from the weight shape alone (<= 128 tiles at the 512-token ubatch, i.e. <= 32 row
        // tiles), never from M: the split changes the f32 summation order, and a prompt must give the same bits
        // however it is cut into ubatches (tests/test_gpu_fullsize.py)
        const int KS = (gv != 13 && mode == 0 && (K / 256) % 2 == 0 && nt <= 32) ? 2 : 1;
        // v5 (TPW = 4: 256-row tiles, each dequantized fragment feeding all 128 tokens' MFMAs) wherever its grid
        // still covers ~7/8 of the CUs; same per-element arithmetic and order as v4 (and KS = 1 on both), so the
        // choice never changes a bit (tools/gemm_ab.py, M = 512, v4 -> v5: gate|up 28672 rows 214.1 -> 188.6 us,
        // gate + up 14336 rows 217.7 -> 201.0; q|k|v 6144 rows 52.3 -> 86.0 on its 96-workgroup grid, so not
        // there).  Variant 14 forces v5.
        const bool v5 = !q5 && (gv == 14 || (gv == 0 && KS == 1 && MT * ((N + 255) / 256) >= 224));
        const int64_t ntw = v5 ? (N + 255) / 256 : nt;
        const unsigned nwg = (unsigned)(MT * ntw * KS);
        const int XG = gv == 12 ? 2 : 1;
        auto launch4 = [&](const void *w, float *y, int64_t ly, const float *r, int64_t lr, const void *w2, float *y2) -> int {
            auto kern = type == KT_Q5_K_RS ? k_gemm_q4v4<KT_Q5_K, 1, 2>
                        : type == KT_Q5_K  ? k_gemm_q4v4<KT_Q5_K, 0, 2>
                        : type == KT_Q4_K_RS ? (v5 ? k_gemm_q4v4<KT_Q4_K, 1, 4> : k_gemm_q4v4<KT_Q4_K, 1, 2>)
                                             : (v5 ? k_gemm_q4v4<KT_Q4_K, 0, 4> : k_gemm_q4v4<KT_Q4_K, 0, 2>);
            hipLaunchKernelGGL(kern, dim3(nwg * (w2 ? 2 : 1)), dim3(512), 0, s, (const uint8_t *)w, K, N, (const uint8_t *)act,
                               M, Mp, MT, y, ly, r, lr, KS, part, XG, (const uint8_t *)w2, y2, (int64_t)N,
                               (const int32_t *)nullptr, 0, (int64_t)0);
            KCPP_CHECK(hipGetLastError());
            if (KS > 1) {
                splitk_finish(part, KS, M, Mp, N, y, ly, r, lr, s);
                KCPP_CHECK(hipGetLastError());
            }
            return 0;
        };
        // GLU (KS = 1): gate and up in one launch
        int rc = launch4(W, Y, ldy, mode == 1 ? nullptr : res, ldr, mode == 1 ? W2 : nullptr, up);
        if (rc || mode != 1) return rc;
        hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if ((type == KT_Q4_K || type == KT_Q4_K_RS) && v3) {
        const int64_t nth = Mp * K / 8 + (Mp / 32) * (K / 256) * 64 + Mp * (K / 256);
        hipLaunchKernelGGL(k_act_frag3, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, s, (const uint8_t *)act, K, M, Mp,
                           (h8v *)a16, dy, (h8v *)bs16);
        KCPP_CHECK(hipGetLastError());
        // measured at M = 512 (tools/gemm_ab.py): 128 x 128 tiles with 8 waves for gate|up (247 vs v2 301 us),
        // 64 x 128 tiles with 4 waves for the 128-192-tile shapes (wo 44.7 vs 46.7, down 131.5 vs 137.2 us)
        const int64_t nt = (N + 127) / 128;
        const bool big = Mp / 128 * nt >= 384;
        const int BMT = big ? 4 : 2;
        const int NWv = (gv == 6 || gv == 7) ? 4 : (big ? 8 : 4);
        const int XG = gv == 8 ? 2 : (gv == 9 ? 4 : (gv == 10 ? 8 : 1));
        const int MT = (int)(Mp / (32 * BMT));
        const int KS = splitk(big, MT * nt);
        const unsigned nwg = (unsigned)(MT * nt * KS);
        auto launch3 = [&](const void *w, float *y, int64_t ly, const float *r, int64_t lr) -> int {
#define KCPP_V3(L_, NW_, B_)                                                                                                 \
    if (gv == 5 || gv == 6) hipLaunchKernelGGL((k_gemm_q4v3<L_, NW_, B_, 2>), dim3(nwg), dim3(64 * NW_), 0, s, (const uint8_t *)w, K, N,      \
                       (const h8v *)a16, dy, (const h8v *)bs16, M, Mp, MT, y, ly, r, lr, KS, part, XG);                      \
    else hipLaunchKernelGGL((k_gemm_q4v3<L_, NW_, B_, 1>), dim3(nwg), dim3(64 * NW_), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, \
                       dy, (const h8v *)bs16, M, Mp, MT, y, ly, r, lr, KS, part, XG)
#define KCPP_V3B(L_, B_) { if (NWv == 4) KCPP_V3(L_, 4, B_); else KCPP_V3(L_, 8, B_); }
            if (type == KT_Q4_K_RS) { if (BMT == 2) KCPP_V3B(1, 2) else KCPP_V3B(1, 4) }
            else { if (BMT == 2) KCPP_V3B(0, 2) else KCPP_V3B(0, 4) }
#undef KCPP_V3B
#undef KCPP_V3
            KCPP_CHECK(hipGetLastError());
            if (KS > 1) {
                splitk_finish(part, KS, M, Mp, N, y, ly, r, lr, s);
                KCPP_CHECK(hipGetLastError());
            }
            return 0;
        };
        int rc = launch3(W, Y, ldy, mode == 1 ? nullptr : res, ldr);
        if (rc || mode != 1) return rc;
        if ((rc = launch3(W2, up, N, nullptr, 0))) return rc;
        hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (type == KT_Q6_K_RS && v3) {
        const int64_t nth = Mp * K / 8 + Mp * (K / 256);
        hipLaunchKernelGGL(k_act_frag6, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, s, (const uint8_t *)act, K, M, Mp,
                           (h8v *)a16, dy, (const int32_t *)nullptr, 0);
        KCPP_CHECK(hipGetLastError());
        const int64_t nt = (N + 127) / 128;
        const bool big = Mp / 128 * nt >= 384;
        // long K (ffn_down, K/256 >= 32, split in two) also takes 128-token x 128-row tiles with 8 waves while that
        // grid still has a workgroup per CU: tools/gemm_ab.py, M = 512, down 14336 x 4096 195.3 -> 171.5 us (v: 34.5
        // stays on 64-token tiles, 49.8 / 53.9 on 128); the tile shape never changes a bit.  Variants 15 / 16 / 17
        // force (BMT, NW) = (4, 4) / (4, 8) / (2, 8).
        const bool longk = K / 256 >= 32 && mode == 0 && (K / 256) % 2 == 0 && Mp / 128 * nt * 2 >= 256;
        const int BMT = gv == 15 || gv == 16 ? 4 : (gv == 17 ? 2 : (big || longk ? 4 : 2));
        const int NWv = gv == 15 ? 4 : (gv == 16 || gv == 17 ? 8 : (big || longk ? 8 : 4));
        const int MT = (int)(Mp / (32 * BMT));
        const int KS = splitk(big, MT * nt);
        const unsigned nwg = (unsigned)(MT * nt * KS);
        auto launch6 = [&](const void *w, float *y, int64_t ly, const float *r, int64_t lr) -> int {
#define KCPP_V6(NW_, B_)                                                                                                   \
    hipLaunchKernelGGL((k_gemm_q6v3<NW_, B_>), dim3(nwg), dim3(64 * NW_), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, \
                       M, Mp, MT, y, ly, r, lr, KS, part, (const int32_t *)nullptr, 0, (int64_t)0)
            if (BMT == 2) { if (NWv == 4) KCPP_V6(4, 2); else KCPP_V6(8, 2); }
            else { if (NWv == 4) KCPP_V6(4, 4); else KCPP_V6(8, 4); }
#undef KCPP_V6
            KCPP_CHECK(hipGetLastError());
            if (KS > 1) {
                splitk_finish(part, KS, M, Mp, N, y, ly, r, lr, s);
                KCPP_CHECK(hipGetLastError());
            }
            return 0;
        };
        int rc = launch6(W, Y, ldy, mode == 1 ? nullptr : res, ldr);
        if (rc || mode != 1) return rc;
        if ((rc = launch6(W2, up, N, nullptr, 0))) return rc;
        hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    const bool rs = type == KT_Q4_K_RS || type == KT_Q5_K_RS || type == KT_Q6_K_RS;       // decode layouts: v2 only
    if (rs || type == KT_Q4_K || type == KT_Q5_K || type == KT_Q6_K) {
        const int64_t nth = Mp * K / 8 + (Mp / 32) * (K / 256) * 64 + Mp * (K / 256);
        hipLaunchKernelGGL(k_act_frag, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, s, (const uint8_t *)act, K, M, Mp,
                           (h8v *)a16, dy, (h8v *)bs16);
        KCPP_CHECK(hipGetLastError());
        const int TMv = (type != KT_Q4_K && type != KT_Q4_K_RS) ? 1 : ((Mp % 256 == 0 && N >= 8192) ? 2 : 1);
        if (TMv == 2 && Mp % 256) return -5;
        const int MT = (int)(Mp / (GB_M * TMv));
        const unsigned nwg = (unsigned)(MT * ((N + GB_N - 1) / GB_N));
        auto launch2 = [&](const void *w, float *y, int64_t ly, const float *r, int64_t lr) -> int {
            switch (type) {
            case KT_Q4_K: if (TMv == 2) hipLaunchKernelGGL((k_gemm_kq<KT_Q4_K, 2, 0>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                else hipLaunchKernelGGL((k_gemm_kq<KT_Q4_K, 1, 0>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            case KT_Q5_K: hipLaunchKernelGGL((k_gemm_kq<KT_Q5_K, 1, 0>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            case KT_Q6_K: hipLaunchKernelGGL((k_gemm_kq<KT_Q6_K, 1, 0>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            case KT_Q4_K_RS: if (TMv == 2) hipLaunchKernelGGL((k_gemm_kq<KT_Q4_K, 2, 1>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                else hipLaunchKernelGGL((k_gemm_kq<KT_Q4_K, 1, 1>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            case KT_Q5_K_RS: hipLaunchKernelGGL((k_gemm_kq<KT_Q5_K, 1, 1>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            default: hipLaunchKernelGGL((k_gemm_kq<KT_Q6_K, 1, 1>), dim3(nwg), dim3(256), 0, s, (const uint8_t *)w, K, N, (const h8v *)a16, dy, (const h8v *)bs16, M, MT, y, ly, r, lr);
                break;
            }
            KCPP_CHECK(hipGetLastError());
            return 0;
        };
        int rc = launch2(W, Y, ldy, mode == 1 ? nullptr : res, ldr);
        if (rc || mode != 1) return rc;
        rc = launch2(W2, up, N, nullptr, 0);
        if (rc) return rc;
        hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    hipLaunchKernelGGL(k_act_to_f16, dim3((unsigned)((K + 1023) / 1024), (unsigned)Mp), dim3(256), 0, s,
                       (const uint8_t *)act, vt, K, M, Mp, a16, dy, bs16);
    KCPP_CHECK(hipGetLastError());
    // v1 split-K (ks1_of: from the weight shape only): a lone workgroup otherwise walks all of K, one load latency a step
    const int KS1 = gv == 21 ? 1 : ks1_of(K, N);
    const dim3 grid((unsigned)((N + GB_N - 1) / GB_N), (unsigned)(Mp / GB_M), (unsigned)KS1);
    const float *s81 = vt == KT_Q8_1 ? act_view(vt, act, K, M, 0).s : nullptr;      // block_q8_1.s [M][K/32]
    auto launch = [&](const void *w, float *y, int64_t ly, const float *r, int64_t lr) -> int {
        switch (type) {
        case KT_Q2_K: hipLaunchKernelGGL(k_gemm<KT_Q2_K>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_Q3_K: hipLaunchKernelGGL(k_gemm<KT_Q3_K>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_Q4_0: hipLaunchKernelGGL(k_gemm<KT_Q4_0>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_Q5_0: hipLaunchKernelGGL(k_gemm<KT_Q5_0>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_Q8_0: hipLaunchKernelGGL(k_gemm<KT_Q8_0>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_Q4_1: hipLaunchKernelGGL(k_gemm<KT_Q4_1>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, s81, part, Mp); break;
        case KT_Q5_1: hipLaunchKernelGGL(k_gemm<KT_Q5_1>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, s81, part, Mp); break;
        case KT_IQ4_NL: hipLaunchKernelGGL(k_gemm<KT_IQ4_NL>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        case KT_IQ4_XS: hipLaunchKernelGGL(k_gemm<KT_IQ4_XS>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
#define KCPP_IQ_GEMM(T) \
        case T: hipLaunchKernelGGL(k_gemm<T>, grid, dim3(256), 0, s, (const uint8_t *)w, K, N, a16, dy, bs16, M, y, ly, r, lr, nullptr, part, Mp); break;
        KCPP_IQ_CASES(KCPP_IQ_GEMM)
#undef KCPP_IQ_GEMM
        default: return -3;
        }
        KCPP_CHECK(hipGetLastError());
        if (KS1 > 1) {
            splitk_finish(part, KS1, M, Mp, N, y, ly, r, lr, s);
            KCPP_CHECK(hipGetLastError());
        }
        return 0;
    };
    int rc = launch(W, Y, ldy, mode == 1 ? nullptr : res, ldr);
    if (rc || mode != 1) return rc;
    rc = launch(W2, up, N, nullptr, 0);
    if (rc) return rc;
    hipLaunchKernelGGL(k_silu_mul_strided, dim3((unsigned)((N * M + 255) / 256)), dim3(256), 0, s, Y, ldy, up, N, M);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
