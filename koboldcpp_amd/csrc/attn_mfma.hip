// attn_mfma.hip -- prefill flash attention on the CDNA4 matrix cores (v_mfma_f32_16x16x32_f16).
//
// Same operator as k_fa_prefill (GGML_OP_FLASH_ATTN_EXT, ggml.c:15667; causal mask, f16 K/V cache,
// Q rounded to f16): softmax(Q K^T * scale) V with an online softmax over 64-key tiles.
//
// Work split: one workgroup = one KV head x 16 queries; its 4 waves are the 4 query heads of the
// GQA group (Llama-3: 32 q heads / 8 kv heads), so every K/V tile staged in LDS serves 4 heads.
// Per wave and 64-key tile:
//   S^T = K . Q^T     (keys x queries)  16 MFMAs: A = K rows from LDS, B = this wave's Q (registers)
//                      -> C layout: lane holds query (lane & 15) and keys 4(lane>>4)+r of each
//                         16-key block, so the softmax statistics of a query are lane-local over 16
//                         values plus two cross-lane steps (xor 16, xor 32);
//   O^T += V^T . P^T  (dims x queries)  16 MFMAs: B = the lane's own P values (f16) taken as the
//                         k-slice {4g..4g+3, 16+4g..16+4g+3} (g = lane>>4) of each 32-key step, A =
//                         V^T rows read from a transposed LDS copy in the same key order.
// P is rounded to f16 for the second product; the CPU reference accumulates V*P in f16 itself
// (ggml_vec_mad_f16), so this stays inside the path's f16 tolerance.
#include "kcpp_common.h"
#include "kcpp_internal.h"

#include <algorithm>
#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define FM_Q 16          // queries per workgroup
#define FM_K 64          // keys per tile
#define FM_SPLIT_T 64    // key-split prefill (k_fa_prefill_mfma3<8, true>): ubatches up to this many tokens,
#define FM_SPLITS 32     // at most this many key splits
#define FM_PQ 132        // split partial of one (query, head): 128 dims, m, l, pad
#define FM_PS (16 * FM_PQ)
#define FM_KP 136        // K tile row pitch (halves): 128 + 8 -> rows 272 B apart (bank spread)
#define FM_VP 72         // V^T tile row pitch (halves): 64 + 8

__global__ void __launch_bounds__(256) k_fa_prefill_mfma(const uint16_t *__restrict__ q16,
                                                         const uint16_t *__restrict__ kc,
                                                         const uint16_t *__restrict__ vc, float *__restrict__ out,
                                                         int T, int H, int HKV, int n_past, float scale) {
    constexpr int D = 128, G = 4;
    __shared__ __attribute__((aligned(16))) uint16_t sk[FM_K * FM_KP];
    __shared__ __attribute__((aligned(16))) uint16_t sv[D * FM_VP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * FM_Q, hk = blockIdx.y, h = hk * G + wave;
    const int EKV = HKV * D;
    const int ql = lane & 15, g = lane >> 4;
    const int qi = q0 + ql;                                   // this lane's query (column)
    const int qpos = n_past + qi;
    // Q fragments (B operand of S^T): Q[qi][32s + 8g + j], 4 dim-steps
    h8 qf[4];
    {
        const int qc = min(qi, T - 1);
        const uint16_t *qp = q16 + ((int64_t)qc * H + h) * D + 8 * g;
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = *(const h8 *)(qp + 32 * s);
    }
    f4 o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;
    const int n_keys = n_past + min(q0 + FM_Q, T);            // keys any query of this block can see
    const int ntile = (n_keys + FM_K - 1) / FM_K;
    for (int kt = 0; kt < ntile; ++kt) {
        const int p0 = kt * FM_K;
        __syncthreads();                                      // previous tile fully consumed
        // stage K tile [64][128] and V^T tile [128][64] (zero rows past the visible keys)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + 256 * i;                    // 1024 16-B pieces per tile
            const int kr = idx >> 4, c8 = idx & 15;
            const int p = p0 + kr;
            uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
            if (p < n_keys) {
                kv = *(const uint4 *)(kc + (int64_t)p * EKV + hk * D + 8 * c8);
                vv = *(const uint4 *)(vc + (int64_t)p * EKV + hk * D + 8 * c8);
            }
            *(uint4 *)(sk + kr * FM_KP + 8 * c8) = kv;
            const uint32_t w4[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                sv[(8 * c8 + 2 * e) * FM_VP + kr] = (uint16_t)(w4[e] & 0xFFFF);
                sv[(8 * c8 + 2 * e + 1) * FM_VP + kr] = (uint16_t)(w4[e] >> 16);
            }
        }
        __syncthreads();
        // S^T for 4 blocks of 16 keys
        f4 sc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            sc[b] = f4{0.f, 0.f, 0.f, 0.f};
            const uint16_t *kp = sk + (16 * b + ql) * FM_KP + 8 * g;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const h8 ka = *(const h8 *)(kp + 32 * s);
                sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ka, qf[s], sc[b], 0, 0, 0);
            }
        }
        // scale + causal mask, tile max of this lane's query
        float mt = -INFINITY;
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = p0 + 16 * b + 4 * g + r;
                const float v = (p <= qpos && p < n_keys) ? sc[b][r] * scale : -INFINITY;
                sc[b][r] = v;
                mt = fmaxf(mt, v);
            }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float m_new = fmaxf(m_run, mt);
        const float alpha = m_run == -INFINITY ? 0.0f : expf(m_run - m_new);
        float ls = 0.0f;
        h8 pb[2];                                             // P^T k-slices for the two 32-key steps
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = sc[b][r] == -INFINITY ? 0.0f : expf(sc[b][r] - m_new);
                ls += e;
                pb[b >> 1][4 * (b & 1) + r] = (_Float16)e;
            }
        ls += __shfl_xor(ls, 16, 64);
        ls += __shfl_xor(ls, 32, 64);
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] *= alpha;
        // O^T += V^T . P^T: dim blocks of 16, key steps of 32 in the lane's k order
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int db = 0; db < 8; ++db) {
                const uint16_t *vp = sv + (16 * db + ql) * FM_VP + 32 * st + 4 * g;
                const uint2 lo = *(const uint2 *)vp;          // keys 32st+4g .. +3
                const uint2 hi = *(const uint2 *)(vp + 16);   // keys 32st+16+4g .. +3
                h8 va;
                const uint32_t w[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    va[2 * e] = __builtin_bit_cast(_Float16, (uint16_t)(w[e] & 0xFFFF));
                    va[2 * e + 1] = __builtin_bit_cast(_Float16, (uint16_t)(w[e] >> 16));
                }
                o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[st], o[db], 0, 0, 0);
            }
        }
    }
    if (qi >= T) return;
    const float inv = 1.0f / l_run;
    float *op = out + ((int64_t)qi * H + h) * D;
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) op[16 * db + 4 * g + r] = o[db][r] * inv;
}

// v2: the same math, key order and summation order as k_fa_prefill_mfma (bit-identical output), restaged:
//   * the next 64-key tile's K/V global loads are issued before the current tile is multiplied (register
//     double buffer), so one tile's HBM/L2 latency hides under the previous tile's MFMAs and softmax;
//   * V is staged row-major with ds_write_b128 like K and read as the transposed A operand of
//     O^T += V^T . P^T by ds_read_b64_tr_b16 (gfx950 hardware transpose: a 16-lane group reads 4 key rows x
//     16 dims and lane i receives dim i of the 4 keys) instead of 8 two-byte LDS stores per 16 B of V.
typedef __fp16 fa_h4 __attribute__((__vector_size__(8)));
__device__ __forceinline__ uint2 ds_tr16(const uint16_t *p) {
    const fa_h4 v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fa_h4 *)(p));
    return __builtin_bit_cast(uint2, v);
}

__global__ void __launch_bounds__(256) k_fa_prefill_mfma2(const uint16_t *__restrict__ q16,
                                                          const uint16_t *__restrict__ kc,
                                                          const uint16_t *__restrict__ vc, float *__restrict__ out,
                                                          int T, int H, int HKV, int n_past, float scale) {
    constexpr int D = 128, G = 4;
    __shared__ __attribute__((aligned(16))) uint16_t sk[FM_K * FM_KP];
    __shared__ __attribute__((aligned(16))) uint16_t sv[FM_K * FM_KP];     // row-major [key][dim]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * FM_Q, hk = blockIdx.y, h = hk * G + wave;
    const int EKV = HKV * D;
    const int ql = lane & 15, g = lane >> 4;
    const int qi = q0 + ql;
    const int qpos = n_past + qi;
    h8 qf[4];
    {
        const int qc = min(qi, T - 1);
        const uint16_t *qp = q16 + ((int64_t)qc * H + h) * D + 8 * g;
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = *(const h8 *)(qp + 32 * s);
    }
    f4 o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;
    const int n_keys = n_past + min(q0 + FM_Q, T);
    const int ntile = (n_keys + FM_K - 1) / FM_K;
    uint4 kn[4], vn[4];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + 256 * i;
            const int p = kt * FM_K + (idx >> 4), c8 = idx & 15;
            kn[i] = make_uint4(0, 0, 0, 0);
            vn[i] = make_uint4(0, 0, 0, 0);
            if (p < n_keys) {
                kn[i] = *(const uint4 *)(kc + (int64_t)p * EKV + hk * D + 8 * c8);
                vn[i] = *(const uint4 *)(vc + (int64_t)p * EKV + hk * D + 8 * c8);
            }
        }
    };
    load(0);
    // transposed-read addresses: lane 4q+p of its 16-lane group -> key row q, dims 4p..4p+3 of a 16-dim block
    const int trq = ql >> 2, trp = ql & 3;
    for (int kt = 0; kt < ntile; ++kt) {
        const int p0 = kt * FM_K;
        __syncthreads();                                      // previous tile fully consumed
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + 256 * i;
            const int kr = idx >> 4, c8 = idx & 15;
            *(uint4 *)(sk + kr * FM_KP + 8 * c8) = kn[i];
            *(uint4 *)(sv + kr * FM_KP + 8 * c8) = vn[i];
        }
        if (kt + 1 < ntile) load(kt + 1);
        __syncthreads();
        f4 sc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            sc[b] = f4{0.f, 0.f, 0.f, 0.f};
            const uint16_t *kp = sk + (16 * b + ql) * FM_KP + 8 * g;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const h8 ka = *(const h8 *)(kp + 32 * s);
                sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ka, qf[s], sc[b], 0, 0, 0);
            }
        }
        float mt = -INFINITY;
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = p0 + 16 * b + 4 * g + r;
                const float v = (p <= qpos && p < n_keys) ? sc[b][r] * scale : -INFINITY;
                sc[b][r] = v;
                mt = fmaxf(mt, v);
            }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float m_new = fmaxf(m_run, mt);
        const float alpha = m_run == -INFINITY ? 0.0f : expf(m_run - m_new);
        float ls = 0.0f;
        h8 pb[2];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = sc[b][r] == -INFINITY ? 0.0f : expf(sc[b][r] - m_new);
                ls += e;
                pb[b >> 1][4 * (b & 1) + r] = (_Float16)e;
            }
        ls += __shfl_xor(ls, 16, 64);
        ls += __shfl_xor(ls, 32, 64);
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] *= alpha;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int db = 0; db < 8; ++db) {
                // keys 32st+4g .. +3 and 32st+16+4g .. +3 of dim 16db + ql (k_fa_prefill_mfma's order)
                const uint2 lo = ds_tr16(sv + (32 * st + 4 * g + trq) * FM_KP + 16 * db + 4 * trp);
                const uint2 hi = ds_tr16(sv + (32 * st + 16 + 4 * g + trq) * FM_KP + 16 * db + 4 * trp);
                h8 va;
                const uint32_t w[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    va[2 * e] = __builtin_bit_cast(_Float16, (uint16_t)(w[e] & 0xFFFF));
                    va[2 * e + 1] = __builtin_bit_cast(_Float16, (uint16_t)(w[e] >> 16));
                }
                o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[st], o[db], 0, 0, 0);
            }
        }
    }
    if (qi >= T) return;
    const float inv = 1.0f / l_run;
    float *op = out + ((int64_t)qi * H + h) * D;
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) op[16 * db + 4 * g + r] = o[db][r] * inv;
}


// v3: v2's work split and MFMA shapes with the tile movement and the softmax rebuilt (v2 spends ~5k cycles per 64-key
// tile against 512 MFMA cycles):
//   * K/V tiles arrive by LDS-DMA (inline asm, so the compiler drains nothing behind our back) into a 4-stage ring
//     three tiles ahead -- no register staging, no ds_write; one DMA instruction = 4 key rows x 256 B (8 lines);
//   * S = K Q^T of tile kt + 1 is issued before tile kt's softmax, so the matrix cores work under the exp2s;
//   * XCD-aware block order: one kv head per XCD, so a head's K/V is read from that XCD's L2 by all its query
//     blocks (v2's order had every XCD stream every head's K/V from the Infinity Cache: ~5 TB/s of re-reads);
//     rows past the visible keys are clamped to the last visible key (finite data; their P is 0);
//   * LDS image [key][16 chunks of 16 B] with chunk c stored at c ^ 2 (key & 7): the K fragment reads and the
//     transposed V reads (ds_read_b64_tr_b16) are both conflict-free;
//   * softmax in the exp2 domain (logits pre-scaled by scale * log2 e, one v_exp_f32 per element instead of expf),
//     the causal / length mask only on tiles that cross the diagonal or the end.
// Same key order and f16 rounding of P as v2; results differ from v2 only by exp2 vs expf rounding (<= 1 ulp of P).
__device__ __forceinline__ uint32_t fa_lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void fa_dma16(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(fa_lds_addr(lds_base))) : "memory", "m0");
}
__device__ __forceinline__ int fa_swz(int row, int c) { return row * 16 + (c ^ ((row & 7) << 1)); }

// NW = 8: two waves per query head, wave w (head w & 3) takes key half hf = w >> 2 of every 64-key tile (2 waves per
// SIMD so one's softmax runs under the other's MFMAs); the halves share each tile's maximum through LDS, so P and the
// running max are v3's, and their (l, O) partial sums are added at the end (only the f32 summation order differs).
//
// SPL (short ubatches, BASELINE config 3's 32 tokens: (T / 16) x HKV workgroups alone leave most CUs idle): the grid
// also splits the keys, ch tiles per workgroup; each split stores its unnormalised (O, m, l) per query and head and
// k_fa_split_merge (next launch) merges the splits in split order.  (An in-launch merge by the last-arriving split
// -- write-through partials, a ticket, device-coherent loads -- measured 15-30 us per layer at 2-16 splits against
// this pair's: every coherent round trip went through HBM.)
// qta (optional, unsplit): the output quantized straight to the KT_Q8_0_TA activation of attn_output (KT_Q8_0_T
// weights): a head's 128 dims are 4 whole Q8_0 blocks, so no other workgroup's output is needed (k_quant_q80's
// rounding); split launches quantize in the merge.
// HM (NW = 8 only; variant 5, A/B): each key half keeps its own running maximum -- no per-tile maximum exchange (one
// barrier per tile instead of two); P is relative to the half's maximum (the same f16 rounding bound), the halves merged
// at the end as before.  tools/fa_ab.py at 512 queries: 16.3 -> 14.7 us (n_past 0), 45.6 -> 41.6 (1536), 79.4 -> 73.3
// (3328), within the kernel test's error bars -- but as the default it took the tiny Q4_1 model's logits just past
// 1.5x the reference's own spread (tests/test_kquants_low.py: 0.0291 vs 0.0283), so variant 4 stays the default
template <int NW, bool SPL, bool HM = false>
__global__ void __launch_bounds__(64 * NW, 1) k_fa_prefill_mfma3(const uint16_t *__restrict__ q16,
                                                                const uint16_t *__restrict__ kc,
                                                                const uint16_t *__restrict__ vc, float *__restrict__ out,
                                                                int T, int H, int HKV, int n_past, float scale,
                                                                float *__restrict__ part, unsigned *__restrict__ tick,
                                                                int ch, int nsp_grid, uint8_t *__restrict__ qta) {
    constexpr int D = 128, G = 4, NST = 4;
    constexpr int NB = NW == 8 ? 2 : 4;               // 16-key blocks per wave and tile
    __shared__ __attribute__((aligned(16))) uint4 sk[NST][FM_K * 16];
    __shared__ __attribute__((aligned(16))) uint4 sv[NST][FM_K * 16];
    __shared__ float s_mx[2][4][16];                  // NW = 8: per key half, head and query: the tile maximum
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hf = NW == 8 ? wave >> 2 : 0;
    // 1-D grid, XCD-aware: blocks b and b + 8 share an XCD, so kv head = b % 8 (+ 8 (b / 8 % (HKV / 8))) keeps every
    // query block of one head on one XCD -- its K/V (n_keys x 512 B) stays in that XCD's L2 instead of every XCD
    // streaming all heads from the Infinity Cache
    int bid = blockIdx.x, sp = 0;
    if constexpr (SPL) {
        const int nb0 = (T + FM_Q - 1) / FM_Q * HKV;
        sp = bid / nb0;
        bid -= sp * nb0;                              // nb0 % 8 == 0 when HKV % 8 == 0: a head keeps its XCD
    }
    int hk, qb;
    if (HKV % 8 == 0) {
        const int j = bid >> 3;
        hk = (bid & 7) + 8 * (j % (HKV / 8));
        qb = j / (HKV / 8);
    } else {
        hk = bid % HKV;
        qb = bid / HKV;
    }
    const int q0 = qb * FM_Q, h = hk * G + (wave & 3);
    const int EKV = HKV * D;
    const int ql = lane & 15, g = lane >> 4;
    const int qi = q0 + ql;
    const int qpos = n_past + qi;
    const float sl2 = scale * 1.4426950408889634f;
    h8 qf[4];
    {
        const int qc = min(qi, T - 1);
        const uint16_t *qp = q16 + ((int64_t)qc * H + h) * D + 8 * g;
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = *(const h8 *)(qp + 32 * s);
    }
    f4 o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.0f;
    const int n_keys = n_past + min(q0 + FM_Q, T);
    const int ntile = (n_keys + FM_K - 1) / FM_K;
    int kt0 = 0, kt1 = ntile;                             // this workgroup's key tiles
    if constexpr (SPL) {
        kt0 = sp * ch;
        kt1 = min(kt0 + ch, ntile);
        if (kt0 >= ntile) return;                         // past this query block's keys (whole workgroup)
    }
    const int qmin = n_past + q0;                         // smallest query position of the block
    // DMA: wave w fetches key rows (64 / NW) w .. +64/NW of the tile (instructions of 4 rows) for K and for V;
    // lane: row 4 i + (lane >> 4) of the instruction, chunk slot lane & 15 <- global chunk (slot ^ 2 (row & 7))
    constexpr int RPW = FM_K / NW, IPW = RPW / 4;
    const int drow = lane >> 4, dslot = lane & 15;
    auto stage = [&](int kt) {
        const int st = kt & (NST - 1);
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int r = RPW * wave + 4 * i + drow;                // row in the tile
            const int p = min(kt * FM_K + r, n_keys - 1);
            const int c = dslot ^ ((r & 7) << 1);
            const int64_t off = (int64_t)p * EKV + hk * D + 8 * c;
            fa_dma16(kc + off, &sk[st][(RPW * wave + 4 * i) * 16]);
            fa_dma16(vc + off, &sv[st][(RPW * wave + 4 * i) * 16]);
        }
    };
    // lane-constant LDS byte offsets (swizzle folded in; the per-tile stage base and the row blocks are immediates):
    // K fragment of step s: row 16 b + ql, chunk 4 s + g -> 4096 b + kofs[s];  V^T read of dim block db: rows
    // 32 s2 + 4 g + trq (+ 16), chunk 2 db + (trp >> 1), half trp & 1 -> 8192 s2 (+ 4096) + vofs[db]
    const int trq = ql >> 2, trp = ql & 3;
    int kofs[4], vofs[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) kofs[s] = 16 * (16 * ql + ((4 * s + g) ^ ((ql & 7) << 1)));
    {
        const int r0 = 4 * g + trq;
#pragma unroll
        for (int db = 0; db < 8; ++db) vofs[db] = 16 * (16 * r0 + ((2 * db + (trp >> 1)) ^ ((r0 & 7) << 1))) + 8 * (trp & 1);
    }
    const int b0 = NB * hf;                                   // this wave's first 16-key block
    // S^T = K Q^T of the wave's key blocks of tile kt (keys x queries), MFMAs only: issued a tile ahead so they run
    // under the softmax; all fragments of two steps read before their MFMAs, step-major (independent chains)
    auto qk = [&](int kt, f4 (&sc)[NB]) {
        const char *skb = (const char *)&sk[kt & (NST - 1)][0] + 4096 * b0;
#pragma unroll
        for (int b = 0; b < NB; ++b) sc[b] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
            h8 ka[2 * NB];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int b = 0; b < NB; ++b) ka[NB * s + b] = *(const h8 *)(skb + 4096 * b + kofs[2 * sp + s]);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    sc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ka[NB * s + b], qf[2 * sp + s], sc[b], 0, 0, 0);
        }
    };
    auto vread = [&](const char *svb, int s2, h8 (&va)[8]) {
#pragma unroll
        for (int db = 0; db < 8; ++db) {
            const uint2 lo = ds_tr16((const uint16_t *)(svb + 8192 * s2 + vofs[db]));
            const uint2 hi = ds_tr16((const uint16_t *)(svb + 8192 * s2 + 4096 + vofs[db]));
            va[db] = __builtin_bit_cast(h8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
    };
    // ring of NST stages, NST - 1 tiles ahead: tile kt + 1's K is read at the top of iteration kt
    for (int t = kt0; t < kt0 + NST - 1 && t < kt1; ++t) stage(t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    f4 sc[NB], sn[NB];
    qk(kt0, sc);
    for (int kt = kt0; kt < kt1; ++kt) {
        const int p0 = kt * FM_K + 16 * b0;
        const bool pre = kt + NST - 1 < kt1;
        if (pre) stage(kt + NST - 1);
        if (kt + 1 < kt1) qk(kt + 1, sn);
        const char *svb = (const char *)&sv[kt & (NST - 1)][0];
        h8 va[8];
        vread(svb, NW == 8 ? hf : 0, va);             // V^T of the first 32 keys: independent of P, read under softmax
        float mt = -INFINITY;
        if (p0 + 16 * NB - 1 > qmin || p0 + 16 * NB > n_keys) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int p = p0 + 16 * b + 4 * g + r;
                    const float v = (p <= qpos && p < n_keys) ? sc[b][r] * sl2 : -INFINITY;
                    sc[b][r] = v;
                    mt = fmaxf(mt, v);
                }
        } else {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sc[b][r] *= sl2;
                    mt = fmaxf(mt, sc[b][r]);
                }
        }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        if constexpr (NW == 8 && !HM) {
            // both key halves take the whole tile's maximum (exchanged through LDS), so P, alpha and the running max
            // are v3's exactly; only the f32 summation of O and l is split in two
            if (g == 0) s_mx[hf][wave & 3][ql] = mt;
            __syncthreads();
            mt = fmaxf(mt, s_mx[hf ^ 1][wave & 3][ql]);
        }
        const float m_new = fmaxf(m_run, mt);
        // m_new = -inf only when every key so far is masked (a half-tile wholly past the diagonal): keep alpha 1
        const float alpha = m_new == -INFINITY ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
        float ls = 0.0f;
        h8 pb[NB / 2];
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = m_new == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(sc[b][r] - m_new);
                ls += e;
                pb[b >> 1][4 * (b & 1) + r] = (_Float16)e;
            }
        ls += __shfl_xor(ls, 16, 64);
        ls += __shfl_xor(ls, 32, 64);
        l_run = l_run * alpha + ls;
        // the running maximum rarely moves after the first tiles: rescale only when some lane's did (alpha = 1
        // leaves o unchanged bit for bit)
        if (__builtin_amdgcn_ballot_w64(m_new != m_run)) {
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] *= alpha;
        }
        m_run = m_new;
#pragma unroll
        for (int db = 0; db < 8; ++db) o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[db], pb[0], o[db], 0, 0, 0);
        if constexpr (NB == 4) {
            vread(svb, 1, va);
#pragma unroll
            for (int db = 0; db < 8; ++db) o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[db], pb[1], o[db], 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) sc[b] = sn[b];
        // tile kt + 2 must have landed before the next iteration reads its K (kt + 3's DMA instructions, issued
        // last, may stay in flight)
        if (pre) {
            if constexpr (IPW == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    if constexpr (NW == 8) {
        // merge the two key halves: wave hf = 1 publishes (m, l, O) in the (now idle) K ring, wave hf = 0 combines
        float *xo = (float *)&sk[0][0] + (wave & 3) * (16 * 130);     // [16 queries][128 dims + m + l]
        if (hf == 1) {
#pragma unroll
            for (int db = 0; db < 8; ++db)
#pragma unroll
                for (int r = 0; r < 4; ++r) xo[ql * 130 + 16 * db + 4 * g + r] = o[db][r];
            if (g == 0) {
                xo[ql * 130 + 128] = m_run;
                xo[ql * 130 + 129] = l_run;
            }
        }
        __syncthreads();
        if (!SPL && hf == 1) return;
        if (hf == 0) {
            const float m1 = xo[ql * 130 + 128], l1 = xo[ql * 130 + 129];
            const float m = fmaxf(m_run, m1);
            const float a0 = m_run == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m_run - m);
            const float a1 = m1 == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(m1 - m);
            l_run = l_run * a0 + l1 * a1;
#pragma unroll
            for (int db = 0; db < 8; ++db)
#pragma unroll
                for (int r = 0; r < 4; ++r) o[db][r] = o[db][r] * a0 + xo[ql * 130 + 16 * db + 4 * g + r] * a1;
            m_run = m;
        }
    }
    if constexpr (SPL) {
        // publish this split's unnormalised (O, m, l) per query and head; k_fa_split_merge (the next launch) merges
        if (hf == 0) {
            float *pp = part + (((int64_t)(qb * HKV + hk) * nsp_grid + sp) * 4 + (wave & 3)) * FM_PS + ql * FM_PQ;
#pragma unroll
            for (int db = 0; db < 8; ++db) *(float4 *)(pp + 16 * db + 4 * g) = make_float4(o[db][0], o[db][1], o[db][2], o[db][3]);
            if (g == 0) *(float4 *)(pp + 128) = make_float4(m_run, l_run, 0.0f, 0.0f);
        }
        return;
    }
    if (qi >= T) return;                                  // (all four lanes of a query leave together)
    const float inv = 1.0f / l_run;
    if (out) {
        float *op = out + ((int64_t)qi * H + h) * D;
#pragma unroll
        for (int db = 0; db < 8; ++db)
#pragma unroll
            for (int r = 0; r < 4; ++r) op[16 * db + 4 * g + r] = o[db][r] * inv;
    }
    if (qta) {
        // Q8_0 block k of this head = dims 32 k .. + 32 = o[2k], o[2k + 1] of the query's 4 lanes (g): element
        // 16 (db - 2k) + 4 g + r -> half db - 2k, byte 4 g + r of the token's 16-byte row (kcpp_common.h KT_Q8_0_TA)
        const int64_t E = (int64_t)H * D, nb = E / 32, ng = (T + 31) / 32, grp = qi >> 5, tok = qi & 31;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) { v[r] = o[2 * k][r] * inv; v[4 + r] = o[2 * k + 1][r] * inv; }
            float am = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
            am = fmaxf(am, __shfl_xor(am, 16, 64));
            am = fmaxf(am, __shfl_xor(am, 32, 64));
            const float id = (am != 0.0f) ? 127.f / am : 0.0f;
            uint32_t pk[2] = {0u, 0u};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                int iv = (int)rintf(__fmul_rn(v[e], id));
                iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
                pk[e >> 2] |= (uint32_t)(iv & 0xFF) << (8 * (e & 3));
            }
            const int64_t ib = (int64_t)h * 4 + k;
            uint8_t *qb8 = qta + (grp * nb + ib) * 1024 + tok * 16 + 4 * g;
            *(uint32_t *)qb8 = pk[0];
            *(uint32_t *)(qb8 + 512) = pk[1];
            if (g == 0) ((float *)(qta + ng * 32 * E))[(grp * nb + ib) * 32 + tok] = h2f(f2h(am / 127.f));
        }
    }
}

static int g_fa_prefill_variant = 0;
extern "C" int kcpp_fa_prefill_set_variant(int v) {
    const int old = g_fa_prefill_variant;
    g_fa_prefill_variant = v;
    return old;
}

// merge of the key splits (SPL): one workgroup per (query block, kv head, head of the group), thread = (query,
// 8-dim chunk); the splits' (m, l) and O chunks loaded together, weights exp2(m_s - max), summed in split order;
// out f32 and / or the KT_Q8_0_TA activation (a Q8_0 block = 4 threads' 32 dims, k_quant_q80's rounding)
__global__ void __launch_bounds__(256) k_fa_split_merge(const float *__restrict__ part, float *__restrict__ out,
                                                        uint8_t *__restrict__ qta, int T, int H, int HKV, int n_past,
                                                        int ch, int nsp_grid) {
    constexpr int D = 128, G = 4;
    const int slot = blockIdx.x >> 2, mh = blockIdx.x & 3, qb = slot / HKV, hk = slot % HKV;
    const int tid = threadIdx.x, mq = tid >> 4, dc = tid & 15;
    const int q0 = qb * FM_Q;
    const int n_keys = n_past + min(q0 + FM_Q, T);
    const int nsp = ((n_keys + FM_K - 1) / FM_K + ch - 1) / ch;
    const float *pm = part + ((int64_t)slot * nsp_grid * 4 + mh) * FM_PS + mq * FM_PQ;
    auto at = [&](int k) { return pm + (int64_t)min(k, nsp - 1) * 4 * FM_PS; };   // branch-free: clamped + weight 0
    float mk[FM_SPLITS], lk[FM_SPLITS];
#pragma unroll
    for (int k = 0; k < FM_SPLITS; ++k) {
        const float2 ml = *(const float2 *)(at(k) + 128);
        mk[k] = k < nsp ? ml.x : -INFINITY;
        lk[k] = k < nsp ? ml.y : 0.0f;
    }
    float4 v[8][2];
    auto chunk = [&](int k0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int c = 0; c < 2; ++c) v[j][c] = *(const float4 *)(at(k0 + j) + 8 * dc + 4 * c);
    };
    chunk(0);
    float mm = -INFINITY;
#pragma unroll
    for (int k = 0; k < FM_SPLITS; ++k) mm = fmaxf(mm, mk[k]);
    float lsum = 0.0f;
#pragma unroll
    for (int k = 0; k < FM_SPLITS; ++k) {
        mk[k] = mk[k] == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mk[k] - mm);
        lsum = lsum + lk[k] * mk[k];
    }
    float ov[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = 0.0f;
#pragma unroll
    for (int k0 = 0; k0 < FM_SPLITS; k0 += 8) {
        if (k0 >= nsp) break;
        if (k0 > 0) chunk(k0);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const float w = mk[k0 + j];
                ov[4 * c] = ov[4 * c] + v[j][c].x * w;
                ov[4 * c + 1] = ov[4 * c + 1] + v[j][c].y * w;
                ov[4 * c + 2] = ov[4 * c + 2] + v[j][c].z * w;
                ov[4 * c + 3] = ov[4 * c + 3] + v[j][c].w * w;
            }
    }
    const int qi = q0 + mq, h = hk * G + mh;
    if (qi >= T) return;                                  // (a query's 16 threads leave together)
    const float inv = 1.0f / lsum;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = ov[e] * inv;
    if (out) {
        float4 *op = (float4 *)(out + ((int64_t)qi * H + h) * D + 8 * dc);
        op[0] = make_float4(ov[0], ov[1], ov[2], ov[3]);
        op[1] = make_float4(ov[4], ov[5], ov[6], ov[7]);
    }
    if (qta) {
        const int64_t E = (int64_t)H * D, nb = E / 32, ng = (T + 31) / 32, grp = qi >> 5, tok = qi & 31;
        float am = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(ov[e]));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        am = fmaxf(am, __shfl_xor(am, 2, 64));
        const float id = (am != 0.0f) ? 127.f / am : 0.0f;
        uint32_t pk[2] = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            int iv = (int)rintf(__fmul_rn(ov[e], id));
            iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
            pk[e >> 2] |= (uint32_t)(iv & 0xFF) << (8 * (e & 3));
        }
        // dims 8 dc .. + 7 of the head = block 2 h*2.. : element 8 (dc & 3) + e of block dc >> 2 -> half (dc & 3) >> 1,
        // bytes 8 (dc & 1) + e
        const int64_t ib = (int64_t)h * 4 + (dc >> 2);
        *(uint2 *)(qta + (grp * nb + ib) * 1024 + ((dc & 3) >> 1) * 512 + tok * 16 + 8 * (dc & 1)) = make_uint2(pk[0], pk[1]);
        if ((dc & 3) == 0) ((float *)(qta + ng * 32 * E))[(grp * nb + ib) * 32 + tok] = h2f(f2h(am / 127.f));
    }
}

// the key-split variant's workspace (kcpp_fa_workspace_bytes reserves it, after the 2 KB header):
// [query block][kv head][split < FM_SPLITS][4 heads][16 queries][FM_PQ] partials for T <= FM_SPLIT_T
extern "C" int64_t kcpp_fa_split_ws_bytes(int H) {
    return KCPP_FA_WS_HEADER + (int64_t)(FM_SPLIT_T / FM_Q) * (H / 4) * FM_SPLITS * 4 * FM_PS * 4;
}

extern "C" int kcpp_flash_attn_prefill_mfma_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out,
                                               void *qta, void *ws, int T, int H, int HKV, int D, int n_past, float scale,
                                               void *stream) {
    if (D != 128 || HKV <= 0 || H != 4 * HKV || (!out && !qta)) return -3;
    const int v = g_fa_prefill_variant ? g_fa_prefill_variant : 4;
    const int nqb = (T + FM_Q - 1) / FM_Q;
    const int nb0 = nqb * HKV;
    if ((v == 4 || v == 5) && ws && T <= FM_SPLIT_T && nb0 <= 512) {
        // keys split so that the grid has ~512 workgroups (at most FM_SPLITS splits of whole 64-key tiles)
        const int ntile = (n_past + T + FM_K - 1) / FM_K;
        const int want = std::min(FM_SPLITS, std::max(1, 512 / nb0));
        const int ch = (ntile + want - 1) / want;
        const int nsp = (ntile + ch - 1) / ch;
        if (nsp > 1) {
            float *part = (float *)((uint8_t *)ws + KCPP_FA_WS_HEADER);
            if (v == 5)
                hipLaunchKernelGGL((k_fa_prefill_mfma3<8, true, true>), dim3(nb0 * nsp), dim3(512), 0, (hipStream_t)stream,
                                   q16, kc, vc, out, T, H, HKV, n_past, scale, part, (unsigned *)nullptr, ch, nsp,
                                   (uint8_t *)nullptr);
            else
                hipLaunchKernelGGL((k_fa_prefill_mfma3<8, true>), dim3(nb0 * nsp), dim3(512), 0, (hipStream_t)stream, q16, kc,
                                   vc, out, T, H, HKV, n_past, scale, part, (unsigned *)nullptr, ch, nsp, (uint8_t *)nullptr);
            KCPP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_fa_split_merge, dim3(nb0 * 4), dim3(256), 0, (hipStream_t)stream, part, out, (uint8_t *)qta,
                               T, H, HKV, n_past, ch, nsp);
            KCPP_CHECK(hipGetLastError());
            return 0;
        }
    }
    if (v == 4 || v == 5) {
        if (v == 5)
            hipLaunchKernelGGL((k_fa_prefill_mfma3<8, false, true>), dim3(nb0), dim3(512), 0, (hipStream_t)stream, q16, kc, vc,
                               out, T, H, HKV, n_past, scale, (float *)nullptr, (unsigned *)nullptr, 0, 1, (uint8_t *)qta);
        else
            hipLaunchKernelGGL((k_fa_prefill_mfma3<8, false>), dim3(nb0), dim3(512), 0, (hipStream_t)stream, q16, kc, vc, out,
                               T, H, HKV, n_past, scale, (float *)nullptr, (unsigned *)nullptr, 0, 1, (uint8_t *)qta);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (!out) return -3;
    return kcpp_flash_attn_prefill_mfma(q16, kc, vc, out, T, H, HKV, D, n_past, scale, stream);
}

extern "C" int kcpp_flash_attn_prefill_mfma(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out,
                                            int T, int H, int HKV, int D, int n_past, float scale, void *stream) {
    if (D != 128 || HKV <= 0 || H != 4 * HKV) return -3;
    const int v = g_fa_prefill_variant ? g_fa_prefill_variant : 4;
    if (v == 3)
        hipLaunchKernelGGL((k_fa_prefill_mfma3<4, false>), dim3((T + FM_Q - 1) / FM_Q * HKV), dim3(256), 0,
                           (hipStream_t)stream, q16, kc, vc, out, T, H, HKV, n_past, scale, (float *)nullptr,
                           (unsigned *)nullptr, 0, 1, (uint8_t *)nullptr);
    else if (v == 4)
        hipLaunchKernelGGL((k_fa_prefill_mfma3<8, false>), dim3((T + FM_Q - 1) / FM_Q * HKV), dim3(512), 0,
                           (hipStream_t)stream, q16, kc, vc, out, T, H, HKV, n_past, scale, (float *)nullptr,
                           (unsigned *)nullptr, 0, 1, (uint8_t *)nullptr);
    else if (v == 5)
        hipLaunchKernelGGL((k_fa_prefill_mfma3<8, false, true>), dim3((T + FM_Q - 1) / FM_Q * HKV), dim3(512), 0,
                           (hipStream_t)stream, q16, kc, vc, out, T, H, HKV, n_past, scale, (float *)nullptr,
                           (unsigned *)nullptr, 0, 1, (uint8_t *)nullptr);
    else if (v == 1)
        hipLaunchKernelGGL(k_fa_prefill_mfma, dim3((T + FM_Q - 1) / FM_Q, HKV), dim3(256), 0, (hipStream_t)stream, q16, kc,
                           vc, out, T, H, HKV, n_past, scale);
    else
        hipLaunchKernelGGL(k_fa_prefill_mfma2, dim3((T + FM_Q - 1) / FM_Q, HKV), dim3(256), 0, (hipStream_t)stream, q16, kc,
                           vc, out, T, H, HKV, n_past, scale);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
