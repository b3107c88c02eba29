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

#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define FM_Q 16          // queries per workgroup
#define FM_K 64          // keys per tile
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

static int g_fa_prefill_variant = 0;
extern "C" int kcpp_fa_prefill_set_variant(int v) {
    const int old = g_fa_prefill_variant;
    g_fa_prefill_variant = v;
    return old;
}

extern "C" int kcpp_flash_attn_prefill_mfma(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out,
                                            int T, int H, int HKV, int D, int n_past, float scale, void *stream) {
    if (D != 128 || HKV <= 0 || H != 4 * HKV) return -3;
    const int v = g_fa_prefill_variant ? g_fa_prefill_variant : 2;
    if (v == 1)
        hipLaunchKernelGGL(k_fa_prefill_mfma, dim3((T + FM_Q - 1) / FM_Q, HKV), dim3(256), 0, (hipStream_t)stream, q16, kc,
                           vc, out, T, H, HKV, n_past, scale);
    else
        hipLaunchKernelGGL(k_fa_prefill_mfma2, dim3((T + FM_Q - 1) / FM_Q, HKV), dim3(256), 0, (hipStream_t)stream, q16, kc,
                           vc, out, T, H, HKV, n_past, scale);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
