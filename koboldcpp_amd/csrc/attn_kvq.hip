// attn_kvq.hip -- quantized KV cache (koboldcpp --quantkv 1 / 2: q8_0 / q4_0 K and V; gpttype_adapter.cpp:1958-1959
// -> llama_kv_cache type_k / type_v; FA only, context shift off, koboldcpp.py:4452).
//
// Reference semantics (CPU):
//   store : K (after RoPE) and V rows go into the cache by ggml_cpy f32 -> Q8_0 / Q4_0, i.e. type_traits[t].from_float:
//           quantize_row_q8_0 (AVX2: d = amax/127, q = round-to-nearest-even(x * 127/amax)) and quantize_row_q4_0_ref
//           (d = max/-8 of the signed extreme, q = min(15, (int8_t)(x/d + 8.5f))), ggml-quants.c:940,1523-1560
//   attend: ggml_compute_forward_flash_attn_ext_f16 with a quantized K: Q is quantized to K's vec_dot_type (Q8_0)
//           from f32 and s = ggml_vec_dot_q{8,4}_0_q8_0(k, q) (sum over 32-blocks of d_k d_q * integer dot); a
//           quantized V is dequantized to f32 and accumulated in f32 (ggml_vec_mad_f32), ggml.c:15750-15840.
// Cache layout here (per layer, internal, 16-B friendly): Q8_0 = qs int8 [n_ctx][EKV] ++ d f16 [n_ctx][EKV/32];
// Q4_0 = qs [n_ctx][EKV/2] (ggml nibble order per 32-block: byte j = elem j | elem j+16 << 4) ++ d f16 [n_ctx][EKV/32].
// The integer parts are exact on both sides (|q_k q_q| sums < 2^24 are exact in f32); only the fp32 order of the
// block combination and of the softmax / V sums differs.
#include "kcpp_common.h"
#include "kcpp_internal.h"

namespace {

__device__ __forceinline__ int8_t *kv_qs(void *c) { return (int8_t *)c; }
__device__ __forceinline__ uint16_t *kv_d(void *c, int type, int64_t n_ctx, int64_t ekv) {
    return (uint16_t *)((uint8_t *)c + (type == KT_Q8_0 ? n_ctx * ekv : n_ctx * ekv / 2));
}

// quantize 32 values: Q8_0 -> 8 words of int8, Q4_0 -> 4 words of nibbles (byte j = elem j | elem j+16 << 4), d
template <int TYPE>
__device__ __forceinline__ void quant32(const float *x, uint32_t *w, uint16_t &dh) {
    if constexpr (TYPE == KT_Q8_0) {
        float am = 0.0f;
        for (int e = 0; e < 32; ++e) am = fmaxf(am, fabsf(x[e]));
        const float d = am / 127.f;
        const float id = am != 0.0f ? 127.f / am : 0.0f;
        for (int k = 0; k < 8; ++k) {
            uint32_t v = 0;
            for (int e = 0; e < 4; ++e) {
                int iv = (int)rintf(__fmul_rn(x[4 * k + e], id));
                iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
                v |= (uint32_t)(iv & 0xFF) << (8 * e);
            }
            w[k] = v;
        }
        dh = f2h_rn(d);
    } else {
        float amax = 0.0f, mx = 0.0f;
        for (int e = 0; e < 32; ++e)
            if (amax < fabsf(x[e])) { amax = fabsf(x[e]); mx = x[e]; }
        const float d = mx / -8.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        for (int k = 0; k < 4; ++k) w[k] = 0;
        for (int j = 0; j < 16; ++j) {
            const float x0 = __fmul_rn(x[j], id), x1 = __fmul_rn(x[16 + j], id);
            const int xi0 = min(15, (int)(int8_t)__fadd_rn(x0, 8.5f)), xi1 = min(15, (int)(int8_t)__fadd_rn(x1, 8.5f));
            w[j >> 2] |= (uint32_t)(xi0 | (xi1 << 4)) << (8 * (j & 3));
        }
        dh = f2h_rn(d);
    }
}

// quantize 32 values into block b of row p of the runtime's cache layout (one thread per block)
template <int TYPE>
__device__ __forceinline__ void quant_block(const float *x, void *cache, int64_t n_ctx, int64_t ekv, int64_t p, int64_t b) {
    uint32_t w[8];
    uint16_t dh;
    quant32<TYPE>(x, w, dh);
    uint32_t *q = (uint32_t *)((uint8_t *)cache + (TYPE == KT_Q8_0 ? p * ekv + b * 32 : p * (ekv / 2) + b * 16));
    for (int k = 0; k < (TYPE == KT_Q8_0 ? 8 : 4); ++k) q[k] = w[k];
    kv_d(cache, TYPE, n_ctx, ekv)[p * (ekv / 32) + b] = dh;
}

// GGML_OP_CPY f32 -> Q8_0 / Q4_0 (ggml_cpy into a quantized cache view: the type's from_float, quantize_row_q8_0 /
// quantize_row_q4_0_ref): n_blocks consecutive 32-blocks of a contiguous f32 source into ggml blocks {f16 d, quants}
template <int TYPE>
__global__ void k_cpy_f32_q(const float *__restrict__ src, int64_t n_blocks, uint8_t *__restrict__ dst) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_blocks) return;
    float x[32];
    for (int e = 0; e < 32; ++e) x[e] = src[b * 32 + e];
    uint32_t w[8];
    uint16_t dh;
    quant32<TYPE>(x, w, dh);
    constexpr int BS = TYPE == KT_Q8_0 ? 34 : 18;
    uint8_t *o = dst + b * BS;
    *(uint16_t *)o = dh;
    for (int k = 0; k < (TYPE == KT_Q8_0 ? 8 : 4); ++k)        // 2-B aligned block: 16-bit stores
        for (int h = 0; h < 2; ++h) *(uint16_t *)(o + 2 + 4 * k + 2 * h) = (uint16_t)(w[k] >> (16 * h));
}

// K and V rows of T tokens (f32, from the q|k|v staging rows: k at column koff, v at voff, row stride ld) into the
// quantized caches at positions n_past + t (or pos_dev[0] + t)
template <int TK, int TV>
__global__ void k_kv_store_q(const float *__restrict__ qkv, int64_t ld, int64_t koff, int64_t voff, int T, int64_t ekv,
                             void *kc, void *vc, int64_t n_ctx, int n_past_arg, const int32_t *__restrict__ pos_dev) {
    const int64_t nb = ekv / 32;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * nb * T) return;
    const int t = (int)(i / (2 * nb));
    const int64_t r = i % (2 * nb);
    const bool isv = r >= nb;
    const int64_t b = isv ? r - nb : r;
    const int64_t p = (pos_dev ? pos_dev[0] : n_past_arg) + t;
    float x[32];
    const float *src = qkv + t * ld + (isv ? voff : koff) + b * 32;
    for (int e = 0; e < 32; ++e) x[e] = src[e];
    if (isv) quant_block<TV>(x, vc, n_ctx, ekv, p, b);
    else quant_block<TK>(x, kc, n_ctx, ekv, p, b);
}

// RoPE of q and k in place in the f32 q|k|v staging rows (same rotation and table as ops.hip k_rope_kv, whose
// f16 rounding the quantized cache must not see: the reference quantizes the f32 rope output)
__global__ void k_rope_qk_inplace(float *__restrict__ qkv, int64_t ld, int H, int HKV, int D, int n_past,
                                  const int32_t *__restrict__ pos_dev, const float2 *__restrict__ rope_tab) {
    const int t = blockIdx.x;
    const int p = (pos_dev ? pos_dev[0] : n_past) + t;
    const int half = D / 2;
    float *row = qkv + (int64_t)t * ld;
    for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < (H + HKV) * half; i += gridDim.y * blockDim.x) {
        const int hh = i / half, ip = i % half;           // heads 0..H-1 are q, H..H+HKV-1 are k (contiguous)
        const float2 cs = rope_tab[(int64_t)p * half + ip];
        float *src = row + (int64_t)hh * D + 2 * ip;
        const float x0 = src[0], x1 = src[1];
        src[0] = __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
        src[1] = __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x));
    }
}

#define FQ_BQ 64
#define FQ_BK 64
// flash attention over quantized caches; grid (ceil(T/64), H), 256 threads; thread (ty, tx): query rows 4ty..4ty+3,
// key columns tx + 16j, output dims tx*DPT..; q f32 at byte strides q_nb1 (query) / q_nb2 (head).
// GG = 0: the runtime's caches (layout above), causal window [0, n_past + t].
// GG = 1: GGML_OP_FLASH_ATTN_EXT's own form (the b1 backend): K / V views of ggml blocks (block_q8_0 / block_q4_0: f16 d
// then the quants) at byte strides nb1 (position) / nb2 (kv head), all n_kv = n_past_arg keys under an explicit f16
// mask row (a -inf key is skipped, otherwise s * scale + mask, ggml.c:15780-15800); null mask = no mask.
struct FqView { int64_t k_nb1, k_nb2, v_nb1, v_nb2; const uint16_t *mask; int64_t mask_ld; };
template <int D, int TK, int TV, int GG>
__global__ void __launch_bounds__(256) k_fa_q(const float *__restrict__ q, int64_t q_nb1, int64_t q_nb2, const void *kc,
                                              const void *vc, float *__restrict__ out, int T, int H, int HKV, int64_t n_ctx,
                                              int n_past_arg, const int32_t *__restrict__ n_past_dev, float scale,
                                              const FqView gv) {
    constexpr int DPT = D / 16, NB = D / 32;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    const int qt = blockIdx.x, h = blockIdx.y;
    const int G = H / HKV, hk = h / G;
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    const int64_t ekv = (int64_t)HKV * D;
    __shared__ float sQ[FQ_BQ][D + 1];                 // Q8_0 integer values of the query
    __shared__ float sQd[FQ_BQ][NB];                   // their block scales (f16-rounded, as GGML_FP16_TO_FP32)
    __shared__ float sK[FQ_BK][D + 1];                 // K integer values (Q8_0: q, Q4_0: nibble - 8)
    __shared__ float sKd[FQ_BK][NB];
    __shared__ float sV[FQ_BK][D];                     // dequantized V
    const int q0 = qt * FQ_BQ;
    // quantize the tile's queries to Q8_0 per 32-block (quantize_row_q8_0 of the f32 q, AVX2 semantics)
    for (int i = tid; i < FQ_BQ * NB; i += 256) {
        const int r = i / NB, b = i % NB;
        float x[32];
        const bool ok = q0 + r < T;
        const float *qr = (const float *)((const char *)q + (int64_t)(q0 + r) * q_nb1 + (int64_t)h * q_nb2) + b * 32;
        for (int e = 0; e < 32; ++e) x[e] = ok ? qr[e] : 0.0f;
        float am = 0.0f;
        for (int e = 0; e < 32; ++e) am = fmaxf(am, fabsf(x[e]));
        const float id = am != 0.0f ? 127.f / am : 0.0f;
        for (int e = 0; e < 32; ++e) {
            int iv = (int)rintf(__fmul_rn(x[e], id));
            iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
            sQ[r][b * 32 + e] = (float)iv;
        }
        sQd[r][b] = h2f(f2h_rn(am / 127.f));
    }
    float m[4], l[4], o[4][DPT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = -INFINITY; l[r] = 0.0f;
#pragma unroll
        for (int j = 0; j < DPT; ++j) o[r][j] = 0.0f;
    }
    const int last_q = min(q0 + FQ_BQ, T) - 1;
    const int kend = GG ? n_past_arg : n_past + last_q + 1;
    const uint16_t *kd = (const uint16_t *)((const uint8_t *)kc + (TK == KT_Q8_0 ? n_ctx * ekv : n_ctx * ekv / 2));
    const uint16_t *vd = (const uint16_t *)((const uint8_t *)vc + (TV == KT_Q8_0 ? n_ctx * ekv : n_ctx * ekv / 2));
    for (int k0 = 0; k0 < kend; k0 += FQ_BK) {
        __syncthreads();
        for (int i = tid; i < FQ_BK * NB; i += 256) {           // one 32-block of K and of V per item
            const int r = i / NB, b = i % NB;
            const int64_t p = k0 + r;
            const bool ok = p < kend;
            const int64_t blk = p * (ekv / 32) + (int64_t)hk * NB + b;   // block index within the cache
            // GG: the ggml block at (position p, kv head hk, block b) of each view: {f16 d, quants}
            const uint8_t *gk = (const uint8_t *)kc + (ok ? p : 0) * gv.k_nb1 + (int64_t)hk * gv.k_nb2 + b * (TK == KT_Q8_0 ? 34 : 18);
            const uint8_t *gvb = (const uint8_t *)vc + (ok ? p : 0) * gv.v_nb1 + (int64_t)hk * gv.v_nb2 + b * (TV == KT_Q8_0 ? 34 : 18);
            float kv[32], vv[32];
            if (TK == KT_Q8_0) {
                const int8_t *s8 = GG ? (const int8_t *)(gk + 2) : (const int8_t *)kc + blk * 32;
                for (int e = 0; e < 32; ++e) kv[e] = ok ? (float)s8[e] : 0.0f;
            } else {
                const uint8_t *s4 = GG ? gk + 2 : (const uint8_t *)kc + blk * 16;
                for (int j = 0; j < 16; ++j) {
                    const int byte = ok ? s4[j] : 0x88;
                    kv[j] = (float)((byte & 0xF) - 8); kv[j + 16] = (float)((byte >> 4) - 8);
                }
            }
            const float dv = ok ? h2f(GG ? *(const uint16_t *)gvb : vd[blk]) : 0.0f;
            if (TV == KT_Q8_0) {
                const int8_t *s8 = GG ? (const int8_t *)(gvb + 2) : (const int8_t *)vc + blk * 32;
                for (int e = 0; e < 32; ++e) vv[e] = ok ? __fmul_rn(dv, (float)s8[e]) : 0.0f;
            } else {
                const uint8_t *s4 = GG ? gvb + 2 : (const uint8_t *)vc + blk * 16;
                for (int j = 0; j < 16; ++j) {
                    const int byte = ok ? s4[j] : 0x88;
                    vv[j] = __fmul_rn(dv, (float)((byte & 0xF) - 8)); vv[j + 16] = __fmul_rn(dv, (float)((byte >> 4) - 8));
                }
            }
            for (int e = 0; e < 32; ++e) { sK[r][b * 32 + e] = kv[e]; sV[r][b * 32 + e] = vv[e]; }
            sKd[r][b] = ok ? h2f(GG ? *(const uint16_t *)gk : kd[blk]) : 0.0f;
        }
        __syncthreads();
        float s[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) s[r][j] = 0.0f;
        for (int b = 0; b < NB; ++b) {
            float isum[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < 4; ++j) isum[r][j] = 0.0f;
            for (int e = 0; e < 32; ++e) {                        // exact: |products| <= 16129, sums < 2^24
                const int d = b * 32 + e;
                float qd[4], kd4[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) qd[r] = sQ[4 * ty + r][d];
#pragma unroll
                for (int j = 0; j < 4; ++j) kd4[j] = sK[tx + 16 * j][d];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < 4; ++j) isum[r][j] = fmaf(qd[r], kd4[j], isum[r][j]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    s[r][j] = fmaf(__fmul_rn(sKd[tx + 16 * j][b], sQd[4 * ty + r][b]), isum[r][j], s[r][j]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qi = q0 + 4 * ty + r;
            const int qpos = n_past + qi;
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = k0 + tx + 16 * j;
                if constexpr (GG) {
                    const float mv = (gv.mask && qi < T && p < kend) ? h2f(gv.mask[(int64_t)qi * gv.mask_ld + p]) : 0.0f;
                    s[r][j] = (qi < T && p < kend && mv != -INFINITY) ? __fadd_rn(s[r][j] * scale, mv) : -INFINITY;
                } else {
                    s[r][j] = (qi < T && p <= qpos) ? s[r][j] * scale : -INFINITY;
                }
                mx = fmaxf(mx, s[r][j]);
            }
            mx = max16_f(mx);
            const float mnew = fmaxf(m[r], mx);
            const float alpha = (mnew == -INFINITY) ? 1.0f : expf(m[r] - mnew);
            float ls = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s[r][j] = (s[r][j] == -INFINITY) ? 0.0f : expf(s[r][j] - mnew);
                ls += s[r][j];
            }
            ls += dpp_f<0xB1>(ls); ls += dpp_f<0x4E>(ls); ls += dpp_f<0x141>(ls); ls += dpp_f<0x140>(ls);
            l[r] = l[r] * alpha + ls;
            m[r] = mnew;
#pragma unroll
            for (int j = 0; j < DPT; ++j) o[r][j] *= alpha;
        }
        for (int src = 0; src < 16; ++src) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kr = src + 16 * j;
                float vr[DPT];
#pragma unroll
                for (int e = 0; e < DPT; ++e) vr[e] = sV[kr][tx * DPT + e];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pr = __shfl(s[r][j], ((16 * ty) & 63) + src, 64);
#pragma unroll
                    for (int e = 0; e < DPT; ++e) o[r][e] = fmaf(pr, vr[e], o[r][e]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int qi = q0 + 4 * ty + r;
        if (qi < T) {
            const float inv = 1.0f / l[r];
#pragma unroll
            for (int e = 0; e < DPT; ++e) out[((int64_t)qi * H + h) * D + tx * DPT + e] = o[r][e] * inv;
        }
    }
}

}  // namespace

extern "C" {

// bytes of one layer's quantized K or V cache
int64_t kcpp_kv_cache_bytes(int type, int64_t n_ctx, int64_t ekv) {
    if (type == KT_F16) return n_ctx * ekv * 2;
    if (type == KT_Q8_0) return n_ctx * ekv + n_ctx * ekv / 16;
    if (type == KT_Q4_0) return n_ctx * ekv / 2 + n_ctx * ekv / 16;
    return -1;
}

int kcpp_rope_qk_inplace(float *qkv, int64_t ld, int T, int H, int HKV, int D, int n_past, const int32_t *pos_dev,
                         const void *rope_tab, void *stream) {
    const int items = (H + HKV) * D / 2;
    hipLaunchKernelGGL(k_rope_qk_inplace, dim3((unsigned)T, (unsigned)((items + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, qkv, ld, H, HKV, D, n_past, pos_dev, (const float2 *)rope_tab);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_kv_store_q(int tk, int tv, const float *qkv, int64_t ld, int64_t koff, int64_t voff, int T, int64_t ekv,
                    void *kc, void *vc, int64_t n_ctx, int n_past, const int32_t *pos_dev, void *stream) {
    if (ekv % 32 || T < 1) return -1;
    const int64_t items = 2 * (ekv / 32) * T;
    const dim3 g((unsigned)((items + 255) / 256));
    hipStream_t s = (hipStream_t)stream;
#define KVS(A, B) hipLaunchKernelGGL((k_kv_store_q<A, B>), g, dim3(256), 0, s, qkv, ld, koff, voff, T, ekv, kc, vc, n_ctx, n_past, pos_dev)
    if (tk == KT_Q8_0 && tv == KT_Q8_0) KVS(KT_Q8_0, KT_Q8_0);
    else if (tk == KT_Q8_0 && tv == KT_Q4_0) KVS(KT_Q8_0, KT_Q4_0);
    else if (tk == KT_Q4_0 && tv == KT_Q8_0) KVS(KT_Q4_0, KT_Q8_0);
    else if (tk == KT_Q4_0 && tv == KT_Q4_0) KVS(KT_Q4_0, KT_Q4_0);
    else return -2;
#undef KVS
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_flash_attn_q(int tk, int tv, const float *q, int64_t ldq, const void *kc, const void *vc, float *out, int T,
                      int H, int HKV, int D, int64_t n_ctx, int n_past, const int32_t *n_past_dev, float scale,
                      void *stream) {
    if (H % HKV || (D != 128 && D != 64)) return -1;
    const dim3 g((unsigned)((T + FQ_BQ - 1) / FQ_BQ), (unsigned)H);
    hipStream_t s = (hipStream_t)stream;
    const FqView gv{0, 0, 0, 0, nullptr, 0};
#define FQ(DD, A, B) hipLaunchKernelGGL((k_fa_q<DD, A, B, 0>), g, dim3(256), 0, s, q, ldq * 4, (int64_t)D * 4, kc, vc, out, T, H, HKV, n_ctx, n_past, n_past_dev, scale, gv)
#define FQD(DD)                                                     \
    if (tk == KT_Q8_0 && tv == KT_Q8_0) FQ(DD, KT_Q8_0, KT_Q8_0);   \
    else if (tk == KT_Q8_0 && tv == KT_Q4_0) FQ(DD, KT_Q8_0, KT_Q4_0); \
    else if (tk == KT_Q4_0 && tv == KT_Q8_0) FQ(DD, KT_Q4_0, KT_Q8_0); \
    else if (tk == KT_Q4_0 && tv == KT_Q4_0) FQ(DD, KT_Q4_0, KT_Q4_0); \
    else return -2;
    if (D == 128) { FQD(128) } else { FQD(64) }
#undef FQD
#undef FQ
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// GGML_OP_FLASH_ATTN_EXT over quantized K / V views (the b1 backend): q f32 [T][H][D] at byte strides q_nb1 / q_nb2,
// K / V views of ggml Q8_0 / Q4_0 blocks at byte strides nb1 (position) / nb2 (kv head), optional f16 mask [T][n_kv]
// (row stride mask_ld elements), out f32 [T][H][D]
int kcpp_flash_attn_ext_q(int tk, int tv, const float *q, int64_t q_nb1, int64_t q_nb2, const void *kc, int64_t k_nb1,
                          int64_t k_nb2, const void *vc, int64_t v_nb1, int64_t v_nb2, const uint16_t *mask,
                          int64_t mask_ld, float *out, int T, int H, int HKV, int D, int n_kv, float scale, void *stream) {
    if (H % HKV || (D != 128 && D != 64) || n_kv < 1 || T < 1) return -1;
    const dim3 g((unsigned)((T + FQ_BQ - 1) / FQ_BQ), (unsigned)H);
    hipStream_t s = (hipStream_t)stream;
    const FqView gv{k_nb1, k_nb2, v_nb1, v_nb2, mask, mask_ld};
#define FQ(DD, A, B) hipLaunchKernelGGL((k_fa_q<DD, A, B, 1>), g, dim3(256), 0, s, q, q_nb1, q_nb2, kc, vc, out, T, H, HKV, (int64_t)0, n_kv, (const int32_t *)nullptr, scale, gv)
#define FQD(DD)                                                     \
    if (tk == KT_Q8_0 && tv == KT_Q8_0) FQ(DD, KT_Q8_0, KT_Q8_0);   \
    else if (tk == KT_Q8_0 && tv == KT_Q4_0) FQ(DD, KT_Q8_0, KT_Q4_0); \
    else if (tk == KT_Q4_0 && tv == KT_Q8_0) FQ(DD, KT_Q4_0, KT_Q8_0); \
    else if (tk == KT_Q4_0 && tv == KT_Q4_0) FQ(DD, KT_Q4_0, KT_Q4_0); \
    else return -2;
    if (D == 128) { FQD(128) } else { FQD(64) }
#undef FQD
#undef FQ
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_cpy_f32_q(int type, const float *src, int64_t n, void *dst, void *stream) {
    if (n % 32) return -1;
    const int64_t nb = n / 32;
    if (nb == 0) return 0;
    const dim3 g((unsigned)((nb + 255) / 256));
    if (type == KT_Q8_0) hipLaunchKernelGGL(k_cpy_f32_q<KT_Q8_0>, g, dim3(256), 0, (hipStream_t)stream, src, nb, (uint8_t *)dst);
    else if (type == KT_Q4_0) hipLaunchKernelGGL(k_cpy_f32_q<KT_Q4_0>, g, dim3(256), 0, (hipStream_t)stream, src, nb, (uint8_t *)dst);
    else return -2;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
