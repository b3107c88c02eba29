// attn_exact.hip -- flash attention in the REFERENCE CPU's arithmetic order (strict-parity mode).
//
// The production kernels (attn.hip, attn_mfma.hip) split the keys over workgroups and accumulate V*P in
// f32.  The reference CPU path, ggml_compute_forward_flash_attn_ext_f16 (ggml/src/ggml.c:15667-15875, F16
// K/V branch), walks the keys of one query row in order with an f16 accumulator:
//     s   = ggml_vec_dot_f16(q16, k16) * scale + mask            (AVX2 order, ggml.c:2258-2290)
//     if s > M: M = s, ms = expf(Mold - M), VKQ16 = f16(VKQ16 * ms)        (ggml_vec_scale_f16, :2501)
//     else:     vs = expf(s - M)
//     VKQ16 = f16(fma(v16, vs, VKQ16))                                     (ggml_vec_mad_f16, FMA build)
//     S = S*ms + vs
//     out = f32(VKQ16) * (1/S)
// Each f16 rounding depends on the previous one, so no key split reproduces it.  At full Llama-3-8B width
// this f16 accumulation moves the residual stream by ~0.6% relative (tests/test_gpu_fullwidth.py), far
// more than the reference's own build-to-build spread.  This kernel reproduces the order exactly:
//   one workgroup per (query row, head), one lane per head dim (D = 128: two waves; D = 64: one);
//   phase 1: the chunk's scores, one lane per key, in the AVX2 lane/accumulator order of ggml_vec_dot_f16
//            (4 accumulators x 8 lanes, FMA, then the GGML_F32x8_REDUCE tree), into LDS;
//   phase 2: every lane walks the chunk's keys serially for its own dim (M and S are computed redundantly
//            and identically by all lanes), exp computed in double and rounded (glibc expf is correctly
//            rounded in practice; the GPU's single-precision expf is not).
// It is a parity instrument, not a fast path: one serial chain per (row, head, dim).  Selected per model by
// kcpp_model_set_fa_exact() or KCPP_FA_EXACT=1 at model creation; off by default.
#include "kcpp_common.h"
#include "kcpp_internal.h"

#define EX_CH 512

__device__ __forceinline__ float ex_exp(float x) { return (float)exp((double)x); }
// f16(x) of an f32 value that must first be rounded to f32: without the register barrier the compiler folds
// f2h(fmaf(a, b, h2f(c))) into one v_fma_mixlo_f16, which rounds the exact result straight to f16 (a single
// rounding where the reference rounds twice, f32 then f16 -- a different result in rare double-rounding cases)
__device__ __forceinline__ uint16_t f2h_of_f32(float x) { return f2h_rn(x); }

// EXT = the ggml op's own form (the b1 backend): q f32 with byte strides (rounded to f16 here, q_to_vec_dot),
// all n_kv keys of the K/V views under an explicit f16 mask row (-inf keys skipped, others s*scale + mask).
// Otherwise the runtime's form: q16 f16 [T][H][D], implicit causal window [0, n_past + t].
template <bool EXT, int EX_D>
__global__ void __launch_bounds__(EX_D) k_fa_exact(const uint16_t *__restrict__ q16, const float *__restrict__ qf32,
                                                   int64_t q_nb1, int64_t q_nb2, const uint16_t *__restrict__ kc,
                                                   const uint16_t *__restrict__ vc, float *__restrict__ out, int H,
                                                   int HKV, int n_past_arg, const int32_t *__restrict__ n_past_dev,
                                                   float scale, const uint16_t *__restrict__ mask, int64_t mask_ld) {
    const int h = blockIdx.x, t = blockIdx.y, d = threadIdx.x;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    // causal: query t (position n_past + t) sees keys 0..n_past+t; EXT: n_past_arg = n_kv, the mask decides
    const int n_kv = EXT ? n_past_arg : n_past + t + 1;
    const uint16_t *mrow = EXT && mask ? mask + (int64_t)t * mask_ld : nullptr;
    const int hk = h / (H / HKV);
    const int64_t ekv = (int64_t)HKV * EX_D;
    __shared__ float qf[EX_D];
    __shared__ float sc[EX_CH];
    if constexpr (EXT) qf[d] = h2f(f2h(((const float *)((const char *)qf32 + t * q_nb1 + h * q_nb2))[d]));
    else qf[d] = h2f(q16[((int64_t)t * H + h) * EX_D + d]);
    __syncthreads();
    float M = -INFINITY, S = 0.0f;
    uint16_t vkq = 0;
    for (int c0 = 0; c0 < n_kv; c0 += EX_CH) {
        const int cnt = min(EX_CH, n_kv - c0);
        for (int j = d; j < cnt; j += EX_D) {
            const float mv = mrow ? h2f(mrow[c0 + j]) : 0.0f;
            if (mv == -INFINITY) { sc[j] = -INFINITY; continue; }      // the reference skips the key entirely
            const uint4 *kr = (const uint4 *)(kc + (int64_t)(c0 + j) * ekv + (int64_t)hk * EX_D);
            float acc[4][8];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int l = 0; l < 8; ++l) acc[a][l] = 0.0f;
#pragma unroll
            for (int i = 0; i < EX_D / 32; ++i) {          // GGML_F16_STEP = 32
#pragma unroll
                for (int a = 0; a < 4; ++a) {                // GGML_F16_ARR = 4 vectors of GGML_F16_EPR = 8
                    const uint4 kv = kr[i * 4 + a];
                    const uint32_t w[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
                    for (int l = 0; l < 8; ++l) {
                        const float kx = h2f((uint16_t)(w[l >> 1] >> (16 * (l & 1))));
                        acc[a][l] = fmaf(kx, qf[i * 32 + a * 8 + l], acc[a][l]);
                    }
                }
            }
            // GGML_F32x8_REDUCE: x0 += x2, x1 += x3; x0 += x1; 128-bit halves; two hadds
#pragma unroll
            for (int l = 0; l < 8; ++l) { acc[0][l] = acc[0][l] + acc[2][l]; acc[1][l] = acc[1][l] + acc[3][l]; }
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[0][l] = acc[0][l] + acc[1][l];
            const float t0 = acc[0][0] + acc[0][4], t1 = acc[0][1] + acc[0][5], t2 = acc[0][2] + acc[0][6],
                        t3 = acc[0][3] + acc[0][7];
            const float s = (t0 + t1) + (t2 + t3);
            sc[j] = s * scale + mv;                        // s*scale, then += mask
        }
        __syncthreads();
        const uint16_t *vr = vc + (int64_t)c0 * ekv + (int64_t)hk * EX_D + d;
        for (int j = 0; j < cnt; ++j) {
            const float s = sc[j];
            if (s == -INFINITY) continue;                  // masked key (a finite score plus a finite mask never is)
            const float v = h2f(vr[(int64_t)j * ekv]);
            float ms = 1.0f, vs = 1.0f;
            if (s > M) {
                const float Mold = M;
                M = s;
                ms = ex_exp(Mold - M);
                vkq = f2h_of_f32(h2f(vkq) * ms);
            } else {
                vs = ex_exp(s - M);
            }
            vkq = f2h_of_f32(fmaf(v, vs, h2f(vkq)));
            S = S * ms + vs;
        }
        __syncthreads();
    }
    const float S_inv = 1.0f / S;
    out[((int64_t)t * H + h) * EX_D + d] = h2f(vkq) * S_inv;
}

// q16 [T][H][D] f16, caches [pos][HKV][D] f16 (row stride HKV*D), out [T][H][D] f32
extern "C" int kcpp_flash_attn_exact(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, int T,
                                     int H, int HKV, int D, int n_past, const int32_t *n_past_dev, float scale,
                                     void *stream) {
    if ((D != 128 && D != 64) || T < 1 || HKV < 1 || H % HKV != 0 || (!n_past_dev && n_past < 0)) return -3;
    if (D == 128)
        hipLaunchKernelGGL((k_fa_exact<false, 128>), dim3(H, T), dim3(128), 0, (hipStream_t)stream, q16, nullptr, 0, 0, kc,
                           vc, out, H, HKV, n_past, n_past_dev, scale, nullptr, 0);
    else
        hipLaunchKernelGGL((k_fa_exact<false, 64>), dim3(H, T), dim3(64), 0, (hipStream_t)stream, q16, nullptr, 0, 0, kc,
                           vc, out, H, HKV, n_past, n_past_dev, scale, nullptr, 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the graph form of GGML_OP_FLASH_ATTN_EXT (as kcpp_flash_attn_ext): q f32 [T][H][D] by byte strides, K/V views
// [n_kv][HKV][D], optional f16 mask [T][n_kv] with row stride mask_ld (elements), out f32 [T][H][D]
extern "C" int kcpp_flash_attn_ext_exact(const float *q, int64_t q_nb1, int64_t q_nb2, const uint16_t *kc,
                                         const uint16_t *vc, const uint16_t *mask, int64_t mask_ld, float *out, int T,
                                         int H, int HKV, int D, int n_kv, float scale, void *stream) {
    if ((D != 128 && D != 64) || T < 1 || HKV < 1 || H % HKV != 0 || n_kv < 1) return -3;
    if (D == 128)
        hipLaunchKernelGGL((k_fa_exact<true, 128>), dim3(H, T), dim3(128), 0, (hipStream_t)stream, nullptr, q, q_nb1, q_nb2,
                           kc, vc, out, H, HKV, n_kv, nullptr, scale, mask, mask_ld);
    else
        hipLaunchKernelGGL((k_fa_exact<true, 64>), dim3(H, T), dim3(64), 0, (hipStream_t)stream, nullptr, q, q_nb1, q_nb2,
                           kc, vc, out, H, HKV, n_kv, nullptr, scale, mask, mask_ld);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
