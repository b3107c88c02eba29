// kcpp_common.h -- shared device helpers for the MI355X (gfx950 / CDNA4) ggml backend.
//
// Wave64 is assumed everywhere (CDNA4); nothing here is a CUDA warp-32 idiom.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/kcpp_synth.h"

#define KCPP_WAVE 64
#define QK_K 256

#define KCPP_CHECK(expr)                                                                 \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            fprintf(stderr, "[kcpp] HIP error %s at %s:%d: %s\n", hipGetErrorName(_e),   \
                    __FILE__, __LINE__, #expr);                                          \
            return -(int)_e - 1000;                                                      \
        }                                                                                \
    } while (0)

// ---------------------------------------------------------------------------------
// wave64 reductions.  __shfl_xor lowers to ds_swizzle/DPP forms for xor masks < 32 and
// to ds_bpermute for 32 on gfx950.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
template <int W, typename T>
__device__ __forceinline__ T group_sum(T v) {     // reduce over aligned groups of W lanes
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }

__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// nearest_int() of ggml-quants.c:1640 with the multiply NOT fused (the reference is built
// -std=c11, i.e. -ffp-contract=off).
__device__ __forceinline__ int nearest_int_mul(float a, float b) {
    float val = __fadd_rn(__fmul_rn(a, b), 12582912.f);
    int i = __float_as_int(val);
    return (i & 0x007fffff) - 0x00400000;
}

// ---------------------------------------------------------------------------------
// GPU weight layout ("kcpp layout").  Same byte size as the ggml layout; blocks are in
// ggml row-major order (row n, block i -> b = n*(K/QK)+i).
//   Q4_K, Q5_K, F32, F16 : identical to ggml (144/176-B blocks are 16-B aligned)
//   Q6_K : [nb][192] ql|qh  ++ [nb][16] scales ++ [nb] fp16 d
//   Q4_0 : [nb][16] qs ++ [nb] fp16 d
//   Q8_0 : [nb][32] qs ++ [nb] fp16 d
__host__ __device__ inline int64_t kl_nblocks(int type, int64_t K, int64_t N) {
    return K / ks_block_elems(type) * N;
}

// Activation buffers (vec_dot_type of the weight; ggml.c:793-959):
//   Q8_K act: qs int8 [M][K] ++ d f32 [M][K/256] ++ bsums int16 [M][K/16]
//   Q8_0 act: qs int8 [M][K] ++ d f32 [M][K/32]  ++ asum  int16 [M][K/32]
struct ActView {
    const int8_t *qs;
    const float *d;
    const int16_t *bs;
    int64_t K;
};
__host__ __device__ inline int64_t act_bytes(int vtype, int64_t K, int64_t M) {
    if (vtype == KT_Q8_K) return M * K + M * (K / 256) * 4 + M * (K / 16) * 2;
    return M * K + M * (K / 32) * 4 + M * (K / 32) * 2;
}
__host__ __device__ inline ActView act_view(int vtype, const void *buf, int64_t K, int64_t M, int64_t c) {
    const int8_t *base = (const int8_t *)buf;
    ActView a;
    a.K = K;
    a.qs = base + c * K;
    if (vtype == KT_Q8_K) {
        a.d = (const float *)(base + M * K) + c * (K / 256);
        a.bs = (const int16_t *)(base + M * K + M * (K / 256) * 4) + c * (K / 16);
    } else {
        a.d = (const float *)(base + M * K) + c * (K / 32);
        a.bs = (const int16_t *)(base + M * K + M * (K / 32) * 4) + c * (K / 32);
    }
    return a;
}
inline int vec_dot_type(int wtype) {
    return (wtype == KT_Q4_0 || wtype == KT_Q8_0) ? KT_Q8_0 : KT_Q8_K;
}
