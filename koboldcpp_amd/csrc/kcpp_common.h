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

// IQ4_NL / IQ4_XS code book (kvalues_iq4nl, ggml-quants.c:3741) as four little-endian dwords
__device__ __forceinline__ int kv_iq4nl(int q) {
    const int8_t t[16] = {-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113};
    return t[q & 15];
}
// four nibble codes (bytes of x, each 0..15) -> their four int8 code-book values: two v_perm_b32 byte lookups into the
// 8-entry halves, picked per byte by the code's bit 3
__device__ __forceinline__ uint32_t iq4nl_lut4(uint32_t x) {
    constexpr uint32_t T0 = 0xBFAD9881u, T1 = 0xF6EADDCFu, T2 = 0x26190D01u, T3 = 0x71594535u;
    const uint32_t sel = x & 0x07070707u;
    const uint32_t lo = __builtin_amdgcn_perm(T1, T0, sel), hi = __builtin_amdgcn_perm(T3, T2, sel);
    const uint32_t m = ((x >> 3) & 0x01010101u) * 0xFFu;
    return (hi & m) | (lo & ~m);
}
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }

// In-launch hand-off payloads as 16-byte vector accesses with the agent-scope (sc1) policy that
// __hip_atomic_{store,load}(..., __HIP_MEMORY_SCOPE_AGENT) puts on single dwords (write-through past the XCD's L2 /
// read from the device-coherent level): one b128 instruction instead of four dword ones.  base must be
// wave-uniform (a buffer resource), off in bytes (< 2 GiB).  MI355X_MICROARCH.md hand-off table, row 1.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t kcpp_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 kcpp_ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ void kcpp_st_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 16);
}
// f32 -> f16 of an already-rounded f32 value.  Without the register barrier the backend folds f2h(a * b) into
// v_fma_mixlo_f16(a, b, 0) -- ONE rounding of the exact product, and +0 for a -0 product -- which is not the
// reference's GGML_FP32_TO_FP16(a * b) (two roundings, sign kept); -ffp-contract=off does not stop it.
__device__ __forceinline__ uint16_t f2h_rn(float x) {
    asm volatile("" : "+v"(x));
    return f2h(x);
}

__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// (cos, sin) of rope pair ip at position p, as ggml_compute_forward_rope_f32 (ggml.c:14272) with
// ggml_rope_cache_init (:14246) and rope_yarn (:14223): theta iterated from the position by theta_scale, the YaRN
// ramp when ext_factor != 0, cos / sin correctly rounded through double (the CPU's glibc cosf / sinf are within 1 ulp
// of that), times mscale.  Shared by the ggml plugin's ROPE kernel and the mat-vec epilogue it is fused into, so both
// give the same bits.
__device__ __forceinline__ void ggml_rope_cs(float p, int64_t ip, const float *ff, float theta_scale, float freq_scale,
                                             float ext_factor, float attn_factor, float mscale_ext, float corr0,
                                             float corr1, float &c, float &s) {
    float theta = p;
    for (int64_t k = 0; k < ip; ++k) theta *= theta_scale;
    const float theta_extrap = theta / (ff ? ff[ip] : 1.0f);
    const float theta_interp = freq_scale * theta_extrap;
    float th = theta_interp, mscale = attn_factor;
    if (ext_factor != 0.0f) {
        const float yy = (ip - corr0) / fmaxf(0.001f, corr1 - corr0);
        const float ramp_mix = (1.0f - fminf(1.0f, fmaxf(0.0f, yy))) * ext_factor;
        th = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
        mscale = mscale_ext;
    }
    c = (float)cos((double)th) * mscale;
    s = (float)sin((double)th) * mscale;
}

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
//   Q8_0_T (KT_Q8_0_T, N % 32 == 0, K % 128 == 0): 32-row tiles; tile t, block b (nb = K / 32 blocks per row):
//          qs at (t nb + b) * 1024: [half h][row r][16 B] = row 32 t + r, bytes 32 b + 16 h .. + 15  (the B operand of
//          v_mfma_i32_32x32x32_i8 for lane 32 h + r, one contiguous 1 KiB wave load), then the d plane at N K:
//          (t nb / 4 + b / 4) * 256 + r * 8 + (b % 4) * 2  (f16: four blocks of a row in one 8-B lane load)
__host__ __device__ inline int64_t kl_nblocks(int type, int64_t K, int64_t N) {
    return K / ks_block_elems(type) * N;
}

// Activation buffers (vec_dot_type of the weight; ggml.c:793-959):
//   Q8_K act: qs int8 [M][K] ++ d f32 [M][K/256] ++ bsums int16 [M][K/16]
//   Q8_0 act: qs int8 [M][K] ++ d f32 [M][K/32]  ++ asum  int16 [M][K/32]
//   Q8_1 act: the Q8_0 act ++ s f32 [M][K/32] (block_q8_1.s = f16(d * sum qs), d before rounding; 4-B aligned)
struct ActView {
    const int8_t *qs;
    const float *d;
    const int16_t *bs;
    const float *s;
    int64_t K;
};
//   Q8_0_TA act (KT_Q8_0_T's vec_dot_type): the Q8_0 quantization of 32-token groups, G = ceil(M / 32):
//          qs int8 [G][K / 32 blocks][half h][32 tokens][16 B] (the A operand of the MFMA, 1 KiB per block) ++
//          d f32 [G][K / 32][32 tokens]; tokens past M are never read back
__host__ __device__ inline int64_t act_bytes(int vtype, int64_t K, int64_t M) {
    if (vtype == KT_Q8_0_TA) return (M + 31) / 32 * 32 * (K + K / 32 * 4);
    if (vtype == KT_Q8_K) return M * K + M * (K / 256) * 4 + M * (K / 16) * 2;
    if (vtype == KT_Q8_1) return M * K + M * (K / 32) * 4 + ((M * (K / 32) * 2 + 3) & ~(int64_t)3) + M * (K / 32) * 4;
    return M * K + M * (K / 32) * 4 + M * (K / 32) * 2;
}
__host__ __device__ inline ActView act_view(int vtype, const void *buf, int64_t K, int64_t M, int64_t c) {
    const int8_t *base = (const int8_t *)buf;
    ActView a;
    a.K = K;
    a.qs = base + c * K;
    a.s = nullptr;
    if (vtype == KT_Q8_1)
        a.s = (const float *)(base + M * K + M * (K / 32) * 4 + ((M * (K / 32) * 2 + 3) & ~(int64_t)3)) + c * (K / 32);
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
    if (wtype == KT_Q4_1 || wtype == KT_Q5_1) return KT_Q8_1;
    if (wtype == KT_Q8_0_T) return KT_Q8_0_TA;
    return (wtype == KT_Q4_0 || wtype == KT_Q5_0 || wtype == KT_Q8_0 || wtype == KT_IQ4_NL) ? KT_Q8_0 : KT_Q8_K;
}

// ---------------------------------------------------------------------------------
// DPP (VALU, no LDS round trip) all-reduce over aligned 16-lane groups:
// quad_perm xor1 (0xB1), quad_perm xor2 (0x4E), row_half_mirror (0x141), row_mirror (0x140).
// After the 4 steps every lane of the group holds the group result (max / int sum exact;
// float sums may differ in rounding between lanes -- read one lane when that matters).
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false)); }

__device__ __forceinline__ int sum16_i(int v) {
    v += dpp_i<0xB1>(v); v += dpp_i<0x4E>(v); v += dpp_i<0x141>(v); v += dpp_i<0x140>(v);
    return v;
}
__device__ __forceinline__ float max16_f(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v)); v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v)); v = fmaxf(v, dpp_f<0x140>(v));
    return v;
}
// (|x|, index, x) arg-max with the smallest index winning ties (commutative + associative,
// so the DPP pairing order does not matter).
template <int CTRL>
__device__ __forceinline__ void amax_step(float &a, int &i, float &x) {
    const float a2 = dpp_f<CTRL>(a), x2 = dpp_f<CTRL>(x);
    const int i2 = dpp_i<CTRL>(i);
    const bool take = a2 > a || (a2 == a && i2 < i);
    a = take ? a2 : a; i = take ? i2 : i; x = take ? x2 : x;
}

// quantize_row_q8_K_ref (ggml-quants.c:3786-3823) of one 256-element super-block held by an
// aligned 16-lane group, lane j holding elements 16j..16j+15 (so bsums[j] is lane-local).
// qs/d/bs point at the super-block's output; l16 = lane & 15.
// VALU-lean form of the reference loop, same bytes:
//  * amax = max |x|; the reference keeps the signed value of the FIRST element reaching it (`ax > amax`): the
//    lane(s) whose own maximum equals amax scan for it, then the smallest index wins across the group;
//  * nearest_int(iscale * x) (ggml-quants.c:1640, multiply not fused) = bits(iscale * x + 1.5 * 2^23) -
//    0x4B400000, so the int8 code is the low byte of those float bits and the 16-element sum is the wrapped sum
//    of the bits minus 16 * 0x4B400000; |iscale * x| <= 127, so the reference's MIN(127, .) never applies.
__device__ __forceinline__ void q8k_quant16(const float (&v)[16], int l16, int8_t *qs, float *d, int16_t *bs) {
    float lm = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) lm = fmaxf(lm, fabsf(v[e]));
    const float am = max16_f(lm);
    if (am == 0.0f) {                                  // uniform over the 16 lanes (one amax)
        *(uint4 *)(qs + 16 * l16) = make_uint4(0, 0, 0, 0);
        bs[l16] = 0;
        if (l16 == 0) *d = 0.0f;
        return;
    }
    int ai = 256;
    float mx = 0.0f;
    if (lm == am) {
#pragma unroll
        for (int e = 15; e >= 0; --e)
            if (fabsf(v[e]) == am) { ai = 16 * l16 + e; mx = v[e]; }
    }
#define KCPP_Q8K_MIN_STEP(CTRL)                                                                  \
    {                                                                                            \
        const int a2 = dpp_i<CTRL>(ai);                                                          \
        const float m2 = dpp_f<CTRL>(mx);                                                        \
        if (a2 < ai) { ai = a2; mx = m2; }                                                       \
    }
    KCPP_Q8K_MIN_STEP(0xB1) KCPP_Q8K_MIN_STEP(0x4E) KCPP_Q8K_MIN_STEP(0x141) KCPP_Q8K_MIN_STEP(0x140)
#undef KCPP_Q8K_MIN_STEP
    const float iscale = -127.f / mx;
    uint32_t w[4], sum = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t bt[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bt[j] = __float_as_uint(__fadd_rn(__fmul_rn(iscale, v[4 * k + j]), 12582912.f));
            sum += bt[j];
        }
        const uint32_t lo = __builtin_amdgcn_perm(bt[1], bt[0], 0x0C0C0400u);   // byte0(bt0) | byte0(bt1) << 8
        const uint32_t hi = __builtin_amdgcn_perm(bt[3], bt[2], 0x0C0C0400u);
        w[k] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);                      // lo.b0 lo.b1 hi.b0 hi.b1
    }
    *(uint4 *)(qs + 16 * l16) = make_uint4(w[0], w[1], w[2], w[3]);
    bs[l16] = (int16_t)(int32_t)(sum - 16u * 0x4B400000u);
    if (l16 == 0) *d = 1.0f / iscale;
}

// 64-lane all-reduce of a double: DPP within rows of 16 (two 32-bit halves per step), then two
// cross-row exchanges.  The summation tree differs from a sequential CPU sum only below 1 ulp of
// double, which is invisible after the (float) rounding the rms_norm callers apply.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xFFFFFFFFll), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Cross-row exchanges on the gfx950 VALU (v_permlane16_swap / v_permlane32_swap): with both operands = v the
// swap returns (row pair's even rows, odd rows) resp. (lower half, upper half), so lane l gets v[l] and
// v[l ^ 16] (v[l ^ 32]) without an LDS round trip (__shfl_xor is a ds_bpermute).  a + b == b + a and
// fmaxf(a, b) == fmaxf(b, a) bitwise, so these equal v (+|max) __shfl_xor(v, 16|32, 64) exactly.
__device__ __forceinline__ float xsum16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xmax16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ double xsum16_d(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)(b & 0xFFFFFFFFll), (unsigned)(b & 0xFFFFFFFFll), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double xsum32_d(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)(b & 0xFFFFFFFFll), (unsigned)(b & 0xFFFFFFFFll), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<0xB1>(v); v += dpp_d<0x4E>(v); v += dpp_d<0x141>(v); v += dpp_d<0x140>(v);
    return xsum32_d(xsum16_d(v));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    v = max16_f(v);
    return xmax32(xmax16(v));
}
__device__ __forceinline__ float wave_sum_f(float v) {
    v += dpp_f<0xB1>(v); v += dpp_f<0x4E>(v); v += dpp_f<0x141>(v); v += dpp_f<0x140>(v);
    return xsum32(xsum16(v));
}
