// gemv_lean.h -- shared parts of the VALU-lean decode mat-vec kernels (gemv_q4k.hip, gemv_rs.hip):
// the activation prologue (rms_norm * w -> Q8_K in LDS, or an already-quantized activation copied to
// LDS) with its global loads issued before the first weight loads, and the epilogue that stores the
// per-lane parked results (residual add / SiLU-GLU / RoPE + f16 K/V cache stores).
#pragma once
#include "gemv_units.h"
#include "kcpp_internal.h"

#include <algorithm>
#include <cstdlib>

namespace lean {

// NT threads per workgroup (MAXC = 16-element chunks per thread: ceil(K / (16 NT)))
// STORE (the ggml plugin's RMS_NORM -> MUL fused into the first consumer, AUX instances): compute() also stores the
// normalised row r = x * scale and the product y = r * w (the two nodes' tensors) where given
template <int PRO, int MAXC, int NT = 256, bool STORE = false>
struct ActPro {               // rms_norm * w -> Q8_K into LDS (see gemv_dec_impl.h); loads first
    float v[MAXC][16];
    float w[PRO == 1 ? MAXC : 1][16];
    __device__ __forceinline__ void load(const DecArgs &a, int64_t xoff = 0) {   // input row a.x + xoff
        const int tid = threadIdx.x, nchunk = (int)(a.K / 16);
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = min(tid + NT * i, nchunk - 1);
            const float4 *p = (const float4 *)(a.x + xoff + 16 * (int64_t)c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 f = p[k];
                v[i][4 * k] = f.x; v[i][4 * k + 1] = f.y; v[i][4 * k + 2] = f.z; v[i][4 * k + 3] = f.w;
            }
            if constexpr (PRO == 1) {
                const float4 *q = (const float4 *)(a.nw + 16 * (int64_t)c);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 f = q[k];
                    w[i][4 * k] = f.x; w[i][4 * k + 1] = f.y; w[i][4 * k + 2] = f.z; w[i][4 * k + 3] = f.w;
                }
            }
        }
    }
    __device__ __forceinline__ void compute(const DecArgs &a, uint8_t *lds, unsigned long long *st_ = nullptr,
                                            float *rout = nullptr, float *yout = nullptr) {
        const int tid = threadIdx.x;
#ifdef KCPP_STAMPS
#define LP_STAMP(ph) if (threadIdx.x == 0 && st_) __hip_atomic_store(&st_[(ph)], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
#define LP_STAMP(ph)
#endif
        if (v[0][0] == 12345.0f && st_) st_[15] = 1;
        LP_STAMP(8);
        const int64_t K = a.K;
        const int nchunk = (int)(K / 16);
        if constexpr (PRO == 1) {
            double ss = 0.0;
#pragma unroll
            for (int i = 0; i < MAXC; ++i)
                if (tid + NT * i < nchunk) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) ss += (double)__fmul_rn(v[i][e], v[i][e]);
                }
            ss = wave_sum_d(ss);
            LP_STAMP(9);
            __shared__ double red[NT / 64];
            if ((tid & 63) == 0) red[tid >> 6] = ss;
            __syncthreads();
            LP_STAMP(10);
            double sum = red[0] + red[1] + red[2] + red[3];
#pragma unroll
            for (int i = 4; i < NT / 64; i += 4) sum += red[i] + red[i + 1] + red[i + 2] + red[i + 3];
            const float scale = 1.0f / sqrtf((float)(sum / (double)K) + a.eps);   // ggml.c:12089
            if constexpr (STORE) {
                if (rout || yout) {
#pragma unroll
                    for (int i = 0; i < MAXC; ++i) {
                        const int c = tid + NT * i;
                        float r16[16];
#pragma unroll
                        for (int e = 0; e < 16; ++e) {
                            r16[e] = __fmul_rn(v[i][e], scale);
                            v[i][e] = __fmul_rn(r16[e], w[i][e]);
                        }
                        if (c < nchunk) {
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                if (rout) ((float4 *)(rout + 16 * (int64_t)c))[k] = make_float4(r16[4 * k], r16[4 * k + 1], r16[4 * k + 2], r16[4 * k + 3]);
                                if (yout) ((float4 *)(yout + 16 * (int64_t)c))[k] = make_float4(v[i][4 * k], v[i][4 * k + 1], v[i][4 * k + 2], v[i][4 * k + 3]);
                            }
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < MAXC; ++i)
#pragma unroll
                        for (int e = 0; e < 16; ++e) v[i][e] = __fmul_rn(__fmul_rn(v[i][e], scale), w[i][e]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < MAXC; ++i)
#pragma unroll
                    for (int e = 0; e < 16; ++e) v[i][e] = __fmul_rn(__fmul_rn(v[i][e], scale), w[i][e]);
            }
        }
        int8_t *qs = (int8_t *)lds;
        float *d = (float *)(lds + K);
        int16_t *bs = (int16_t *)(lds + K + K / 256 * 4);
#ifndef KCPP_PROBE_NOQUANT
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = tid + NT * i;
            if (c < nchunk) q8k_quant16(v[i], c & 15, qs + (c >> 4) * 256, d + (c >> 4), bs + (c >> 4) * 16);
        }
#else   // timing probe only (wrong results, finite: an all-zero activation): the prologue without its quantization
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = tid + NT * i;
            if (c < nchunk) {
                *(uint4 *)(qs + 16 * c) = make_uint4(v[i][0] == 1234.5f, 0, 0, 0);
                if ((c & 15) == 0) d[c >> 4] = 0.0f;
                bs[c] = 0;
            }
        }
#endif
        LP_STAMP(11);
        __syncthreads();
        LP_STAMP(12);
#undef LP_STAMP
    }
};


// quantized activation (M = 1, <= 20 KB, multiple of 16 B) -> LDS through registers
struct ActCopy {
    uint4 r[5];
    __device__ __forceinline__ void load(const uint8_t *act, int abytes) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = min(((int)threadIdx.x + 256 * i) * 16, abytes - 16);
            r[i] = *(const uint4 *)(act + o);
        }
    }
    __device__ __forceinline__ void store(uint8_t *lds, int abytes) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = ((int)threadIdx.x + 256 * i) * 16;
            if (o < abytes) *(uint4 *)(lds + o) = r[i];
        }
        __syncthreads();
    }
};

// column c of a Q8_K activation buffer with Mt columns (qs [Mt][K] ++ d [Mt][K/256] ++ bsums [Mt][K/16]) ->
// the single-column LDS image qs[K] ++ d[K/256] ++ bsums[K/16]; NT threads, K <= NT * QPT * 16 (and the
// K / 256 + K / 32 scale words <= NT * SPT): 256 threads x (4, 2) cover K 16384, 512 x (4, 3) K 32768 (XL)
template <int NT = 256, int QPT = 4, int SPT = 2>
struct ActCopyCol {
    uint4 q[QPT];
    uint32_t s[SPT];
    __device__ __forceinline__ void load(const uint8_t *act, int K, int64_t Mt, int64_t c) {
        const int tid = threadIdx.x, nq = K / 16, ns = K / 256 + K / 32;
        const uint8_t *qs = act + c * K;
        const uint32_t *d = (const uint32_t *)(act + Mt * K) + c * (K / 256);
        const uint32_t *bs = (const uint32_t *)(act + Mt * K + Mt * (K / 256) * 4) + c * (K / 32);
#pragma unroll
        for (int i = 0; i < QPT; ++i) q[i] = *(const uint4 *)(qs + 16 * min(tid + NT * i, nq - 1));
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int j = min(tid + NT * i, ns - 1);
            s[i] = j < K / 256 ? d[j] : bs[j - K / 256];
        }
    }
    __device__ __forceinline__ void store(uint8_t *lds, int K) {
        const int tid = threadIdx.x, nq = K / 16, ns = K / 256 + K / 32;
#pragma unroll
        for (int i = 0; i < QPT; ++i)
            if (tid + NT * i < nq) *(uint4 *)(lds + 16 * (tid + NT * i)) = q[i];
#pragma unroll
        for (int i = 0; i < SPT; ++i)
            if (tid + NT * i < ns) ((uint32_t *)(lds + K))[tid + NT * i] = s[i];
        __syncthreads();
    }
};

// store R parked results of group slot_g (rows row0.. of segment seg)
template <int R, int MODE, bool AUX = false>
__device__ __forceinline__ void store_group(const DecArgs &a, int seg, int row0, const float (&slot)[R],
                                            float *aux0 = nullptr, uint16_t *auxh = nullptr, RopeP rp = RopeP{}) {
    if constexpr (MODE != 2) {
        float *Y = seg == 0 ? a.Y[0] : (seg == 1 ? a.Y[1] : a.Y[2]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float v = (MODE == 0 && a.escale) ? __fmul_rn(slot[r], a.escale[0]) : slot[r];
            if (MODE == 0 && a.pre) v = __fadd_rn(a.pre[row0 + r], v);
            if constexpr (AUX && MODE == 0) {      // the ggml plugin's MUL_MAT -> ADD: the product node's tensor too
                const float rv = a.res ? a.res[row0 + r] : 0.0f;
                if (aux0) aux0[row0 + r] = v;
                if (auxh && !rp.out) auxh[row0 + r] = f2h_rn(v);
                Y[row0 + r] = a.res ? __fadd_rn(v, rv) : v;
                if constexpr (R % 2 == 0) {
                    if (rp.out && (r & 1)) {          // MUL_MAT -> ROPE (-> CPY): the pair (row0 + r - 1, row0 + r)
                        const int row = row0 + r - 1;
                        float c, s;
                        ggml_rope_cs((float)rp.pos[0], (int64_t)((row % rp.D) / 2), rp.ff, rp.theta_scale, rp.freq_scale,
                                     rp.ext_factor, rp.attn_factor, rp.mscale_ext, rp.corr0, rp.corr1, c, s);
                        const float x0 = slot[r - 1], x1 = v;
                        const float o0 = __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, s));
                        const float o1 = __fadd_rn(__fmul_rn(x0, s), __fmul_rn(x1, c));
                        rp.out[row] = o0;
                        rp.out[row + 1] = o1;
                        if (auxh) { auxh[row] = f2h_rn(o0); auxh[row + 1] = f2h_rn(o1); }
                    }
                }
            } else {
                Y[row0 + r] = ((MODE == 0 || MODE == 3) && a.res) ? __fadd_rn(v, a.res[row0 + r]) : v;
            }
        }
    } else {
        const int role = seg == 0 ? a.role[0] : (seg == 1 ? a.role[1] : a.role[2]);
        const int p = a.pos[0];
        if (role == 2) {
#pragma unroll
            for (int r = 0; r < R; ++r) a.vc[(int64_t)p * a.ekv + row0 + r] = f2h(slot[r]);
        } else {
            const int hd = a.D / 2;
#pragma unroll
            for (int r = 0; r < R; r += 2) {          // rows (2i, 2i+1): a RoPE pair (NORM mode)
                const int row = row0 + r;
                const float2 cs = a.rope_tab[(int64_t)p * hd + (row % a.D) / 2];
                const float x0 = slot[r], x1 = slot[r + 1];
                const float o0 = __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
                const float o1 = __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x));
                const uint32_t pk = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
                if (role == 0) *(uint32_t *)(a.q16 + row) = pk;
                else *(uint32_t *)(a.kc + (int64_t)p * a.ekv + row) = pk;
            }
        }
    }
}

}  // namespace lean
