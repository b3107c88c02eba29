// gemv_dec_impl.h -- the single-token decode mat-vec with its neighbours fused in.
// Included once per quant type by gemv_dec_<type>.hip (parallel compilation).
//
// The reference runs, per layer, rms_norm -> mul -> quantize_q8_1 -> mul_mat_vec_q (x3) -> rope (x2)
// -> cpy K/V into the cache as separate ggml nodes, each a kernel launch (ggml-cuda.cu:2145-2349,
// norm.cu:101, quantize.cu:4, mmvq.cu:50, rope.cu:31, cpy.cu:34).  On MI355X a decode token is
// launch/latency bound before it is bandwidth bound, so one launch here does:
//   prologue  (PRO=1) rms_norm(x)*w -> Q8_K (or Q8_0) activation, computed per workgroup into LDS
//             while the workgroup's first weight loads are already in flight;  (PRO=2) quantize
//             only (ffn_down input);  (PRO=0) activation already quantized in global memory.
//   body      up to three weight segments of one quant type (e.g. wq|wk|wv), R rows per wave,
//             the same integer unit dots as gemv.hip (CPU vec_dot semantics).
//   epilogue  MODE 0: y (+ residual);  MODE 1: silu(gate)*up;  MODE 2: RoPE (table built exactly
//             like ggml_rope_cache_init) + f16 store of q, and of K/V straight into the cache.
#pragma once
#include "gemv_units.h"
#include "kcpp_internal.h"

#include <algorithm>
#include <cstdlib>



__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    return xsum32(xsum16(v));
}

// Q8_0 quantization (AVX2 quantize_row_q8_0, ggml-quants.c:940-1000) of 16 elements held by one lane,
// two lanes per 32-block.  Writes qs (16 B), and lane-even writes d (f16-rounded, as float) and asum.
__device__ __forceinline__ void q80_quant16(const float (&v)[16], int l16, int8_t *qs16, float *dblk, int16_t *sblk) {
    float am = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) am = fmaxf(am, fabsf(v[e]));
    am = fmaxf(am, dpp_f<0xB1>(am));                 // partner lane (xor 1) holds the other half
    const float d = am / 127.f;
    const float id = (am != 0.0f) ? 127.f / am : 0.0f;
    int q[16], s = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int iv = (int)rintf(__fmul_rn(v[e], id));
        q[e] = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
        s += q[e];
    }
    s += dpp_i<0xB1>(s);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)(q[4 * k] & 0xFF) | ((uint32_t)(q[4 * k + 1] & 0xFF) << 8) |
               ((uint32_t)(q[4 * k + 2] & 0xFF) << 16) | ((uint32_t)(q[4 * k + 3] & 0xFF) << 24);
    *(uint4 *)qs16 = make_uint4(w[0], w[1], w[2], w[3]);
    if ((l16 & 1) == 0) { *dblk = h2f(f2h(d)); *sblk = (int16_t)s; }
}

// activation prologue into LDS: layout identical to the global act buffer with M = 1.
// Single pass: each thread keeps its <= MAXC chunks of 16 inputs in registers across the
// sum-of-squares block reduction (rms_norm, ggml.c:12059-12103) and the quantization.
template <int VT, int PRO, int MAXC>
__device__ __forceinline__ void prologue(const DecArgs &a, uint8_t *lds) {
    // MAXC chunks of 16 per thread: K <= 256 * 16 * MAXC
    const int tid = threadIdx.x;
    const int64_t K = a.K;
    const int nchunk = (int)(K / 16);
    float v[MAXC][16];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = tid + 256 * i;
        if (c < nchunk) {
            const float4 *p = (const float4 *)(a.x + 16 * (int64_t)c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 f = p[k];
                v[i][4 * k] = f.x; v[i][4 * k + 1] = f.y; v[i][4 * k + 2] = f.z; v[i][4 * k + 3] = f.w;
            }
        }
    }
    if constexpr (PRO == 1) {
        double ss = 0.0;
#pragma unroll
        for (int i = 0; i < MAXC; ++i)
            if (tid + 256 * i < nchunk) {
#pragma unroll
                for (int e = 0; e < 16; ++e) ss += (double)__fmul_rn(v[i][e], v[i][e]);
            }
        ss = wave_sum_d(ss);
        __shared__ double red[4];
        if ((tid & 63) == 0) red[tid >> 6] = ss;
        __syncthreads();
        const double sum = red[0] + red[1] + red[2] + red[3];
        const float mean = (float)(sum / (double)K);
        const float scale = 1.0f / sqrtf(mean + a.eps);   // ggml.c:12089
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = tid + 256 * i;
            if (c < nchunk) {
                const float4 *wp = (const float4 *)(a.nw + 16 * (int64_t)c);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 f = wp[k];
                    v[i][4 * k] = __fmul_rn(__fmul_rn(v[i][4 * k], scale), f.x);
                    v[i][4 * k + 1] = __fmul_rn(__fmul_rn(v[i][4 * k + 1], scale), f.y);
                    v[i][4 * k + 2] = __fmul_rn(__fmul_rn(v[i][4 * k + 2], scale), f.z);
                    v[i][4 * k + 3] = __fmul_rn(__fmul_rn(v[i][4 * k + 3], scale), f.w);
                }
            }
        }
    }
    int8_t *qs = (int8_t *)lds;
    float *d = (float *)(lds + K);
    int16_t *bs = (int16_t *)(lds + K + (VT == KT_Q8_K ? K / 256 : K / 32) * 4);
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = tid + 256 * i;
        if (c < nchunk) {                          // uniform per aligned 16-lane group
            if constexpr (VT == KT_Q8_K) {
                const int sb = c >> 4;
                q8k_quant16(v[i], c & 15, qs + sb * 256, d + sb, bs + sb * 16);
            } else {
                q80_quant16(v[i], c & 15, qs + 16 * c, d + (c >> 1), bs + (c >> 1));
            }
        }
    }
    __syncthreads();
}

// copy an already-quantized global activation (M = 1) into LDS (PRO == 0)
__device__ __forceinline__ void act_to_lds(const uint8_t *__restrict__ act, uint8_t *lds, int64_t bytes) {
    for (int64_t i = (int64_t)threadIdx.x * 16; i < bytes; i += (int64_t)blockDim.x * 16) {
        if (i + 16 <= bytes) *(uint4 *)(lds + i) = *(const uint4 *)(act + i);
        else for (int64_t j = i; j < bytes; ++j) lds[j] = act[j];
    }
    __syncthreads();
}

// Persistent-style: each wave walks row groups g = wave_id, wave_id + n_waves, ...  All K-slices
// (IT = ceil(units_per_row / 64)) of a group's R rows are loaded at once, and the loads of group
// g + n_waves are issued before group g is computed (two register buffers), so a wave keeps
// 2 x IT x R units (48-80 B each per lane) in flight.
template <int TYPE, int R, int MODE, int PRO, int MC, int IT>
__global__ void __launch_bounds__(256) k_gemv_dec(const DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_act[];
    const int KB_BID = (int)blockIdx.x, KB_NBLK = (int)gridDim.x;
#define KB_ARGS a
#include "gemv_dec_body.inc"
#undef KB_ARGS
}

// grid and LDS of k_gemv_dec<TYPE, R, MODE, PRO, ...> for a (launch_dec_it's rule)
template <int TYPE, int R, int PRO>
static int64_t dec_grid(const DecArgs &a, size_t &lds) {
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) ntot += a.N[i];
    const int max_blocks = a.K > 4096 ? 512 : 1024;
    const int64_t groups = ntot / R;
    const int vt = (TYPE == KT_Q4_0 || TYPE == KT_Q5_0 || TYPE == KT_Q8_0 || TYPE == KT_IQ4_NL) ? KT_Q8_0 : KT_Q8_K;
    lds = PRO ? (size_t)act_bytes(vt, a.K, 1) + 16 : 0;
    return std::min<int64_t>((groups + 3) / 4, max_blocks);
}

template <int TYPE, int R, int MODE, int PRO, int MC, int IT>
static int launch_dec_it(const DecArgs &a, hipStream_t s) {
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % R) return -5;
        ntot += a.N[i];
    }
    if (PRO != 0 && a.K > 4096 * MC) return -6;
    // 1024 workgroups for K = n_embd shapes (the output head prefers more), 512 for the K = n_ff
    // quantize-prologue shape (ffn_down: 20.6 vs 26.8 us measured)
    size_t lds = 0;
    const int64_t nblk = dec_grid<TYPE, R, PRO>(a, lds);
    hipLaunchKernelGGL((k_gemv_dec<TYPE, R, MODE, PRO, MC, IT>), dim3((unsigned)nblk), dim3(256), lds, s, a);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// IT = K-slices per lane: K/E/64 (Q4_K K=4096 -> 1, K=14336 -> 4; Q4_0/Q8_0 double).
// The ffn_down prologue (PRO 2) covers K = n_ff: IT 2..8; everything else K = n_embd: IT 1..4.
template <int TYPE, int R, int MODE, int PRO, int MC>
static int launch_dec(const DecArgs &a, hipStream_t s) {
    const int64_t upr = a.K / Unit<TYPE>::ELEMS;
    const int64_t it = (upr + 63) / 64;
    if constexpr (PRO == 2) {
        if (it <= 2) return launch_dec_it<TYPE, R, MODE, PRO, MC, 2>(a, s);
        if (it <= 4) return launch_dec_it<TYPE, R, MODE, PRO, MC, 4>(a, s);
        if (it <= 8) return launch_dec_it<TYPE, R, MODE, PRO, MC, 8>(a, s);
    } else {
        if (it <= 1) return launch_dec_it<TYPE, R, MODE, PRO, MC, 1>(a, s);
        if (it <= 2) return launch_dec_it<TYPE, R, MODE, PRO, MC, 2>(a, s);
        if (it <= 4) return launch_dec_it<TYPE, R, MODE, PRO, MC, 4>(a, s);
    }
    return -8;
}

// only the (mode, prologue, rows, chunk) combinations the runtime uses are instantiated
template <int TYPE>
int dispatch_mode(const DecArgs &a, int mode, int pro, int rows_per_wave, hipStream_t s) {
    const int64_t mc = (a.K + 4095) / 4096;
    if (mode == 2) {
        if (pro != 1) return -7;
        return mc <= 1 ? launch_dec<TYPE, 2, 2, 1, 1>(a, s) : launch_dec<TYPE, 2, 2, 1, 2>(a, s);
    }
    if (mode == 1) {
        if (pro != 1) return -7;
        if (rows_per_wave >= 2) return mc <= 1 ? launch_dec<TYPE, 2, 1, 1, 1>(a, s) : launch_dec<TYPE, 2, 1, 1, 2>(a, s);
        return mc <= 1 ? launch_dec<TYPE, 1, 1, 1, 1>(a, s) : launch_dec<TYPE, 1, 1, 1, 2>(a, s);
    }
    if (pro == 0) {
        if (rows_per_wave >= 4) return launch_dec<TYPE, 4, 0, 0, 1>(a, s);
        if (rows_per_wave >= 2) return launch_dec<TYPE, 2, 0, 0, 1>(a, s);
        return launch_dec<TYPE, 1, 0, 0, 1>(a, s);
    }
    if (pro == 1) {
        if (rows_per_wave >= 2) return mc <= 1 ? launch_dec<TYPE, 2, 0, 1, 1>(a, s) : launch_dec<TYPE, 2, 0, 1, 2>(a, s);
        return mc <= 1 ? launch_dec<TYPE, 1, 0, 1, 1>(a, s) : launch_dec<TYPE, 1, 0, 1, 2>(a, s);
    }
    if (mc <= 2) return launch_dec<TYPE, 1, 0, 2, 2>(a, s);
    if (mc <= 4) return launch_dec<TYPE, 1, 0, 2, 4>(a, s);
    return launch_dec<TYPE, 1, 0, 2, 8>(a, s);
}

