// ops.hip -- norm / rope / KV-store / elementwise / embedding kernels.
//
// Semantics follow the CPU ops (reference ggml/src/ggml.c):
//   rms_norm  ggml_compute_forward_rms_norm_f32  :12059  (double accumulation of float x*x)
//   rope      ggml_compute_forward_rope_f32      :14272  (NORM mode, iterated theta *= theta_scale)
//   KV store  ggml_cpy f32->f16 (RNE)            src/llama.cpp:9180-9202
//   silu      x/(1+exp(-x)), then * up           src/llama.cpp:9289-9414
// Fusions (MI355X-first, one launch instead of 2-4 ggml nodes): rms_norm * w -> Q8_K quantize;
// rope(q) + rope(k) + f16 store of K/V into the cache.
#include "kcpp_common.h"
#include "kcpp_internal.h"

// ---------------------------------------------------------------- rms_norm (+ weight, + quantize)
// One workgroup per row, ne0/16 threads, 16 consecutive elements per thread: an aligned 16-lane
// group is exactly one Q8_K super-block, so the fused quantization needs only DPP steps.
// part (optional): x is first formed from KS split-K partials [KS][Mp][ne0] summed in split order plus res, exactly as
// gemm.hip k_splitk_reduce does, and stored at xout -- the reduce and the norm of the next layer step in one launch
__global__ void __launch_bounds__(1024) k_rms_norm(const float *__restrict__ x, int64_t ldx, const float *__restrict__ w,
                                                   float *__restrict__ y, int64_t ldy, uint8_t *__restrict__ qout,
                                                   int64_t ne0, int64_t nrows, float eps, int q80 = 0,
                                                   const float *__restrict__ part = nullptr, int KS = 1, int64_t Mp = 0,
                                                   float *__restrict__ xout = nullptr, const float *__restrict__ res = nullptr,
                                                   int64_t ldr = 0) {
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = (blockDim.x + 63) >> 6;
    const int64_t e0 = (int64_t)tid * 16;
    const bool active = e0 < ne0;                    // block is >= 64 threads even for small rows
    float v[16];
    if (part) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float4 g = active ? *(const float4 *)(part + r * ne0 + e0 + 4 * k) : make_float4(0, 0, 0, 0);
            for (int sp = 1; sp < KS; ++sp) {
                const float4 h = active ? *(const float4 *)(part + ((int64_t)sp * Mp + r) * ne0 + e0 + 4 * k)
                                        : make_float4(0, 0, 0, 0);
                g = make_float4(__fadd_rn(g.x, h.x), __fadd_rn(g.y, h.y), __fadd_rn(g.z, h.z), __fadd_rn(g.w, h.w));
            }
            if (res && active) {
                const float4 h = *(const float4 *)(res + r * ldr + e0 + 4 * k);
                g = make_float4(__fadd_rn(g.x, h.x), __fadd_rn(g.y, h.y), __fadd_rn(g.z, h.z), __fadd_rn(g.w, h.w));
            }
            if (active) *(float4 *)(xout + r * ldx + e0 + 4 * k) = g;
            v[4 * k] = g.x; v[4 * k + 1] = g.y; v[4 * k + 2] = g.z; v[4 * k + 3] = g.w;
        }
    } else {
        const float4 *src = (const float4 *)(x + r * ldx + e0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 f = active ? src[k] : make_float4(0, 0, 0, 0);
            v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
        }
    }
    double ss = 0.0;
#pragma unroll
    for (int e = 0; e < 16; ++e) ss += (double)__fmul_rn(v[e], v[e]);
    ss = wave_sum(ss);
    __shared__ double red[16];
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    double sum = 0.0;
    for (int i = 0; i < nw; ++i) sum += red[i];
    const float mean = (float)(sum / (double)ne0);
    const float scale = 1.0f / sqrtf(mean + eps);
    if (!active) return;
    float wv[16];
    if (w) {
        const float4 *wp = (const float4 *)(w + e0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 f = wp[k];
            wv[4 * k] = f.x; wv[4 * k + 1] = f.y; wv[4 * k + 2] = f.z; wv[4 * k + 3] = f.w;
        }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        v[e] = __fmul_rn(v[e], scale);
        if (w) v[e] = __fmul_rn(v[e], wv[e]);
    }
    if (y) {
        float4 *dst = (float4 *)(y + r * ldy + e0);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    if (qout && q80) {                                 // Q8_0 as k_quant_q80 (AVX2 semantics), a lane pair per block
        const int64_t nb = ne0 / 32, ib = tid >> 1;
        float am = 0.0f;
#pragma unroll
        for (int e = 0; e < 16; ++e) am = fmaxf(am, fabsf(v[e]));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        const float dd = am / 127.f;
        const float id = (am != 0.0f) ? 127.f / am : 0.0f;
        int qv[16], sq = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int iv = (int)rintf(__fmul_rn(v[e], id));
            qv[e] = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
            sq += qv[e];
        }
        sq += __shfl_xor(sq, 1, 64);
        int pk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            pk[k] = (qv[4 * k] & 0xFF) | ((qv[4 * k + 1] & 0xFF) << 8) | ((qv[4 * k + 2] & 0xFF) << 16) | ((qv[4 * k + 3] & 0xFF) << 24);
        if (q80 == 2) {      // the tile layout's activation (KT_Q8_0_TA, kcpp_common.h): 32-token groups, fragment order
            const int64_t g = r >> 5, tok = r & 31, ng = (nrows + 31) / 32;
            *(int4 *)((int8_t *)qout + (g * nb + ib) * 1024 + (tid & 1) * 512 + tok * 16) = make_int4(pk[0], pk[1], pk[2], pk[3]);
            if ((tid & 1) == 0) ((float *)(qout + ng * 32 * ne0))[(g * nb + ib) * 32 + tok] = h2f(f2h(dd));
            return;
        }
        int *qs = (int *)((int8_t *)qout + r * ne0 + e0);
#pragma unroll
        for (int k = 0; k < 4; ++k) qs[k] = pk[k];
        if ((tid & 1) == 0) {
            ((float *)(qout + nrows * ne0))[r * nb + ib] = h2f(f2h(dd));   // the dot uses GGML_FP16_TO_FP32(y.d)
            ((int16_t *)(qout + nrows * ne0 + nrows * nb * 4))[r * nb + ib] = (int16_t)sq;
        }
    } else if (qout) {
        const int64_t nsb = ne0 / 256, sb = tid >> 4;
        int8_t *qs = (int8_t *)qout + r * ne0 + sb * 256;
        float *d = (float *)(qout + nrows * ne0) + r * nsb + sb;
        int16_t *bs = (int16_t *)(qout + nrows * ne0 + nrows * nsb * 4) + r * (ne0 / 16) + sb * 16;
        q8k_quant16(v, tid & 15, qs, d, bs);
    }
}

// ---------------------------------------------------------------- rope + KV store
// qkv row layout per token: q [H*D] | k [HKV*D] | v [HKV*D] at stride ldqkv.
// Outputs: q_out f32 [T][H][D] (roped), q16 f16 copy (FA operand), K/V caches f16 [pos][HKV*D].
// rope_tab [pos][D/2] (cos, sin) is built on the host exactly as ggml_rope_cache_init
// (ggml.c:14246) computes it, so the rotation is bit-identical to the CPU op.
__global__ void k_rope_kv(const float *__restrict__ qkv, int64_t ldqkv, float *__restrict__ q_out,
                          uint16_t *__restrict__ q16, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
                          int H, int HKV, int D, int n_past, const int32_t *__restrict__ pos_dev,
                          const float2 *__restrict__ rope_tab) {
    const int t = blockIdx.x;
    const int p = pos_dev ? pos_dev[t] : n_past + t;
    const int half = D / 2;
    const int npairs_q = H * half, npairs_k = HKV * half;
    const float *row = qkv + (int64_t)t * ldqkv;
    const int64_t EKV = (int64_t)HKV * D;
    for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < npairs_q + npairs_k + (int)EKV; i += gridDim.y * blockDim.x) {
        if (i < npairs_q + npairs_k) {
            const bool isq = i < npairs_q;
            const int pi = isq ? i : i - npairs_q;
            const int hh = pi / half, ip = pi % half;
            const float2 cs = rope_tab[(int64_t)p * half + ip];
            const float c = cs.x, s = cs.y;
            const float *src = isq ? row + (int64_t)hh * D + 2 * ip : row + (int64_t)H * D + (int64_t)hh * D + 2 * ip;
            const float x0 = src[0], x1 = src[1];
            const float o0 = __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, s));
            const float o1 = __fadd_rn(__fmul_rn(x0, s), __fmul_rn(x1, c));
            if (isq) {
                const int64_t o = ((int64_t)t * H + hh) * D + 2 * ip;
                if (q_out) { q_out[o] = o0; q_out[o + 1] = o1; }
                if (q16) { q16[o] = f2h(o0); q16[o + 1] = f2h(o1); }
            } else {
                const int64_t o = (int64_t)p * EKV + (int64_t)hh * D + 2 * ip;
                kc[o] = f2h(o0); kc[o + 1] = f2h(o1);
            }
        } else {
            const int e = i - npairs_q - npairs_k;
            vc[(int64_t)p * EKV + e] = f2h(row[(int64_t)(H + HKV) * D + e]);
        }
    }
}

// ---------------------------------------------------------------- elementwise / embedding
__global__ void k_add(float *__restrict__ y, const float *__restrict__ a, const float *__restrict__ b, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __fadd_rn(a[i], b[i]);
}
__global__ void k_silu_mul(float *__restrict__ y, const float *__restrict__ g, const float *__restrict__ u, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { const float x = g[i]; y[i] = (x / (1.0f + expf(-x))) * u[i]; }
}


// K-shift of a layer's cache rows (llama.cpp build_k_shift + ggml_compute_forward_rope_f16, mode NORM; koboldcpp
// context shifting, gpttype_adapter.cpp:1504-1571): ks = f16(rope_f32(f32(kc), cs)) per adjacent pair, vs = vc.
// rows = positions x n_head_kv, D elements each; cs = (cos, sin) per pair for the shift distance.
__global__ void k_kv_shift(const uint32_t *__restrict__ kc, const uint32_t *__restrict__ vc, uint32_t *__restrict__ ks,
                           uint32_t *__restrict__ vs, int64_t npairs, int half_d, const float2 *__restrict__ cs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const uint32_t kk = kc[i];
    const float2 c = cs[i % half_d];
    const float x0 = h2f((uint16_t)(kk & 0xFFFF)), x1 = h2f((uint16_t)(kk >> 16));
    const uint16_t y0 = f2h(__fsub_rn(__fmul_rn(x0, c.x), __fmul_rn(x1, c.y)));
    const uint16_t y1 = f2h(__fadd_rn(__fmul_rn(x0, c.y), __fmul_rn(x1, c.x)));
    ks[i] = (uint32_t)y0 | ((uint32_t)y1 << 16);
    vs[i] = vc[i];
}

extern "C" {

int kcpp_rms_norm(const float *x, int64_t ldx, const float *w, float *y, int64_t ldy, void *q8k_out, int64_t ne0,
                  int64_t nrows, float eps, void *stream) {
    if (ne0 % 256 || ne0 > 16384) return -1;
    const unsigned nthr = (unsigned)(ne0 / 16 < 64 ? 64 : ne0 / 16);
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned)nrows), dim3(nthr), 0, (hipStream_t)stream, x, ldx, w, y,
                       ldy, (uint8_t *)q8k_out, ne0, nrows, eps);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// split-K partials [KS][Mp][ne0] (+ res) -> x (stored at x, row stride ldx) -> rms_norm * w -> the Q8_K activation:
// k_splitk_reduce followed by kcpp_rms_norm(x, ..., q8k_out), bit for bit, in one launch
int kcpp_reduce_rms_norm(const float *part, int KS, int64_t Mp, const float *res, int64_t ldr, float *x, int64_t ldx,
                         const float *w, void *q8k_out, int64_t ne0, int64_t nrows, float eps, void *stream) {
    if (ne0 % 256 || ne0 > 16384 || !part || KS < 1 || !x || !q8k_out) return -1;
    const unsigned nthr = (unsigned)(ne0 / 16 < 64 ? 64 : ne0 / 16);
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned)nrows), dim3(nthr), 0, (hipStream_t)stream, (const float *)x, ldx, w,
                       (float *)nullptr, (int64_t)0, (uint8_t *)q8k_out, ne0, nrows, eps, 0, part, KS, Mp, x, res, ldr);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_rms_norm_q80(const float *x, int64_t ldx, const float *w, void *q80_out, int64_t ne0, int64_t nrows, float eps,
                      void *stream) {
    if (ne0 % 256 || ne0 > 16384 || !q80_out) return -1;
    const unsigned nthr = (unsigned)(ne0 / 16 < 64 ? 64 : ne0 / 16);
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned)nrows), dim3(nthr), 0, (hipStream_t)stream, x, ldx, w, (float *)nullptr,
                       (int64_t)0, (uint8_t *)q80_out, ne0, nrows, eps, 1);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// rms_norm * w -> the KT_Q8_0_TA activation of KT_Q8_0_T weights (same values as kcpp_rms_norm_q80)
int kcpp_rms_norm_q80t(const float *x, int64_t ldx, const float *w, void *q80t_out, int64_t ne0, int64_t nrows, float eps,
                       void *stream) {
    if (ne0 % 256 || ne0 > 16384 || !q80t_out) return -1;
    const unsigned nthr = (unsigned)(ne0 / 16 < 64 ? 64 : ne0 / 16);
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned)nrows), dim3(nthr), 0, (hipStream_t)stream, x, ldx, w, (float *)nullptr,
                       (int64_t)0, (uint8_t *)q80t_out, ne0, nrows, eps, 2);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_rope_kv(const float *qkv, int64_t ldqkv, float *q_out, uint16_t *q16, uint16_t *kc, uint16_t *vc, int T, int H,
                 int HKV, int D, int n_past, const int32_t *pos_dev, const void *rope_tab, void *stream) {
    const int items = H * D / 2 + HKV * D / 2 + HKV * D;
    hipLaunchKernelGGL(k_rope_kv, dim3((unsigned)T, (unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream, qkv,
                       ldqkv, q_out, q16, kc, vc, H, HKV, D, n_past, pos_dev, (const float2 *)rope_tab);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_kv_shift_rows(const uint16_t *kc, const uint16_t *vc, uint16_t *ks, uint16_t *vs, int64_t rows, int D,
                       const float *cs, void *stream) {
    if (D % 2 || rows < 0) return -1;
    const int64_t np = rows * D / 2;
    if (np == 0) return 0;
    hipLaunchKernelGGL(k_kv_shift, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, (hipStream_t)stream, (const uint32_t *)kc,
                       (const uint32_t *)vc, (uint32_t *)ks, (uint32_t *)vs, np, D / 2, (const float2 *)cs);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_add(float *y, const float *a, const float *b, int64_t n, void *stream) {
    hipLaunchKernelGGL(k_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y, a, b, n);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
int kcpp_silu_mul(float *y, const float *g, const float *u, int64_t n, void *stream) {
    hipLaunchKernelGGL(k_silu_mul, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y, g, u, n);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
