// moe.hip -- mixture-of-experts pieces around the expert mat-vecs / GEMMs (GGML_OP_MUL_MAT_ID path).
//
// Reference: llm_build_moe_ffn (src/llama.cpp:9416-9520) and its CUDA execution ggml_cuda_mul_mat_id
// (ggml/src/ggml-cuda.cu:2003-2139), which copies the expert ids to the host and synchronizes on every
// MoE mat-mul.  Here:
//   * k_moe_route: router logits (F16 weights: the activation rounded to f16 first, as the CPU's
//     vec_dot_f16 does; or F32), softmax (ggml_float sum), top-k by the CPU argsort's exchange order,
//     weights normalized by their sum -- one workgroup per token (wave w: experts w, w+4, ..., all loads of
//     an expert in flight at once), results stay on the device;
//   * decode reads the expert id inside the expert mat-vec kernels (DecArgs.eid), so a whole token
//     remains one hipGraph replay with no host round trip;
//   * prefill groups tokens per expert on the host (one sync per layer, like the reference) and runs
//     each expert as a dense GEMM over its gathered rows; k_moe_scatter writes w * out into the token's
//     top-k slot, and k_moe_combine sums the slots in top-k order and adds the residual
//     (ggml_add chain over the weighted experts view, then ggml_add(moe_out, ffn_inp)).
#include "kcpp_common.h"
#include "kcpp_internal.h"

#define MOE_MAX_EXPERT 64

// NORM: x is the residual stream and the router input is rms_norm(x) * nw computed here exactly as k_rms_norm
// does for K <= 4096 (same thread -> element map, double partial sums in the same order), one launch less
template <int WT, bool NORM = false>
__global__ void __launch_bounds__(256) k_moe_route(const float *__restrict__ x, int64_t ldx, const void *__restrict__ w,
                                                   int K, int NE, int NU, int32_t *__restrict__ ids,
                                                   float *__restrict__ wts, const float *__restrict__ nw = nullptr,
                                                   float eps = 0.0f) {
    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float *xr = x + (int64_t)t * ldx;
    __shared__ float s_logit[MOE_MAX_EXPERT];
    __shared__ float s_part[4][8];
    if (NE <= 8) {
        // all experts at once: thread tid owns elements 16 tid .. +15 of every 4096-element chunk, the loads of
        // all NE router rows in flight together (one memory round trip per chunk)
        float acc[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        float nscale = 1.0f;
        // NORM (K <= 4096, one chunk): the router rows' loads go out first -- they do not wait for the norm -- so
        // the weight and residual round trips overlap
        float4 wpre[NORM ? 8 : 1][4], gpre[4];
        if constexpr (NORM) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                gpre[u] = 16 * tid + 4 * u < K ? *(const float4 *)(nw + 16 * tid + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int e = 0; e < 8; ++e)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = 16 * tid + 4 * u;
                    wpre[e][u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (e < NE && i < K) {
                        if constexpr (WT == KT_F16) {
                            const uint2 h = *(const uint2 *)((const uint16_t *)w + (int64_t)e * K + i);
                            wpre[e][u] = make_float4(h2f(h.x & 0xFFFF), h2f(h.x >> 16), h2f(h.y & 0xFFFF), h2f(h.y >> 16));
                        } else {
                            wpre[e][u] = *(const float4 *)((const float *)w + (int64_t)e * K + i);
                        }
                    }
                }
        }
        if constexpr (NORM) {                            // K <= 4096: one chunk, elements 16 tid .. +15
            double ss = 0.0;
            if (16 * tid < K) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4 f = *(const float4 *)(xr + 16 * tid + 4 * u);
                    ss += (double)__fmul_rn(f.x, f.x); ss += (double)__fmul_rn(f.y, f.y);
                    ss += (double)__fmul_rn(f.z, f.z); ss += (double)__fmul_rn(f.w, f.w);
                }
            }
            ss = wave_sum(ss);
            __shared__ double red[4];
            if (lane == 0) red[wave] = ss;
            __syncthreads();
            double sum = 0.0;
            for (int i = 0; i < 4; ++i) sum += red[i];
            const float mean = (float)(sum / (double)K);
            nscale = 1.0f / sqrtf(mean + eps);
        }
        for (int i0 = 16 * tid; i0 < K; i0 += 4096) {
            float4 xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                xv[u] = i0 + 4 * u < K ? *(const float4 *)(xr + i0 + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (NORM) {
                    if (i0 + 4 * u < K) {
                        const float4 g = gpre[u];
                        xv[u] = make_float4(__fmul_rn(__fmul_rn(xv[u].x, nscale), g.x), __fmul_rn(__fmul_rn(xv[u].y, nscale), g.y),
                                            __fmul_rn(__fmul_rn(xv[u].z, nscale), g.z), __fmul_rn(__fmul_rn(xv[u].w, nscale), g.w));
                    }
                }
                if constexpr (WT == KT_F16)   // ggml converts src1 to the F16 vec_dot_type
                    xv[u] = make_float4(h2f(f2h_rn(xv[u].x)), h2f(f2h_rn(xv[u].y)), h2f(f2h_rn(xv[u].z)), h2f(f2h_rn(xv[u].w)));
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (e >= NE) break;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = i0 + 4 * u;
                    if (i >= K) break;
                    float4 wv;
                    if constexpr (NORM) {
                        wv = wpre[e][u];
                    } else if constexpr (WT == KT_F16) {
                        const uint2 h = *(const uint2 *)((const uint16_t *)w + (int64_t)e * K + i);
                        wv = make_float4(h2f(h.x & 0xFFFF), h2f(h.x >> 16), h2f(h.y & 0xFFFF), h2f(h.y >> 16));
                    } else {
                        wv = *(const float4 *)((const float *)w + (int64_t)e * K + i);
                    }
                    acc[e] = fmaf(xv[u].x, wv.x, acc[e]);
                    acc[e] = fmaf(xv[u].y, wv.y, acc[e]);
                    acc[e] = fmaf(xv[u].z, wv.z, acc[e]);
                    acc[e] = fmaf(xv[u].w, wv.w, acc[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (e >= NE) break;
            const float v = wave_sum(acc[e]);
            if (lane == 0) s_part[wave][e] = v;
        }
        __syncthreads();
        if (tid < NE) s_logit[tid] = (s_part[0][tid] + s_part[1][tid]) + (s_part[2][tid] + s_part[3][tid]);
    } else {
    // wave w: experts w, w+4, ...; lane: 4 consecutive elements per 256-element step, 4 steps in flight
    for (int e = wave; e < NE; e += 4) {
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int i0 = 4 * lane; i0 < K; i0 += 1024) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + 256 * u;
                if (i >= K) break;
                float4 xv = *(const float4 *)(xr + i);
                float4 wv;
                if constexpr (WT == KT_F16) {
                    // ggml converts src1 to the F16 vec_dot_type
                    xv = make_float4(h2f(f2h_rn(xv.x)), h2f(f2h_rn(xv.y)), h2f(f2h_rn(xv.z)), h2f(f2h_rn(xv.w)));
                    const uint2 h = *(const uint2 *)((const uint16_t *)w + (int64_t)e * K + i);
                    wv = make_float4(h2f(h.x & 0xFFFF), h2f(h.x >> 16), h2f(h.y & 0xFFFF), h2f(h.y >> 16));
                } else {
                    wv = *(const float4 *)((const float *)w + (int64_t)e * K + i);
                }
                acc[u] = fmaf(xv.x, wv.x, acc[u]);
                acc[u] = fmaf(xv.y, wv.y, acc[u]);
                acc[u] = fmaf(xv.z, wv.z, acc[u]);
                acc[u] = fmaf(xv.w, wv.w, acc[u]);
            }
        }
        const float a = wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
        if (lane == 0) s_logit[e] = a;
    }
    }
    __syncthreads();
    if (tid != 0) return;
    if (NE <= 8) {      // register arrays (constant indices after unrolling; the generic path keeps p / idx in scratch)
        moe_topk8(s_logit, NE, NU, ids + t * NU, wts + t * NU);
        return;
    }
    float p[MOE_MAX_EXPERT];
    float mx = -INFINITY;
    for (int e = 0; e < NE; ++e) {
        p[e] = s_logit[e];
        mx = fmaxf(mx, p[e]);
    }
    double sum = 0.0;                                    // ggml_vec_soft_max_f32: ggml_float sum
    for (int e = 0; e < NE; ++e) { p[e] = expf(p[e] - mx); sum += (double)p[e]; }
    const float inv = (float)(1.0 / sum);
    for (int e = 0; e < NE; ++e) p[e] *= inv;
    int idx[MOE_MAX_EXPERT];
    for (int e = 0; e < NE; ++e) idx[e] = e;
    for (int j = 0; j < NU; ++j)                         // argsort descending (exchange order), first NU
        for (int k = j + 1; k < NE; ++k)
            if (p[idx[j]] < p[idx[k]]) { const int tmp = idx[j]; idx[j] = idx[k]; idx[k] = tmp; }
    double ws = 0.0;
    for (int j = 0; j < NU; ++j) ws += (double)p[idx[j]];
    const float wsum = (float)ws;
    for (int j = 0; j < NU; ++j) {
        ids[t * NU + j] = idx[j];
        wts[t * NU + j] = p[idx[j]] / wsum;
    }
}

__global__ void k_moe_gather(const float *__restrict__ src, int64_t lds, const int32_t *__restrict__ rows, int n,
                             int64_t E, float *__restrict__ dst) {
    const int i = blockIdx.y;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && c < E) dst[(int64_t)i * E + c] = src[(int64_t)rows[i] * lds + c];
}

__global__ void k_moe_scatter(float *__restrict__ dst, int64_t ldd, const float *__restrict__ src,
                              const int32_t *__restrict__ rows, const float *__restrict__ w, int n, int64_t E) {
    const int i = blockIdx.y;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && c < E) {
        const float v = src[(int64_t)i * E + c];
        dst[(int64_t)rows[i] * ldd + c] = w ? __fmul_rn(v, w[i]) : v;          // w null: plain row scatter
    }
}

// x[t] = ((slot0[t] + slot1[t]) + ...) + x[t]
__global__ void k_moe_combine(float *__restrict__ x, const float *__restrict__ slots, int64_t slot_stride, int nu,
                              int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float acc = slots[i];
    for (int j = 1; j < nu; ++j) acc = __fadd_rn(acc, slots[j * slot_stride + i]);
    x[i] = __fadd_rn(acc, x[i]);
}

extern "C" {

int kcpp_moe_route_norm(const float *x, int64_t ldx, const float *norm_w, float eps, const void *w_router, int wtype,
                        int64_t K, int n_expert, int k, int32_t *ids, float *weights, int T, void *stream) {
    if (n_expert < 1 || n_expert > 8 || k < 1 || k > n_expert || K > 4096 || K % 16 || ldx % 4) return -3;
    hipStream_t s = (hipStream_t)stream;
    if (wtype == KT_F16)
        hipLaunchKernelGGL((k_moe_route<KT_F16, true>), dim3(T), dim3(256), 0, s, x, ldx, w_router, (int)K, n_expert, k, ids,
                           weights, norm_w, eps);
    else if (wtype == KT_F32)
        hipLaunchKernelGGL((k_moe_route<KT_F32, true>), dim3(T), dim3(256), 0, s, x, ldx, w_router, (int)K, n_expert, k, ids,
                           weights, norm_w, eps);
    else
        return -3;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_moe_route(const float *x, int64_t ldx, const void *w_router, int wtype, int64_t K, int n_expert, int k,
                   int32_t *ids, float *weights, int T, void *stream) {
    if (n_expert < 1 || n_expert > MOE_MAX_EXPERT || k < 1 || k > n_expert) return -1;
    if (K % 4 || ldx % 4) return -1;                    // float4 / 4-half loads
    hipStream_t s = (hipStream_t)stream;
    if (wtype == KT_F16)
        hipLaunchKernelGGL((k_moe_route<KT_F16, false>), dim3(T), dim3(256), 0, s, x, ldx, w_router, (int)K, n_expert, k, ids, weights);
    else if (wtype == KT_F32)
        hipLaunchKernelGGL((k_moe_route<KT_F32, false>), dim3(T), dim3(256), 0, s, x, ldx, w_router, (int)K, n_expert, k, ids, weights);
    else
        return -3;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_moe_gather(const float *src, int64_t lds, const int32_t *rows, int n, int64_t E, float *dst, void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_moe_gather, dim3((unsigned)((E + 255) / 256), n), dim3(256), 0, (hipStream_t)stream, src, lds,
                       rows, n, E, dst);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_moe_scatter(float *dst, int64_t ldd, const float *src, const int32_t *rows, const float *w, int n, int64_t E,
                     void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_moe_scatter, dim3((unsigned)((E + 255) / 256), n), dim3(256), 0, (hipStream_t)stream, dst, ldd,
                       src, rows, w, n, E);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_moe_combine(float *x, const float *slots, int64_t slot_stride, int k, int64_t n, void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_moe_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, slots,
                       slot_stride, k, n);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
