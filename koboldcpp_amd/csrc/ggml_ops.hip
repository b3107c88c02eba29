// ggml_ops.hip -- general-layout (ne/nb strided) kernels for the ggml graph nodes the b1 backend
// (csrc/ggml_backend.cpp) executes outside the fused Llama runtime.  Each follows the CPU op of the
// reference (ggml/src/ggml.c) it replaces:
//   binary add/sub/mul/div  ggml_compute_forward_add/mul/div_f32 (src1 broadcast by modulo)
//   unary silu              ggml_vec_silu_f32 (x / (1 + exp(-x)))
//   cpy / dup / cont        ggml_compute_forward_dup (f32 <-> f16, RNE), element order preserved
//   scale                   ggml_compute_forward_scale_f32 :11857
//   rms_norm                ggml_compute_forward_rms_norm_f32 :12059 (ggml_float sum)
//   rope (NORM / NEOX)      ggml_compute_forward_rope_f32 :14272 + ggml_rope_cache_init :14246
//   soft_max (+mask, scale) ggml_compute_forward_soft_max_f32 :13909 (ggml_float sum)
//   argsort                 ggml_compute_forward_argsort_f32 (exchange order, ties keep CPU order)
//   sum_rows                ggml_compute_forward_sum_rows_f32 (ggml_float sum)
//   get_rows (f32 / f16)    ggml_compute_forward_get_rows_f32/_f16
//   mul_mat F16 / F32 src0  ggml_compute_forward_mul_mat with vec_dot_type F16 (src1 rounded to f16)
// Row-parallel: blockIdx.y walks the (i1, i2, i3) rows, threads walk i0, so the 64-bit index
// arithmetic is per row, not per element.
#include "kcpp_common.h"
#include "kcpp_internal.h"

struct TD {
    int64_t ne[4];
    int64_t nb[4];
};
static TD td_of(const kcpp_tdesc *t) {
    TD d;
    for (int i = 0; i < 4; ++i) { d.ne[i] = t->ne[i]; d.nb[i] = t->nb[i]; }
    return d;
}
static int64_t nrows_of(const kcpp_tdesc *t) { return t->ne[1] * t->ne[2] * t->ne[3]; }
static dim3 row_grid(int64_t ne0, int64_t nrows, int threads = 256) {
    const int64_t gx = std::min<int64_t>((ne0 + threads - 1) / threads, 64);
    return dim3((unsigned)std::max<int64_t>(gx, 1), (unsigned)std::min<int64_t>(std::max<int64_t>(nrows, 1), 65535));
}

__device__ __forceinline__ void row3(int64_t r, const int64_t *ne, int64_t &i1, int64_t &i2, int64_t &i3) {
    i1 = r % ne[1];
    const int64_t q = r / ne[1];
    i2 = q % ne[2];
    i3 = q / ne[2];
}

// ---------------------------------------------------------------- binary (src1 broadcast)
template <int OP>
__global__ void k_bin(const char *__restrict__ a, TD ta, const char *__restrict__ b, TD tb, char *__restrict__ d, TD td,
                      int64_t nrows) {
    for (int64_t r = blockIdx.y; r < nrows; r += gridDim.y) {
        int64_t i1, i2, i3;
        row3(r, td.ne, i1, i2, i3);
        const char *ar = a + i1 * ta.nb[1] + i2 * ta.nb[2] + i3 * ta.nb[3];
        const char *br = b + (i1 % tb.ne[1]) * tb.nb[1] + (i2 % tb.ne[2]) * tb.nb[2] + (i3 % tb.ne[3]) * tb.nb[3];
        char *dr = d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
        const bool bfull = tb.ne[0] == td.ne[0];
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < td.ne[0]; i0 += (int64_t)gridDim.x * blockDim.x) {
            const float x = *(const float *)(ar + i0 * ta.nb[0]);
            const float y = *(const float *)(br + (bfull ? i0 : i0 % tb.ne[0]) * tb.nb[0]);
            float v;
            if constexpr (OP == KCPP_BIN_ADD) v = __fadd_rn(x, y);
            else if constexpr (OP == KCPP_BIN_SUB) v = __fsub_rn(x, y);
            else if constexpr (OP == KCPP_BIN_MUL) v = __fmul_rn(x, y);
            else v = __fdiv_rn(x, y);
            *(float *)(dr + i0 * td.nb[0]) = v;
        }
    }
}

// ---------------------------------------------------------------- unary / scale
template <int OP>
__global__ void k_unary(const char *__restrict__ a, TD ta, char *__restrict__ d, TD td, float param, int64_t nrows) {
    for (int64_t r = blockIdx.y; r < nrows; r += gridDim.y) {
        int64_t i1, i2, i3;
        row3(r, td.ne, i1, i2, i3);
        const char *ar = a + i1 * ta.nb[1] + i2 * ta.nb[2] + i3 * ta.nb[3];
        char *dr = d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < td.ne[0]; i0 += (int64_t)gridDim.x * blockDim.x) {
            const float x = *(const float *)(ar + i0 * ta.nb[0]);
            float v;
            if constexpr (OP == KCPP_UN_SILU) v = x / (1.0f + expf(-x));
            else if constexpr (OP == KCPP_UN_SCALE) v = __fmul_rn(x, param);
            else if constexpr (OP == KCPP_UN_NEG) v = -x;
            else v = x > 0.0f ? x : 0.0f;                  // relu
            *(float *)(dr + i0 * td.nb[0]) = v;
        }
    }
}

// ---------------------------------------------------------------- cpy (f32/f16 both sides)
template <typename TS, typename TDST>
__device__ __forceinline__ TDST cvt(TS v);
template <> __device__ __forceinline__ float cvt<float, float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t cvt<float, uint16_t>(float v) { return f2h(v); }
template <> __device__ __forceinline__ float cvt<uint16_t, float>(uint16_t v) { return h2f(v); }
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, uint16_t>(uint16_t v) { return v; }

template <typename TS, typename TDST>
__global__ void k_cpy(const char *__restrict__ s, TD ts, char *__restrict__ d, TD td, int same, int64_t nrows) {
    for (int64_t r = blockIdx.y; r < nrows; r += gridDim.y) {
        int64_t i1, i2, i3;
        row3(r, ts.ne, i1, i2, i3);
        const char *sr = s + i1 * ts.nb[1] + i2 * ts.nb[2] + i3 * ts.nb[3];
        const int64_t lrow = ((i3 * ts.ne[2] + i2) * ts.ne[1] + i1) * ts.ne[0];
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < ts.ne[0]; i0 += (int64_t)gridDim.x * blockDim.x) {
            int64_t o;
            if (same) {
                o = i0 * td.nb[0] + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
            } else {                                     // same element order, other shape
                int64_t L = lrow + i0;
                const int64_t j0 = L % td.ne[0]; L /= td.ne[0];
                const int64_t j1 = L % td.ne[1]; L /= td.ne[1];
                const int64_t j2 = L % td.ne[2]; const int64_t j3 = L / td.ne[2];
                o = j0 * td.nb[0] + j1 * td.nb[1] + j2 * td.nb[2] + j3 * td.nb[3];
            }
            *(TDST *)(d + o) = cvt<TS, TDST>(*(const TS *)(sr + i0 * ts.nb[0]));
        }
    }
}

// ---------------------------------------------------------------- rms_norm (any row length)
// sum over a row of (double)(x*x): thread t accumulates elements t, t + 256, ... in ascending order (16 loads in
// flight, not one dependent load per step -- a single-row norm is one workgroup's latency chain), then the wave sums
// and ((w0 + w1) + (w2 + w3)).  256 threads; rows of nb0 bytes per element (4: contiguous).
__device__ __forceinline__ double row_sumsq(const float *xr, int64_t ne0, int64_t nb0) {
    const char *xb = (const char *)xr;
    double ss = 0.0;
    for (int64_t i0 = threadIdx.x; i0 < ne0; i0 += 256 * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int64_t i = i0 + 256 * u;
            v[u] = i < ne0 ? *(const float *)(xb + i * nb0) : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (i0 + 256 * u < ne0) ss += (double)__fmul_rn(v[u], v[u]);
    }
    ss = wave_sum(ss);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const double sum = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return sum;
}

// rows of up to 4096 (a multiple of 16): the decode mat-vec prologue's own order (lean::ActPro, PRO 1) -- thread t
// sums chunk t (elements 16t .. 16t + 15) in order, wave_sum_d, then ((w0 + w1) + w2) + w3 -- so a norm fused into
// the consumer's prologue gives these kernels' bits (ggml_backend.cpp fuse_norm_into)
__device__ __forceinline__ double row_sumsq16(const float *xr, int64_t ne0, float (&v)[16]) {
    const int tid = threadIdx.x;
    const bool live = tid < ne0 / 16;
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = live ? xr[16 * tid + e] : 0.0f;
    double ss = 0.0;
    if (live) {
#pragma unroll
        for (int e = 0; e < 16; ++e) ss += (double)__fmul_rn(v[e], v[e]);
    }
    ss = wave_sum_d(ss);
    __shared__ double red16[4];
    if ((tid & 63) == 0) red16[tid >> 6] = ss;
    __syncthreads();
    const double sum = red16[0] + red16[1] + red16[2] + red16[3];
    __syncthreads();
    return sum;
}

__global__ void __launch_bounds__(256) k_rms_norm_g(const char *__restrict__ x, TD tx, char *__restrict__ y, TD ty,
                                                    float eps, int64_t nrows) {
    for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row3(r, tx.ne, i1, i2, i3);
        const float *xr = (const float *)(x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
        float *yr = (float *)(y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
        if (tx.ne[0] % 16 == 0 && tx.ne[0] <= 4096) {
            float v[16];
            const double sum = row_sumsq16(xr, tx.ne[0], v);
            const float scale = 1.0f / sqrtf((float)(sum / (double)tx.ne[0]) + eps);
            if (threadIdx.x < tx.ne[0] / 16) {
#pragma unroll
                for (int e = 0; e < 16; ++e) yr[16 * threadIdx.x + e] = __fmul_rn(v[e], scale);
            }
            continue;
        }
        const double sum = row_sumsq(xr, tx.ne[0], 4);
        const float mean = (float)(sum / (double)tx.ne[0]);
        const float scale = 1.0f / sqrtf(mean + eps);
        for (int64_t i = threadIdx.x; i < tx.ne[0]; i += 256) yr[i] = __fmul_rn(xr[i], scale);
    }
}

// rms_norm and the MUL by a broadcast weight that follows it (build_norm, src/llama.cpp: ggml_mul(ggml_rms_norm(x),
// w)) in one launch: both nodes' outputs are written, each element the unfused pair's bits (r = x * scale rounded,
// then y = r * w rounded, the norm row before the product row per element -- an in-place y over r ends the same).
// Rows of x, r, y, w contiguous (nb[0] = 4); w broadcast over rows by modulo as k_bin.
__global__ void __launch_bounds__(256) k_rms_norm_mul_g(const char *__restrict__ x, TD tx, char *r, TD tr, char *y, TD ty,
                                                        const char *__restrict__ w, TD tw, float eps, int64_t nrows) {
    for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
        int64_t i1, i2, i3;
        row3(row, tx.ne, i1, i2, i3);
        const float *xr = (const float *)(x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
        float *rr = (float *)(r + i1 * tr.nb[1] + i2 * tr.nb[2] + i3 * tr.nb[3]);
        float *yr = (float *)(y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
        const float *wr = (const float *)(w + (i1 % tw.ne[1]) * tw.nb[1] + (i2 % tw.ne[2]) * tw.nb[2] + (i3 % tw.ne[3]) * tw.nb[3]);
        const bool wfull = tw.ne[0] == ty.ne[0];
        if (tx.ne[0] % 16 == 0 && tx.ne[0] <= 4096) {      // the mat-vec prologue's order (row_sumsq16)
            float v[16], wv[16];
            const bool live = threadIdx.x < tx.ne[0] / 16;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t i = 16 * threadIdx.x + e;
                wv[e] = live ? wr[wfull ? i : i % tw.ne[0]] : 0.0f;
            }
            const double sum = row_sumsq16(xr, tx.ne[0], v);
            const float scale = 1.0f / sqrtf((float)(sum / (double)tx.ne[0]) + eps);
            if (live) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int64_t i = 16 * threadIdx.x + e;
                    const float rv = __fmul_rn(v[e], scale);
                    rr[i] = rv;
                    yr[i] = __fmul_rn(rv, wv[e]);
                }
            }
            continue;
        }
        if (tx.ne[0] <= 256 * 16) {
            // one pass (rows up to 4096): x and w loaded once, up front; the same sums in the same order as below
            float xv[16], wv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int64_t i = threadIdx.x + 256 * u;
                xv[u] = i < tx.ne[0] ? xr[i] : 0.0f;
                wv[u] = i < tx.ne[0] ? wr[wfull ? i : i % tw.ne[0]] : 0.0f;
            }
            double ss = 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (threadIdx.x + 256 * u < tx.ne[0]) ss += (double)__fmul_rn(xv[u], xv[u]);
            ss = wave_sum(ss);
            __shared__ double red1[4];
            if ((threadIdx.x & 63) == 0) red1[threadIdx.x >> 6] = ss;
            __syncthreads();
            const double sum1 = (red1[0] + red1[1]) + (red1[2] + red1[3]);
            __syncthreads();
            const float scale1 = 1.0f / sqrtf((float)(sum1 / (double)tx.ne[0]) + eps);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int64_t i = threadIdx.x + 256 * u;
                if (i >= tx.ne[0]) break;
                const float v = __fmul_rn(xv[u], scale1);
                rr[i] = v;
                yr[i] = __fmul_rn(v, wv[u]);
            }
            continue;
        }
        const double sum = row_sumsq(xr, tx.ne[0], 4);
        const float mean = (float)(sum / (double)tx.ne[0]);
        const float scale = 1.0f / sqrtf(mean + eps);
        // 8 elements per thread in flight (x and w loaded before the stores; an in-place r / y over x reads each
        // element before its own thread writes it)
        for (int64_t i0 = threadIdx.x; i0 < tx.ne[0]; i0 += 256 * 8) {
            float xv[8], wv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + 256 * u;
                xv[u] = i < tx.ne[0] ? xr[i] : 0.0f;
                wv[u] = i < tx.ne[0] ? wr[wfull ? i : i % tw.ne[0]] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t i = i0 + 256 * u;
                if (i >= tx.ne[0]) break;
                const float v = __fmul_rn(xv[u], scale);
                rr[i] = v;
                yr[i] = __fmul_rn(v, wv[u]);
            }
        }
    }
}

// ---------------------------------------------------------------- rope
// thread = one pair (i0 = 2 ip); theta iterated from the position exactly as ggml_rope_cache_init,
// cos / sin correctly rounded through double (the CPU's glibc cosf / sinf are within 1 ulp of that).
__global__ void k_rope(const char *__restrict__ x, TD tx, char *__restrict__ y, TD ty, const int32_t *__restrict__ pos,
                       const float *__restrict__ ff, int n_dims, int neox, float freq_scale, float ext_factor,
                       float attn_factor, float mscale_ext, float corr0, float corr1, float theta_scale, int64_t nrows,
                       uint16_t *__restrict__ h16 = nullptr) {
    // h16 (the ggml plugin's ROPE -> CPY fusion): y contiguous, each value also stored as f16 at its linear index
    for (int64_t r = blockIdx.y; r < nrows; r += gridDim.y) {
        int64_t i1, i2, i3;
        row3(r, tx.ne, i1, i2, i3);
        const char *xr = x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3];
        char *yr = y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3];
        const float p = (float)pos[i2];
        for (int64_t ip = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ip < tx.ne[0] / 2; ip += (int64_t)gridDim.x * blockDim.x) {
            const int64_t i0 = 2 * ip;
            if (i0 >= n_dims) {                            // tail beyond n_dims: copied
                const float t0 = *(const float *)(xr + i0 * tx.nb[0]), t1 = *(const float *)(xr + (i0 + 1) * tx.nb[0]);
                *(float *)(yr + i0 * ty.nb[0]) = t0;
                *(float *)(yr + (i0 + 1) * ty.nb[0]) = t1;
                if (h16) { h16[r * tx.ne[0] + i0] = f2h_rn(t0); h16[r * tx.ne[0] + i0 + 1] = f2h_rn(t1); }
                continue;
            }
            float c, s;
            ggml_rope_cs(p, ip, ff, theta_scale, freq_scale, ext_factor, attn_factor, mscale_ext, corr0, corr1, c, s);
            const int64_t ia = neox ? ip : i0, ib = neox ? ip + n_dims / 2 : i0 + 1;
            const float x0 = *(const float *)(xr + ia * tx.nb[0]), x1 = *(const float *)(xr + ib * tx.nb[0]);
            const float o0 = __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, s)), o1 = __fadd_rn(__fmul_rn(x0, s), __fmul_rn(x1, c));
            *(float *)(yr + ia * ty.nb[0]) = o0;
            *(float *)(yr + ib * ty.nb[0]) = o1;
            if (h16) { h16[r * tx.ne[0] + ia] = f2h_rn(o0); h16[r * tx.ne[0] + ib] = f2h_rn(o1); }
        }
    }
}

// ---------------------------------------------------------------- soft_max (+ mask row i1 % mask_rows)
template <bool MF16>
__global__ void __launch_bounds__(256) k_soft_max(const char *__restrict__ x, TD tx, const void *__restrict__ mask,
                                                  int64_t mask_ld, int64_t mask_rows, char *__restrict__ y, TD ty,
                                                  float scale, int64_t nrows) {
    __shared__ float redf[4];
    __shared__ double redd[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row3(r, tx.ne, i1, i2, i3);
        const float *xr = (const float *)(x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
        float *yr = (float *)(y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
        const int64_t mrow = r % mask_rows;
        auto wv = [&](int64_t i) {
            float v = __fmul_rn(xr[i], scale);
            if (mask) v = __fadd_rn(v, MF16 ? h2f(((const uint16_t *)mask)[mrow * mask_ld + i])
                                            : ((const float *)mask)[mrow * mask_ld + i]);
            return v;
        };
        float mx = -INFINITY;
        for (int64_t i = threadIdx.x; i < tx.ne[0]; i += 256) mx = fmaxf(mx, wv(i));
        mx = wave_max(mx);
        if (lane == 0) redf[wave] = mx;
        __syncthreads();
        mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
        double sum = 0.0;
        for (int64_t i = threadIdx.x; i < tx.ne[0]; i += 256) {
            const float w = wv(i);
            const float e = w == -INFINITY ? 0.0f : expf(w - mx);
            yr[i] = e;
            sum += (double)e;
        }
        sum = wave_sum(sum);
        if (lane == 0) redd[wave] = sum;
        __syncthreads();
        const float inv = (float)(1.0 / ((redd[0] + redd[1]) + (redd[2] + redd[3])));
        for (int64_t i = threadIdx.x; i < tx.ne[0]; i += 256) yr[i] = __fmul_rn(yr[i], inv);
        __syncthreads();
    }
}

// ---------------------------------------------------------------- argsort / sum_rows (one thread per row)
__global__ void k_argsort(const char *__restrict__ x, TD tx, int32_t *__restrict__ d, int64_t ld, int desc,
                          int64_t nrows) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    int64_t i1, i2, i3;
    row3(r, tx.ne, i1, i2, i3);
    const float *xr = (const float *)(x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
    int32_t *dr = d + r * ld;
    const int n = (int)tx.ne[0];
    for (int j = 0; j < n; ++j) dr[j] = j;
    for (int j = 0; j < n; ++j)
        for (int k = j + 1; k < n; ++k) {
            const float a = xr[dr[j]], b = xr[dr[k]];
            if (desc ? a < b : a > b) { const int32_t t = dr[j]; dr[j] = dr[k]; dr[k] = t; }
        }
}

__global__ void k_sum_rows(const char *__restrict__ x, TD tx, char *__restrict__ y, TD ty, int64_t nrows) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    int64_t i1, i2, i3;
    row3(r, tx.ne, i1, i2, i3);
    const char *xr = x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3];
    double s = 0.0;
    for (int64_t i = 0; i < tx.ne[0]; ++i) s += (double)*(const float *)(xr + i * tx.nb[0]);
    *(float *)(y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]) = (float)s;
}

// ---------------------------------------------------------------- get_rows (f32 / f16 source -> f32)
// dst row (i10, i11, i12) = src0 row (ids[i10, i11, i12], i11, i12)
template <bool F16>
__global__ void k_get_rows_g(const char *__restrict__ s, TD ts, const char *__restrict__ ids, TD ti,
                             char *__restrict__ d, TD td, int64_t nrows) {
    for (int64_t r = blockIdx.y; r < nrows; r += gridDim.y) {
        int64_t i10, i11, i12;
        row3(r, td.ne, i10, i11, i12);           // dst dims 1..3 = ids dims 0..2
        const int64_t row = min(max((int64_t)*(const int32_t *)(ids + i10 * ti.nb[0] + i11 * ti.nb[1] + i12 * ti.nb[2]),
                                    (int64_t)0), ts.ne[1] - 1);   // clamped: a bad id cannot fault the device
        const char *sr = s + row * ts.nb[1] + i11 * ts.nb[2] + i12 * ts.nb[3];
        char *dr = d + i10 * td.nb[1] + i11 * td.nb[2] + i12 * td.nb[3];
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < td.ne[0]; i0 += (int64_t)gridDim.x * blockDim.x) {
            const float v = F16 ? h2f(*(const uint16_t *)(sr + i0 * ts.nb[0])) : *(const float *)(sr + i0 * ts.nb[0]);
            *(float *)(dr + i0 * td.nb[0]) = v;
        }
    }
}

// ---------------------------------------------------------------- mul_mat with F16 / F32 src0
// one wave per dst element (n, m, batch); src0 broadcast over src1's dims 2/3 by ratio (ggml rule)
template <bool F16, bool ROUND_X = F16>
__global__ void __launch_bounds__(256) k_mul_mat_f(const char *__restrict__ w, TD tw, const char *__restrict__ x, TD tx,
                                                   char *__restrict__ d, TD td) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t m = blockIdx.y;
    const int64_t b = blockIdx.z;                     // i12 + ne12 * i13
    if (n >= td.ne[0]) return;
    const int64_t i12 = b % tx.ne[2], i13 = b / tx.ne[2];
    const int64_t i02 = i12 / (tx.ne[2] / tw.ne[2]), i03 = i13 / (tx.ne[3] / tw.ne[3]);
    const char *wr = w + n * tw.nb[1] + i02 * tw.nb[2] + i03 * tw.nb[3];
    const char *xr = x + m * tx.nb[1] + i12 * tx.nb[2] + i13 * tx.nb[3];
    float acc = 0.0f;
    for (int64_t k = lane; k < tw.ne[0]; k += 64) {
        float xv = *(const float *)(xr + k * tx.nb[0]);
        float wv;
        if (F16) { if (ROUND_X) xv = h2f(f2h(xv)); wv = h2f(*(const uint16_t *)(wr + k * tw.nb[0])); }
        else wv = *(const float *)(wr + k * tw.nb[0]);
        acc = fmaf(xv, wv, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) *(float *)(d + n * td.nb[0] + m * td.nb[1] + i12 * td.nb[2] + i13 * td.nb[3]) = acc;
}

__global__ void k_rows_move(const char *__restrict__ src, const int64_t *__restrict__ soffs, int64_t sld,
                            char *__restrict__ dst, const int64_t *__restrict__ doffs, int64_t dld, int64_t K) {
    const int64_t i = blockIdx.y, e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= K) return;
    const float *s = (const float *)(src + (soffs ? soffs[i] : i * sld));
    float *d = (float *)(dst + (doffs ? doffs[i] : i * dld));
    d[e] = s[e];
}

extern "C" {

int kcpp_ggml_binary(int op, const void *a, const kcpp_tdesc *ta, const void *b, const kcpp_tdesc *tb, void *d,
                     const kcpp_tdesc *td, void *stream) {
    const int64_t nr = nrows_of(td);
    if (nr == 0 || td->ne[0] == 0) return 0;
    for (int i = 0; i < 4; ++i) if (tb->ne[i] < 1 || td->ne[i] % tb->ne[i]) return -1;
    const dim3 g = row_grid(td->ne[0], nr);
    hipStream_t s = (hipStream_t)stream;
#define KB(OP) hipLaunchKernelGGL(k_bin<OP>, g, dim3(256), 0, s, (const char *)a, td_of(ta), (const char *)b, td_of(tb), (char *)d, td_of(td), nr)
    switch (op) {
    case KCPP_BIN_ADD: KB(KCPP_BIN_ADD); break;
    case KCPP_BIN_SUB: KB(KCPP_BIN_SUB); break;
    case KCPP_BIN_MUL: KB(KCPP_BIN_MUL); break;
    case KCPP_BIN_DIV: KB(KCPP_BIN_DIV); break;
    default: return -2;
    }
#undef KB
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_unary(int op, const void *a, const kcpp_tdesc *ta, void *d, const kcpp_tdesc *td, float param,
                    void *stream) {
    const int64_t nr = nrows_of(td);
    if (nr == 0 || td->ne[0] == 0) return 0;
    const dim3 g = row_grid(td->ne[0], nr);
    hipStream_t s = (hipStream_t)stream;
#define KU(OP) hipLaunchKernelGGL(k_unary<OP>, g, dim3(256), 0, s, (const char *)a, td_of(ta), (char *)d, td_of(td), param, nr)
    switch (op) {
    case KCPP_UN_SILU: KU(KCPP_UN_SILU); break;
    case KCPP_UN_SCALE: KU(KCPP_UN_SCALE); break;
    case KCPP_UN_NEG: KU(KCPP_UN_NEG); break;
    case KCPP_UN_RELU: KU(KCPP_UN_RELU); break;
    default: return -2;
    }
#undef KU
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_cpy(int stype, const void *src, const kcpp_tdesc *ts, int dtype, void *dst, const kcpp_tdesc *td,
                  void *stream) {
    const int64_t nr = nrows_of(ts);
    if (nr == 0 || ts->ne[0] == 0) return 0;
    int same = 1;
    for (int i = 0; i < 4; ++i) same &= ts->ne[i] == td->ne[i];
    const dim3 g = row_grid(ts->ne[0], nr);
    hipStream_t s = (hipStream_t)stream;
    const char *sp = (const char *)src;
    char *dp = (char *)dst;
    if (stype == KT_F32 && dtype == KT_F32)
        hipLaunchKernelGGL((k_cpy<float, float>), g, dim3(256), 0, s, sp, td_of(ts), dp, td_of(td), same, nr);
    else if (stype == KT_F32 && dtype == KT_F16)
        hipLaunchKernelGGL((k_cpy<float, uint16_t>), g, dim3(256), 0, s, sp, td_of(ts), dp, td_of(td), same, nr);
    else if (stype == KT_F16 && dtype == KT_F32)
        hipLaunchKernelGGL((k_cpy<uint16_t, float>), g, dim3(256), 0, s, sp, td_of(ts), dp, td_of(td), same, nr);
    else if (stype == KT_F16 && dtype == KT_F16)
        hipLaunchKernelGGL((k_cpy<uint16_t, uint16_t>), g, dim3(256), 0, s, sp, td_of(ts), dp, td_of(td), same, nr);
    else
        return -2;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_rms_norm(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, float eps, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    hipLaunchKernelGGL(k_rms_norm_g, dim3((unsigned)std::min<int64_t>(nr, 65535)), dim3(256), 0, (hipStream_t)stream,
                       (const char *)x, td_of(tx), (char *)y, td_of(ty), eps, nr);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_rms_norm_mul(const void *x, const kcpp_tdesc *tx, void *r, const kcpp_tdesc *tr, void *y,
                           const kcpp_tdesc *ty, const float *w, const kcpp_tdesc *tw, float eps, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    if (tx->nb[0] != 4 || tr->nb[0] != 4 || ty->nb[0] != 4 || tw->nb[0] != 4) return -2;
    hipLaunchKernelGGL(k_rms_norm_mul_g, dim3((unsigned)std::min<int64_t>(nr, 65535)), dim3(256), 0, (hipStream_t)stream,
                       (const char *)x, td_of(tx), (char *)r, td_of(tr), (char *)y, td_of(ty), (const char *)w, td_of(tw),
                       eps, nr);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// host-side constants exactly as the CPU op computes them (ggml.c:14321-14324, rope_yarn :14223):
// out = {theta_scale, corr0, corr1, mscale_ext}
void kcpp_ggml_rope_consts(int n_dims, int n_ctx_orig, float freq_base, float freq_scale, float attn_factor,
                           float beta_fast, float beta_slow, float *out) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    auto corr_dim = [&](float n_rot) {
        return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float)M_PI)) / (2 * logf(freq_base));
    };
    const float start = floorf(corr_dim(beta_fast)), end = ceilf(corr_dim(beta_slow));
    out[0] = theta_scale;
    out[1] = fmaxf(0.0f, start);
    out[2] = fminf((float)(n_dims - 1), end);
    out[3] = attn_factor * (1.0f + 0.1f * logf(1.0f / freq_scale));
}

int kcpp_ggml_rope(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, const int32_t *pos,
                   const float *freq_factors, int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale,
                   float ext_factor, float attn_factor, float beta_fast, float beta_slow, void *stream) {
    return kcpp_ggml_rope_f16(x, tx, y, ty, nullptr, pos, freq_factors, n_dims, mode, n_ctx_orig, freq_base, freq_scale,
                              ext_factor, attn_factor, beta_fast, beta_slow, stream);
}

int kcpp_ggml_rope_f16(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, void *y16, const int32_t *pos,
                       const float *freq_factors, int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale,
                       float ext_factor, float attn_factor, float beta_fast, float beta_slow, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    if (n_dims > tx->ne[0] || n_dims % 2 || tx->nb[0] != 4) return -1;
    if (mode != 0 && mode != 2) return -2;
    float cst[4];
    kcpp_ggml_rope_consts(n_dims, n_ctx_orig, freq_base, freq_scale, attn_factor, beta_fast, beta_slow, cst);
    const float theta_scale = cst[0], corr0 = cst[1], corr1 = cst[2], mscale_ext = cst[3];
    const dim3 g = row_grid(tx->ne[0] / 2, nr, 64);
    hipLaunchKernelGGL(k_rope, g, dim3(64), 0, (hipStream_t)stream, (const char *)x, td_of(tx), (char *)y, td_of(ty), pos,
                       freq_factors, n_dims, mode == 2 ? 1 : 0, freq_scale, ext_factor, attn_factor, mscale_ext, corr0,
                       corr1, theta_scale, nr, (uint16_t *)y16);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_soft_max(const void *x, const kcpp_tdesc *tx, const void *mask, int mask_type, int64_t mask_ld,
                       int64_t mask_rows, void *y, const kcpp_tdesc *ty, float scale, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    const dim3 g((unsigned)std::min<int64_t>(nr, 65535));
    if (mask_rows < 1) mask_rows = 1;
    if (mask && mask_type == KT_F16)
        hipLaunchKernelGGL(k_soft_max<true>, g, dim3(256), 0, (hipStream_t)stream, (const char *)x, td_of(tx), mask,
                           mask_ld, mask_rows, (char *)y, td_of(ty), scale, nr);
    else if (!mask || mask_type == KT_F32)
        hipLaunchKernelGGL(k_soft_max<false>, g, dim3(256), 0, (hipStream_t)stream, (const char *)x, td_of(tx), mask,
                           mask_ld, mask_rows, (char *)y, td_of(ty), scale, nr);
    else
        return -2;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_argsort(const void *x, const kcpp_tdesc *tx, int32_t *d, int64_t ld, int desc, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    hipLaunchKernelGGL(k_argsort, dim3((unsigned)((nr + 63) / 64)), dim3(64), 0, (hipStream_t)stream, (const char *)x,
                       td_of(tx), d, ld, desc, nr);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_sum_rows(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, void *stream) {
    const int64_t nr = nrows_of(tx);
    if (nr == 0) return 0;
    hipLaunchKernelGGL(k_sum_rows, dim3((unsigned)((nr + 63) / 64)), dim3(64), 0, (hipStream_t)stream, (const char *)x,
                       td_of(tx), (char *)y, td_of(ty), nr);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_get_rows(int stype, const void *src, const kcpp_tdesc *ts, const int32_t *ids, const kcpp_tdesc *ti,
                       void *dst, const kcpp_tdesc *td, void *stream) {
    const int64_t nr = nrows_of(td);
    if (nr == 0) return 0;
    const dim3 g = row_grid(td->ne[0], nr);
    if (stype == KT_F32)
        hipLaunchKernelGGL(k_get_rows_g<false>, g, dim3(256), 0, (hipStream_t)stream, (const char *)src, td_of(ts),
                           (const char *)ids, td_of(ti), (char *)dst, td_of(td), nr);
    else if (stype == KT_F16)
        hipLaunchKernelGGL(k_get_rows_g<true>, g, dim3(256), 0, (hipStream_t)stream, (const char *)src, td_of(ts),
                           (const char *)ids, td_of(ti), (char *)dst, td_of(td), nr);
    else
        return -2;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_ggml_mul_mat_f(int wtype, const void *w, const kcpp_tdesc *tw, const float *x, const kcpp_tdesc *tx, float *d,
                        const kcpp_tdesc *td, void *stream) {
    if (td->ne[0] == 0 || td->ne[1] == 0) return 0;
    if (tx->ne[2] % tw->ne[2] || tx->ne[3] % tw->ne[3] || tx->ne[1] > 65535) return -1;
    const dim3 g((unsigned)((td->ne[0] + 3) / 4), (unsigned)td->ne[1], (unsigned)(tx->ne[2] * tx->ne[3]));
    if (wtype == KT_F16)
        hipLaunchKernelGGL((k_mul_mat_f<true, true>), g, dim3(256), 0, (hipStream_t)stream, (const char *)w, td_of(tw),
                           (const char *)x, td_of(tx), (char *)d, td_of(td));
    else if (wtype == KCPP_MM_F16_X32)
        hipLaunchKernelGGL((k_mul_mat_f<true, false>), g, dim3(256), 0, (hipStream_t)stream, (const char *)w, td_of(tw),
                           (const char *)x, td_of(tx), (char *)d, td_of(td));
    else if (wtype == KT_F32)
        hipLaunchKernelGGL(k_mul_mat_f<false>, g, dim3(256), 0, (hipStream_t)stream, (const char *)w, td_of(tw),
                           (const char *)x, td_of(tx), (char *)d, td_of(td));
    else
        return -2;
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// row moves of the MoE mat-mul (ggml_cuda_mul_mat_id's k_copy_src1_to_contiguous / k_copy_dst_from_contiguous,
// ggml-cuda.cu:1954-2001): dst row i = src row i, rows addressed by byte offsets (soffs / doffs) or by a stride
int kcpp_rows_move_f32(const void *src, const int64_t *soffs, int64_t sld, void *dst, const int64_t *doffs, int64_t dld,
                       int64_t K, int n, void *stream) {
    if (n <= 0 || K <= 0) return 0;
    hipLaunchKernelGGL(k_rows_move, dim3((unsigned)((K + 255) / 256), (unsigned)n), dim3(256), 0, (hipStream_t)stream,
                       (const char *)src, soffs, sld, (char *)dst, doffs, dld, K);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
