// gemv.hip -- quantized mat-vec / small-batch mat-mul for the decode path.
//
// Replaces the reference's MMVQ path (ggml/src/ggml-cuda/mmvq.cu:50-202 + vecdotq.cuh) and
// computes exactly the CPU vec_dot semantics (ggml-quants.c:3922,5519,7714,8282,8919):
// integer block dots of the *CPU* activation quantization (Q8_K per 256 for K-quants,
// Q8_0 per 32 for Q4_0/Q8_0), so only fp32 summation order differs from the oracle.
//
// Layout (MI355X-first, not a port of the 32-lane MMVQ): one wave64 owns R output rows; its
// 64 lanes split the row's K dimension into 64-element "units" (one 16-B aligned slice of
// a super-block), every lane issues dwordx4 loads, integer dots use v_dot4_i32_i8, and the
// per-row reduction is a wave64 butterfly.  NC (<= 8) activation columns share one pass
// over the weights.
#include "kcpp_common.h"
#include "kcpp_internal.h"

#include <cstring>

#include "gemv_units.h"

// ---------------------------------------------------------------- kernel
// mode 0: Y[c][n] = dot (+ res[c][n] if res)      mode 1 (GLU): Y[c][n] = silu(dot(W,n)) * dot(W2,n)
// ex (MoE, optional): the expert slice W + e * ebytes with e = ex.eid[0] read on the device (clamped to
// [0, n_exp)), and mode 0's product scaled by ex.escale[0] (the router weight: llm_build_moe_ffn's ggml_mul)
struct GemvExpert {
    const int32_t *eid;
    int64_t ebytes;
    int n_exp;
    const float *escale;
};
template <int TYPE, int R, int NC, int MODE>
__global__ void __launch_bounds__(256) k_gemv(const uint8_t *__restrict__ W, const uint8_t *__restrict__ W2,
                                              int64_t K, int64_t N, const uint8_t *__restrict__ act, int64_t M,
                                              int64_t Mtot, int64_t c0,
                                              float *__restrict__ Y, int64_t ldy, const float *res, int64_t ldr,
                                              const GemvExpert ex) {
    using A = typename ActOf<TYPE>::T;
    if (ex.eid) {
        int e = __builtin_amdgcn_readfirstlane(ex.eid[0]);
        e = e < 0 ? 0 : (e >= ex.n_exp ? ex.n_exp - 1 : e);
        W += (int64_t)e * ex.ebytes;
        if (W2) W2 += (int64_t)e * ex.ebytes;
    }
    const float esc = ex.escale ? ex.escale[0] : 1.0f;
    constexpr int E = Unit<TYPE>::ELEMS;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t row0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wave) * (MODE == 1 ? 1 : R);
    if (row0 >= N) return;
    const int64_t upr = K / E;
    const int64_t nb = K / ks_block_elems(TYPE) * N;
    const int vt = (TYPE == KT_Q4_1 || TYPE == KT_Q5_1) ? KT_Q8_1
                 : (TYPE == KT_Q4_0 || TYPE == KT_Q5_0 || TYPE == KT_Q8_0 || TYPE == KT_IQ4_NL) ? KT_Q8_0 : KT_Q8_K;
    constexpr int RR = MODE == 1 ? 2 : R;
    float acc[RR][NC];
#pragma unroll
    for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[r][c] = 0.0f;

    for (int u = lane; u < upr; u += 64) {
        Unit<TYPE> w[RR];
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            if constexpr (MODE == 1) load_unit<TYPE>(w[r], r == 0 ? W : W2, nb, row0, upr, u);
            else {
                const int64_t row = row0 + r < N ? row0 + r : N - 1;
                load_unit<TYPE>(w[r], W, nb, row, upr, u);
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < M) {
                const ActView av = act_view(vt, act, K, Mtot, c0 + c);
                A x;
                load_act(av, u, x);
#pragma unroll
                for (int r = 0; r < RR; ++r) acc[r][c] += unit_dot(w[r], u, x);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[r][c] = wave_sum(acc[r][c]);
    if (lane == 0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= M) break;
            if constexpr (MODE == 1) {
                const float g = acc[0][c], up = acc[1][c];
                Y[(c0 + c) * ldy + row0] = (g / (1.0f + expf(-g))) * up;
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int64_t n = row0 + r;
                    if (n < N) {
                        const float v = ex.escale ? __fmul_rn(acc[r][c], esc) : acc[r][c];
                        Y[(c0 + c) * ldy + n] = v + (res ? res[(c0 + c) * ldr + n] : 0.0f);
                    }
                }
            }
        }
    }
}

template <int TYPE, int R, int MODE>
static int launch_gemv_t(const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, int64_t Mtot,
                         int64_t c0, float *Y, int64_t ldy, const float *res, int64_t ldr, hipStream_t s,
                         const GemvExpert &ex) {
    const int rows_per_block = 4 * (MODE == 1 ? 1 : R);
    dim3 grid((unsigned)((N + rows_per_block - 1) / rows_per_block)), block(256);
#define KCPP_GEMV_CASE(NCV)                                                                                    \
    hipLaunchKernelGGL((k_gemv<TYPE, R, NCV, MODE>), grid, block, 0, s, (const uint8_t *)W, (const uint8_t *)W2, K, N, \
                       (const uint8_t *)act, M, Mtot, c0, Y, ldy, res, ldr, ex)
    if (M == 1) KCPP_GEMV_CASE(1);
    else if (M == 2) KCPP_GEMV_CASE(2);
    else if (M <= 4) KCPP_GEMV_CASE(4);
    else KCPP_GEMV_CASE(8);
#undef KCPP_GEMV_CASE
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// columns [c0, c0+M) of an activation buffer holding Mtot columns; eid != null: expert-indexed (see GemvExpert)
int gemv_cols(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, int64_t Mtot,
              int64_t c0, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *stream,
              const int32_t *eid, int64_t ebytes, int n_exp, const float *escale) {
    hipStream_t s = (hipStream_t)stream;
    const GemvExpert ex{eid, ebytes, n_exp, escale};
    if (M < 1 || M > 8) return -1;
    if (type == KT_Q4_K_RS || type == KT_Q5_K_RS || type == KT_Q6_K_RS) {   // decode layouts: one RS mat-vec launch per column
        if (eid) return -3;
        for (int64_t c = 0; c < M; ++c) {
            DecArgs a;
            memset(&a, 0, sizeof a);
            a.K = K; a.nseg = 1; a.W[0] = (const uint8_t *)W; a.W2 = (const uint8_t *)W2; a.N[0] = N;
            a.Y[0] = Y + c * ldy; a.res = res ? res + c * ldr : nullptr;
            a.act = (const uint8_t *)act; a.act_mtot = Mtot; a.act_col = c0 + c;
            const int rc = kcpp_gemv_rs(type, &a, mode, 0, stream);
            if (rc) return rc;
        }
        return 0;
    }
    const int64_t E = ks_block_elems(type) == 32 ? 32 : 64;
    if (K % ks_block_elems(type) || K / E < 1) return -2;
#define KCPP_T(T)                                                                   \
    case T:                                                                         \
        return mode == 1 ? launch_gemv_t<T, 1, 1>(W, W2, K, N, act, M, Mtot, c0, Y, ldy, res, ldr, s, ex) \
                         : launch_gemv_t<T, 2, 0>(W, W2, K, N, act, M, Mtot, c0, Y, ldy, res, ldr, s, ex);
    switch (type) {
        KCPP_T(KT_Q4_K)
        KCPP_T(KT_Q5_K)
        KCPP_T(KT_Q6_K)
        KCPP_T(KT_Q3_K)
        KCPP_T(KT_Q2_K)
        KCPP_T(KT_Q4_0)
        KCPP_T(KT_Q5_0)
        KCPP_T(KT_Q4_1)
        KCPP_T(KT_Q5_1)
        KCPP_T(KT_IQ4_NL)
        KCPP_T(KT_IQ4_XS)
        KCPP_T(KT_Q8_0)
        KCPP_IQ_CASES(KCPP_T)
    default: return -3;
    }
#undef KCPP_T
}

extern "C" {

// y[c][n] (+)= sum_k W[n][k] x[c][k] for c < M <= 8, act = kcpp_quantize_act output.
// mode 0: plain (+res), mode 1: GLU silu(W.x)*(W2.x)
int kcpp_gemv(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
              int64_t ldy, const float *res, int64_t ldr, int mode, void *stream) {
    if (type == KT_Q8_0_T) return -3;            // the tile layout runs through kcpp_gemm at every M (its workspace)
    return gemv_cols(type, W, W2, K, N, act, M, M, 0, Y, ldy, res, ldr, mode, stream);
}

// the same for one activation column with the weight slice of a device-resident expert id (MoE decode of the
// types without a fused decode mat-vec: Q4_1 / Q5_1 / IQ*): W + e * ebytes, e = eid[0] clamped to [0, n_exp);
// mode 0 scales the product by escale[0] when given
int kcpp_gemv_expert(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, float *Y,
                     const int32_t *eid, int64_t ebytes, int n_exp, const float *escale, int mode, void *stream) {
    if (!eid || n_exp < 1) return -1;
    return gemv_cols(type, W, W2, K, N, act, 1, 1, 0, Y, N, nullptr, 0, mode, stream, eid, ebytes, n_exp, escale);
}

}  // extern "C"
