// gemv_q6k.hip -- VALU-lean single-token Q6_K mat-vec (decode): ffn_down / attn_v of the Q4_K_M
// "more bits" layers and the output head (430 MB for Llama-3-8B: the largest single read of a token).
//
// Unit = 64 elements of one super-block (ggml-common.h:321 block_q6_K; kcpp layout = structure of arrays
// [nb][192] ql|qh ++ [nb][16] scales ++ [nb] d): u -> (sb = u>>2, half h = (u>>1)&1, quarter lq = u&1),
// elements 128h + 16lq + 32p + [0,16) for planes p = 0..3 (dequantize_row_q6_K, ggml-quants.c:2978).
// Per lane the (h, lq) pair is constant (64 % 4 == 0), so only the 8 scale bytes of half h are loaded and
// the four signed scales sc[8h + lq + 2p] are two signed bit-field extracts per word.  The integer dot
// is exact: q6 in [0, 64) is a valid signed int8 operand of v_dot4_i32_i8, and the -32 offset is applied
// through the activation's 16-element sums (sum (q-32) a = sum q a - 32 bsum), as the CPU kernel does.
#include "gemv_lean.h"

namespace {

struct ActU6 {                // the lane's 4 planes x 16 int8, super-block d, 4 plane bsums
    int4 a[4];
    float d;
    int bs[4];
};
__device__ __forceinline__ void act_unit6(const uint8_t *lds, int K, int u, ActU6 &x) {
    const int sb = u >> 2, h = (u >> 1) & 1, lq = u & 1;
    const int e0 = sb * 256 + 128 * h + 16 * lq;
#pragma unroll
    for (int p = 0; p < 4; ++p) x.a[p] = *(const int4 *)(lds + e0 + 32 * p);
    x.d = ((const float *)(lds + K))[sb];
    const int16_t *bs = (const int16_t *)(lds + K + (K / 256) * 4);
#pragma unroll
    for (int p = 0; p < 4; ++p) x.bs[p] = bs[(e0 >> 4) + 2 * p];
}

struct W6 { uint4 qa, qb, qh; uint2 sc; uint32_t d; };

__device__ __forceinline__ float q6k_unit(const W6 &w, const ActU6 &x, int lq) {
    const uint32_t la[4] = {w.qa.x, w.qa.y, w.qa.z, w.qa.w};
    const uint32_t lb[4] = {w.qb.x, w.qb.y, w.qb.z, w.qb.w};
    const uint32_t hh[4] = {w.qh.x, w.qh.y, w.qh.z, w.qh.w};
    const int a0[4] = {x.a[0].x, x.a[0].y, x.a[0].z, x.a[0].w};
    const int a1[4] = {x.a[1].x, x.a[1].y, x.a[1].z, x.a[1].w};
    const int a2[4] = {x.a[2].x, x.a[2].y, x.a[2].z, x.a[2].w};
    const int a3[4] = {x.a[3].x, x.a[3].y, x.a[3].z, x.a[3].w};
    int d0 = 0, d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t p0 = (la[i] & 0x0F0F0F0Fu) | ((hh[i] << 4) & 0x30303030u);
        const uint32_t p1 = (lb[i] & 0x0F0F0F0Fu) | ((hh[i] << 2) & 0x30303030u);
        const uint32_t p2 = ((la[i] >> 4) & 0x0F0F0F0Fu) | (hh[i] & 0x30303030u);
        const uint32_t p3 = ((lb[i] >> 4) & 0x0F0F0F0Fu) | ((hh[i] >> 2) & 0x30303030u);
        d0 = sdot4((int)p0, a0[i], d0);
        d1 = sdot4((int)p1, a1[i], d1);
        d2 = sdot4((int)p2, a2[i], d2);
        d3 = sdot4((int)p3, a3[i], d3);
    }
    // sc[8h + lq + 2p]: bytes lq, lq + 2 of the half's two scale words (8 B loaded at 8h)
    const int sh = 8 * lq;
    const int s0 = __builtin_amdgcn_sbfe((int)w.sc.x, sh, 8), s1 = __builtin_amdgcn_sbfe((int)w.sc.x, sh + 16, 8);
    const int s2 = __builtin_amdgcn_sbfe((int)w.sc.y, sh, 8), s3 = __builtin_amdgcn_sbfe((int)w.sc.y, sh + 16, 8);
    const int sumi = __mul24(s0, d0 - 32 * x.bs[0]) + __mul24(s1, d1 - 32 * x.bs[1]) + __mul24(s2, d2 - 32 * x.bs[2]) +
                     __mul24(s3, d3 - 32 * x.bs[3]);
    return x.d * (h2f((uint16_t)w.d) * (float)sumi);
}

}  // namespace

// PF: prefetch the next group's weights while computing this one (two register buffers); only worth
// its registers when a wave streams several groups (gate|up, output head), not at one group per wave.
template <int IT, int R, int MODE, int PRO, int MC, int PF>
__global__ void __launch_bounds__(256) k_gemv_q6k(const DecArgs a) {
    constexpr int RR = MODE == 1 ? 2 * R : R;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = (int)a.K, upr = K / 64, nsb = K / 256;
    const int N0 = (int)a.N[0], N1 = a.nseg > 1 ? (int)a.N[1] : 0, N2 = a.nseg > 2 ? (int)a.N[2] : 0;
    const int ngroups = (N0 + N1 + N2) / R;
    const int nw = (int)gridDim.x * 4;
    const int wid = (int)blockIdx.x * 4 + wave;
    const int64_t eoff = a.eid ? (int64_t)__builtin_amdgcn_readfirstlane(a.eid[0]) * a.ebytes : 0;   // MoE slice
    const int abytes = K + K / 256 * 4 + K / 16 * 2;
    const int h = (lane >> 1) & 1, lq = lane & 1;
    const uint32_t oq = 64u * h + 16u * lq, oh = 128u + 32u * h + 16u * lq, os = 8u * h;

    auto group_rows = [&](int g, int &seg, int &row0) {
        const int r = g * R;
        seg = r < N0 ? 0 : (r < N0 + N1 ? 1 : 2);
        row0 = seg == 0 ? r : (seg == 1 ? r - N0 : r - N0 - N1);
    };
    struct Buf { W6 w[IT][RR]; };
    auto issue = [&](int g, Buf &b) {
        int seg, row0;
        group_rows(g, seg, row0);
        const uint8_t *W = (seg == 0 ? a.W[0] : (seg == 1 ? a.W[1] : a.W[2])) + eoff;
        const int64_t NB = (int64_t)nsb * (seg == 0 ? N0 : (seg == 1 ? N1 : N2));   // blocks of the tensor
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint8_t *T = (MODE == 1 && r >= R) ? a.W2 + eoff : W;
            const int64_t b0 = (int64_t)(row0 + (r % R)) * nsb;
            const uint8_t *qp = T + b0 * 192, *sp = T + NB * 192 + b0 * 16, *dp = T + NB * 208 + b0 * 2;
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const uint32_t sb = (uint32_t)(min(lane + 64 * it, upr - 1) >> 2);
                b.w[it][r].qa = ld_nt(qp + sb * 192u + oq);
                b.w[it][r].qb = ld_nt(qp + sb * 192u + oq + 32u);
                b.w[it][r].qh = ld_nt(qp + sb * 192u + oh);
                b.w[it][r].sc = *(const uint2 *)(sp + sb * 16u + os);
                b.w[it][r].d = *(const uint16_t *)(dp + sb * 2u);
            }
        }
    };

    Buf ba, bb;
    const int g0 = min(wid, ngroups - 1);
    if constexpr (PRO != 0) {
        lean::ActPro<PRO, MC> pro;
        pro.load(a);
        issue(g0, ba);
        pro.compute(a, lds);
    } else {
        lean::ActCopy cp;
        cp.load(a.act, abytes);
        issue(g0, ba);
        cp.store(lds, abytes);
    }
    ActU6 xr;
    if constexpr (IT == 1) act_unit6(lds, K, lane, xr);

    float slot[R];
#pragma unroll
    for (int r = 0; r < R; ++r) slot[r] = 0.0f;
    int slot_g = -1;
    auto compute = [&](int g, const Buf &b, int k) {
        float acc[RR];
#pragma unroll
        for (int r = 0; r < RR; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int u0 = lane + 64 * it;
            ActU6 x;
            if constexpr (IT == 1) x = xr;
            else act_unit6(lds, K, min(u0, upr - 1), x);
#pragma unroll
            for (int r = 0; r < RR; ++r) {
                const float p = q6k_unit(b.w[it][r], x, lq);
                acc[r] += (IT == 1 || u0 < upr) ? p : 0.0f;
            }
        }
#pragma unroll
        for (int r = 0; r < RR; ++r) acc[r] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_f(acc[r]))));
        const bool mine = lane == k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float v;
            if constexpr (MODE == 1) v = (acc[r] / (1.0f + expf(-acc[r]))) * acc[R + r];
            else v = acc[r];
            slot[r] = mine ? v : slot[r];
        }
        slot_g = mine ? g : slot_g;
    };
    int k = 0;
    if constexpr (PF) {
        for (int g = wid; g < ngroups; g += 2 * nw, k += 2) {
            const int g1 = g + nw, g2 = g + 2 * nw;
            issue(min(g1, ngroups - 1), bb);
            compute(g, ba, k);
            if (g1 >= ngroups) break;
            issue(min(g2, ngroups - 1), ba);
            compute(g1, bb, k + 1);
        }
    } else {
        for (int g = wid; g < ngroups; g += nw, ++k) {
            if (k) issue(g, ba);
            compute(g, ba, k);
        }
    }
    if (slot_g < 0) return;
    int seg, row0;
    group_rows(slot_g, seg, row0);
    lean::store_group<R, MODE>(a, seg, row0, slot);
}

namespace {
template <int IT, int R, int MODE, int PRO, int MC, int PF>
int launch_q6k(const DecArgs &a, hipStream_t s) {
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % R) return -5;
        ntot += a.N[i];
    }
    const int64_t groups = ntot / R;
    static const int max_blocks = getenv("KCPP_Q6K_BLOCKS") ? atoi(getenv("KCPP_Q6K_BLOCKS")) : 1024;
    int64_t nblk = std::min<int64_t>((groups + 3) / 4, max_blocks);
    nblk = std::max<int64_t>(nblk, (groups + 255) / 256);    // <= 64 groups per wave (result slots)
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    hipLaunchKernelGGL((k_gemv_q6k<IT, R, MODE, PRO, MC, PF>), dim3((unsigned)nblk), dim3(256), (size_t)abytes + 16, s, a);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
}  // namespace

// -3 = not covered (caller falls back to gemv_dec_impl.h)
extern "C" int kcpp_gemv_q6k(const void *args, int mode, int pro, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    if (a.nseg < 1 || a.nseg > 3) return -3;
    static const int r_env = getenv("KCPP_Q6K_R") ? atoi(getenv("KCPP_Q6K_R")) : 0;
    if (a.K == 4096) {
        if (mode == 0 && pro == 1) {                  // output head
            if (r_env == 1) return launch_q6k<1, 1, 0, 1, 1, 1>(a, s);
            if (r_env == 4) return launch_q6k<1, 4, 0, 1, 1, 1>(a, s);
            return launch_q6k<1, 2, 0, 1, 1, 1>(a, s);
        }
        if (mode == 2 && pro == 1) return launch_q6k<1, 2, 2, 1, 1, 0>(a, s);
        if (mode == 0 && pro == 0) return launch_q6k<1, 1, 0, 0, 1, 0>(a, s);
        if (mode == 1 && pro == 1) return launch_q6k<1, 1, 1, 1, 1, 1>(a, s);
        return -3;
    }
    if (a.K == 14336 && mode == 0 && pro == 2) return launch_q6k<4, 1, 0, 2, 4, 0>(a, s);
    return -3;
}
