// attn_dec.h -- the single-token split-KV attention body (one workgroup = one split of one kv head, 4 waves), used
// by the stand-alone decode kernel k_fa_dec4 (attn.hip).
//
// Split sp of NS owns keys [p0, p1) of [0, n_kv).  Wave w streams 16-key groups base = p0 + 16 w + 64 j: lane
// (kq = lane >> 4, sub = lane & 15) holds 16 B (8 dims) of K and of V for keys base + 4 i + kq, i < 4 -- every load
// instruction is 1 KiB contiguous per wave.  Scores: 8-dim partial dot, 16-lane DPP reduction; online softmax per
// wave in the exp2 domain (m, l wave-uniform); O: each lane accumulates its 8 dims over its row's keys, rows summed
// once at the end, waves merged in LDS.  Partials: O [H][NS][128], (m, l) [H][NS] (m = -inf for an empty split).
#pragma once
#include "kcpp_common.h"

namespace fadec {

constexpr int D = 128;

template <int G>
struct State {
    float qv[G][8];
    float m[G], l[G], acc[G][8];
};

template <int G>
__device__ __forceinline__ void init(State<G> &st) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
        st.m[g] = -INFINITY; st.l[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) st.acc[g][e] = 0.0f;
    }
}

// q of the G heads of kv head hk, dims sub*8 .. +7, from 16-B words (plain or write-through loads)
template <int G>
__device__ __forceinline__ void set_q(State<G> &st, int g, const uint4 qq) {
    const uint32_t w4[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { st.qv[g][2 * e] = h2f(w4[e] & 0xFFFF); st.qv[g][2 * e + 1] = h2f(w4[e] >> 16); }
}

// q of head g from 8 f32 values (the graph form's f32 Q), rounded to f16 first as the reference's q_to_vec_dot
template <int G>
__device__ __forceinline__ void set_q_f32(State<G> &st, int g, const float4 a, const float4 b) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) st.qv[g][e] = h2f(f2h(v[e]));
}

// one 16-key group (keys base + 4 i + kq, i < 4; keys >= p1 masked), sc2 = scale * log2(e).  madd (optional): the
// row's additive mask times log2(e), -inf = key skipped (its V never enters, as the CPU skips it)
template <int G>
__device__ __forceinline__ void consume(State<G> &st, int base, int p1, int kq, float sc2, const uint4 *kk, const uint4 *vv,
                                        const float *madd = nullptr) {
    float s[G][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w4[4] = {kk[i].x, kk[i].y, kk[i].z, kk[i].w};
        float kf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { kf[2 * e] = h2f(w4[e] & 0xFFFF); kf[2 * e + 1] = h2f(w4[e] >> 16); }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float sc = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sc = fmaf(st.qv[g][e], kf[e], sc);
            s[g][i] = sc;
        }
    }
    // 16-lane row sums of all G x 4 partial dots, interleaved (independent DPP chains)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[g][i] += dpp_f<0xB1>(s[g][i]);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[g][i] += dpp_f<0x4E>(s[g][i]);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[g][i] += dpp_f<0x141>(s[g][i]);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s[g][i] += dpp_f<0x140>(s[g][i]);
            if (madd) {
                const bool ok = base + 4 * i + kq < p1 && madd[i] != -INFINITY;
                s[g][i] = ok ? __fadd_rn(s[g][i] * sc2, madd[i]) : -INFINITY;
            } else {
                s[g][i] = base + 4 * i + kq < p1 ? s[g][i] * sc2 : -INFINITY;
            }
        }
    float mx[G], al[G];
#pragma unroll
    for (int g = 0; g < G; ++g) mx[g] = fmaxf(fmaxf(s[g][0], s[g][1]), fmaxf(s[g][2], s[g][3]));
#pragma unroll
    for (int g = 0; g < G; ++g) mx[g] = xmax16(mx[g]);
#pragma unroll
    for (int g = 0; g < G; ++g) mx[g] = xmax32(mx[g]);
    float ls[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        // finite when a key of the group is valid (without a mask: key base + kq (i = 0) of row 0 is); a group whose
        // keys are all masked keeps m = -inf and contributes nothing (mr = 0 keeps exp2 away from -inf - -inf)
        const float mn = fmaxf(st.m[g], mx[g]);
        const float mr = mn == -INFINITY ? 0.0f : mn;
        al[g] = __builtin_amdgcn_exp2f(st.m[g] - mr);     // m = -inf -> 0
        ls[g] = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s[g][i] = __builtin_amdgcn_exp2f(s[g][i] - mr);   // -inf -> 0
            ls[g] += s[g][i];
        }
        st.m[g] = mn;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) ls[g] = xsum16(ls[g]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        st.l[g] = fmaf(st.l[g], al[g], xsum32(ls[g]));
#pragma unroll
        for (int e = 0; e < 8; ++e) st.acc[g][e] *= al[g];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // keys >= p1 carry weight exp2(-inf) = 0; their V words (clamped or stale rows) are zeroed so a non-finite
        // value there cannot turn 0 * v into NaN
        const bool vok = base + 4 * i + kq < p1 && (!madd || madd[i] != -INFINITY);
        const uint32_t w4[4] = {vok ? vv[i].x : 0u, vok ? vv[i].y : 0u, vok ? vv[i].z : 0u, vok ? vv[i].w : 0u};
        float vf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { vf[2 * e] = h2f(w4[e] & 0xFFFF); vf[2 * e + 1] = h2f(w4[e] >> 16); }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e = 0; e < 8; ++e) st.acc[g][e] = fmaf(s[g][i], vf[e], st.acc[g][e]);
    }
}

template <int G, int NW = 4>
struct Smem {
    float o[NW][G][D];
    float ml[NW][G][2];
    float w[NW][G], L[G];
};

// rows (kq) hold disjoint keys: park every row's 8 dims in LDS, reduce rows and the NW waves in one pass; write the
// split's partial O and (M, L) of heads hk * G + g.  FINAL (one split holds every key): write O / L to part_o as the
// attention output [H][128] instead -- what k_fa_comb4 makes of a lone split, bit for bit (weight exp2(0) = 1)
template <int G, int NW = 4, bool FINAL = false>
__device__ __forceinline__ void finish(State<G> &st, Smem<G, NW> &sm, int hk, int sp, int NS, float *__restrict__ part_o,
                                       float2 *__restrict__ part_ml) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) st.acc[g][e] = xsum16(st.acc[g][e]);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) st.acc[g][e] = xsum32(st.acc[g][e]);
    if (kq == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            *(float4 *)&sm.o[wave][g][sub * 8] = make_float4(st.acc[g][0], st.acc[g][1], st.acc[g][2], st.acc[g][3]);
            *(float4 *)&sm.o[wave][g][sub * 8 + 4] = make_float4(st.acc[g][4], st.acc[g][5], st.acc[g][6], st.acc[g][7]);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) { sm.ml[wave][g][0] = st.m[g]; sm.ml[wave][g][1] = st.l[g]; }
    }
    __syncthreads();
    if (tid < G) {                                        // per-head wave weights and the split's (M, L)
        const int g = tid;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = fmaxf(M, sm.ml[w][g][0]);
        float L = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float wt = M == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(sm.ml[w][g][0] - M);
            sm.w[w][g] = wt;
            L = fmaf(wt, sm.ml[w][g][1], L);
        }
        sm.L[g] = L;
        if (!FINAL) part_ml[(int64_t)(hk * G + g) * NS + sp] = make_float2(M, L);
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += 64 * NW) {
        const int g = i / D, d = i % D;
        float O = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) O = fmaf(sm.w[w][g], sm.o[w][g][d], O);
        if (FINAL) part_o[(int64_t)(hk * G + g) * D + d] = O / sm.L[g];
        else part_o[((int64_t)(hk * G + g) * NS + sp) * D + d] = O;
    }
}

}  // namespace fadec
