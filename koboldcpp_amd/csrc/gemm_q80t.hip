// gemm_q80t.hip -- the Q8_0 mat-mul on the tile layout KT_Q8_0_T (kcpp_common.h), every batch size from one token up.
//
// BASELINE config 3 (Llama-3-8B Q8_0, ubatches of 32 tokens) is HBM-bound: 232 MB of weights per layer for 32 tokens.
// The SoA Q8_0 layout keeps each row's blocks together, so the v_mfma_i32_32x32x32_i8 B operand of a 32-row tile
// (lane 32 h + r = row r, bytes 32 b + 16 h of block b) is 32 rows x 32 B scattered over 32 cache lines per wave
// load; staged through LDS it ran at 1.4-2.2 TB/s (k_gemm_q80s2), straight from the rows at 1.6-2.9 TB/s
// (tools/q80_pattern_probe.hip).  KT_Q8_0_T stores every (tile, block) as that operand, 1 KiB contiguous, and the
// activation (KT_Q8_0_TA) likewise per 32-token group: each wave streams its weight fragments straight into MFMA
// registers, two 4-block units in flight, no LDS staging and no barrier in the loop -- 4.4-4.9 TB/s in the same
// probe.
//
// Work split (from the weight shape only, never M, so a token's bits do not depend on the batch it came in):
//   workgroup = one 32-row tile x one K range (S = 2 ranges when the matrix has < 256 tiles) x one 32-token group;
//   its WV waves split the K range (MODE 1: waves 0 .. WV/2-1 gate, the rest up, each over the whole K);
//   per block: exact int32 block dot by the MFMA, then tot += (float)sumi * (d_w * d_x) -- ggml_vec_dot_q8_0_q8_0's
//   per-block scaling (ggml-quants.c:5519) -- in block order; waves summed in wave order through LDS; the two K
//   ranges of an S = 2 tile are added by whichever workgroup arrives second (an agent-scope ticket; a + b = b + a).
// Epilogues: MODE 0 Y (+ residual); MODE 1 h = silu(g) u, quantized straight to the KT_Q8_0_TA activation of the
// down projection (the tile's 32 rows are one Q8_0 block of h per token: k_quant_q80's rounding), or f32 h.
// Workgroup -> tile placement keeps every workgroup of a tile on one XCD (blockIdx % 8; speed only).
#include "kcpp_common.h"
#include "kcpp_internal.h"

#include <algorithm>

#ifndef Q80T_RING
#define Q80T_RING 2              // loop per mode (bit MODE set: the branch-free Q80T_P-deep ring): tools/q80t_sweep.py
#endif
#ifndef Q80T_P
#define Q80T_P 2                 // weight units in flight per wave (even: the x pair alternates with the ring slot)
#endif
#define Q80T_SMAX 8              // K ranges per tile at most (split-K tickets)
#ifndef Q80T_GLU_WV
#define Q80T_GLU_WV 4
#endif

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ i32x4 ld_frag_nt(const uint8_t *p) {   // weights: read once per launch (nt-weights)
    const v4u x = __builtin_nontemporal_load((const v4u *)p);
    return i32x4{(int)x[0], (int)x[1], (int)x[2], (int)x[3]};
}

struct Q80TArgs {
    const uint8_t *W[3];     // KT_Q8_0_T weights, segment rows back to back in the output columns (q|k|v)
    int64_t N[3];            // rows per segment, multiples of 32
    int nseg;
    const uint8_t *W2;       // MODE 1: up (gate = W[0])
    int64_t K, M;
    const uint8_t *act;      // KT_Q8_0_TA activation of the M tokens
    float *Y;                // MODE 0 output (MODE 1 without qout: f32 h)
    int64_t ldy;
    const float *res;        // MODE 0 residual
    int64_t ldr;
    uint8_t *qout;           // MODE 1: KT_Q8_0_TA activation of h (K_down = N[0])
    float *part;             // S = 2: [tile][group][split][1024] partial tiles
    unsigned *tick;          // S = 2: [tile][group] arrival tickets, zero between launches (the second arriver resets)
    int64_t ntile;           // 32-row tiles (MODE 1: of the gate)
    int S, Z;                // K ranges per tile, 32-token groups
    // MODE 0 q|k|v epilogue with rope_tab: rope(q) -> q16 [t][nq], rope(k) -> kc, v -> vc ([pos][nkv], f16) as
    // ops.hip k_rope_kv stores them; Y is not written
    const float2 *rope_tab;
    uint16_t *q16, *kc, *vc;
    const int32_t *pos;      // positions per token (graph replay), else n_past + t
    int n_past, hd;
    int64_t nq, nkv;
};

template <int MODE, int WV, bool RING = ((Q80T_RING >> MODE) & 1) != 0>
__global__ void __launch_bounds__(64 * WV) k_q80t(const Q80TArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = a.S, Z = a.Z;
    const int64_t L = blockIdx.x;
    int64_t q = L >> 3;
    const int64_t z = q % Z;
    q /= Z;
    const int split = (int)(q % S);
    const int64_t tile = (q / S) * 8 + (L & 7);
    if (tile >= a.ntile) return;
    const int64_t K = a.K, nb = K / 32, nu = nb / 4;                 // 4-block units
    // the tile's segment (q|k|v launches): local tile, output column offset, weight, rows
    int64_t tl = tile, coff = 0;
    const uint8_t *W = a.W[0];
    int64_t Ns = a.N[0];
    if (MODE == 0 && a.nseg > 1 && tl >= a.N[0] / 32) {
        tl -= a.N[0] / 32; coff = a.N[0]; W = a.W[1]; Ns = a.N[1];
        if (a.nseg > 2 && tl >= a.N[1] / 32) { tl -= a.N[1] / 32; coff += a.N[1]; W = a.W[2]; Ns = a.N[2]; }
    }
    const int64_t u0 = nu * split / S, u1 = nu * (split + 1) / S;    // this workgroup's units
    // wave w's units: MODE 0 a WV-th of the range, MODE 1 a (WV/2)-th for its matrix (gate: waves < WV/2)
    constexpr int WP = MODE == 1 ? WV / 2 : WV;
    const int wp = wave % WP;
    const int64_t wu0 = u0 + (u1 - u0) * wp / WP, wu1 = u0 + (u1 - u0) * (wp + 1) / WP;
    if (MODE == 1 && wave >= WP) W = a.W2;
    float *dxs = (float *)lds;                                       // token scales of the units [u0, u1): [block][32]
    float *red = dxs + (u1 - u0) * 128;                              // [WV][16][64] per-wave sums
    const int64_t ng = (a.M + 31) / 32;
    const uint8_t *wq = W + tl * nb * 1024 + lane * 16;              // block b at + b * 1024
    const uint8_t *wd = W + Ns * K + tl * nu * 256 + (lane & 31) * 8;   // unit u at + u * 256
    float tot[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) tot[r] = 0.0f;
    if constexpr (RING) {
        // lanes of tokens past M read their k-half's token-0 bytes (cache lines the live lanes fetch anyway: at M = 1 the
        // wave moves 32 B of activation per block, not 1 KiB) and zero them
        const bool xlive = z * 32 + (lane & 31) < a.M;
        const uint8_t *aq = a.act + z * nb * 1024 + (xlive ? lane : (lane & 32)) * 16;
        const int xm = xlive ? -1 : 0;
        // weight fragments Q80T_P units (4 blocks each) ahead of the MFMA, activation fragments (L2-resident) one unit
        // ahead; the loop body is branch-free (unit indices clamped to the wave's last unit, a clamped unit's scale zeroed)
        // so the per-block MFMA + epilogue stays one scheduling region with one accumulator live
        struct WUnit { i32x4 w[4]; uint2 d; };
        struct XUnit { i32x4 x[4]; };
        const int64_t ulast = wu1 - 1;
        f2 tot2[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) tot2[r] = f2{0.0f, 0.0f};
        auto loadw = [&](int64_t u, WUnit &U) {
            u = u < ulast ? u : ulast;
#pragma unroll
            for (int i = 0; i < 4; ++i) U.w[i] = ld_frag_nt(wq + (4 * u + i) * 1024);
            U.d = *(const uint2 *)(wd + u * 256);
        };
        auto loadx = [&](int64_t u, XUnit &X) {
            u = u < ulast ? u : ulast;
#pragma unroll
            for (int i = 0; i < 4; ++i) X.x[i] = *(const i32x4 *)(aq + (4 * u + i) * 1024) & xm;
        };
        auto comp = [&](int64_t u, const WUnit &U, const XUnit &X) {
            const bool live = u <= ulast;
            u = live ? u : ulast;
            const float dw[4] = {live ? h2f((uint16_t)(U.d.x & 0xFFFF)) : 0.0f, live ? h2f((uint16_t)(U.d.x >> 16)) : 0.0f,
                                 live ? h2f((uint16_t)(U.d.y & 0xFFFF)) : 0.0f, live ? h2f((uint16_t)(U.d.y >> 16)) : 0.0f};
            auto mf = [&](int i) {
                i32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0;
                i32x4 xv = X.x[i], wv = U.w[i];
                asm volatile("" : "+v"(xv), "+v"(wv));   // not hoisted above the previous block's epilogue
                return __builtin_amdgcn_mfma_i32_32x32x32_i8(xv, wv, acc, 0, 0, 0);
            };
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const i32x16 acc = mf(i);
                const float *sd = dxs + ((u - u0) * 4 + i) * 32 + 4 * kg;
                const f2 dw2 = {dw[i], dw[i]};
#pragma unroll
                for (int c = 0; c < 4; ++c) {                // packed f32 pairs: v_pk_mul_f32 + v_pk_fma_f32
                    const float4 d4 = *(const float4 *)(sd + 8 * c);
                    const f2 s0 = dw2 * f2{d4.x, d4.y}, s1 = dw2 * f2{d4.z, d4.w};
                    tot2[2 * c] = __builtin_elementwise_fma(f2{(float)acc[4 * c], (float)acc[4 * c + 1]}, s0, tot2[2 * c]);
                    tot2[2 * c + 1] =
                        __builtin_elementwise_fma(f2{(float)acc[4 * c + 2], (float)acc[4 * c + 3]}, s1, tot2[2 * c + 1]);
                }
#pragma unroll
                for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(tot2[r]));  // ... and its epilogue done here: one
                asm volatile("" ::: "memory");                                  // accumulator live at a time
            }
        };
        WUnit wr[Q80T_P];
        XUnit xa, xb;
        if (wu0 < wu1) {
#pragma unroll
            for (int i = 0; i < Q80T_P; ++i) loadw(wu0 + i, wr[i]);
            loadx(wu0, xa);
        }
        {   // the token scales go to LDS while the first units' fragments are in flight
            const float4 *src = (const float4 *)(a.act + ng * 32 * K) + (z * nb + 4 * u0) * 8;
            float4 *dst = (float4 *)dxs;
            for (int64_t i = tid; i < (u1 - u0) * 32; i += 64 * WV) dst[i] = src[i];
        }
        __syncthreads();
        for (int64_t u = wu0; u < wu1; u += Q80T_P) {
#pragma unroll
            for (int i = 0; i < Q80T_P; ++i) {     // unrolled: ring slot i and the x pair are static registers
                XUnit &xc = (i & 1) ? xb : xa, &xn = (i & 1) ? xa : xb;
                loadx(u + i + 1, xn);
                asm volatile("" ::: "memory");       // loads stay where they are issued (in flight across the compute)
                comp(u + i, wr[i], xc);
                loadw(u + i + Q80T_P, wr[i]);
                asm volatile("" ::: "memory");
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) { tot[2 * r] = tot2[r].x; tot[2 * r + 1] = tot2[r].y; }
    } else {
        const uint8_t *aq = a.act + z * nb * 1024 + lane * 16;
        // lanes of tokens past M read no activation (at M = 1 the wave fetches 32 B of it per block, not 1 KiB)
        const bool xlive = z * 32 + (lane & 31) < a.M;
        struct Unit { i32x4 w[4], x[4]; uint2 d; };
        auto load = [&](int64_t u, Unit &U) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                U.w[i] = ld_frag_nt(wq + (4 * u + i) * 1024);
                U.x[i] = xlive ? *(const i32x4 *)(aq + (4 * u + i) * 1024) : i32x4{0, 0, 0, 0};
            }
            U.d = *(const uint2 *)(wd + u * 256);
        };
        auto comp = [&](int64_t u, const Unit &U) {
            const float dw[4] = {h2f((uint16_t)(U.d.x & 0xFFFF)), h2f((uint16_t)(U.d.x >> 16)), h2f((uint16_t)(U.d.y & 0xFFFF)),
                                 h2f((uint16_t)(U.d.y >> 16))};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                i32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0;
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(U.x[i], U.w[i], acc, 0, 0, 0);
                const float *sd = dxs + ((u - u0) * 4 + i) * 32 + 4 * kg;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 d4 = *(const float4 *)(sd + 8 * c);
                    const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        tot[4 * c + e] = fmaf((float)acc[4 * c + e], __fmul_rn(dw[i], dv[e]), tot[4 * c + e]);
                    }
                }
            }
        };
        Unit ua, ub;
        if (wu0 < wu1) load(wu0, ua);
        if (wu0 + 1 < wu1) load(wu0 + 1, ub);
        {   // the token scales go to LDS while the first two units' fragments are in flight
            const float4 *src = (const float4 *)(a.act + ng * 32 * K) + (z * nb + 4 * u0) * 8;
            float4 *dst = (float4 *)dxs;
            for (int64_t i = tid; i < (u1 - u0) * 32; i += 64 * WV) dst[i] = src[i];
        }
        __syncthreads();
        for (int64_t u = wu0; u < wu1; u += 2) {
            if (u > wu0 && u + 1 < wu1) load(u + 1, ub);
            comp(u, ua);
            if (u + 1 >= wu1) break;
            if (u + 2 < wu1) load(u + 2, ua);
            comp(u + 1, ub);
        }
    }
    // waves summed in wave order: element (token t, row j) of lane l, r: t = (r & 3) + 8 (r >> 2) + 4 (l >> 5), j = l & 31
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = tot[r];
    __syncthreads();
    if constexpr (MODE == 1) {
        float *hs = red + WV * 1024;                                 // h [token][row]
        for (int idx = tid; idx < 1024; idx += 64 * WV) {
            float g = red[idx], u = red[WP * 1024 + idx];
#pragma unroll
            for (int w = 1; w < WP; ++w) {
                g = __fadd_rn(g, red[w * 1024 + idx]);
                u = __fadd_rn(u, red[(WP + w) * 1024 + idx]);
            }
            const int r = idx >> 6, l = idx & 63;
            const int t = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), j = l & 31;
            hs[t * 32 + j] = (g / (1.0f + expf(-g))) * u;
        }
        __syncthreads();
        if (!a.qout) {
            for (int idx = tid; idx < 1024; idx += 64 * WV) {
                const int t = idx >> 5, j = idx & 31;
                if (z * 32 + t < a.M) a.Y[(z * 32 + t) * a.ldy + tile * 32 + j] = hs[idx];
            }
            return;
        }
        // Q8_0 of h per token over the tile's 32 rows (k_quant_q80's AVX2 rounding): 8 threads per token, 4 rows each
        if (tid < 256) {
            const int t = tid >> 3, sub = tid & 7;
            const float4 v4 = *(const float4 *)(hs + t * 32 + 4 * sub);
            const float v[4] = {v4.x, v4.y, v4.z, v4.w};
            float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            am = fmaxf(am, __shfl_xor(am, 4, 64));
            const float id = (am != 0.0f) ? 127.f / am : 0.0f;
            int pk = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                int iv = (int)rintf(__fmul_rn(v[e], id));
                iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
                pk |= (iv & 0xFF) << (8 * e);
            }
            const int64_t nbh = a.ntile;                             // h's Q8_0 blocks per token
            *(int *)(a.qout + (z * nbh + tile) * 1024 + (sub >> 2) * 512 + t * 16 + 4 * (sub & 3)) = pk;
            if (sub == 0) ((float *)(a.qout + ng * 32 * (nbh * 32)))[(z * nbh + tile) * 32 + t] = h2f(f2h(am / 127.f));
        }
        return;
    } else {
        __shared__ unsigned s_old;
        if (S > 1) {
            // publish this K range's partial (write-through stores, drained), then one agent-scope ticket per workgroup;
            // the second arriver adds the other partial (MI355X_MICROARCH.md hand-off table, row 1)
            float *pp = a.part + ((tile * Z + z) * S + split) * 1024;
            for (int idx = tid; idx < 1024; idx += 64 * WV) {
                float v = red[idx];
#pragma unroll
                for (int w = 1; w < WV; ++w) v = __fadd_rn(v, red[w * 1024 + idx]);
                __hip_atomic_store(pp + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            unsigned *tk = a.tick + tile * 64 + z;
            if (tid == 0) s_old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            if (s_old != (unsigned)(S - 1)) return;                   // the last arriver sums the S ranges
            if (tid == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const float *po = a.part + (tile * Z + z) * S * 1024;
        for (int idx = tid; idx < 1024; idx += 64 * WV) {
            float v = red[idx];
#pragma unroll
            for (int w = 1; w < WV; ++w) v = __fadd_rn(v, red[w * 1024 + idx]);
            if (S > 1) {     // in range order whichever workgroup arrived last (S = 2: a + b = b + a)
                const float own = v;
                v = split == 0 ? own : __hip_atomic_load(po + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (int k = 1; k < S; ++k)
                    v = __fadd_rn(v, k == split ? own : __hip_atomic_load(po + k * 1024 + idx, __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_AGENT));
            }
            const int r = idx >> 6, l = idx & 63;
            const int64_t t = z * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            const int64_t n = coff + tl * 32 + (l & 31);
            if (a.rope_tab) {
                // k_rope_kv's rotation of the adjacent pair (n & ~1, n | 1): the partner is lane l ^ 1, same token
                const float pv = __shfl_xor(v, 1, 64);
                if (t < a.M) {
                    const int64_t p = a.pos ? a.pos[t] : a.n_past + t;
                    if (n < a.nq + a.nkv) {
                        const int64_t nr = n < a.nq ? n : n - a.nq;
                        const float2 cs = a.rope_tab[p * (a.hd / 2) + (nr % a.hd) / 2];
                        const bool odd = n & 1;
                        const float x0 = odd ? pv : v, x1 = odd ? v : pv;
                        const float o = odd ? __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x))
                                            : __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
                        if (n < a.nq) a.q16[t * a.nq + n] = f2h_rn(o);
                        else a.kc[p * a.nkv + nr] = f2h_rn(o);
                    } else {
                        a.vc[p * a.nkv + (n - a.nq - a.nkv)] = f2h_rn(v);
                    }
                }
                continue;
            }
            if (t < a.M) a.Y[t * a.ldy + n] = a.res ? __fadd_rn(v, a.res[t * a.ldr + n]) : v;
        }
    }
}

// split / wave choice from the weight shape alone (KCPP_Q80T_SHAPE="S,WV" / KCPP_Q80T_GLU="WV": tools/q80t_sweep.py)
void q80t_shape(int mode, int64_t ntile, int64_t nu, int &S, int &WV) {
    static int ov_s = -1, ov_wv = 0, ov_glu = 0;
    if (ov_s < 0) {
        ov_s = 0;
        if (const char *e = getenv("KCPP_Q80T_SHAPE")) sscanf(e, "%d,%d", &ov_s, &ov_wv);
        if (const char *e = getenv("KCPP_Q80T_GLU")) ov_glu = atoi(e);
    }
    if (mode == 1) { S = 1; WV = ov_glu == 4 || ov_glu == 8 ? ov_glu : Q80T_GLU_WV; return; }
    if (ov_s >= 1 && ov_s <= Q80T_SMAX && (ov_wv == 1 || ov_wv == 2 || ov_wv == 4 || ov_wv == 8)) {
        S = ntile <= 256 ? ov_s : 1;
        WV = ov_wv;
        while (WV > 1 && nu / S < WV) WV /= 2;
        return;
    }
    // tools/q80t_sweep.py (Llama-3-8B shapes, M = 1 and 32): q|k|v (192 tiles) S 1 x 8 waves 10.6 us vs 15.8 at S 2; wo /
    // down (128 tiles) S 2 x 8 waves 9.0 / 16.9 us, the best of S 1-2 x 2-8 waves
    S = ntile < 160 && nu >= 16 ? 2 : 1;
    WV = ntile * S >= 512 ? 4 : 8;
    while (WV > 1 && nu / S < WV) WV /= 2;
}

}  // namespace

// workspace of kcpp_gemm for KT_Q8_0_T: the S = 2 tickets at a FIXED place (the first 64 KB: [tile < 256][group < 64]
// words, zero when the workspace is first used and left zero by every launch, whatever shape ran before), then the
// partial tiles of a split shape
constexpr int64_t Q80T_TICK_BYTES = 256 * 64 * 4;
static_assert(Q80T_SMAX <= 8, "partials sized for 8 ranges");
extern "C" {
int64_t kcpp_q80t_ws_bytes(int64_t K, int64_t N, int64_t M) {
    const int64_t ntile = N / 32, Z = (M + 31) / 32;
    int S, WV;
    q80t_shape(0, ntile, K / 128, S, WV);
    // partial tiles only where the shape splits K (S > 1; GLU, mode 1, never splits): the output head (4008 tiles) and
    // the fused gate|up need none, so the workspace is the tickets plus the split projections' partials
    return Q80T_TICK_BYTES + (S > 1 ? ntile * Z * S * 4096 : 0);
}

// mode 0: Y = W act (+ res); mode 1: h = silu(W act) * (W2 act) as f32 (Y) or as the KT_Q8_0_TA activation (qout)
static int q80t_launch(Q80TArgs &a, const void *const *Ws, const int64_t *Ns, int nseg, const void *W2, int64_t K,
                       const void *act, int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode,
                       void *qout, void *ws, void *stream) {
    if (nseg < 1 || nseg > 3 || K % 128 || M < 1 || (mode == 1 && (nseg != 1 || !W2))) return -1;
    int64_t ntot = 0;
    for (int i = 0; i < nseg; ++i) {
        if (Ns[i] % 32 || Ns[i] <= 0) return -1;
        a.W[i] = (const uint8_t *)Ws[i];
        a.N[i] = Ns[i];
        ntot += Ns[i];
    }
    a.nseg = nseg; a.W2 = (const uint8_t *)W2; a.K = K; a.M = M; a.act = (const uint8_t *)act;
    a.Y = Y; a.ldy = ldy; a.res = res; a.ldr = ldr; a.qout = (uint8_t *)qout;
    a.ntile = ntot / 32;
    a.Z = (int)((M + 31) / 32);
    int S, WV;
    q80t_shape(mode, a.ntile, K / 128, S, WV);
    if (S > 1 && a.Z > 64) { S = 1; WV = 8; }            // beyond the ticket capacity (2048 tokens): one K range
    a.S = S;
    if (S > 1) {
        if (!ws) return -2;
        a.tick = (unsigned *)ws;                           // [tile][group], tile < 256 when S = 2
        a.part = (float *)((uint8_t *)ws + Q80T_TICK_BYTES);
    }
    const int64_t units = (K / 128 + S - 1) / S;
    const size_t smem = (size_t)units * 512 + (size_t)WV * 4096 + (mode == 1 ? 4096 : 0);
    const int64_t nblk = (a.ntile + 7) / 8 * 8 * S * a.Z;
    hipStream_t s = (hipStream_t)stream;
#define Q80T_L(MD, W_) hipLaunchKernelGGL((k_q80t<MD, W_>), dim3((unsigned)nblk), dim3(64 * W_), smem, s, a)
    if (mode == 1 && WV == 8) Q80T_L(1, 8);
    else if (mode == 1) Q80T_L(1, 4);
    else if (WV == 8) Q80T_L(0, 8);
    else if (WV == 4) Q80T_L(0, 4);
    else if (WV == 2) Q80T_L(0, 2);
    else Q80T_L(0, 1);
#undef Q80T_L
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_gemm_q80t(const void *const *Ws, const int64_t *Ns, int nseg, const void *W2, int64_t K, const void *act,
                   int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *qout, void *ws,
                   void *stream) {
    Q80TArgs a;
    memset(&a, 0, sizeof a);
    return q80t_launch(a, Ws, Ns, nseg, W2, K, act, M, Y, ldy, res, ldr, mode, qout, ws, stream);
}

// q|k|v = W act with k_rope_kv fused into the epilogue: rope(q) -> q16 [M][H D], rope(k) / v -> the f16 caches at
// positions pos[t] (or n_past + t); the f32 q|k|v rows are not written
int kcpp_gemm_q80t_qkv_rope(const void *const *Ws, const int64_t *Ns, int64_t K, const void *act, int64_t M,
                            const void *rope_tab, int n_past, const int32_t *pos_dev, int head_dim, uint16_t *q16,
                            uint16_t *kc, uint16_t *vc, void *ws, void *stream) {
    if (!rope_tab || !q16 || !kc || !vc || head_dim <= 0 || head_dim % 2 || Ns[0] % head_dim || Ns[1] % head_dim ||
        Ns[1] != Ns[2])
        return -1;
    Q80TArgs a;
    memset(&a, 0, sizeof a);
    a.rope_tab = (const float2 *)rope_tab;
    a.q16 = q16; a.kc = kc; a.vc = vc; a.pos = pos_dev; a.n_past = n_past; a.hd = head_dim;
    a.nq = Ns[0]; a.nkv = Ns[1];
    return q80t_launch(a, Ws, Ns, 3, nullptr, K, act, M, nullptr, 0, nullptr, 0, 0, nullptr, ws, stream);
}
}  // extern "C"
