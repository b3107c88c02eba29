// dec_engine.hip -- single-token decode of a whole stage (all its layers) as ONE persistent launch.
//
// The launch chain it replaces (runtime.cpp forward_layers_dec: per layer q|k|v, attention, combine, wo, gate|up,
// down = six dependent launches) pays every launch's ramp and drain: 1.66 ms per Llama-3-8B token against 0.81 ms
// for its bytes at 6.3 TB/s.  The reference pays one launch per ggml node (ggml-cuda.cu:2654-2676,
// mmvq.cu:50-130, fattn-vec-f16.cuh + fattn-common.cuh:523).  Here every CU runs the whole layer sequence, and the
// dependency edges between the ops are hand-offs inside the launch, so the weight bytes of the NEXT op are already
// in flight while an edge resolves (MI355X_MICROARCH.md, prefetch-credit / engine-vs-launches).
//
// Geometry: one 512-thread workgroup per CU (NB = the CU count, all resident at once; the dynamic LDS request
// admits one workgroup per CU).  Waves 0..6 are COMPUTE waves: they only ever issue weight / cached-K/V loads
// (plain non-temporal loads into registers, issued ahead of the edge they wait behind) and read LDS.  Wave 7 is the
// CONTROL wave: it polls the edge counters, loads every handed-off byte (write-through `sc1` loads), stages it in
// LDS, and does every global store of the workgroup (write-through `sc1` stores) and the arrive.  Because vector
// loads return in order per wave, a poll issued by a wave behind its own weight loads would wait for those weights;
// the control wave has nothing else outstanding, so it sees an edge as soon as it resolves.  Barriers do not drain
// VMEM, so the compute waves' prefetched weights stay in flight across them.
//
// Hand-off protocol (MI355X_MICROARCH.md "Valid forms", first row of the sc1 table; cdna_hip_programming.md
// Guideline 16): payload stored write-through (sc1) by the control wave only, `s_waitcnt vmcnt(0)`, then ONE lane's
// agent-scope atomic add on the edge counter; the consumer's control wave polls the counter with sc1 loads (s_sleep
// between polls), then loads the payload with sc1 loads only (no acquire fence needed), stages it in LDS and
// releases the compute waves with a workgroup barrier.  The counters are zeroed ahead of every launch (a memset node
// of the decode graph), so an edge's target is its arrival count.  Every poll is bounded; a timeout sets the error word, after which every poll of every workgroup returns at once, so the grid
// always drains (the host reads the word, reports, and resets the counters).
//
// Per layer, with NB = 256, Llama-3-8B shapes (E 4096, F 14336, 32 q / 8 kv heads of 128):
//   Q  (q|k|v)  CU b: kv-head group hk = b % HKV, part j = b / HKV of the group's 768 rows (512 q, 128 k, 128 v):
//               24 rows; rms_norm(x)*w -> Q8_K; RoPE; f16 q / K / V stores.  Edge cQ[hk]: 32 arrivals.
//   A  (attn)   CU b: split sp = b / HKV of kv head hk (32 splits, the key partition of k_fa_dec4); cached keys
//               prefetched before the edge, the new key patched in after it.  Edge cA[hk]: 32 arrivals.
//   C  (merge)  CUs with sp < 2: unit u = 2 hk + sp merges heads 2u, 2u+1 (one Q8_K super-block of the attention
//               output, as k_fa_comb4<QUANT>).  Edge cC: H/2 arrivals.
//   O  (wo)     CU b: rows [16 b, 16 b + 16), x += wo . attn.  Edge cO (8 shards): NB arrivals.
//   G  (glu)    CU b: rows [56 b, 56 b + 56) of gate and up, h = silu(g) * u.  Edge cG (8 shards): NB arrivals.
//   D  (down)   CU b: rows [16 b, ...), x += down . Q8_K(h).  Edge cD (8 shards): NB arrivals = next layer's x.
// Rows of a CU are split over the 7 compute waves in contiguous runs; every row's dot is computed exactly as the
// stand-alone k_gemv_rs computes it (same lane -> piece map, same per-lane order, same wave reduction), so q|k|v,
// wo, gate|up and down are bit-identical to the launch chain; only the attention's key-to-wave split differs.
#include "attn_dec.h"
#include "gemv_rs.h"

#include <algorithm>
#include <cstdlib>

using namespace rs;

namespace eng {

constexpr int NW = 8, NC = 7, CTL = 7, NT = 512;
constexpr int NWA = 4;                            // attention waves (k_fa_dec4's 4-wave key assignment)
constexpr unsigned kSpinMax = 1u << 19;          // polls (each >= one sc1 round trip): ~0.5 s
constexpr int SLOTS = 48;                         // counters per layer, one 128-B line each
enum { S_Q = 0, S_A = 8, S_C = 16, S_O = 24, S_G = 32, S_D = 40 };

struct Layer {
    const uint8_t *wq, *wk, *wv, *wo, *wg, *wu, *wd;
    const float *attn_norm, *ffn_norm;
    uint16_t *kc, *vc;
    int tv, td;            // attn_v / ffn_down: 0 = Q4_K_RS, 1 = Q6_K_RS
};

struct Args {
    const Layer *layers;
    int nl;
    float *x;                 // [E] residual stream
    uint16_t *q16;            // [H * 128] rope'd q (f16)
    float *part_o;            // [H][NS][128]
    float2 *part_ml;          // [H][NS]
    uint8_t *act;             // Q8_K image of the attention output: qs [E] ++ d [E/256] ++ bsums [E/16]
    float *h;                 // [F]
    unsigned *sync;           // nl * SLOTS counters (128-B lines) ++ the error word
    const int32_t *pos;       // {position, epoch}
    const float2 *rope_tab;   // [n_ctx][64] (cos, sin)
    float eps, kq_scale;
    int opt;                  // edge ordering per phase (2 bits each, Q O G D): 0 together, 1 store first, 2 arrive first
    float *dbg;               // diagnostics (tests only, null in the product): the merged attention rows in f32
    unsigned long long *stamps;   // diagnostics (tools/engine_stamps.py, null in the product): [NB][nl][32] clocks
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, 0x7fffffff, 0x00020000);
}
// write-through (sc1) 16-B load / store at byte offset `off` of a wave-uniform base (buffer instructions: vector path)
__device__ __forceinline__ uint4 ld_sc1(__amdgpu_buffer_rsrc_t r, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int off, uint4 v) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 16);
}
__device__ __forceinline__ void st_sc1_u32(void *p, uint32_t v) {
    __hip_atomic_store((uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f32(float *p, float v) { st_sc1_u32(p, __float_as_uint(v)); }

__device__ __forceinline__ unsigned *counter(unsigned *sync, int l, int s) { return sync + ((size_t)l * SLOTS + s) * 32; }

// lanes of one wave exchanging data through LDS: the compiler may otherwise reorder one lane's LDS access past another
// lane's (diverged branches are not ordered across lanes), so every such hand-off inside the control wave goes
// through this (a wavefront fence pair around the wave barrier; no instruction is emitted for the barrier itself)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// control wave: wait until the sum of n consecutive counters (lanes < n) reaches `target` (wrap-safe)
__device__ __forceinline__ void poll(const unsigned *c0, int n, unsigned target, unsigned *err, unsigned code, int lane) {
    for (unsigned it = 0;; ++it) {
        unsigned v = lane < n ? __hip_atomic_load(c0 + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
        for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        v = __builtin_amdgcn_readfirstlane(v);
        if ((int)(v - target) >= 0) return;
        if ((it & 31) == 31 &&
            __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u)
            return;                                   // another workgroup gave up: drain
        if (it > kSpinMax) {
            if (lane == 0 && __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                // diagnostics of the first timeout: what the poll saw, what it waited for, where
                __hip_atomic_store(err + 1, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(err + 2, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(err + 3, (unsigned)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// control wave, after its write-through stores: drain them, then one lane arrives
__device__ __forceinline__ void arrive(unsigned *c, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ one K-row of a Q4_K_RS / Q6_K_RS matrix in a lane
template <int K>
struct Row {
    static constexpr int NSB = K / 256;
    static constexpr int NP4 = NSB * 8, NP6 = NSB * 4;
    static constexpr int NI4 = (NP4 + 63) / 64, NI6 = (NP6 + 63) / 64;
    static constexpr int NU6 = 3 * NI6 + (NI6 + 1) / 2;          // A, B, C per piece; (sc, d) pairs packed
    static constexpr int NU = 2 * NI4 > NU6 ? 2 * NI4 : NU6;
    uint4 u[NU];
};
template <int K>
__device__ __forceinline__ void load_row(Row<K> &b, const uint8_t *W, int row, bool q6, int lane) {
    using R = Row<K>;
    if (!q6) {
        const uint8_t *rp = W + (int64_t)row * (R::NSB * 144);
#pragma unroll
        for (int i = 0; i < R::NI4; ++i) {
            const int p = min(lane + 64 * i, R::NP4 - 1);
            b.u[2 * i] = ld_nt(rp + 16 * (p >> 3));
            b.u[2 * i + 1] = ld_nt(rp + 16 * R::NSB + 16 * p);
        }
    } else {
        const uint8_t *rp = W + (int64_t)row * (R::NSB * 210);
#pragma unroll
        for (int i = 0; i < R::NI6; ++i) {
            const int p = min(lane + 64 * i, R::NP6 - 1);
            b.u[3 * i] = ld_nt(rp + 16 * p);
            b.u[3 * i + 1] = ld_nt(rp + 64 * R::NSB + 16 * p);
            b.u[3 * i + 2] = ld_nt(rp + 128 * R::NSB + 16 * p);
            const uint32_t sc = __builtin_nontemporal_load((const uint32_t *)(rp + 192 * R::NSB + 4 * p));
            const uint32_t d = __builtin_nontemporal_load((const uint16_t *)(rp + 208 * R::NSB + 2 * (p >> 2)));
            uint4 &pk = b.u[3 * R::NI6 + (i >> 1)];
            if (i & 1) { pk.z = sc; pk.w = d; } else { pk.x = sc; pk.y = d; }
        }
    }
}
template <int K>
__device__ __forceinline__ void zero_row(Row<K> &b) {
#pragma unroll
    for (int i = 0; i < Row<K>::NU; ++i) b.u[i] = make_uint4(0, 0, 0, 0);
}
// activation slices of a K = E phase (both vec_dot layouts of the Q8_K image), held in registers
template <int K>
struct ActE {
    typename RS<KT_Q4_K_RS>::Act a4[Row<K>::NI4];
    typename RS<KT_Q6_K_RS>::Act a6[Row<K>::NI6];
};
template <int K>
__device__ __forceinline__ void load_act(ActE<K> &x, const uint8_t *act, int lane, bool q4, bool q6) {
    using R = Row<K>;
    if (q4) {
        const auto lc = RS<KT_Q4_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI4; ++i) RS<KT_Q4_K_RS>::act(act, K, min(RS<KT_Q4_K_RS>::sb_of(lane, i), R::NSB - 1), lc, x.a4[i]);
    }
    if (q6) {
        const auto lc = RS<KT_Q6_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI6; ++i) RS<KT_Q6_K_RS>::act(act, K, min(RS<KT_Q6_K_RS>::sb_of(lane, i), R::NSB - 1), lc, x.a6[i]);
    }
}
// the row's dot with the held activation: k_gemv_rs's per-lane order and wave reduction
template <int K>
__device__ __forceinline__ float dot_row(const Row<K> &b, const ActE<K> &x, bool q6, int lane) {
    using R = Row<K>;
    float acc = 0.0f;
    if (!q6) {
        const auto lc = RS<KT_Q4_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI4; ++i) {
            const bool ok = (R::NI4 * 64 == R::NP4) || lane + 64 * i < R::NP4;
            typename RS<KT_Q4_K_RS>::W w;
            w.h = b.u[2 * i]; w.q = b.u[2 * i + 1];
            const float p = RS<KT_Q4_K_RS>::dot(w, x.a4[i], lc);
            acc += ok ? p : 0.0f;
        }
    } else {
        const auto lc = RS<KT_Q6_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI6; ++i) {
            const bool ok = (R::NI6 * 64 == R::NP6) || lane + 64 * i < R::NP6;
            typename RS<KT_Q6_K_RS>::W w;
            const uint4 &pk = b.u[3 * R::NI6 + (i >> 1)];
            w.A = b.u[3 * i]; w.B = b.u[3 * i + 1]; w.C = b.u[3 * i + 2];
            w.sc = (i & 1) ? pk.z : pk.x; w.d = (i & 1) ? pk.w : pk.y;
            const float p = RS<KT_Q6_K_RS>::dot(w, x.a6[i], lc);
            acc += ok ? p : 0.0f;
        }
    }
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_f(acc))));
}
// the same with the activation read from LDS per piece (the K = F down projection: too many slices to hold)
template <int K>
__device__ __forceinline__ float dot_row_lds(const Row<K> &b, const uint8_t *act, bool q6, int lane) {
    using R = Row<K>;
    float acc = 0.0f;
    if (!q6) {
        const auto lc = RS<KT_Q4_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI4; ++i) {
            const bool ok = (R::NI4 * 64 == R::NP4) || lane + 64 * i < R::NP4;
            typename RS<KT_Q4_K_RS>::Act xa;
            RS<KT_Q4_K_RS>::act(act, K, min(RS<KT_Q4_K_RS>::sb_of(lane, i), R::NSB - 1), lc, xa);
            typename RS<KT_Q4_K_RS>::W w;
            w.h = b.u[2 * i]; w.q = b.u[2 * i + 1];
            const float p = RS<KT_Q4_K_RS>::dot(w, xa, lc);
            acc += ok ? p : 0.0f;
        }
    } else {
        const auto lc = RS<KT_Q6_K_RS>::lane_consts(lane);
#pragma unroll
        for (int i = 0; i < R::NI6; ++i) {
            const bool ok = (R::NI6 * 64 == R::NP6) || lane + 64 * i < R::NP6;
            typename RS<KT_Q6_K_RS>::Act xa;
            RS<KT_Q6_K_RS>::act(act, K, min(RS<KT_Q6_K_RS>::sb_of(lane, i), R::NSB - 1), lc, xa);
            typename RS<KT_Q6_K_RS>::W w;
            const uint4 &pk = b.u[3 * R::NI6 + (i >> 1)];
            w.A = b.u[3 * i]; w.B = b.u[3 * i + 1]; w.C = b.u[3 * i + 2];
            w.sc = (i & 1) ? pk.z : pk.x; w.d = (i & 1) ? pk.w : pk.y;
            const float p = RS<KT_Q6_K_RS>::dot(w, xa, lc);
            acc += ok ? p : 0.0f;
        }
    }
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_f(acc))));
}


// contiguous run of items [s, e) of a CU's R items for compute wave w
__device__ __forceinline__ void wave_run(int R, int w, int &s, int &e) { s = w * R / NC; e = (w + 1) * R / NC; }

// Q8_K of the f32 staging row xs[K] into the LDS image act (all 512 threads; 16 lanes per super-block)
template <int K>
__device__ __forceinline__ void quant_lds(const float *xs, uint8_t *act, int tid) {
    for (int c = tid; c < K / 16; c += NT) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 f = *(const float4 *)(xs + 16 * c + 4 * k);
            v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
        }
        q8k_quant16(v, c & 15, (int8_t *)act + (c >> 4) * 256, (float *)(act + K) + (c >> 4),
                    (int16_t *)(act + K + K / 256 * 4) + (c >> 4) * 16);
    }
}

// control wave: the rms_norm scale of the f32 row xs[E] gathered in LDS (ggml_compute_forward_rms_norm_f32: f32
// squares summed in double, ggml.c:12089; lane order = the k_gemv_rs norm prologue's, so the bits agree)
template <int E>
__device__ __forceinline__ float ctl_scale(const float *xs, float eps, int lane) {
    constexpr int NL = E / 256;                       // 16-B words per lane
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const float4 v = *(const float4 *)(xs + 4 * (lane + 64 * k));
        ss += (double)__fmul_rn(v.x, v.x) + (double)__fmul_rn(v.y, v.y) + (double)__fmul_rn(v.z, v.z) +
              (double)__fmul_rn(v.w, v.w);
    }
    ss = wave_sum_d(ss);
    return 1.0f / sqrtf((float)(ss / (double)E) + eps);
}
// Q8_K of rms_norm(xs) * w (w staged in LDS at nws) into the LDS image act (all 512 threads; 16 lanes per super-block)
template <int K>
__device__ __forceinline__ void quant_lds_norm(const float *xs, const float *nws, float scale, uint8_t *act, int tid) {
    for (int c = tid; c < K / 16; c += NT) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 f = *(const float4 *)(xs + 16 * c + 4 * k), w = *(const float4 *)(nws + 16 * c + 4 * k);
            v[4 * k] = __fmul_rn(__fmul_rn(f.x, scale), w.x);
            v[4 * k + 1] = __fmul_rn(__fmul_rn(f.y, scale), w.y);
            v[4 * k + 2] = __fmul_rn(__fmul_rn(f.z, scale), w.z);
            v[4 * k + 3] = __fmul_rn(__fmul_rn(f.w, scale), w.w);
        }
        q8k_quant16(v, c & 15, (int8_t *)act + (c >> 4) * 256, (float *)(act + K) + (c >> 4),
                    (int16_t *)(act + K + K / 256 * 4) + (c >> 4) * 16);
    }
}
// control wave: n16 16-B words from a wave-uniform base into LDS by write-through (sc1) LDS-DMA (no registers), then
// drained (the caller's barrier then publishes them to the other waves)
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void dma16_sc1(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_base))) : "memory", "m0");
}
__device__ __forceinline__ void dma16_plain(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_base))) : "memory", "m0");
}
// control wave: issue (no wait) the LDS-DMA of n16 16-B words of read-only data (norm weights: cached)
__device__ __forceinline__ void ctl_fetch(void *dst, const void *src, int n16, int lane) {
    for (int k = 0; 64 * k < n16; ++k)
        if (64 * k + lane < n16) dma16_plain((const uint8_t *)src + 16 * (64 * k + lane), (uint8_t *)dst + 1024 * k);
}
// control wave: a vector produced in 8 contiguous shards (shard s by the CUs [NB/8 s, NB/8 (s + 1)), whose arrivals
// count on the s-th counter from c0) gathered into LDS by write-through LDS-DMA, each shard requested as soon as
// its producers have arrived (the later shards' polls overlap the earlier shards' copies); drained at the end.
// n16 / 8 is a multiple of 64 (host-checked shapes).  `wait` false: no polls (the launch's input).
__device__ __forceinline__ void ctl_gather8(void *dst, const void *src, const unsigned *c0, int n16, unsigned per,
                                            bool wait, unsigned *err, unsigned code, int lane) {
    const int W = n16 / 8;
    unsigned done = wait ? 0u : 0xffu;
    if (!wait)
        for (int k = 0; 64 * k < n16; ++k)
            dma16_sc1((const uint8_t *)src + 16 * (64 * k + lane), (uint8_t *)dst + 1024 * k);
    for (unsigned it = 0; done != 0xffu; ++it) {
        // one load of all 8 counters per round; the shards that completed since the last round are requested
        const unsigned v = lane < 8 ? __hip_atomic_load(c0 + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned ready = (unsigned)__ballot(lane < 8 && (int)(v - per) >= 0) & ~done & 0xffu;
        for (unsigned m = ready; m; m &= m - 1) {
            const int sh = __builtin_ctz(m);
            for (int k = 0; 64 * k < W; ++k)
                dma16_sc1((const uint8_t *)src + 16 * (sh * W + 64 * k + lane), (uint8_t *)dst + 16 * (sh * W + 64 * k));
        }
        done |= ready;
        if (ready) continue;
        if ((it & 31) == 31 &&
            __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u)
            break;                                        // another workgroup gave up: drain
        if (it > kSpinMax) {
            if (lane == 0 && __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                __hip_atomic_store(err + 1, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(err + 2, per, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(err + 3, (unsigned)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// control wave: issue the write-through LDS-DMA of n16 16-B words (no wait)
__device__ __forceinline__ void ctl_copy_issue(void *dst, const void *src, int n16, int lane) {
    for (int k = 0; 64 * k < n16; ++k) {
        if (64 * k + lane < n16) dma16_sc1((const uint8_t *)src + 16 * (64 * k + lane), (uint8_t *)dst + 1024 * k);
        if (k >= 56) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");      // (vmcnt counts to 63)
    }
}
__device__ __forceinline__ void ctl_copy(void *dst, const void *src, int n16, int lane) {
#ifdef ENG_REGCOPY
    const auto r = rsrc(src);
#pragma unroll 1
    for (int c0 = 0; c0 < n16; c0 += 512) {
        uint4 u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = c0 + lane + 64 * k;
            u[k] = c < n16 ? ld_sc1(r, 16 * c) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = c0 + lane + 64 * k;
            if (c < n16) *(uint4 *)((uint8_t *)dst + 16 * c) = u[k];
        }
    }
    return;
#endif
    ctl_copy_issue(dst, src, n16, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 16 B per lane of streamed-once data (cached K/V) into LDS at lds_base + 16 lane (LDS-DMA, non-temporal)
__device__ __forceinline__ void dma16(const void *g, const void *lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g),
                 "s"(__builtin_amdgcn_readfirstlane(lds_addr(lds_base))) : "memory", "m0");
}

// ------------------------------------------------------------------ the engine
template <int E, int F, int H, int HKV>
struct Geo {
    static constexpr int D = 128, G = H / HKV, EKV = HKV * D;
    static constexpr int RG = (G + 2) * D;                       // q|k|v rows per kv-head group
    static constexpr int NB = 256;                               // compiled for 256 CUs (host checks)
    static constexpr int CG = NB / HKV;                          // CUs per group = attention splits
    static constexpr int RQ = ((RG + CG - 1) / CG + 1) & ~1;     // q|k|v rows per CU (even: RoPE pairs)
    static constexpr int RO = (E + NB - 1) / NB;                 // wo / down rows per CU
    static constexpr int RF = (F + NB - 1) / NB;                 // gate|up rows per CU
    static constexpr int MQ = (RQ + NC - 1) / NC, MO = (RO + NC - 1) / NC, MG = (2 * RF + NC - 1) / NC;
    static constexpr int WG = 4, WD = 1;                         // rows in flight: gate|up items, down rows
    static constexpr int ACTE = E + E / 256 * 4 + E / 16 * 2, ACTF = F + F / 256 * 4 + F / 16 * 2;
    // LDS map (bytes)
    static constexpr int L_XS = 0;                               // f32 [F] staging (norm output, h); attention smem
    static constexpr int L_ACT = (F * 4 + 255) & ~255;           // Q8_K image (K <= F)
    static constexpr int L_KV = 0;                               // attention: 7 waves x 2 chunks x 8 KB of K/V
    static constexpr int L_SO = NC * 16384;                      // attention merge (f32 partials of the waves)
    static constexpr int L_RES0 = L_SO + ((NC * G * D * 4 + NC * G * 16 + G * D * 4 + G * 8 + 255) & ~255);
    static constexpr int L_RES1 = L_ACT + ((ACTF + 255) & ~255);
    static constexpr int L_RES = L_RES0 > L_RES1 ? L_RES0 : L_RES1;   // f32 [2 RF] per-item results
    static constexpr int L_Q = L_RES + ((8 * RF + 255) & ~255);  // f16 q [G][D], new K [D], new V [D]
    static constexpr int L_MISC = L_Q + 2 * G * D + 4 * D;       // small control words
    static constexpr int LDS = L_MISC + 1024;
    static constexpr int LDS_REQ = LDS > 96 * 1024 ? LDS : 96 * 1024;   // one workgroup per CU
};

// the q|k|v rows of compute wave `wave` of CU b in flight (group rows [jq RQ + s, jq RQ + e) of kv-head group hk)
template <int E, class GG>
__device__ __forceinline__ void issue_qkv(Row<E> (&wq)[GG::MQ], const Layer &L, int b, int wave, int lane) {
    constexpr int G = GG::G, D = GG::D;
    const int hk = b % (GG::CG == 0 ? 1 : (GG::NB / GG::CG)), jq = b / (GG::NB / GG::CG);
    int s, e;
    wave_run(GG::RQ, wave == CTL ? 0 : wave, s, e);
    if (wave == CTL) e = s;
#pragma unroll
    for (int i = 0; i < GG::MQ; ++i) {
        const int gr = jq * GG::RQ + s + i;
        if (s + i < e && gr < GG::RG) {
            const uint8_t *W;
            int row;
            bool q6 = false;
            if (gr < G * D) { W = L.wq; row = hk * G * D + gr; }
            else if (gr < (G + 1) * D) { W = L.wk; row = hk * D + gr - G * D; }
            else { W = L.wv; row = hk * D + gr - (G + 1) * D; q6 = L.tv != 0; }
            load_row<E>(wq[i], W, row, q6, lane);
        } else {
            zero_row<E>(wq[i]);
        }
    }
}

#define ESTAMP(k)                                                                                                     \
    if (a.stamps && tid == CTL * 64) a.stamps[((size_t)b * a.nl + l) * 32 + (k)] = __builtin_amdgcn_s_memrealtime();

template <int E, int F, int H, int HKV>
__global__ void __launch_bounds__(512, 1) k_engine(const Args a) {
    using GG = Geo<E, F, H, HKV>;
    constexpr int D = GG::D, G = GG::G, EKV = GG::EKV, RG = GG::RG, CG = GG::CG, RQ = GG::RQ, RO = GG::RO, RF = GG::RF;
    constexpr int NS = CG;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    float *xs = (float *)(lds + GG::L_XS);
    uint8_t *act = lds + GG::L_ACT;
    float *res = (float *)(lds + GG::L_RES);
    float *nws = xs + E;                                          // the norm weights, staged beside xs
    float *sscale = (float *)(lds + GG::L_MISC);                  // the rms_norm scale
    uint16_t *sq = (uint16_t *)(lds + GG::L_Q), *snk = sq + G * D, *snv = snk + D;

    const int np = a.pos[0];
    unsigned *err = a.sync + (size_t)a.nl * SLOTS * 32;
    const float sc2 = a.kq_scale * 1.4426950408889634f;
    const int b0 = blockIdx.x, lane0 = threadIdx.x & 63, wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Row<E> wq[GG::MQ];
    issue_qkv<E, GG>(wq, a.layers[0], b0, wave0, lane0);      // (the control wave's run is empty: zeros)
    float xres = 0.0f;            // control wave, lane j < RO: this CU's residual row j (it alone writes those rows)
    if (wave0 == CTL && lane0 < RO && b0 * RO + lane0 < E) xres = a.x[b0 * RO + lane0];
    for (int l = 0; l < a.nl; ++l) {
        // the workgroup / wave / lane ids laundered per layer: every per-layer index derived from them is computed
        // here, not hoisted out of the layer loop (hoisted, the row indices and masks of all six phases stay live
        // across the whole loop and spill)
        int b = b0, wave = wave0, lane = lane0;
        asm volatile("" : "+s"(b), "+s"(wave));
        asm volatile("" : "+v"(lane));
        const int tid = 64 * wave + lane;
        const bool ctl = wave == CTL;
        const int hk = b % HKV, jq = b / HKV;                     // q|k|v group and part; attention head and split
        // attention: this CU's split of the keys and, within it, k_fa_dec4's own assignment -- waves 0..3 take the
        // 16-key groups p0 + 16 w + 64 j -- so that the split's (m, l, O) partial is k_fa_dec4's bit for bit (and with
        // it the merge, the wo input and every later op: the engine equals the launch chain exactly)
        const int nkv = np + 1, per = (nkv + NS - 1) / NS;
        const int p0 = min(jq * per, nkv), p1 = min(p0 + per, nkv);
        const int k0 = p0 + 16 * wave;
        const int nch = (wave < NWA && k0 < p1) ? (p1 - k0 + 63) / 64 : 0;
        const int sub = lane & 15, kq = lane >> 4;
        int qs_, qe_;
        wave_run(RQ, ctl ? 0 : wave, qs_, qe_);
        if (ctl) qe_ = qs_;
        const Layer L = a.layers[l];
        // ======================================================== Q: attn_norm -> q|k|v -> RoPE, f16 stores
        ESTAMP(0)
        if (ctl) {
            ctl_fetch(nws, L.attn_norm, E / 4, lane);
            ctl_gather8(xs, a.x, counter(a.sync, l > 0 ? l - 1 : 0, S_D), E / 4, GG::NB / 8, l > 0, err, 1u, lane);
            ESTAMP(1)
            const float sc = ctl_scale<E>(xs, a.eps, lane);
            if (lane == 0) *sscale = sc;
            ESTAMP(2)
        }
        __syncthreads();
        quant_lds_norm<E>(xs, nws, *sscale, act, tid);
        __syncthreads();
        ESTAMP(3)
        if (!ctl) {
            ActE<E> xa;
            load_act<E>(xa, act, lane, true, L.tv != 0);
            // (rolled, the row buffers rotating: the whole layer loop has to fit the instruction cache)
#pragma unroll 1
            for (int i = 0; i < GG::MQ; ++i) {
                const int gr = jq * RQ + qs_ + i;
                if (qs_ + i < qe_ && gr < RG) {
                    const bool q6 = gr >= (G + 1) * D && L.tv != 0;
                    const float v = dot_row<E>(wq[0], xa, q6, lane);
                    if (lane == 0) res[qs_ + i] = v;
                }
#pragma unroll
                for (int j = 0; j + 1 < GG::MQ; ++j) wq[j] = wq[j + 1];
            }
        }
        // compute waves: the attention's cached keys (not this token's: this phase writes it) go in flight by LDS-DMA
        // (no registers held across the edge): wave slot = 2 chunks of 16 keys, chunk = 4 K + 4 V wave loads of
        // 1 KiB, lane (kq, sub) -> 16 B (8 dims) of key base + 4 i + kq, stored lane-linear
        const uint16_t *kb = L.kc + hk * D + sub * 8, *vb = L.vc + hk * D + sub * 8;
        uint8_t *kvs = lds + GG::L_KV + (wave < NWA ? wave : 0) * 16384;
        auto dma_chunk = [&](int base, int slot) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int p = base + 4 * i + kq;
                p = (p < p1 && p != np) ? p : p0;              // any row in bounds (replaced at the read)
                dma16(kb + (int64_t)p * EKV, kvs + slot * 8192 + i * 1024);
                dma16(vb + (int64_t)p * EKV, kvs + slot * 8192 + 4096 + i * 1024);
            }
        };
        __syncthreads();    // (behind the barrier: nothing of the q|k|v dots is live beside them)
        ESTAMP(4)
        const int ordq = a.opt & 3;
        if (ordq == 0) {
            if (nch > 0) dma_chunk(k0, 0);
            if (nch > 1) dma_chunk(k0 + 64, 1);
        }
        if (ctl) {          // RoPE (NORM pairs, the rope table) + f16 q / K / V stores, write-through
            const int n = min(RQ, RG - jq * RQ);
            if (lane < n / 2) {
                const int gr = jq * RQ + 2 * lane;
                const float x0 = res[2 * lane], x1 = res[2 * lane + 1];
                uint32_t pk;
                uint16_t *dst;
                if (gr >= (G + 1) * D) {
                    pk = (uint32_t)f2h(x0) | ((uint32_t)f2h(x1) << 16);
                    dst = L.vc + (int64_t)np * EKV + hk * D + gr - (G + 1) * D;
                } else {
                    const int row = gr < G * D ? hk * G * D + gr : hk * D + gr - G * D;
                    const float2 cs = a.rope_tab[(int64_t)np * (D / 2) + (row % D) / 2];
                    const float o0 = __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
                    const float o1 = __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x));
                    pk = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
                    dst = gr < G * D ? a.q16 + row : L.kc + (int64_t)np * EKV + row;
                }
                st_sc1_u32(dst, pk);
            }
            if (ordq != 1) arrive(counter(a.sync, l, S_Q + hk), lane);
        }
        if (ordq != 0) {
            __syncthreads();
            if (nch > 0) dma_chunk(k0, 0);
            if (nch > 1) dma_chunk(k0 + 64, 1);
            if (ctl && ordq == 1) arrive(counter(a.sync, l, S_Q + hk), lane);
        }
        if (ctl) { ESTAMP(5) }
        // ======================================================== A: split jq of kv head hk
        if (ctl) {
            poll(counter(a.sync, l, S_Q + hk), 1, CG, err, 2u, lane);
            ESTAMP(6)
            // q of the G heads (G * 256 B) and, in the split holding it, the new key's K and V rows (256 B each)
            const auto rq = rsrc(a.q16 + hk * G * D);
            for (int c = lane; c < G * D / 8; c += 64) *(uint4 *)(sq + 8 * c) = ld_sc1(rq, 16 * c);
            if (np >= p0 && np < p1 && lane < 32) {
                const uint16_t *src = (lane < 16 ? L.kc : L.vc) + (int64_t)np * EKV + hk * D;
                *(uint4 *)((lane < 16 ? snk : snv) + 8 * (lane & 15)) = ld_sc1(rsrc(src), 16 * (lane & 15));
            }
        }
        __syncthreads();
        ESTAMP(7)
        fadec::State<G> st;
        fadec::init(st);
        if (!ctl && nch > 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) fadec::set_q(st, g, *(const uint4 *)(sq + g * D + sub * 8));
            for (int c = 0; c < nch; ++c) {
                const int base = k0 + 64 * c, slot = c & 1;
                if (c + 1 < nch) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint4 kk[4], vv[4];
                const uint8_t *src = kvs + slot * 8192 + lane * 16;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int p = base + 4 * i + kq;
                    uint4 k = *(const uint4 *)(src + i * 1024), v = *(const uint4 *)(src + 4096 + i * 1024);
                    if (p >= p1) { k = make_uint4(0, 0, 0, 0); v = k; }
                    else if (p == np) { k = *(const uint4 *)(snk + sub * 8); v = *(const uint4 *)(snv + sub * 8); }
                    kk[i] = k; vv[i] = v;
                }
                fadec::consume(st, base, p1, kq, sc2, kk, vv);
                if (c + 2 < nch) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this slot's reads are done
                    dma_chunk(base + 128, slot);
                }
            }
        }
        int os_, oe_;
        wave_run(RO, ctl ? 0 : wave, os_, oe_);
        if (ctl) oe_ = os_;
        Row<E> wo[GG::MO];
        {   // merge the compute waves' (m, l, O) in LDS (the attention smem lives in the staging area)
            float *so = (float *)(lds + GG::L_SO);        // [NWA][G][D]
            float2 *sml = (float2 *)(so + NC * G * D);    // [NWA][G]
            float *sw = (float *)(sml + NC * G);          // [NWA][G]
            float *sout = sw + NC * G;                    // [G][D]
            float2 *sML = (float2 *)(sout + G * D);       // [G]
            if (wave < NWA) {        // fadec::finish's order: rows, then the 4 waves in LDS
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
                        *(float4 *)&so[(wave * G + g) * D + sub * 8] = make_float4(st.acc[g][0], st.acc[g][1], st.acc[g][2], st.acc[g][3]);
                        *(float4 *)&so[(wave * G + g) * D + sub * 8 + 4] = make_float4(st.acc[g][4], st.acc[g][5], st.acc[g][6], st.acc[g][7]);
                    }
                }
                if (lane == 0) {
#pragma unroll
                    for (int g = 0; g < G; ++g) sml[wave * G + g] = make_float2(st.m[g], st.l[g]);
                }
            }
            __syncthreads();
            ESTAMP(8)
            // compute waves: wo rows in flight (consumed after the merge edge; issued behind this barrier so that
            // they are not live beside the attention state)
#pragma unroll
            for (int i = 0; i < GG::MO; ++i)
                if (os_ + i < oe_ && b * RO + os_ + i < E) load_row<E>(wo[i], L.wo, b * RO + os_ + i, false, lane);
                else zero_row<E>(wo[i]);
            if (tid < G) {
                float M = -INFINITY;
#pragma unroll
                for (int w = 0; w < NWA; ++w) M = fmaxf(M, sml[w * G + tid].x);
                float Ls = 0.0f;
#pragma unroll
                for (int w = 0; w < NWA; ++w) {
                    const float wt = M == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(sml[w * G + tid].x - M);
                    sw[w * G + tid] = wt;
                    Ls = fmaf(wt, sml[w * G + tid].y, Ls);
                }
                sML[tid] = make_float2(M, Ls);
            }
            __syncthreads();
            for (int i = tid; i < G * D; i += NT) {
                const int g = i / D, d = i % D;
                float O = 0.0f;
#pragma unroll
                for (int w = 0; w < NWA; ++w) O = fmaf(sw[w * G + g], so[(w * G + g) * D + d], O);
                sout[i] = O;
            }
            __syncthreads();
            if (ctl) {      // partials [H][NS][D] and (M, L) [H][NS], write-through
                const auto ro = rsrc(a.part_o);
                for (int c = lane; c < G * D / 4; c += 64) {
                    const int g = c / (D / 4), d4 = c % (D / 4);
                    const float4 o = *(const float4 *)&sout[g * D + 4 * d4];
                    st_sc1(ro, 4 * (((hk * G + g) * NS + jq) * D + 4 * d4),
                           make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(o.w)));
                }
                if (lane < G) {
                    const float2 ml = sML[lane];
                    __hip_atomic_store((uint64_t *)(a.part_ml + (hk * G + lane) * NS + jq),
                                       (uint64_t)__float_as_uint(ml.x) | ((uint64_t)__float_as_uint(ml.y) << 32),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                arrive(counter(a.sync, l, S_A + hk), lane);
                ESTAMP(9)
            }
        }
        // ======================================================== C: merge heads 2u, 2u+1 -> one Q8_K super-block
        if (ctl && jq < 2) {
            const int u = 2 * hk + jq;                    // (2u) / G == hk for G = 4
            poll(counter(a.sync, l, S_A + hk), 1, NS, err, 3u, lane);
            ESTAMP(10)
            const int hl = lane >> 5, c = lane & 31, hh = 2 * u + hl;
            float *cw = xs;                               // [2][NS] split weights
            float *cres = xs + 2 * NS;                    // [256] merged output
            float Lh;
            // the two heads' partials [2][NS][D] into LDS by DMA (32 KB: no registers), issued first: the (m, l) loads
            // below return behind them
            float *cpo = xs + 1024;
            ctl_copy_issue(cpo, a.part_o + (int64_t)(2 * u) * NS * D, 2 * NS * D / 4, lane);
            {
                float2 ml = make_float2(-INFINITY, 0.0f);
                if (c < NS) {
                    const uint64_t v = __hip_atomic_load((const uint64_t *)(a.part_ml + hh * NS + c), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    ml = make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
                }
                const float M = xmax16(max16_f(ml.x));
                const float wt = ml.x == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(ml.x - M);
                if (c < NS) cw[hl * NS + c] = wt;
                wave_sync();
                float t = wt * ml.y;
                t += dpp_f<0xB1>(t); t += dpp_f<0x4E>(t); t += dpp_f<0x141>(t); t += dpp_f<0x140>(t);
                Lh = xsum16(t);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            float4 O0 = make_float4(0, 0, 0, 0), O1 = O0, O2 = O0, O3 = O0;
            auto fma4 = [](float w, float4 o, float4 &acc) {
                acc.x = fmaf(w, o.x, acc.x); acc.y = fmaf(w, o.y, acc.y); acc.z = fmaf(w, o.z, acc.z); acc.w = fmaf(w, o.w, acc.w);
            };
            const float *po = cpo + hl * NS * D + 4 * c;
#pragma unroll 4
            for (int s = 0; s < NS; s += 4) {
                fma4(cw[hl * NS + s], *(const float4 *)(po + (s + 0) * D), O0);
                fma4(cw[hl * NS + s + 1], *(const float4 *)(po + (s + 1) * D), O1);
                fma4(cw[hl * NS + s + 2], *(const float4 *)(po + (s + 2) * D), O2);
                fma4(cw[hl * NS + s + 3], *(const float4 *)(po + (s + 3) * D), O3);
            }
            float4 r;
            r.x = ((O0.x + O1.x) + (O2.x + O3.x)) / Lh;
            r.y = ((O0.y + O1.y) + (O2.y + O3.y)) / Lh;
            r.z = ((O0.z + O1.z) + (O2.z + O3.z)) / Lh;
            r.w = ((O0.w + O1.w) + (O2.w + O3.w)) / Lh;
            *(float4 *)&cres[hl * D + 4 * c] = r;
            wave_sync();
            if (a.dbg) {
                a.dbg[u * 256 + hl * D + 4 * c] = r.x; a.dbg[u * 256 + hl * D + 4 * c + 1] = r.y;
                a.dbg[u * 256 + hl * D + 4 * c + 2] = r.z; a.dbg[u * 256 + hl * D + 4 * c + 3] = r.w;
                if (c == 0) { a.dbg[E + 4 * u + 2 * hl] = Lh; a.dbg[E + 4 * u + 2 * hl + 1] = cw[hl * NS]; }
            }
            // Q8_K of the 256 merged values: lanes 0..15 hold 16 each (q8k_quant16 into this lane's own LDS words,
            // read back by the same lane), then write-through stores: qs 16 B per lane, bsums paired into dwords
            // through a register shuffle, d by lane 0
            uint8_t *cq = (uint8_t *)(cres + 256);        // qs [256] ++ d ++ bsums [16]
            uint4 qv = make_uint4(0, 0, 0, 0);
            int bsv = 0;
            float dv = 0.0f;
            if (lane < 16) {
                float v[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = cres[16 * lane + k];
                q8k_quant16(v, lane, (int8_t *)cq, (float *)(cq + 256), (int16_t *)(cq + 320));
                qv = *(const uint4 *)(cq + 16 * lane);
                bsv = ((const int16_t *)(cq + 320))[lane];
                if (lane == 0) dv = *(const float *)(cq + 256);  // written by lane 0 only
            }
            const int bs_hi = __shfl_down(bsv, 1, 64);
            if (lane < 16) st_sc1(rsrc(a.act), u * 256 + 16 * lane, qv);
            if (lane < 16 && (lane & 1) == 0)
                st_sc1_u32(a.act + E + E / 256 * 4 + u * 32 + 2 * lane, (uint32_t)(uint16_t)bsv | ((uint32_t)bs_hi << 16));
            if (lane == 0) st_sc1_u32(a.act + E + 4 * u, __float_as_uint(dv));
            arrive(counter(a.sync, l, S_C), lane);
            ESTAMP(11)
        }
        // ======================================================== O: x += wo . attn
        if (ctl) {
            poll(counter(a.sync, l, S_C), 1, (H / 2), err, 4u, lane);
            ESTAMP(12)
            ctl_copy(act, a.act, GG::ACTE / 16, lane);
            ESTAMP(13)
        }
        __syncthreads();
        if (!ctl) {
            ActE<E> xa;
            load_act<E>(xa, act, lane, true, false);
#pragma unroll
            for (int i = 0; i < GG::MO; ++i)
                if (os_ + i < oe_ && b * RO + os_ + i < E) {
                    const float v = dot_row<E>(wo[i], xa, false, lane);
                    if (lane == 0) res[os_ + i] = v;
                }
        }
        // compute waves: the first gate|up rows in flight
        int gs_, ge_;
        wave_run(2 * RF, ctl ? 0 : wave, gs_, ge_);
        if (ctl) ge_ = gs_;
        Row<E> wg[GG::WG];
        auto glu_item = [&](int it, const uint8_t *&W, int &row) {
            W = (it & 1) ? L.wu : L.wg;
            row = b * RF + (it >> 1);
        };
        __syncthreads();    // (issued behind the barrier: not live beside wo's rows and activation)
        ESTAMP(14)
        const int ordo = (a.opt >> 2) & 3;
        if (ctl) {
            if (lane < RO && b * RO + lane < E) {
                xres = __fadd_rn(res[lane], xres);
                st_sc1_f32(a.x + b * RO + lane, xres);
            }
            if (ordo != 1) arrive(counter(a.sync, l, S_O + (b >> 5)), lane);
        }
        if (ordo != 0) __syncthreads();
#pragma unroll
        for (int i = 0; i < GG::WG; ++i) {
            const int it = gs_ + i;
            const uint8_t *W; int row;
            glu_item(it, W, row);
            if (it < ge_ && row < F) load_row<E>(wg[i], W, row, false, lane);
            else zero_row<E>(wg[i]);
        }
        if (ctl) {
            if (ordo == 1) arrive(counter(a.sync, l, S_O + (b >> 5)), lane);
            ESTAMP(15)
        }
        // ======================================================== G: ffn_norm -> gate|up -> silu(g) * u
        if (ctl) {
            ctl_fetch(nws, L.ffn_norm, E / 4, lane);
            ctl_gather8(xs, a.x, counter(a.sync, l, S_O), E / 4, GG::NB / 8, true, err, 5u, lane);
            ESTAMP(16)
            const float sc = ctl_scale<E>(xs, a.eps, lane);
            if (lane == 0) *sscale = sc;
            ESTAMP(17)
        }
        __syncthreads();
        quant_lds_norm<E>(xs, nws, *sscale, act, tid);
        __syncthreads();
        ESTAMP(18)
        if (!ctl) {
            ActE<E> xa;
            load_act<E>(xa, act, lane, true, false);
            static_assert(GG::MG % GG::WG == 0, "gate|up ring");
#pragma unroll 1
            for (int i0 = 0; i0 < GG::MG; i0 += GG::WG) {
#pragma unroll
                for (int j = 0; j < GG::WG; ++j) {
                    const int i = i0 + j, it = gs_ + i;
                    const uint8_t *W; int row;
                    glu_item(it, W, row);
                    if (it < ge_ && row < F) {
                        const float v = dot_row<E>(wg[j], xa, false, lane);
                        if (lane == 0) res[it] = v;
                        const int it2 = it + GG::WG;
                        const uint8_t *W2; int row2;
                        glu_item(it2, W2, row2);
                        if (i + GG::WG < GG::MG && it2 < ge_ && row2 < F) load_row<E>(wg[j], W2, row2, false, lane);
                        else zero_row<E>(wg[j]);
                    }
                }
            }
        }
        // compute waves: the first down rows in flight
        int ds_, de_;
        wave_run(RO, ctl ? 0 : wave, ds_, de_);
        if (ctl) de_ = ds_;
        const bool d6 = L.td != 0;
        Row<F> wd[GG::WD];
        __syncthreads();
        ESTAMP(19)
        const int ordg = (a.opt >> 4) & 3;
        if (ctl) {
            const int n = min(RF, F - b * RF);
            if (lane < n) {
                const float g = res[2 * lane], u = res[2 * lane + 1];
                st_sc1_f32(a.h + b * RF + lane, (g / (1.0f + expf(-g))) * u);
            }
            if (ordg != 1) arrive(counter(a.sync, l, S_G + (b >> 5)), lane);
        }
        if (ordg != 0) __syncthreads();
#pragma unroll
        for (int i = 0; i < GG::WD; ++i)
            if (ds_ + i < de_ && b * RO + ds_ + i < E) load_row<F>(wd[i], L.wd, b * RO + ds_ + i, d6, lane);
            else zero_row<F>(wd[i]);
        if (ctl) {
            if (ordg == 1) arrive(counter(a.sync, l, S_G + (b >> 5)), lane);
            ESTAMP(20)
        }
        // ======================================================== D: x += down . Q8_K(h)
        if (ctl) {
            ctl_gather8(xs, a.h, counter(a.sync, l, S_G), F / 4, GG::NB / 8, true, err, 6u, lane);
            ESTAMP(21)
            ESTAMP(22)
        }
        __syncthreads();
        quant_lds<F>(xs, act, tid);
        __syncthreads();
        ESTAMP(23)
        if (!ctl) {
            static_assert(GG::WD == 1, "down: one row in flight per wave");
#pragma unroll 1
            for (int i = 0; i < GG::MO; ++i)
                if (ds_ + i < de_ && b * RO + ds_ + i < E) {
                    const float v = dot_row_lds<F>(wd[0], act, d6, lane);
                    if (lane == 0) res[ds_ + i] = v;
                    if (i + 1 < GG::MO && ds_ + i + 1 < de_ && b * RO + ds_ + i + 1 < E)
                        load_row<F>(wd[0], L.wd, b * RO + ds_ + i + 1, d6, lane);
                    else
                        zero_row<F>(wd[0]);
                }
        }
        __syncthreads();
        ESTAMP(24)
        const int ordd = (a.opt >> 6) & 3;
        if (ctl) {
            if (lane < RO && b * RO + lane < E) {
                xres = __fadd_rn(res[lane], xres);
                st_sc1_f32(a.x + b * RO + lane, xres);
            }
            if (ordd != 1) arrive(counter(a.sync, l, S_D + (b >> 5)), lane);
        }
        if (ordd != 0) __syncthreads();
        if (l + 1 < a.nl) issue_qkv<E, GG>(wq, a.layers[l + 1], b, wave, lane);
        else
#pragma unroll
            for (int i = 0; i < GG::MQ; ++i) zero_row<E>(wq[i]);
        if (ctl) {
            if (ordd == 1) arrive(counter(a.sync, l, S_D + (b >> 5)), lane);
            ESTAMP(25)
        }
    }
}

}  // namespace eng

using namespace eng;

static float *g_dbg = nullptr;
static unsigned long long *g_stamps = nullptr;
// tools only: [NB][nl][32] s_memrealtime stamps of every workgroup's control wave at the phase points (null: off)
extern "C" void kcpp_engine_set_stamps(void *p) { g_stamps = (unsigned long long *)p; }
// tests only: a device buffer of E + 64 floats the next launches write their merged attention rows into (null: off)
extern "C" void kcpp_engine_set_debug(void *p) { g_dbg = (float *)p; }

// bytes of the engine's counter block for nl layers (zeroed once; counters are monotonic across tokens)
extern "C" int64_t kcpp_engine_sync_bytes(int nl) { return ((int64_t)nl * SLOTS + 1) * 128; }

// the geometry the engine is compiled for (host check before choosing it): 1 = covered
extern "C" int kcpp_engine_supported(int E, int F, int H, int HKV, int D, int ncu) {
    return E == 4096 && F == 14336 && H == 32 && HKV == 8 && D == 128 && ncu == Geo<4096, 14336, 32, 8>::NB;
}

// one persistent launch for layers [0, nl) of the table at `layers_dev` (eng::Layer records on the device)
extern "C" int kcpp_engine_decode(const void *layers_dev, int nl, float *x, uint16_t *q16, void *fa_ws, void *act,
                                  float *h, unsigned *sync, const int32_t *pos, const void *rope_tab, float eps,
                                  float kq_scale, int E, int F, int H, int HKV, void *stream) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -1;
    if (!kcpp_engine_supported(E, F, H, HKV, 128, ncu) || nl < 1) return -3;
    using GG = Geo<4096, 14336, 32, 8>;
    static bool attr = false;
    if (!attr) {
        KCPP_CHECK(hipFuncSetAttribute((const void *)k_engine<4096, 14336, 32, 8>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, GG::LDS_REQ));
        attr = true;
    }
    Args a;
    a.layers = (const Layer *)layers_dev;
    a.nl = nl;
    a.x = x;
    a.q16 = q16;
    a.part_o = (float *)((uint8_t *)fa_ws + KCPP_FA_WS_HEADER);
    a.part_ml = (float2 *)(a.part_o + (int64_t)H * GG::CG * 128);
    a.act = (uint8_t *)act;
    a.h = h;
    a.sync = sync;
    a.pos = pos;
    a.rope_tab = (const float2 *)rope_tab;
    a.eps = eps;
    a.kq_scale = kq_scale;
    a.dbg = g_dbg;
    a.stamps = g_stamps;
    static const int opt = [] { const char *e = getenv("KCPP_ENGINE_OPT"); return e ? atoi(e) : 0; }();
    a.opt = opt;
    hipLaunchKernelGGL((k_engine<4096, 14336, 32, 8>), dim3(GG::NB), dim3(NT), GG::LDS_REQ, (hipStream_t)stream, a);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// record size of the device layer table (host side fills eng::Layer through kcpp_engine_layer)
extern "C" int kcpp_engine_layer_bytes(void) { return (int)sizeof(Layer); }
extern "C" void kcpp_engine_layer(void *rec, const void *wq, const void *wk, const void *wv, const void *wo,
                                  const void *wg, const void *wu, const void *wd, const float *attn_norm,
                                  const float *ffn_norm, uint16_t *kc, uint16_t *vc, int v_q6, int down_q6) {
    Layer &L = *(Layer *)rec;
    L.wq = (const uint8_t *)wq; L.wk = (const uint8_t *)wk; L.wv = (const uint8_t *)wv; L.wo = (const uint8_t *)wo;
    L.wg = (const uint8_t *)wg; L.wu = (const uint8_t *)wu; L.wd = (const uint8_t *)wd;
    L.attn_norm = attn_norm; L.ffn_norm = ffn_norm;
    L.kc = kc; L.vc = vc;
    L.tv = v_q6; L.td = down_q6;
}

// the error word (0 = every poll of every launch since the last reset completed)
extern "C" int kcpp_engine_error(const unsigned *sync, int nl, void *stream) {
    unsigned e = 0;
    if (hipMemcpyAsync(&e, sync + (size_t)nl * SLOTS * 32, 4, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return -1;
    return (int)e;
}
