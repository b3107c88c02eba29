// attn.hip -- flash attention over the F16 KV cache (GGML_OP_FLASH_ATTN_EXT).
//
// Semantics: ggml_compute_forward_flash_attn_ext_f16 (reference ggml/src/ggml.c:15667-15875):
// Q is rounded to f16 (q_to_vec_dot), s = (q16 . k16) * scale + mask, softmax over the
// causal window, V-weighted sum.  The CPU accumulates V in f16 (ggml_vec_mad_f16); we keep
// f32 accumulators (strictly more accurate; parity within the f16 rounding of the CPU path).
// The reference GPU path (ggml/src/ggml-cuda/fattn-vec-f16.cuh:4-299) is a 32-lane vector
// kernel with half accumulators; this is a wave64 split-KV design instead:
//   decode  : k_fa_decode  grid (chunks of 256 keys, kv-head, query) -> partial (O, m, l)
//             k_fa_combine one 256-thread block per (query, head pair) -> f32 out (+Q8_K quant)
//   prefill : k_fa_prefill tiled 64 queries x 64 keys per step, online softmax.
#include "kcpp_common.h"
#include "kcpp_internal.h"

#include <algorithm>
#include <cstdlib>

#define FA_CHUNK 64
#define FA_MAXG 8
#define FA_WS_TICKETS 256
#define FA_MAX_CHUNKS 2048
static void *g_fa_stamps = nullptr;       // diagnostic stamp buffer (tools only; kcpp_fa_set_stamps)          // k_fa_combine's chunk-weight table: 2048 x 64 = 131072 keys

// K/V cache layout: [pos][HKV][D] f16, row stride EKV = HKV*D elements.
// Query layout: q16 [T][H][D] f16.  Query t sits at absolute position n_past + t.
// One workgroup = (128-key chunk, kv head, query); its G = H/HKV query heads share every K/V row
// (GQA).  Wave w owns keys 32w..32w+31.  Scores: 16 lanes x 16 B per K row; P.V: lane owns two
// dims and reads one dword of each V row (no cross-lane reduction).  The last workgroup of a
// (query, kv head) to finish -- an agent-scope release/acquire ticket (cdna_hip_programming.md
// Guideline 16) -- merges the chunk partials and, for G >= 2, quantizes the heads' output to
// Q8_K for wo (replaces the reference's separate flash_attn_combine_results launch,
// ggml/src/ggml-cuda/fattn-common.cuh:523).
template <int D, int G, bool FUSED>
__global__ void __launch_bounds__(256) k_fa_decode(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                   const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                   float2 *__restrict__ part_ml, int *__restrict__ tickets,
                                                   float *__restrict__ out, uint8_t *__restrict__ qout, int T, int H,
                                                   int HKV, int n_past_arg, const int32_t *__restrict__ n_past_dev,
                                                   int n_chunks, float scale, const uint16_t *__restrict__ mask,
                                                   int64_t mask_ld, int64_t kv_ld, int64_t kv_hs) {
    static_assert(D == 128, "head dim 128");
    const int c = blockIdx.x, hk = blockIdx.y, t = blockIdx.z;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    // implicit causal window [0, n_past + t] (mask_ld < 0), or the ggml op's explicit form: all n_kv
    // (= n_past_arg) keys under the mask (none if mask is null)
    const int kend = mask_ld >= 0 ? n_past_arg : n_past + t + 1;   // exclusive
    if (c * FA_CHUNK >= kend) return;                    // chunk unused by this query (graph-static grid)
    const int nused = (kend - 1) / FA_CHUNK + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p0 = c * FA_CHUNK;
    const int p1 = min(p0 + FA_CHUNK, kend);              // exclusive
    const uint16_t *mrow = mask ? mask + (int64_t)t * mask_ld : nullptr;
    __shared__ float s_sc[G][FA_CHUNK];
    __shared__ float s_red[4][G][D];
    __shared__ float s_m[G], s_l[G];
    __shared__ int s_last;

    const int sub = lane & 15, kq = lane >> 4;
    float qv[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint4 qq = *(const uint4 *)(q16 + ((int64_t)t * H + hk * G + g) * D + sub * 8);
        const uint32_t w4[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { qv[g][2 * i] = h2f(w4[i] & 0xFFFF); qv[g][2 * i + 1] = h2f(w4[i] >> 16); }
    }
    constexpr int KPW = FA_CHUNK / 4;                    // keys per wave
    uint4 kk[KPW / 4];
#pragma unroll
    for (int i = 0; i < KPW / 4; ++i) {
        const int p = p0 + KPW * wave + 4 * i + kq;
        kk[i] = p < p1 ? *(const uint4 *)(kc + (int64_t)p * kv_ld + hk * kv_hs + sub * 8) : make_uint4(0, 0, 0, 0);
    }
    uint32_t vv[KPW];
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
        const int p = p0 + KPW * wave + i;
        // masked keys are skipped like the CPU does (their V never enters the sum, even if not finite)
        const bool use = p < p1 && !(mrow && mrow[p] == 0xFC00);
        vv[i] = use ? *(const uint32_t *)(vc + (int64_t)p * kv_ld + hk * kv_hs + 2 * lane) : 0u;
    }
#pragma unroll
    for (int i = 0; i < KPW / 4; ++i) {
        const int p = p0 + KPW * wave + 4 * i + kq;
        const uint32_t w4[4] = {kk[i].x, kk[i].y, kk[i].z, kk[i].w};
        float kf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { kf[2 * e] = h2f(w4[e] & 0xFFFF); kf[2 * e + 1] = h2f(w4[e] >> 16); }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float sc = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sc = fmaf(qv[g][e], kf[e], sc);
            sc += dpp_f<0xB1>(sc); sc += dpp_f<0x4E>(sc); sc += dpp_f<0x141>(sc); sc += dpp_f<0x140>(sc);
            if (sub == 0) {
                float sv = -INFINITY;
                if (p < p1) sv = mrow ? (mrow[p] == 0xFC00 ? -INFINITY : sc * scale + h2f(mrow[p])) : sc * scale;
                s_sc[g][p - p0] = sv;
            }
        }
    }
    __syncthreads();
    // softmax statistics of the chunk, one wave per head (lanes cover FA_CHUNK keys)
    for (int g = wave; g < G; g += 4) {
        float m = -INFINITY;
        for (int i = lane; i < FA_CHUNK; i += 64) m = fmaxf(m, s_sc[g][i]);
        m = wave_max_dpp(m);
        float l = 0.0f;
        for (int i = lane; i < FA_CHUNK; i += 64) {
            const float sv = s_sc[g][i];
            const float e = (sv == -INFINITY) ? 0.0f : expf(sv - m);
            s_sc[g][i] = e;
            l += e;
        }
        l = wave_sum_f(l);
        if (lane == 0) { s_m[g] = m; s_l[g] = l; }
    }
    __syncthreads();
    float acc[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g][0] = acc[g][1] = 0.0f;
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
        const float v0 = h2f(vv[i] & 0xFFFF), v1 = h2f(vv[i] >> 16);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float pr = s_sc[g][KPW * wave + i];
            acc[g][0] = fmaf(pr, v0, acc[g][0]);
            acc[g][1] = fmaf(pr, v1, acc[g][1]);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) { s_red[wave][g][2 * lane] = acc[g][0]; s_red[wave][g][2 * lane + 1] = acc[g][1]; }
    __syncthreads();
    for (int i = threadIdx.x; i < G * D; i += 256) {
        const int g = i / D, d = i % D;
        const float o = s_red[0][g][d] + s_red[1][g][d] + s_red[2][g][d] + s_red[3][g][d];
        part_o[(((int64_t)t * H + hk * G + g) * n_chunks + c) * D + d] = o;
    }
    if (threadIdx.x < G) part_ml[((int64_t)t * H + hk * G + threadIdx.x) * n_chunks + c] = make_float2(s_m[threadIdx.x], s_l[threadIdx.x]);
    if constexpr (!FUSED) return;
    // ---- ticket: the last chunk of (t, hk) to finish merges the partials
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(&tickets[t * HKV + hk], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == nused - 1;
        if (s_last) {
            __hip_atomic_store(&tickets[t * HKV + hk], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!s_last) return;
    // chunk weights exp(m_c - M) per head; the denominators
    __shared__ float s_w[G][4096 / FA_CHUNK * 4];
    for (int g = wave; g < G; g += 4) {
        const float2 *ml = part_ml + ((int64_t)t * H + hk * G + g) * n_chunks;
        float M = -INFINITY;
        for (int cc = lane; cc < nused; cc += 64) M = fmaxf(M, ml[cc].x);
        M = wave_max_dpp(M);
        float L = 0.0f;
        for (int cc = lane; cc < nused; cc += 64) {
            const float2 v = ml[cc];
            const float wgt = v.x == -INFINITY ? 0.0f : expf(v.x - M);
            s_w[g][cc] = wgt;
            L = fmaf(wgt, v.y, L);
        }
        L = wave_sum_f(L);
        if (lane == 0) s_l[g] = L;
    }
    __syncthreads();
    float *s_out = &s_red[0][0][0];                        // reuse: G*D floats
    for (int i = threadIdx.x; i < G * D; i += 256) {
        const int g = i / D, d = i % D;
        const float *po = part_o + ((int64_t)t * H + hk * G + g) * n_chunks * D + d;
        float O0 = 0.0f, O1 = 0.0f, O2 = 0.0f, O3 = 0.0f;
        int cc = 0;
        for (; cc + 4 <= nused; cc += 4) {
            O0 = fmaf(s_w[g][cc], po[(int64_t)cc * D], O0);
            O1 = fmaf(s_w[g][cc + 1], po[(int64_t)(cc + 1) * D], O1);
            O2 = fmaf(s_w[g][cc + 2], po[(int64_t)(cc + 2) * D], O2);
            O3 = fmaf(s_w[g][cc + 3], po[(int64_t)(cc + 3) * D], O3);
        }
        for (; cc < nused; ++cc) O0 = fmaf(s_w[g][cc], po[(int64_t)cc * D], O0);
        const float r = ((O0 + O1) + (O2 + O3)) / s_l[g];
        s_out[i] = r;
        if (out) out[(int64_t)t * H * D + (int64_t)(hk * G + g) * D + d] = r;
    }
    if (qout == nullptr || G * D < 256) return;
    __syncthreads();
    // quantize the G*D outputs (G*D/256 Q8_K super-blocks of this kv head's query heads)
    const int nsbk = G * D / 256;
    if ((int)threadIdx.x < nsbk * 16) {
        const int sbl = threadIdx.x >> 4, l16 = threadIdx.x & 15;
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = s_out[sbl * 256 + 16 * l16 + k];
        const int64_t E = (int64_t)H * D, nsb = E / 256;
        const int64_t sbg = (int64_t)hk * nsbk + sbl;      // super-block index within the row
        int8_t *qs = (int8_t *)qout + (int64_t)t * E + sbg * 256;
        float *dp = (float *)(qout + (int64_t)T * E) + (int64_t)t * nsb + sbg;
        int16_t *bs = (int16_t *)(qout + (int64_t)T * E + (int64_t)T * nsb * 4) + (int64_t)t * (E / 16) + sbg * 16;
        q8k_quant16(v, l16, qs, dp, bs);
    }
}

// ---------------------------------------------------------------- decode v2: split-KV + in-launch merge
// One token (T = 1).  Grid (NS splits, kv head), 512 threads, one workgroup per CU at NS = 32 x 8 kv heads.
// Split sp owns keys [p0, p1) of the causal window [0, n_past]; it streams them in 128-key sub-chunks, the
// next one's loads issued before the current one is used (wave w: keys 16w + 4i + (lane >> 4), i < 4; a 16-lane row holds one K row and one V row, 8 dims per
// lane), keeps an online softmax per wave, merges its 4 waves in LDS and publishes (m, l, O) of its G
// heads WRITE-THROUGH (sc1 stores), then adds to the kv head's ticket.  The split whose add comes last
// merges all NS partials with sc1 loads (MI355X_MICROARCH.md, visibility table row 1: one lane per storing
// workgroup adds to one unsharded counter after every storing wave's vmcnt(0) + barrier; the last adder
// loads), writes the f32 output and the Q8_K activation of wo, and resets the ticket.  Replaces the
// reference's flash_attn_vec_ext + flash_attn_combine_results pair (fattn-vec-f16.cuh:4-299,
// fattn-common.cuh:523) and this file's k_fa_decode + k_fa_combine pair (two launches, 1 MB of partials).
typedef unsigned long long fa_u64;
typedef unsigned int fa_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sc1_f2(float2 *p, float2 v) {
    __hip_atomic_store((fa_u64 *)p, ((fa_u64)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_sc1_f2(const float2 *p) {
    const fa_u64 x = __hip_atomic_load((fa_u64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((uint32_t)x), __uint_as_float((uint32_t)(x >> 32)));
}

#define FA2_NS 32
// FA2_W waves per workgroup (16 FA2_W-key sub-chunks): 8, or 4 at G = 8 (register budget)
template <int G, int FA2_W = (G == 8 ? 4 : 8)>
__global__ void __launch_bounds__(64 * FA2_W) k_fa_dec2(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                 const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                 float2 *__restrict__ part_ml, unsigned *__restrict__ tickets,
                                                 float *__restrict__ out, uint8_t *__restrict__ qout, int H, int HKV,
                                                 int n_past_arg, const int32_t *__restrict__ n_past_dev, float scale,
                                                 int probe, int64_t kv_ld, int64_t kv_hs,
                                                 unsigned long long *__restrict__ stamps) {
    constexpr int D = 128;
    // diagnostic phase stamps (tools/fa_dec_bench.py): s_memrealtime (100 MHz, chip-wide) per workgroup,
    // written by lane 0 of wave 0 with a vector store; stamps == nullptr in every product launch
    const int wg_id = blockIdx.y * gridDim.x + blockIdx.x;
#define FA_STAMP(ph)                                                                                   \
    if (stamps && threadIdx.x == 0) {                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
        __hip_atomic_store(&stamps[wg_id * 8 + (ph)], t_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    }
    FA_STAMP(0);
    const int sp = blockIdx.x, NS = gridDim.x, hk = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    const int nkv = n_past + 1;
    const int per = ((nkv + NS - 1) / NS + 3) & ~3;
    const int p0 = min(sp * per, nkv), p1 = min(p0 + per, nkv);
    __shared__ float s_o[FA2_W][G][D];
    __shared__ float s_m[FA2_W][G], s_l[FA2_W][G];
    __shared__ int s_last;

    float qv[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint4 qq = *(const uint4 *)(q16 + (int64_t)(hk * G + g) * D + sub * 8);
        const uint32_t w4[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { qv[g][2 * i] = h2f(w4[i] & 0xFFFF); qv[g][2 * i + 1] = h2f(w4[i] >> 16); }
    }
    if (stamps) { if (qv[0][0] == 12345.0f) stamps[0] = 0; FA_STAMP(1); }
    float m[G], l[G], acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        m[g] = -INFINITY; l[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = 0.0f;
    }
    const uint16_t *kb = kc + hk * kv_hs + sub * 8, *vb = vc + hk * kv_hs + sub * 8;
    uint4 kk[4], vv[4];
    auto load_kv = [&](int c0, uint4 (&kr)[4], uint4 (&vr)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = c0 + 16 * wave + 4 * i + kq;
            kr[i] = p < p1 ? *(const uint4 *)(kb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = c0 + 16 * wave + 4 * i + kq;
            vr[i] = p < p1 ? *(const uint4 *)(vb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
        }
    };
    constexpr bool PF = true;                                       // register budget of the prefetch
    if (PF && p0 < p1) load_kv(p0, kk, vv);
    for (int c0 = p0; c0 < p1; c0 += 16 * FA2_W) {
        uint4 kn[4], vn[4];
        const bool nxt = PF && c0 + 16 * FA2_W < p1;
        if (nxt) load_kv(c0 + 16 * FA2_W, kn, vn);
        if (!PF) load_kv(c0, kk, vv);
        float sc[G][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t w4[4] = {kk[i].x, kk[i].y, kk[i].z, kk[i].w};
            float kf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) { kf[2 * e] = h2f(w4[e] & 0xFFFF); kf[2 * e + 1] = h2f(w4[e] >> 16); }
            const bool valid = c0 + 16 * wave + 4 * i + kq < p1;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float s = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) s = fmaf(qv[g][e], kf[e], s);
                s += dpp_f<0xB1>(s); s += dpp_f<0x4E>(s); s += dpp_f<0x141>(s); s += dpp_f<0x140>(s);
                sc[g][i] = valid ? s * scale : -INFINITY;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float cm = fmaxf(fmaxf(sc[g][0], sc[g][1]), fmaxf(sc[g][2], sc[g][3]));
            cm = xmax32(xmax16(cm));
            const float mn = fmaxf(m[g], cm);
            if (mn == -INFINITY) continue;                          // nothing valid yet (wave-uniform)
            const float alpha = m[g] == -INFINITY ? 0.0f : expf(m[g] - mn);
            m[g] = mn;
            float pr[4];
            float ls = 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) { pr[i] = sc[g][i] == -INFINITY ? 0.0f : expf(sc[g][i] - mn); ls += pr[i]; }
            l[g] = fmaf(l[g], alpha, ls);                           // lane-partial over its own keys
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[g][e] *= alpha;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t w4[4] = {vv[i].x, vv[i].y, vv[i].z, vv[i].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    acc[g][2 * e] = fmaf(pr[i], h2f(w4[e] & 0xFFFF), acc[g][2 * e]);
                    acc[g][2 * e + 1] = fmaf(pr[i], h2f(w4[e] >> 16), acc[g][2 * e + 1]);
                }
            }
        }
        if (nxt) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { kk[i] = kn[i]; vv[i] = vn[i]; }
        }
    }
    FA_STAMP(2);
    // wave merge over its 4 key rows (kq): m is wave-uniform, l and acc are per row
#pragma unroll
    for (int g = 0; g < G; ++g) {
        l[g] = xsum32(xsum16(l[g]));
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = xsum32(xsum16(acc[g][e]));
        if (kq == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) s_o[wave][g][sub * 8 + e] = acc[g][e];
        }
        if (lane == 0) { s_m[wave][g] = m[g]; s_l[wave][g] = l[g]; }
    }
    __syncthreads();
    // workgroup merge of the waves -> this split's partial, published write-through (16-B sc1 stores)
    float2 *pml = part_ml + ((int64_t)hk * NS + sp) * G;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(part_o, 0, 0x7FFFFFFF, 0x00020000);
    for (int j = tid; j < G * D / 4; j += 64 * FA2_W) {
        const int g = (4 * j) / D, d = (4 * j) % D;
        float M = s_m[0][g];
#pragma unroll
        for (int w = 1; w < FA2_W; ++w) M = fmaxf(M, s_m[w][g]);
        float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (M != -INFINITY) {
#pragma unroll
            for (int w = 0; w < FA2_W; ++w) {
                const float wt = s_m[w][g] == -INFINITY ? 0.0f : expf(s_m[w][g] - M);
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = fmaf(wt, s_o[w][g][d + e], o[e]);
            }
        }
        const fa_v4u v = {__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, prs, (int)((((int64_t)hk * NS + sp) * G * D + g * D + d) * 4), 0, 16);
    }
    if (tid < G) {
        const int g = tid;
        float M = s_m[0][g];
#pragma unroll
        for (int w = 1; w < FA2_W; ++w) M = fmaxf(M, s_m[w][g]);
        float L = 0.0f;
        if (M != -INFINITY) {
#pragma unroll
            for (int w = 0; w < FA2_W; ++w) L = fmaf(s_m[w][g] == -INFINITY ? 0.0f : expf(s_m[w][g] - M), s_l[w][g], L);
        }
        st_sc1_f2(pml + g, make_float2(M, L));
    }
    FA_STAMP(3);
    if (tickets == nullptr) {                                       // partials only (combine kernel follows)
        if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(4); }
        return;
    }
    if (probe != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FA_STAMP(4);
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&tickets[hk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned)(NS - 1);
        if (s_last) __hip_atomic_store(&tickets[hk], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    FA_STAMP(5);
    if (!s_last || probe == 3) return;
    // ---- last split of this kv head: merge the NS partials (sc1 loads only).  SS adjacent lanes share one
    // 4-dim quad of one head, each loading every SS-th split (16-B loads, all issued before use), then
    // reduce over the SS lanes: every thread of the workgroup has <= PER partials in flight.
    float *s_res = &s_o[0][0][0];                                  // reuse: G*D floats
    {
        constexpr int NQ = G * D / 4, NT = 64 * FA2_W;
        constexpr int SS = NT / NQ >= 1 ? NT / NQ : 1, PER = (FA2_NS + SS - 1) / SS;
        if (tid < NQ * SS) {
            const int q = tid / SS, sub = tid % SS;
            const int g = q / (D / 4), d = 4 * (q % (D / 4));
            float2 ml[PER];
            fa_v4u ov[PER];
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const int s2 = sub + SS * k;
                ml[k] = s2 < NS ? ld_sc1_f2(part_ml + ((int64_t)hk * NS + s2) * G + g) : make_float2(-INFINITY, 0.0f);
                ov[k] = s2 < NS ? __builtin_amdgcn_raw_buffer_load_b128(prs, (int)((((int64_t)hk * NS + s2) * G * D + g * D + d) * 4), 0, 16)
                                : fa_v4u{0u, 0u, 0u, 0u};
            }
            float M = -INFINITY;
#pragma unroll
            for (int k = 0; k < PER; ++k) M = fmaxf(M, ml[k].x);
#pragma unroll
            for (int o_ = 1; o_ < SS; o_ <<= 1) M = fmaxf(M, __shfl_xor(M, o_, 64));
            float L = 0.0f, o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const float wt = ml[k].x == -INFINITY ? 0.0f : expf(ml[k].x - M);
                L = fmaf(wt, ml[k].y, L);
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = fmaf(wt, __uint_as_float(ov[k][e]), o[e]);
            }
#pragma unroll
            for (int o_ = 1; o_ < SS; o_ <<= 1) {
                L += __shfl_xor(L, o_, 64);
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] += __shfl_xor(o[e], o_, 64);
            }
            if (sub == 0) {
                const float4 r = make_float4(o[0] / L, o[1] / L, o[2] / L, o[3] / L);
                *(float4 *)&s_res[g * D + d] = r;
                if (out) *(float4 *)(out + (int64_t)(hk * G + g) * D + d) = r;
            }
        }
    }
    FA_STAMP(6);
    if (qout == nullptr || G * D < 256) return;
    __syncthreads();
    const int nsbk = G * D / 256;
    if (tid < nsbk * 16) {
        const int sbl = tid >> 4, l16 = tid & 15;
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = s_res[sbl * 256 + 16 * l16 + k];
        const int64_t E = (int64_t)H * D, nsb = E / 256;
        const int64_t sbg = (int64_t)hk * nsbk + sbl;
        int8_t *qs = (int8_t *)qout + sbg * 256;
        float *dp = (float *)(qout + E) + sbg;
        int16_t *bs = (int16_t *)(qout + E + nsb * 4) + sbg * 16;
        q8k_quant16(v, l16, qs, dp, bs);
    }
    if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(7); }
#undef FA_STAMP
}

// combine of k_fa_dec2's partials (decode v3 = k_fa_dec2 without tickets + this): one 256-thread workgroup
// per head pair (= one Q8_K block of 256); 4 adjacent lanes share a 4-dim quad of one head and each loads
// every 4th split (<= 8 x 16-B O loads + 8 x 8-B (m, l) loads per thread, all issued before use), then
// reduce over the 4 lanes.  One barrier, before the Q8_K quantization of the pair's 256 outputs.
template <int G, bool QUANT>
__global__ void __launch_bounds__(256) k_fa_combine2(const float *__restrict__ part_o, const float2 *__restrict__ part_ml,
                                                    float *__restrict__ out, uint8_t *__restrict__ qout, int H, int NS) {
    constexpr int D = 128, SS = 4, PER = FA2_NS / SS;
    const int pair = blockIdx.x, tid = threadIdx.x;
    const int hl = tid >> 7, r = tid & 127, q = r >> 2, sub = r & 3;
    const int h = 2 * pair + hl, hk = h / G, g = h % G, d = 4 * q;
    __shared__ float s_res[2 * D];
    float2 ml[PER];
    float4 ov[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int s2 = sub + SS * k;
        ml[k] = s2 < NS ? part_ml[((int64_t)hk * NS + s2) * G + g] : make_float2(-INFINITY, 0.0f);
        ov[k] = s2 < NS ? *(const float4 *)(part_o + (((int64_t)hk * NS + s2) * G + g) * D + d) : make_float4(0, 0, 0, 0);
    }
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < PER; ++k) M = fmaxf(M, ml[k].x);
    M = fmaxf(M, __shfl_xor(M, 1, 64));
    M = fmaxf(M, __shfl_xor(M, 2, 64));
    float L = 0.0f, o0 = 0.0f, o1 = 0.0f, o2 = 0.0f, o3 = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const float wt = ml[k].x == -INFINITY ? 0.0f : expf(ml[k].x - M);
        L = fmaf(wt, ml[k].y, L);
        o0 = fmaf(wt, ov[k].x, o0); o1 = fmaf(wt, ov[k].y, o1);
        o2 = fmaf(wt, ov[k].z, o2); o3 = fmaf(wt, ov[k].w, o3);
    }
#pragma unroll
    for (int x = 1; x <= 2; x <<= 1) {
        L += __shfl_xor(L, x, 64);
        o0 += __shfl_xor(o0, x, 64); o1 += __shfl_xor(o1, x, 64);
        o2 += __shfl_xor(o2, x, 64); o3 += __shfl_xor(o3, x, 64);
    }
    if (sub == 0) {
        const float4 res = make_float4(o0 / L, o1 / L, o2 / L, o3 / L);
        *(float4 *)&s_res[hl * D + d] = res;
        if (out) *(float4 *)(out + (int64_t)h * D + d) = res;
    }
    if constexpr (QUANT) {
        __syncthreads();
        if (tid < 16) {
            float v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = s_res[16 * tid + k];
            const int64_t E = (int64_t)H * D, nsb = E / 256;
            q8k_quant16(v, tid, (int8_t *)qout + pair * 256, (float *)(qout + E) + pair,
                        (int16_t *)(qout + E + nsb * 4) + pair * 16);
        }
    }
}

#define FA_STAMP(ph)                                                                                   \
    if (stamps && threadIdx.x == 0) {                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
        __hip_atomic_store(&stamps[wg_id * 8 + (ph)], t_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    }
// ---------------------------------------------------------------- decode v4: streaming splits + wide combine
// One token.  Grid (NS splits, kv head), 256 threads.  Split sp owns keys [sp*per, (sp+1)*per) of [0, n_past].
// Wave w streams 16-key groups base = p0 + 16 w + 64 j: lane (kq = lane >> 4, sub = lane & 15) loads 16 B
// (8 dims) of K and of V for keys base + 4 i + kq, i < 4 -- every load instruction 1 KiB contiguous per wave --
// and the next group's 8 loads are issued before the current one is used.  Scores: 8-dim partial dot, 16-lane
// DPP reduction; online softmax per wave (m, l wave-uniform); O: each lane accumulates its 8 dims over its
// row's keys, rows summed once at the end (permlane swaps), waves merged in LDS.  Partials: O [H][NS][128],
// (m, l) [H][NS] (m = -inf for an empty split).
template <int G, bool MERGE>
__global__ void __launch_bounds__(256) k_fa_dec4(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                 const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                 float2 *__restrict__ part_ml, int H, int n_past_arg,
                                                 const int32_t *__restrict__ n_past_dev, int NS, float scale,
                                                 int64_t kv_ld, int64_t kv_hs, unsigned long long *stamps,
                                                 unsigned *__restrict__ tickets, float *__restrict__ out) {
    constexpr int D = 128;
    const int sp = blockIdx.x, hk = blockIdx.y;
    const int wg_id = blockIdx.y * gridDim.x + blockIdx.x;
    FA_STAMP(0);
    const int nkv = (n_past_dev ? n_past_dev[0] : n_past_arg) + 1;
    const int per = (nkv + NS - 1) / NS;
    const int p0 = sp * per, p1 = min(p0 + per, nkv);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
    __shared__ float s_o[4][G][D];
    __shared__ float s_ml[4][G][2];
    __shared__ float s_w[4][G], s_L[G];
    // scores in the exp2 domain: s2 = (q . k) * scale * log2(e); partial m in the same domain
    const float sc2 = scale * 1.4426950408889634f;
    float qv[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint4 qq = *(const uint4 *)(q16 + (int64_t)(hk * G + g) * D + sub * 8);
        const uint32_t w4[4] = {qq.x, qq.y, qq.z, qq.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) { qv[g][2 * e] = h2f(w4[e] & 0xFFFF); qv[g][2 * e + 1] = h2f(w4[e] >> 16); }
    }
    if (stamps) { if (qv[0][0] == 12345.0f) stamps[0] = 0; FA_STAMP(1); }
    const uint16_t *kb = kc + (int64_t)hk * kv_hs + sub * 8, *vb = vc + (int64_t)hk * kv_hs + sub * 8;
    float m[G], l[G], acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        m[g] = -INFINITY; l[g] = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = 0.0f;
    }
    uint4 ka[4], va[4], kn[4], vn[4];
    auto issue = [&](int base, uint4 *kk, uint4 *vv) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = base + 4 * i + kq;
            const bool ok = p < p1;
            kk[i] = ok ? *(const uint4 *)(kb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
            vv[i] = ok ? *(const uint4 *)(vb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
        }
    };
    auto consume = [&](int base, const uint4 *kk, const uint4 *vv) {
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
                for (int e = 0; e < 8; ++e) sc = fmaf(qv[g][e], kf[e], sc);
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
                s[g][i] = base + 4 * i + kq < p1 ? s[g][i] * sc2 : -INFINITY;
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
            const float mn = fmaxf(m[g], mx[g]);           // finite: key base + kq (i = 0) of row 0 is valid
            al[g] = __builtin_amdgcn_exp2f(m[g] - mn);     // m = -inf -> 0
            ls[g] = 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s[g][i] = __builtin_amdgcn_exp2f(s[g][i] - mn);   // -inf -> 0
                ls[g] += s[g][i];
            }
            m[g] = mn;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) ls[g] = xsum16(ls[g]);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            l[g] = fmaf(l[g], al[g], xsum32(ls[g]));
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[g][e] *= al[g];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t w4[4] = {vv[i].x, vv[i].y, vv[i].z, vv[i].w};
            float vf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) { vf[2 * e] = h2f(w4[e] & 0xFFFF); vf[2 * e + 1] = h2f(w4[e] >> 16); }
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(s[g][i], vf[e], acc[g][e]);
        }
    };
    int base = p0 + 16 * wave;
    if (base < p1) issue(base, ka, va);
    for (; base < p1; base += 128) {
        const int b1 = base + 64;
        if (b1 < p1) issue(b1, kn, vn);
        consume(base, ka, va);
        if (stamps && base == p0 + 16 * wave) { if (acc[0][0] == 12345.0f) stamps[0] = 0; FA_STAMP(2); }
        if (b1 >= p1) break;
        if (b1 + 64 < p1) issue(b1 + 64, ka, va);
        consume(b1, kn, vn);
    }
    FA_STAMP(3);
    // rows (kq) hold disjoint keys: park every row's 8 dims in LDS, reduce rows and waves in one pass
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = xsum16(acc[g][e]);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = xsum32(acc[g][e]);
    if (kq == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            *(float4 *)&s_o[wave][g][sub * 8] = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
            *(float4 *)&s_o[wave][g][sub * 8 + 4] = make_float4(acc[g][4], acc[g][5], acc[g][6], acc[g][7]);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) { s_ml[wave][g][0] = m[g]; s_ml[wave][g][1] = l[g]; }
    }
    __syncthreads();
    if (tid < G) {                                        // per-head wave weights and the split's (M, L)
        const int g = tid;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) M = fmaxf(M, s_ml[w][g][0]);
        float L = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const float wt = M == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(s_ml[w][g][0] - M);
            s_w[w][g] = wt;
            L = fmaf(wt, s_ml[w][g][1], L);
        }
        s_L[g] = L;
        part_ml[(int64_t)(hk * G + g) * NS + sp] = make_float2(M, L);
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += 256) {
        const int g = i / D, d = i % D;
        float O = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) O = fmaf(s_w[w][g], s_o[w][g][d], O);
        part_o[((int64_t)(hk * G + g) * NS + sp) * D + d] = O;
    }
    FA_STAMP(4);
    if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(5); }
    if constexpr (MERGE) {
        // the last split of this kv head to finish merges all NS partials (release / agent-scope ticket /
        // acquire, as k_fa_decode's fused form) and writes the f32 attention output
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned prev = __hip_atomic_fetch_add(&tickets[hk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = prev == (unsigned)(NS - 1);
            if (s_last) {
                __hip_atomic_store(&tickets[hk], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (!s_last) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        FA_STAMP(6);
        // split weights: wave w forms exp2(m_s - M) of heads w, w + 4 in LDS (NS <= 64 = one lane each)
        __shared__ float s_sw[G][64];
        __shared__ float s_sl[G];
        for (int g = wave; g < G; g += 4) {
            const float2 v = lane < NS ? part_ml[(int64_t)(hk * G + g) * NS + lane] : make_float2(-INFINITY, 0.0f);
            const float M = wave_max_dpp(v.x);
            const float wt = v.x == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(v.x - M);
            s_sw[g][lane] = wt;
            const float L = wave_sum_f(wt * v.y);
            if (lane == 0) s_sl[g] = L;
        }
        __syncthreads();
        for (int i = tid; i < G * D; i += 256) {
            const int g = i / D, d = i % D;
            const float *po = part_o + (int64_t)(hk * G + g) * NS * D + d;
            float ov[64];
#pragma unroll
            for (int s2 = 0; s2 < 64; ++s2) ov[s2] = s2 < NS ? po[(int64_t)s2 * D] : 0.0f;
            float O0 = 0.0f, O1 = 0.0f, O2 = 0.0f, O3 = 0.0f;
#pragma unroll
            for (int s2 = 0; s2 < 64; s2 += 4) {
                O0 = fmaf(s_sw[g][s2], ov[s2], O0);
                O1 = fmaf(s_sw[g][s2 + 1], ov[s2 + 1], O1);
                O2 = fmaf(s_sw[g][s2 + 2], ov[s2 + 2], O2);
                O3 = fmaf(s_sw[g][s2 + 3], ov[s2 + 3], O3);
            }
            out[(int64_t)(hk * G + g) * D + d] = ((O0 + O1) + (O2 + O3)) / s_sl[g];
        }
        if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(7); }
    }
}

// combine of k_fa_dec4's partials (m in the exp2 domain): grid (H / 2), 256 threads = 2 heads x 128 dims
// (one Q8_K block of 256 when quantizing); thread (head, d) issues all NS partial loads of its dim (<= 64, in
// flight together); one wave per head forms the split weights exp2(m_s - M) in LDS.
template <bool QUANT>
__global__ void __launch_bounds__(256) k_fa_comb4(const float *__restrict__ part_o, const float2 *__restrict__ part_ml,
                                                  float *__restrict__ out, uint8_t *__restrict__ qout, int H, int NS,
                                                  unsigned long long *stamps) {
    constexpr int D = 128, MAXS = 64;
    const int pair = blockIdx.x, tid = threadIdx.x;
    const int wg_id = 2048 + blockIdx.x;
    FA_STAMP(0);
    const int hl = tid >> 7, d = tid & 127, h = 2 * pair + hl;
    __shared__ float s_w[2][MAXS];
    __shared__ float s_l[2];
    __shared__ float s_res[2 * D];
    const float *po = part_o + (int64_t)h * NS * D + d;
    float ov[MAXS];
#pragma unroll
    for (int s = 0; s < MAXS; ++s) ov[s] = s < NS ? po[(int64_t)s * D] : 0.0f;
    if (d < 64) {                                        // wave 0 / 2: split weights of head hl
        const float2 v = d < NS ? part_ml[(int64_t)h * NS + d] : make_float2(-INFINITY, 0.0f);
        const float M = wave_max_dpp(v.x);
        const float wt = v.x == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(v.x - M);
        s_w[hl][d] = wt;
        const float L = wave_sum_f(wt * v.y);
        if (d == 0) s_l[hl] = L;
    }
    __syncthreads();
    FA_STAMP(1);
    float O0 = 0.0f, O1 = 0.0f, O2 = 0.0f, O3 = 0.0f;
#pragma unroll
    for (int s = 0; s < MAXS; s += 4) {
        O0 = fmaf(s_w[hl][s], ov[s], O0);
        O1 = fmaf(s_w[hl][s + 1], ov[s + 1], O1);
        O2 = fmaf(s_w[hl][s + 2], ov[s + 2], O2);
        O3 = fmaf(s_w[hl][s + 3], ov[s + 3], O3);
    }
    const float res = ((O0 + O1) + (O2 + O3)) / s_l[hl];
    FA_STAMP(2);
    if (out) out[(int64_t)h * D + d] = res;
    if constexpr (QUANT) {
        s_res[tid] = res;
        __syncthreads();
        if (tid < 16) {
            float v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = s_res[16 * tid + k];
            const int64_t E = (int64_t)H * D, nsb = E / 256;
            q8k_quant16(v, tid, (int8_t *)qout + pair * 256, (float *)(qout + E) + pair,
                        (int16_t *)(qout + E + nsb * 4) + pair * 16);
        }
    }
    if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(3); }
}

#undef FA_STAMP

// split count of k_fa_dec4: one workgroup per CU (256 / HKV splits; measured at 3850 cached keys,
// tools/fa_dec_bench.py: 7.8 us vs 8.7 at 512 workgroups).  Independent of the context size, so the key
// partition -- and the result, bit for bit -- depends on the cached keys only (empty splits exit early).
static int fa4_splits(int n_kv_max, int HKV) {
    (void)n_kv_max;
    static const int ns_env = getenv("KCPP_FA4_NS") ? atoi(getenv("KCPP_FA4_NS")) : 0;
    const int ns = ns_env > 0 ? ns_env : 256 / HKV;
    return std::max(1, std::min(ns, 64));
}

static int fa4_launch(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                      float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                      int n_kv_max, float scale, hipStream_t s) {
    const int G = H / HKV;
    const int NS = fa4_splits(n_kv_max, HKV);
    float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
    float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
    const dim3 grid(NS, HKV);
    // in-launch merge by the last split of each kv head: opt-in only -- measured 17.9 vs 12.3 us per layer at 3850
    // keys (tools/fa_dec_bench.py variant 4 vs 3: the agent-scope ticket lands ~5 us after the partial stores and
    // the single merging workgroup per kv head reads its 64 KB of partials in ~4.6 us), the combine launch is cheaper
    static const int merge_env = getenv("KCPP_FA4_MERGE") ? atoi(getenv("KCPP_FA4_MERGE")) : 0;
    const bool merge = merge_env && qout == nullptr && out != nullptr && HKV * 4 <= FA_WS_TICKETS;
    unsigned *tk = (unsigned *)ws;
    unsigned long long *st = (unsigned long long *)g_fa_stamps;
#define KCPP_FA4_CASE(GG)                                                                                               \
    case GG:                                                                                                            \
        if (merge) hipLaunchKernelGGL((k_fa_dec4<GG, true>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past, n_past_dev, NS, scale, kv_ld, kv_hs, st, tk, out); \
        else hipLaunchKernelGGL((k_fa_dec4<GG, false>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past, n_past_dev, NS, scale, kv_ld, kv_hs, st, tk, out); \
        break;
    switch (G) {
        KCPP_FA4_CASE(1) KCPP_FA4_CASE(2) KCPP_FA4_CASE(4) KCPP_FA4_CASE(8)
    default: return -1;
    }
#undef KCPP_FA4_CASE
    KCPP_CHECK(hipGetLastError());
    if (merge) return 0;
    if (qout) hipLaunchKernelGGL(k_fa_comb4<true>, dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS, (unsigned long long *)g_fa_stamps);
    else hipLaunchKernelGGL(k_fa_comb4<false>, dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, H, NS, (unsigned long long *)g_fa_stamps);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// combine split-KV partials; one 1024-thread workgroup covers two heads (= one Q8_K block of 256).
// Latency-bound (a few hundred KB from L2), so it is built for memory-level parallelism: every
// thread issues its 16 partial-O loads (4 threads per output dim split the chunks) together with
// the chunk (m, l) loads, then the chunk weights exp(m_c - M) are formed in LDS and applied.
template <bool QUANT>
__global__ void __launch_bounds__(1024) k_fa_combine(const float *__restrict__ part_o, const float2 *__restrict__ part_ml,
                                                     float *__restrict__ out, uint8_t *__restrict__ qout, int T, int H,
                                                     int D, int n_past_arg, const int32_t *__restrict__ n_past_dev,
                                                     int n_chunks_alloc, int masked) {
    constexpr int MAXCH = FA_MAX_CHUNKS;               // 128k context
    const int t = blockIdx.y;
    const int pair = blockIdx.x;                       // heads 2*pair, 2*pair+1
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hl = tid >> 9, r = tid & 511, d = r & 127, cg = r >> 7;
    const int h = 2 * pair + hl;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    const int nch = masked ? (n_past_arg - 1) / FA_CHUNK + 1    // explicit mask: all n_kv keys
                           : (n_past + t) / FA_CHUNK + 1;     // chunks this query actually used
    __shared__ float s_w[2][MAXCH];
    __shared__ float s_red[16];
    __shared__ float s_sum[2][4][128];
    const float2 *ml = part_ml + ((int64_t)t * H + h) * n_chunks_alloc;
    const float *po = part_o + ((int64_t)t * H + h) * n_chunks_alloc * 128 + d;
    // (m, l) of chunk r (r < nch), and this thread's first 16 O partials, all in flight together
    const float2 mlv = r < nch ? ml[r] : make_float2(-INFINITY, 0.0f);
    float ov[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int c = cg + 4 * k;
        ov[k] = c < nch ? po[(int64_t)c * 128] : 0.0f;
    }
    // M = max_c m_c per head: waves 0-7 hold head 0's chunks, 8-15 head 1's (chunks beyond 512: strided)
    float mloc = mlv.x;
    for (int c = r + 512; c < nch; c += 512) mloc = fmaxf(mloc, ml[c].x);
    float M = wave_max(mloc);
    if (lane == 0) s_red[wave] = M;
    __syncthreads();
    M = s_red[8 * hl];
#pragma unroll
    for (int w = 1; w < 8; ++w) M = fmaxf(M, s_red[8 * hl + w]);
    const float wgt = mlv.x == -INFINITY ? 0.0f : expf(mlv.x - M);
    if (r < MAXCH) s_w[hl][r] = wgt;
    float lsum = wgt * mlv.y;
    for (int c = r + 512; c < nch; c += 512) {
        const float2 v = ml[c];
        const float w2 = v.x == -INFINITY ? 0.0f : expf(v.x - M);
        s_w[hl][c] = w2;
        lsum = fmaf(w2, v.y, lsum);
    }
    float L = wave_sum(lsum);
    __syncthreads();                                   // s_red reuse + s_w visible
    if (lane == 0) s_red[wave] = L;
    __syncthreads();
    L = 0.0f;
#pragma unroll
    for (int w = 0; w < 8; ++w) L += s_red[8 * hl + w];
    float O = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int c = cg + 4 * k;
        if (c < nch) O = fmaf(s_w[hl][c], ov[k], O);
    }
    for (int c0 = 64; c0 < nch; c0 += 64) {            // contexts beyond 64 chunks
#pragma unroll 4
        for (int k = 0; k < 16; ++k) {
            const int c = c0 + cg + 4 * k;
            if (c < nch) O = fmaf(s_w[hl][c], po[(int64_t)c * 128], O);
        }
    }
    s_sum[hl][cg][d] = O;
    __syncthreads();
    if (cg == 0) {
        const float res = ((s_sum[hl][0][d] + s_sum[hl][1][d]) + (s_sum[hl][2][d] + s_sum[hl][3][d])) / L;
        const int64_t e = (int64_t)t * H * 128 + (int64_t)h * 128 + d;
        if (out) out[e] = res;
        s_sum[hl][0][d] = res;
    }
    if constexpr (QUANT) {
        __syncthreads();
        if (tid < 16) {                                // lane j holds elements 16j..16j+15 of the block
            float v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int e = 16 * tid + k;
                v[k] = s_sum[e >> 7][0][e & 127];
            }
            const int64_t E = (int64_t)H * 128;
            const int64_t nsb = E / 256;
            int8_t *qs = (int8_t *)qout + (int64_t)t * E + pair * 256;
            float *dp = (float *)(qout + (int64_t)T * E) + (int64_t)t * nsb + pair;
            int16_t *bs = (int16_t *)(qout + (int64_t)T * E + (int64_t)T * nsb * 4) + (int64_t)t * (E / 16) + pair * 16;
            q8k_quant16(v, tid, qs, dp, bs);
        }
    }
}

// ---------------------------------------------------------------- prefill (tiled, online softmax)
// grid (ceil(T/64), H), block 256.  Thread (ty = tid/16, tx = tid%16): query rows 4*ty..4*ty+3,
// S columns tx + 16*j (j<4) and O dims tx*8 .. tx*8+7 (8 dims).
#define FP_BQ 64
#define FP_BK 64
// D = 128 or 64 (TinyLlama-class heads): thread tx owns DPT = D / 16 output dims; n_past from n_past_dev when given
// (single-token decode replayed from a graph)
template <int D>
__global__ void __launch_bounds__(256) k_fa_prefill(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                    const uint16_t *__restrict__ vc, float *__restrict__ out, int T,
                                                    int H, int HKV, int n_past_arg, float scale,
                                                    const uint16_t *__restrict__ mask, int64_t mask_ld, int n_kv,
                                                    const int32_t *__restrict__ n_past_dev) {
    constexpr int DPT = D / 16;
    const int n_past = n_past_dev ? n_past_dev[0] : n_past_arg;
    const int qt = blockIdx.x, h = blockIdx.y;
    const int G = H / HKV, hk = h / G;
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    const int64_t EKV = (int64_t)HKV * D;
    __shared__ float sQ[FP_BQ][D + 1];
    __shared__ float sK[FP_BK][D + 1];
    __shared__ float sV[FP_BK][D];
    const int q0 = qt * FP_BQ;
    for (int i = tid; i < FP_BQ * D; i += 256) {
        const int r = i / D, d = i % D;
        sQ[r][d] = (q0 + r < T) ? h2f(q16[((int64_t)(q0 + r) * H + h) * D + d]) : 0.0f;
    }
    float m[4], l[4], o[4][DPT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = -INFINITY; l[r] = 0.0f;
#pragma unroll
        for (int j = 0; j < DPT; ++j) o[r][j] = 0.0f;
    }
    const int last_q = min(q0 + FP_BQ, T) - 1;
    const bool expl = mask_ld >= 0;                       // explicit ggml mask form (mask may be null)
    const int kend = expl ? n_kv : n_past + last_q + 1;   // keys needed by this tile (exclusive)
    __shared__ int s_dead[FP_BK];
    for (int k0 = 0; k0 < kend; k0 += FP_BK) {
        __syncthreads();
        if (expl && mask && tid < FP_BK) {               // keys masked for every query of the tile are skipped
            int dead = 1;                                // (their V may be anything, as on the CPU)
            const int p = k0 + tid;
            for (int qi = q0; qi <= last_q && dead && p < kend; ++qi) dead = mask[(int64_t)qi * mask_ld + p] == 0xFC00;
            s_dead[tid] = dead;
        }
        __syncthreads();
        for (int i = tid; i < FP_BK * D / 2; i += 256) {
            const int r = i / (D / 2), d2 = i % (D / 2);
            const int p = k0 + r;
            uint32_t kk = 0, vv = 0;
            if (p < kend) {
                kk = *(const uint32_t *)(kc + (int64_t)p * EKV + hk * D + 2 * d2);
                if (!(expl && mask && s_dead[r])) vv = *(const uint32_t *)(vc + (int64_t)p * EKV + hk * D + 2 * d2);
            }
            sK[r][2 * d2] = h2f(kk & 0xFFFF); sK[r][2 * d2 + 1] = h2f(kk >> 16);
            sV[r][2 * d2] = h2f(vv & 0xFFFF); sV[r][2 * d2 + 1] = h2f(vv >> 16);
        }
        __syncthreads();
        float s[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) s[r][j] = 0.0f;
        for (int d = 0; d < D; ++d) {
            float qd[4], kd[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) qd[r] = sQ[4 * ty + r][d];
#pragma unroll
            for (int j = 0; j < 4; ++j) kd[j] = sK[tx + 16 * j][d];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < 4; ++j) s[r][j] = fmaf(qd[r], kd[j], s[r][j]);
        }
        // online softmax per query row; the 16 threads of a row-group (same ty) share rows
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qi = q0 + 4 * ty + r;
            const int qpos = n_past + qi;
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = k0 + tx + 16 * j;
                if (expl) {
                    const uint16_t mv = (qi < T && p < kend) ? (mask ? mask[(int64_t)qi * mask_ld + p] : (uint16_t)0)
                                                             : (uint16_t)0xFC00;
                    s[r][j] = mv == 0xFC00 ? -INFINITY : s[r][j] * scale + h2f(mv);
                } else {
                    s[r][j] = (qi < T && p <= qpos) ? s[r][j] * scale : -INFINITY;
                }
                mx = fmaxf(mx, s[r][j]);
            }
            mx = fmaxf(mx, __shfl_xor(mx, 1, 64)); mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 4, 64)); mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
            const float mnew = fmaxf(m[r], mx);
            const float alpha = (mnew == -INFINITY) ? 1.0f : expf(m[r] - mnew);
            float ls = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s[r][j] = (s[r][j] == -INFINITY) ? 0.0f : expf(s[r][j] - mnew);
                ls += s[r][j];
            }
            ls += __shfl_xor(ls, 1, 64); ls += __shfl_xor(ls, 2, 64);
            ls += __shfl_xor(ls, 4, 64); ls += __shfl_xor(ls, 8, 64);
            l[r] = l[r] * alpha + ls;
            m[r] = mnew;
#pragma unroll
            for (int j = 0; j < DPT; ++j) o[r][j] *= alpha;
        }
        // O += P V : P row r lives across the 16 tx-threads of the group (4 cols each)
        for (int src = 0; src < 16; ++src) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kr = src + 16 * j;
                float vr[DPT];
#pragma unroll
                for (int e = 0; e < DPT; ++e) vr[e] = sV[kr][tx * DPT + e];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pr = __shfl(s[r][j], ((16 * ty) & 63) + src, 64);
#pragma unroll
                    for (int e = 0; e < DPT; ++e) o[r][e] = fmaf(pr, vr[e], o[r][e]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int qi = q0 + 4 * ty + r;
        if (qi < T) {
            const float inv = 1.0f / l[r];
#pragma unroll
            for (int e = 0; e < DPT; ++e) out[((int64_t)qi * H + h) * D + tx * DPT + e] = o[r][e] * inv;
        }
    }
}

extern "C" {

// partial O + (m, l) per (query, head, chunk) + one ticket per (query, kv head).  The tickets must be
// zero before first use (allocate zeroed); the merging workgroup resets its ticket.
int64_t kcpp_fa_workspace_bytes(int T, int H, int n_kv_max) {
    const int64_t nch = (n_kv_max + FA_CHUNK - 1) / FA_CHUNK;
    // partial slots: T x nch chunks (k_fa_decode), at least the 64 splits k_fa_dec4 may use
    const int64_t slots = std::max<int64_t>((int64_t)T * nch, 64);
    return 256 + (int64_t)H * slots * (128 * 4 + 8) + (int64_t)T * H * 4 + 256;
}
// the first 256 B of the workspace are the decode-v2 tickets (one per kv head, zero between launches)

// out f32 [T][H][D] (may be null), qout Q8_K act [T][H*D] (may be null), ws from kcpp_fa_workspace_bytes
// n_past_dev (optional): device-resident n_past (graph-replayable decode); then n_kv_max
// bounds the grid and the kernels read the real n_past from memory.
int kcpp_flash_attn(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qout, void *ws,
                    int T, int H, int HKV, int D, int n_past, const int32_t *n_past_dev, int n_kv_max, float scale,
                    int force_path, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if ((D != 128 && D != 64) || H % HKV || (H % 2)) return -1;
    if (D == 64) {       // 64-dim heads (TinyLlama class): the tiled kernel for decode and prefill alike
        if (!out) return -2;
        hipLaunchKernelGGL(k_fa_prefill<64>, dim3((T + FP_BQ - 1) / FP_BQ, H), dim3(256), 0, s, q16, kc, vc, out, T, H,
                           HKV, n_past, scale, nullptr, -1, 0, n_past_dev);
        KCPP_CHECK(hipGetLastError());
        if (qout) return kcpp_quantize_act(KT_Q8_K, out, (int64_t)H * D, qout, (int64_t)H * D, T, stream);
        return 0;
    }
    if (H / HKV > FA_MAXG) return -1;
    const bool use_decode = force_path == 1 || force_path == 4 || force_path == 5 || (force_path == 0 && T <= 16);
    static const int v2_env = getenv("KCPP_FA_V2") ? atoi(getenv("KCPP_FA_V2")) : 0;   // in-launch merge: slower end to end (422 vs 443 tok/s)
    const int G0 = H / HKV;
    static const int v3_env = getenv("KCPP_FA_V3") ? atoi(getenv("KCPP_FA_V3")) : 0;
    const bool v3 = (v3_env || force_path == 5) && !(force_path == 4);
    static const int fa4_env = getenv("KCPP_FA4") ? atoi(getenv("KCPP_FA4")) : 1;
    if (use_decode && T == 1 && (force_path == 0 || force_path == 1) && fa4_env && !v2_env && !v3_env && (G0 == 1 || G0 == 2 || G0 == 4 || G0 == 8) &&
        (qout == nullptr || G0 >= 2))
        return fa4_launch(q16, kc, vc, (int64_t)HKV * 128, 128, out, qout, ws, H, HKV, n_past, n_past_dev,
                          n_past_dev ? n_kv_max : n_past + 1, scale, s);
    if (use_decode && T == 1 && (v2_env || v3 || force_path == 4) && HKV <= 64 && (G0 == 1 || G0 == 2 || G0 == 4 || G0 == 8) && (qout == nullptr || G0 >= 2)) {
        const int nkv = n_past_dev ? n_kv_max : n_past + 1;
        const int NS = std::max(1, std::min(FA2_NS, (nkv + 127) / 128));   // >= 1 sub-chunk of 128 keys per split
        static const int nomerge_env = getenv("KCPP_FA2_NOMERGE") ? atoi(getenv("KCPP_FA2_NOMERGE")) : 0;
        const int nomerge = v3 ? 1 : nomerge_env;
        unsigned *tickets = nomerge == 1 ? nullptr : (unsigned *)ws;
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
        const dim3 grid(NS, HKV);
        switch (G0) {
        case 1: hipLaunchKernelGGL(k_fa_dec2<1>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, nomerge, (int64_t)HKV * 128, (int64_t)128, nullptr); break;
        case 2: hipLaunchKernelGGL(k_fa_dec2<2>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, nomerge, (int64_t)HKV * 128, (int64_t)128, nullptr); break;
        case 4: hipLaunchKernelGGL(k_fa_dec2<4>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, nomerge, (int64_t)HKV * 128, (int64_t)128, nullptr); break;
        default: hipLaunchKernelGGL(k_fa_dec2<8>, grid, dim3(256), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, nomerge, (int64_t)HKV * 128, (int64_t)128, nullptr); break;
        }
        KCPP_CHECK(hipGetLastError());
        if (v3) {
#define KCPP_FA_C2(GG)                                                                                                     \
    case GG:                                                                                                               \
        if (qout) hipLaunchKernelGGL((k_fa_combine2<GG, true>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS); \
        else hipLaunchKernelGGL((k_fa_combine2<GG, false>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS);    \
        break;
            switch (G0) { KCPP_FA_C2(1) KCPP_FA_C2(2) KCPP_FA_C2(4) KCPP_FA_C2(8) }
#undef KCPP_FA_C2
            KCPP_CHECK(hipGetLastError());
        }
        return 0;
    }
    if (use_decode) {
        ws = (uint8_t *)ws + FA_WS_TICKETS;
        const int nkv = n_past_dev ? n_kv_max : n_past + T;
        const int nch = (nkv + FA_CHUNK - 1) / FA_CHUNK;
        if (nch > FA_MAX_CHUNKS) return -4;              // combine's chunk-weight table (128k context)
        float *po = (float *)ws;
        float2 *pml = (float2 *)(po + (int64_t)T * H * nch * 128);
        const dim3 grid(nch, HKV, T);
        int *tickets = (int *)(pml + (int64_t)T * H * nch);
        const int G = H / HKV;
        static const int fuse_env = getenv("KCPP_FA_FUSED") ? atoi(getenv("KCPP_FA_FUSED")) : 0;
        const bool fused = fuse_env && G >= 2 && nch <= 4096 / FA_CHUNK * 4;   // (its merge table: 16k keys)
#define KCPP_FA_CASE(GG)                                                                                       \
    case GG:                                                                                                   \
        if (fused)                                                                                             \
            hipLaunchKernelGGL((k_fa_decode<128, GG, true>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, tickets, \
                               out, (uint8_t *)qout, T, H, HKV, n_past, n_past_dev, nch, scale, nullptr, -1,   \
                               (int64_t)HKV * 128, (int64_t)128);                                          \
        else                                                                                                   \
            hipLaunchKernelGGL((k_fa_decode<128, GG, false>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, tickets, \
                               out, (uint8_t *)qout, T, H, HKV, n_past, n_past_dev, nch, scale, nullptr, -1,   \
                               (int64_t)HKV * 128, (int64_t)128);                                          \
        break;
        switch (G) {
            KCPP_FA_CASE(1)
            KCPP_FA_CASE(2)
            KCPP_FA_CASE(4)
            KCPP_FA_CASE(8)
        default: return -3;
        }
#undef KCPP_FA_CASE
        KCPP_CHECK(hipGetLastError());
        if (!fused) {
            if (qout)
                hipLaunchKernelGGL(k_fa_combine<true>, dim3(H / 2, T), dim3(1024), 0, s, po, pml, out, (uint8_t *)qout, T,
                                   H, D, n_past, n_past_dev, nch, 0);
            else
                hipLaunchKernelGGL(k_fa_combine<false>, dim3(H / 2, T), dim3(1024), 0, s, po, pml, out, (uint8_t *)nullptr,
                                   T, H, D, n_past, n_past_dev, nch, 0);
        }
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (!out) return -2;
    // prefill: MFMA kernel (attn_mfma.hip) for GQA groups of 4 (force_path 3, or auto), else FMA tiles (2)
    static const int mfma_env = getenv("KCPP_FA_MFMA") ? atoi(getenv("KCPP_FA_MFMA")) : 1;
    int rc = -3;
    if (force_path == 3 || (force_path == 0 && mfma_env))
        rc = kcpp_flash_attn_prefill_mfma(q16, kc, vc, out, T, H, HKV, D, n_past, scale, stream);
    if (rc == -3 && force_path == 3) return -3;
    if (rc == -3)
        hipLaunchKernelGGL(k_fa_prefill<128>, dim3((T + FP_BQ - 1) / FP_BQ, H), dim3(256), 0, s, q16, kc, vc, out, T, H, HKV,
                           n_past, scale, nullptr, -1, 0, (const int32_t *)nullptr);
    else if (rc)
        return rc;
    KCPP_CHECK(hipGetLastError());
    if (qout) return kcpp_quantize_act(KT_Q8_K, out, (int64_t)H * D, qout, (int64_t)H * D, T, stream);
    return 0;
}

// single-token decode attention with explicit cache strides (elements): key p of kv head hk starts at
// kc + p * kv_ld + hk * kv_hs.  Position-major ggml view: kv_ld = HKV*D, kv_hs = D; head-major: kv_ld = D,
// kv_hs = n_ctx*D.  variant 0: 64-key chunks + k_fa_combine; 1: NS splits, last arriver merges in-launch;
// 2: NS splits + k_fa_combine2.  (tools/fa_dec_bench.py)

void kcpp_fa_set_stamps(void *p) { g_fa_stamps = p; }     // diagnostic stamp buffer of k_fa_dec2 (tools only)
int kcpp_fa_decode_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                      float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                      int n_kv_max, float scale, int variant, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int G = H / HKV;
    if (H % HKV || !(G == 1 || G == 2 || G == 4 || G == 8) || (H % 2) || HKV > 64) return -1;
    if (qout && G < 2) return -1;
    const int nkv = n_past_dev ? n_kv_max : n_past + 1;
    if (variant == 0) {
        const int nch = (nkv + FA_CHUNK - 1) / FA_CHUNK;
        if (nch > FA_MAX_CHUNKS) return -4;
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)H * nch * 128);
        const dim3 grid(nch, HKV, 1);
#define KCPP_FA_CASE(GG)                                                                                         \
    case GG:                                                                                                     \
        hipLaunchKernelGGL((k_fa_decode<128, GG, false>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, nullptr, out, \
                           (uint8_t *)qout, 1, H, HKV, n_past, n_past_dev, nch, scale, nullptr, -1, kv_ld, kv_hs); \
        break;
        switch (G) { KCPP_FA_CASE(1) KCPP_FA_CASE(2) KCPP_FA_CASE(4) KCPP_FA_CASE(8) }
#undef KCPP_FA_CASE
        KCPP_CHECK(hipGetLastError());
        if (qout) hipLaunchKernelGGL(k_fa_combine<true>, dim3(H / 2, 1), dim3(1024), 0, s, po, pml, out, (uint8_t *)qout, 1, H, 128, n_past, n_past_dev, nch, 0);
        else hipLaunchKernelGGL(k_fa_combine<false>, dim3(H / 2, 1), dim3(1024), 0, s, po, pml, out, (uint8_t *)nullptr, 1, H, 128, n_past, n_past_dev, nch, 0);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (variant >= 10 && variant <= 13) {         // timing probes (tools/fa_dec_bench.py): pieces of variant 3
        const int NS = fa4_splits(nkv, HKV);
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
        const int32_t *npd = variant == 12 ? nullptr : n_past_dev;
        const int np = variant == 12 ? nkv - 1 : n_past;
        if (variant != 11 && G == 4)
            hipLaunchKernelGGL((k_fa_dec4<4, false>), dim3(NS, HKV), dim3(256), 0, s, q16, kc, vc, po, pml, H, np, npd, NS, scale, kv_ld, kv_hs, (unsigned long long *)g_fa_stamps, (unsigned *)ws, out);
        if (variant == 11 || variant == 13)
            hipLaunchKernelGGL(k_fa_comb4<true>, dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS, (unsigned long long *)g_fa_stamps);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (variant == 3) return fa4_launch(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, nkv, scale, s);
    if (variant == 4) return fa4_launch(q16, kc, vc, kv_ld, kv_hs, out, nullptr, ws, H, HKV, n_past, n_past_dev, nkv, scale, s);
    const int NS = std::max(1, std::min(FA2_NS, (nkv + 127) / 128));
    unsigned *tickets = variant == 1 ? (unsigned *)ws : nullptr;
    float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
    float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
    const dim3 grid(NS, HKV);
    const int probe = variant == 1 ? 0 : 1;
    switch (G) {
    case 1: hipLaunchKernelGGL(k_fa_dec2<1>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, probe, kv_ld, kv_hs, (unsigned long long *)g_fa_stamps); break;
    case 2: hipLaunchKernelGGL(k_fa_dec2<2>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, probe, kv_ld, kv_hs, (unsigned long long *)g_fa_stamps); break;
    case 4: hipLaunchKernelGGL(k_fa_dec2<4>, grid, dim3(512), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, probe, kv_ld, kv_hs, (unsigned long long *)g_fa_stamps); break;
    default: hipLaunchKernelGGL(k_fa_dec2<8>, grid, dim3(256), 0, s, q16, kc, vc, po, pml, tickets, out, (uint8_t *)qout, H, HKV, n_past, n_past_dev, scale, probe, kv_ld, kv_hs, (unsigned long long *)g_fa_stamps); break;
    }
    KCPP_CHECK(hipGetLastError());
    if (variant == 2) {
#define KCPP_FA_C2(GG)                                                                                                     \
    case GG:                                                                                                               \
        if (qout) hipLaunchKernelGGL((k_fa_combine2<GG, true>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS); \
        else hipLaunchKernelGGL((k_fa_combine2<GG, false>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, NS);    \
        break;
        switch (G) { KCPP_FA_C2(1) KCPP_FA_C2(2) KCPP_FA_C2(4) KCPP_FA_C2(8) }
#undef KCPP_FA_C2
        KCPP_CHECK(hipGetLastError());
    }
    return 0;
}

// GGML_OP_FLASH_ATTN_EXT as the ggml graph states it (the b1 backend path): q f32 [D][T][H] with byte
// strides (q_nb1 between queries, q_nb2 between heads), K/V f16 cache views [n_kv][HKV][D] (row stride
// HKV*D), mask f16 [T_pad][n_kv] (row stride mask_ld elements, 0 / -inf, may be null = no mask), out f32
// [T][H][D].  Q is rounded to f16 first (q_to_vec_dot of ggml_compute_forward_flash_attn_ext_f16,
// ggml.c:15667); keys whose mask is -inf are skipped.  ws: kcpp_fa_workspace_bytes(T, H, n_kv) + T*H*D*2.
int64_t kcpp_fa_ext_workspace_bytes(int T, int H, int n_kv, int D) {
    return ((kcpp_fa_workspace_bytes(T, H, n_kv) + 255) & ~(int64_t)255) + (int64_t)T * H * D * 2 + 256;
}

__global__ void k_q_to_f16(const char *__restrict__ q, int64_t nb1, int64_t nb2, int T, int H, int D,
                           uint16_t *__restrict__ q16) {
    const int t = blockIdx.x, h = blockIdx.y;
    for (int d = threadIdx.x; d < D; d += blockDim.x)
        q16[((int64_t)t * H + h) * D + d] = f2h(((const float *)(q + t * nb1 + h * nb2))[d]);
}

int kcpp_flash_attn_ext(const float *q, int64_t q_nb1, int64_t q_nb2, const uint16_t *kc, const uint16_t *vc,
                        const uint16_t *mask, int64_t mask_ld, float *out, void *ws, int T, int H, int HKV, int D,
                        int n_kv, float scale, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (D != 128 || H % HKV || H / HKV > FA_MAXG || (H % 2) || n_kv < 1) return -1;
    uint16_t *q16 = (uint16_t *)((uint8_t *)ws + ((kcpp_fa_workspace_bytes(T, H, n_kv) + 255) & ~(int64_t)255));
    hipLaunchKernelGGL(k_q_to_f16, dim3(T, H), dim3(128), 0, s, (const char *)q, q_nb1, q_nb2, T, H, D, q16);
    KCPP_CHECK(hipGetLastError());
    if (mask_ld < 0) mask_ld = 0;
    if (T <= 16) {
        const int nch = (n_kv + FA_CHUNK - 1) / FA_CHUNK;
        if (nch > FA_MAX_CHUNKS) return -4;
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)T * H * nch * 128);
        int *tickets = (int *)(pml + (int64_t)T * H * nch);
        const dim3 grid(nch, HKV, T);
#define KCPP_FA_CASE(GG)                                                                                          \
    case GG:                                                                                                      \
        hipLaunchKernelGGL((k_fa_decode<128, GG, false>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, tickets, out, \
                           (uint8_t *)nullptr, T, H, HKV, n_kv, nullptr, nch, scale, mask, mask_ld,                \
                           (int64_t)HKV * 128, (int64_t)128);                                                     \
        break;
        switch (H / HKV) {
            KCPP_FA_CASE(1)
            KCPP_FA_CASE(2)
            KCPP_FA_CASE(4)
            KCPP_FA_CASE(8)
        default: return -3;
        }
#undef KCPP_FA_CASE
        KCPP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(k_fa_combine<false>, dim3(H / 2, T), dim3(1024), 0, s, po, pml, out, (uint8_t *)nullptr, T, H,
                           D, n_kv, nullptr, nch, 1);
    } else {
        hipLaunchKernelGGL(k_fa_prefill<128>, dim3((T + FP_BQ - 1) / FP_BQ, H), dim3(256), 0, s, q16, kc, vc, out, T, H,
                           HKV, 0, scale, mask, mask_ld, n_kv, (const int32_t *)nullptr);
    }
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
