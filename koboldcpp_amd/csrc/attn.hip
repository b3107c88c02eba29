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
#include "attn_dec.h"
#include "kcpp_common.h"
#include "kcpp_internal.h"
#include "gemv_units.h"

#include <algorithm>
#include <cstdlib>

#define FA_CHUNK 64
#define FA_MAXG 8
#define FA_WS_TICKETS KCPP_FA_WS_HEADER     // workspace header (kcpp_internal.h)
#define FA_MAX_CHUNKS 2048          // k_fa_combine's chunk-weight table: 2048 x 64 = 131072 keys
static void *g_fa_stamps = nullptr;       // diagnostic stamp buffer (tools only; kcpp_fa_set_stamps)

// K/V cache layout: [pos][HKV][D] f16, row stride EKV = HKV*D elements.
// Query layout: q16 [T][H][D] f16.  Query t sits at absolute position n_past + t.
// One workgroup = (64-key chunk, kv head, query); its G = H/HKV query heads share every K/V row
// (GQA).  Scores: 16 lanes x 16 B per K row; P.V: lane owns two dims and reads one dword of each V
// row (no cross-lane reduction).  Partials (O, m, l) per chunk, merged by k_fa_combine (the role of the
// reference's flash_attn_combine_results, ggml/src/ggml-cuda/fattn-common.cuh:523).  Used for 2..16
// queries (single-token decode runs k_fa_dec4) and by the ggml-op form.
template <int D, int G>
__global__ void __launch_bounds__(256) k_fa_decode(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                   const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                   float2 *__restrict__ part_ml, int T, int H,
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
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p0 = c * FA_CHUNK;
    const int p1 = min(p0 + FA_CHUNK, kend);              // exclusive
    const uint16_t *mrow = mask ? mask + (int64_t)t * mask_ld : nullptr;
    __shared__ float s_sc[G][FA_CHUNK];
    __shared__ float s_red[4][G][D];
    __shared__ float s_m[G], s_l[G];

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
template <int G, bool NT>
__global__ void __launch_bounds__(256) k_fa_dec4(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                 const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                 float2 *__restrict__ part_ml, int H, int n_past_arg,
                                                 const int32_t *__restrict__ n_past_dev, int NS, float scale,
                                                 int64_t kv_ld, int64_t kv_hs, unsigned long long *stamps) {
    constexpr int D = 128;
    const int sp = blockIdx.x, hk = blockIdx.y;
    const int wg_id = blockIdx.y * gridDim.x + blockIdx.x;
    FA_STAMP(0);
    const int nkv = (n_past_dev ? n_past_dev[0] : n_past_arg) + 1;
    const int per = (nkv + NS - 1) / NS;
    const int p0 = sp * per, p1 = min(p0 + per, nkv);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
    __shared__ fadec::Smem<G> sm;
    // scores in the exp2 domain: s2 = (q . k) * scale * log2(e); partial m in the same domain
    const float sc2 = scale * 1.4426950408889634f;
    fadec::State<G> st;
#pragma unroll
    for (int g = 0; g < G; ++g) fadec::set_q(st, g, *(const uint4 *)(q16 + (int64_t)(hk * G + g) * D + sub * 8));
    if (stamps) { if (st.qv[0][0] == 12345.0f) stamps[0] = 0; FA_STAMP(1); }
    const uint16_t *kb = kc + (int64_t)hk * kv_hs + sub * 8, *vb = vc + (int64_t)hk * kv_hs + sub * 8;
    fadec::init(st);
    uint4 ka[4], va[4], kn[4], vn[4];
    auto issue = [&](int base, uint4 *kk, uint4 *vv) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = base + 4 * i + kq;
            const bool ok = p < p1;
            if constexpr (NT) {      // K/V rows are read once per token: non-temporal (MI355X_MICROARCH.md nt-weights)
                kk[i] = ok ? ld_nt(kb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
                vv[i] = ok ? ld_nt(vb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
            } else {
                kk[i] = ok ? *(const uint4 *)(kb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
                vv[i] = ok ? *(const uint4 *)(vb + (int64_t)p * kv_ld) : make_uint4(0, 0, 0, 0);
            }
        }
    };
    int base = p0 + 16 * wave;
    if (base < p1) issue(base, ka, va);
    for (; base < p1; base += 128) {
        const int b1 = base + 64;
        if (b1 < p1) issue(b1, kn, vn);
        fadec::consume(st, base, p1, kq, sc2, ka, va);
        if (stamps && base == p0 + 16 * wave) { if (st.acc[0][0] == 12345.0f) stamps[0] = 0; FA_STAMP(2); }
        if (b1 >= p1) break;
        if (b1 + 64 < p1) issue(b1 + 64, ka, va);
        fadec::consume(st, b1, p1, kq, sc2, kn, vn);
    }
    FA_STAMP(3);
    fadec::finish(st, sm, hk, sp, NS, part_o, part_ml);
    FA_STAMP(4);
    if (stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); FA_STAMP(5); }
}

// ---------------------------------------------------------------- decode v5: every K/V load in flight from entry
// k_fa_dec4 issued its first 16-key group only after the n_past word arrived (the split range depends on it), and its
// loads sat in lane-conditional branches, so the compiler could not count them: the q conversion waited for nearly
// all of the first group and the second group went out only after the first had landed -- two dependent HBM round
// trips per wave plus the n_past one in front.  Here the key partition does not depend on n_past: 64-key chunks,
// chunk c on split c % NS (chunks sp, sp + NS, ...), wave w owning keys 64 c + 16 w .. + 15 of each, so split sp's
// first chunk is issued at entry beside q (rows clamped to the cache's n_rows), its second as soon as n_past is
// known (rows clamped to n_past), and every load is unconditional (rows past the keys clamp to a valid row and are
// masked by their score), which keeps the compiler's vmcnt accounting exact: two chunks per wave in flight, q waited
// for alone.  Partials as k_fa_dec4 (O [H][NS][128], (m, l) [H][NS], m = -inf for a split without keys); the merge
// is k_fa_comb4.
// GRAPH (the ggml plugin's FLASH_ATTN_EXT with one query, kcpp_flash_attn_ext_dec): q f32 at qf (head stride qf_hs
// floats), rounded to f16 in the kernel; the f16 mask row added to the scores, -inf keys skipped.
// FINAL (short contexts, NS = 1, kcpp_flash_attn force_path 7): one workgroup per kv head walks every key and writes
// the attention output itself (part_o = out [H][128]) -- no combine launch
template <int G, bool NT, int NW = 4, bool GRAPH = false, bool FINAL = false>
__global__ void __launch_bounds__(64 * NW) k_fa_dec5(const uint16_t *__restrict__ q16, const uint16_t *__restrict__ kc,
                                                     const uint16_t *__restrict__ vc, float *__restrict__ part_o,
                                                     float2 *__restrict__ part_ml, int H, int n_past_arg,
                                                     const int32_t *__restrict__ n_past_dev, int NS, float scale,
                                                     int64_t kv_ld, int64_t kv_hs, int n_rows,
                                                     const float *__restrict__ qf = nullptr, int64_t qf_hs = 0,
                                                     const uint16_t *__restrict__ mask = nullptr) {
    constexpr int D = 128, CK = 16 * NW;              // keys per chunk: 16 per wave
    const int sp = blockIdx.x, hk = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
    __shared__ fadec::Smem<G, NW> sm;
    const float sc2 = scale * 1.4426950408889634f;    // scores in the exp2 domain
    uint4 qraw[GRAPH ? 1 : G];
    float4 qfa[GRAPH ? G : 1], qfb[GRAPH ? G : 1];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if constexpr (GRAPH) {
            const float4 *qp = (const float4 *)(qf + (int64_t)(hk * G + g) * qf_hs + sub * 8);
            qfa[g] = qp[0];
            qfb[g] = qp[1];
        } else {
            qraw[g] = *(const uint4 *)(q16 + (int64_t)(hk * G + g) * D + sub * 8);
        }
    }
    const uint16_t *kb = kc + (int64_t)hk * kv_hs + sub * 8, *vb = vc + (int64_t)hk * kv_hs + sub * 8;
    uint4 ka[4], va[4], kn[4], vn[4];
    uint32_t ma[GRAPH ? 4 : 1], mb[GRAPH ? 4 : 1];      // mask words (f16) of the group's keys
    auto issue = [&](int base, int lim, uint4 *kk, uint4 *vv, uint32_t *mm) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t p = min(base + 4 * i + kq, lim);
            if constexpr (GRAPH) mm[i] = mask[p];
            if constexpr (NT) {
                kk[i] = ld_nt(kb + p * kv_ld);
                vv[i] = ld_nt(vb + p * kv_ld);
            } else {
                kk[i] = *(const uint4 *)(kb + p * kv_ld);
                vv[i] = *(const uint4 *)(vb + p * kv_ld);
            }
        }
    };
    issue(CK * sp + 16 * wave, n_rows - 1, ka, va, ma);
    const int nkv = (n_past_dev ? n_past_dev[0] : n_past_arg) + 1;
    const int lim = nkv - 1;
    issue(CK * (sp + NS) + 16 * wave, lim, kn, vn, mb);
    fadec::State<G> st;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if constexpr (GRAPH) fadec::set_q_f32(st, g, qfa[g], qfb[g]);
        else fadec::set_q(st, g, qraw[g]);
    }
    fadec::init(st);
    const float l2e = 1.4426950408889634f;
    auto madd = [&](const uint32_t *mm, float *out) {    // the mask times log2(e); -inf stays -inf
#pragma unroll
        for (int i = 0; i < 4; ++i) out[i] = h2f((uint16_t)mm[i]) * l2e;
    };
    const int nch = (nkv + CK - 1) / CK;
    for (int c = sp; c < nch; c += 2 * NS) {
        const int b0 = CK * c + 16 * wave;
        float md[4];
        if constexpr (GRAPH) madd(ma, md);
        if (b0 < nkv) fadec::consume(st, b0, nkv, kq, sc2, ka, va, GRAPH ? md : nullptr);
        issue(CK * (c + 2 * NS) + 16 * wave, lim, ka, va, ma);
        if (c + NS >= nch) break;
        const int b1 = CK * (c + NS) + 16 * wave;
        if constexpr (GRAPH) madd(mb, md);
        if (b1 < nkv) fadec::consume(st, b1, nkv, kq, sc2, kn, vn, GRAPH ? md : nullptr);
        issue(CK * (c + 3 * NS) + 16 * wave, lim, kn, vn, mb);
    }
    fadec::finish<G, NW, FINAL>(st, sm, hk, sp, NS, part_o, part_ml);
}

// combine of k_fa_dec4's partials (m in the exp2 domain): grid (H / 2), 256 threads = 2 heads x 128 dims
// (one Q8_K block of 256 when quantizing); thread (head, d) issues all NS partial loads of its dim (<= 64, in
// flight together); one wave per head forms the split weights exp2(m_s - M) in LDS.
// QUANT 1: qout = the Q8_K activation; 2: the KT_Q8_0_TA activation of one token (8 Q8_0 blocks per head pair)
template <int QUANT, int NS>
__global__ void __launch_bounds__(256) k_fa_comb4(const float *__restrict__ part_o, const float2 *__restrict__ part_ml,
                                                  float *__restrict__ out, uint8_t *__restrict__ qout, int H,
                                                  unsigned long long *stamps, unsigned *reset) {
    constexpr int D = 128, MAXS = 64;
    const int pair = blockIdx.x, tid = threadIdx.x;
    if (reset && pair == 0 && tid < 15) reset[32 * tid] = 0;   // (a caller's counters: reset once consumed)
    const int wg_id = 2048 + blockIdx.x;
    FA_STAMP(0);
    const int hl = tid >> 7, d = tid & 127, h = 2 * pair + hl;
    __shared__ float s_w[2][MAXS];
    __shared__ float s_l[2];
    __shared__ float s_res[2 * D];
    const float *po = part_o + (int64_t)h * NS * D + d;
    float ov[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ov[s] = po[(int64_t)s * D];
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
    for (int s = 0; s < NS; s += 4) {
        O0 = fmaf(s_w[hl][s], ov[s], O0);
        O1 = fmaf(s_w[hl][s + 1], ov[s + 1], O1);
        O2 = fmaf(s_w[hl][s + 2], ov[s + 2], O2);
        O3 = fmaf(s_w[hl][s + 3], ov[s + 3], O3);
    }
    const float res = ((O0 + O1) + (O2 + O3)) / s_l[hl];
    FA_STAMP(2);
    if (out) out[(int64_t)h * D + d] = res;
    if constexpr (QUANT == 2) {
        s_res[tid] = res;
        __syncthreads();
        if (tid < 16) {                                  // half (tid & 1) of block tid >> 1: k_quant_q80's rounding
            float v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = s_res[16 * tid + k];
            float am = 0.0f;
#pragma unroll
            for (int k = 0; k < 16; ++k) am = fmaxf(am, fabsf(v[k]));
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            const float id = (am != 0.0f) ? 127.f / am : 0.0f;
            uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                int iv = (int)rintf(__fmul_rn(v[k], id));
                iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
                pk[k >> 2] |= (uint32_t)(iv & 0xFF) << (8 * (k & 3));
            }
            const int64_t E = (int64_t)H * D, ib = (int64_t)pair * 8 + (tid >> 1);
            *(uint4 *)(qout + ib * 1024 + (tid & 1) * 512) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            if ((tid & 1) == 0) ((float *)(qout + 32 * E))[ib * 32] = h2f(f2h(am / 127.f));
        }
    } else if constexpr (QUANT == 1) {
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

// split count of k_fa_dec4: one workgroup per CU (256 / HKV splits, rounded down to a power of two in [4, 64];
// measured at 3850 cached keys, tools/fa_dec_bench.py: 7.8 us vs 8.7 at 512 workgroups).  Independent of the
// context size, so the key partition -- and the result, bit for bit -- depends on the cached keys only.
static int fa4_splits(int HKV) {
    int ns = 4;
    while (ns < 64 && 2 * ns * HKV <= 256) ns *= 2;
    return ns;
}

template <int G, int NS>
static void fa4_dispatch(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                         float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                         float scale, hipStream_t s, int qkind, int n_rows, bool v5) {
    float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
    float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
    unsigned long long *st = (unsigned long long *)g_fa_stamps;
    static const bool nt = [] { const char *e = getenv("KCPP_FA_NT"); return !e || atoi(e) != 0; }();
    if (v5 && n_rows > 0) {
        if (nt)
            hipLaunchKernelGGL((k_fa_dec5<G, true>), dim3(NS, HKV), dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past,
                               n_past_dev, NS, scale, kv_ld, kv_hs, n_rows);
        else
            hipLaunchKernelGGL((k_fa_dec5<G, false>), dim3(NS, HKV), dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past,
                               n_past_dev, NS, scale, kv_ld, kv_hs, n_rows);
    } else if (nt) {
        hipLaunchKernelGGL((k_fa_dec4<G, true>), dim3(NS, HKV), dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past,
                           n_past_dev, NS, scale, kv_ld, kv_hs, st);
    } else {
        hipLaunchKernelGGL((k_fa_dec4<G, false>), dim3(NS, HKV), dim3(256), 0, s, q16, kc, vc, po, pml, H, n_past,
                           n_past_dev, NS, scale, kv_ld, kv_hs, st);
    }
    if (qout && qkind == 2)
        hipLaunchKernelGGL((k_fa_comb4<2, NS>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, st,
                           (unsigned *)nullptr);
    else if (qout) hipLaunchKernelGGL((k_fa_comb4<1, NS>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)qout, H, st,
                                      (unsigned *)nullptr);
    else hipLaunchKernelGGL((k_fa_comb4<0, NS>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, H, st,
                            (unsigned *)nullptr);
}

template <int G>
static int fa4_dispatch_ns(int NS, const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld,
                           int64_t kv_hs, float *out, void *qout, void *ws, int H, int HKV, int n_past,
                           const int32_t *n_past_dev, float scale, hipStream_t s, int qkind, int n_rows, bool v5) {
    switch (NS) {
    case 4: fa4_dispatch<G, 4>(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 8: fa4_dispatch<G, 8>(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 16: fa4_dispatch<G, 16>(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 32: fa4_dispatch<G, 32>(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 64: fa4_dispatch<G, 64>(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    default: return -1;
    }
    return 0;
}

// single-token decode: k_fa_dec5 (k_fa_dec4 when the cache's row count n_rows is not known, or for A/B with v5 off) +
// k_fa_comb4; partials behind FA_WS_TICKETS in ws.  n_rows: rows the K/V views hold (n_ctx), >= n_past + 1.
static bool fa_dec5_default() {
    static const bool on = [] { const char *e = getenv("KCPP_FA_DEC"); return !e || atoi(e) != 4; }();
    return on;
}
// short contexts (n_kv <= KCPP_FA_SHORT_MAX): k_fa_dec5<FINAL> on one 8-wave workgroup per kv head, the output written
// directly (one launch instead of split + combine; at a few hundred keys the split grid mostly holds empty splits and
// the combine is a whole dependent launch).  The caller decides by the host-known position (graphs per regime).
static int fa_short_launch(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                           float *out, int H, int HKV, int n_past, const int32_t *n_past_dev, float scale, hipStream_t s,
                           int n_rows) {
    const int G = H / HKV;
#define KCPP_FS(G_)                                                                                                   \
    hipLaunchKernelGGL((k_fa_dec5<G_, true, 8, false, true>), dim3(1, HKV), dim3(512), 0, s, q16, kc, vc, out,         \
                       (float2 *)nullptr, H, n_past, n_past_dev, 1, scale, kv_ld, kv_hs, n_rows, (const float *)nullptr, \
                       (int64_t)0, (const uint16_t *)nullptr)
    switch (G) {
    case 1: KCPP_FS(1); break;
    case 2: KCPP_FS(2); break;
    case 4: KCPP_FS(4); break;
    case 8: KCPP_FS(8); break;
    default: return -3;
    }
#undef KCPP_FS
    KCPP_CHECK(hipGetLastError());
    return 0;
}

static int fa4_launch(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                      float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                      float scale, hipStream_t s, int qkind, int n_rows, bool v5) {
    const int G = H / HKV;
    const int NS = fa4_splits(HKV);
    if (!qout && !out) return -1;
    int rc = -1;
    switch (G) {
    case 1: rc = fa4_dispatch_ns<1>(NS, q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 2: rc = fa4_dispatch_ns<2>(NS, q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 4: rc = fa4_dispatch_ns<4>(NS, q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    case 8: rc = fa4_dispatch_ns<8>(NS, q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, qkind, n_rows, v5); break;
    default: return -1;
    }
    if (rc) return rc;
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

// partial O + (m, l) per (query, head, chunk / split) behind a 256-B header
int64_t kcpp_fa_workspace_bytes(int T, int H, int n_kv_max) {
    const int64_t nch = (n_kv_max + FA_CHUNK - 1) / FA_CHUNK;
    // partial slots: T x nch chunks (k_fa_decode), at least the 64 splits k_fa_dec4 may use
    const int64_t slots = std::max<int64_t>((int64_t)T * nch, 64);
    return std::max<int64_t>(FA_WS_TICKETS + (int64_t)H * slots * (128 * 4 + 8) + (int64_t)T * H * 4 + 256,
                             kcpp_fa_split_ws_bytes(H));      // the key-split prefill (attn_mfma.hip)
}

// single-token decode attention (k_fa_dec4 + k_fa_comb4) whose combine writes the KT_Q8_0_TA activation of one token
// (attn_output in the KT_Q8_0_T layout) instead of a separate kcpp_quantize_act; out f32 may be null.  -3: not covered
int kcpp_flash_attn_dec_ta(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qta, void *ws,
                           int H, int HKV, int D, int n_past, const int32_t *n_past_dev, int n_kv_max, float scale,
                           void *stream) {
    if (D != 128 || H % HKV || H % 2 || !qta) return -3;
    const int G = H / HKV;
    if (!(G == 2 || G == 4 || G == 8)) return -3;
    return fa4_launch(q16, kc, vc, (int64_t)HKV * 128, 128, out, qta, ws, H, HKV, n_past, n_past_dev, scale,
                      (hipStream_t)stream, 2, n_past_dev ? n_kv_max : n_past + 1, fa_dec5_default());
}

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
    // force_path 0: auto (T <= 16 decode kernels, else prefill), 1: decode kernels, 2: tiled prefill, 3: MFMA
    // prefill, 6: the 64-key-chunk decode kernel even for T = 1 (tests)
    const bool use_decode = force_path == 1 || force_path == 6 || (force_path == 0 && T <= 16);
    const int G0 = H / HKV;
    if (force_path == 7) {       // single-pass decode (short contexts: the caller keeps n_kv <= KCPP_FA_SHORT_MAX)
        if (T != 1 || !out || qout) return -1;
        return fa_short_launch(q16, kc, vc, (int64_t)HKV * 128, 128, out, H, HKV, n_past, n_past_dev, scale, s,
                               n_past_dev ? n_kv_max : n_past + 1);
    }
    if (use_decode && T == 1 && force_path != 6 && (G0 == 1 || G0 == 2 || G0 == 4 || G0 == 8) && (qout == nullptr || G0 >= 2))
        return fa4_launch(q16, kc, vc, (int64_t)HKV * 128, 128, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, 1,
                          n_past_dev ? n_kv_max : n_past + 1, fa_dec5_default());
    if (use_decode) {
        ws = (uint8_t *)ws + FA_WS_TICKETS;
        const int nkv = n_past_dev ? n_kv_max : n_past + T;
        const int nch = (nkv + FA_CHUNK - 1) / FA_CHUNK;
        if (nch > FA_MAX_CHUNKS) return -4;              // combine's chunk-weight table (128k context)
        float *po = (float *)ws;
        float2 *pml = (float2 *)(po + (int64_t)T * H * nch * 128);
        const dim3 grid(nch, HKV, T);
#define KCPP_FA_CASE(GG)                                                                                       \
    case GG:                                                                                                   \
        hipLaunchKernelGGL((k_fa_decode<128, GG>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, T, H, HKV,     \
                           n_past, n_past_dev, nch, scale, nullptr, -1, (int64_t)HKV * 128, (int64_t)128);     \
        break;
        switch (G0) {
            KCPP_FA_CASE(1)
            KCPP_FA_CASE(2)
            KCPP_FA_CASE(4)
            KCPP_FA_CASE(8)
        default: return -3;
        }
#undef KCPP_FA_CASE
        KCPP_CHECK(hipGetLastError());
        if (qout)
            hipLaunchKernelGGL(k_fa_combine<true>, dim3(H / 2, T), dim3(1024), 0, s, po, pml, out, (uint8_t *)qout, T,
                               H, D, n_past, n_past_dev, nch, 0);
        else
            hipLaunchKernelGGL(k_fa_combine<false>, dim3(H / 2, T), dim3(1024), 0, s, po, pml, out, (uint8_t *)nullptr,
                               T, H, D, n_past, n_past_dev, nch, 0);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (!out) return -2;
    // prefill: MFMA kernel (attn_mfma.hip) for GQA groups of 4 (force_path 3, or auto), else FMA tiles (2)
    int rc = -3;
    if (force_path == 3 || force_path == 0)
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
// kv_hs = n_ctx*D.  variant 0: 64-key chunks + k_fa_combine; 3: k_fa_dec4 + k_fa_comb4 (round 5's production pair);
// 5: k_fa_dec5 + k_fa_comb4 (the production pair; n_kv_max = the views' row count); 8: the short-context single launch
// (one workgroup per kv head, no combine).  A/B entry for tools/fa_dec_bench.py.
void kcpp_fa_set_stamps(void *p) { g_fa_stamps = p; }     // diagnostic stamp buffer of k_fa_dec4 / k_fa_comb4 (tools only)
int kcpp_fa_decode_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                      float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                      int n_kv_max, float scale, int variant, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int G = H / HKV;
    if (H % HKV || !(G == 1 || G == 2 || G == 4 || G == 8) || (H % 2) || HKV > 64) return -1;
    if (qout && G < 2) return -1;
    const int nkv = n_past_dev ? n_kv_max : n_past + 1;
    if (variant == 3 || variant == 5)
        return fa4_launch(q16, kc, vc, kv_ld, kv_hs, out, qout, ws, H, HKV, n_past, n_past_dev, scale, s, 1, nkv,
                          variant == 5);
    if (variant == 8) {                     // the short-context single launch (kcpp_flash_attn force_path 7)
        if (qout || !out) return -1;
        return fa_short_launch(q16, kc, vc, kv_ld, kv_hs, out, H, HKV, n_past, n_past_dev, scale, s, nkv);
    }
    if (variant == 6 || variant == 7) {     // A/B (tools/fa_dec_bench.py): k_fa_dec5 at NS splits (KCPP_FA_NS) x NW waves
        // (KCPP_FA_NW), G = 4; 7: without the combine (the split kernel alone)
        const int NS = getenv("KCPP_FA_NS") ? atoi(getenv("KCPP_FA_NS")) : 32;
        const int NW = getenv("KCPP_FA_NW") ? atoi(getenv("KCPP_FA_NW")) : 4;
        if (G != 4 || !out) return -1;
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
#define KCPP_D6(NW_) hipLaunchKernelGGL((k_fa_dec5<4, true, NW_>), dim3(NS, HKV), dim3(64 * NW_), 0, s, q16, kc, vc, po, pml, \
                                        H, n_past, n_past_dev, NS, scale, kv_ld, kv_hs, nkv)
        if (NW == 4) KCPP_D6(4);
        else if (NW == 8) KCPP_D6(8);
        else if (NW == 16) KCPP_D6(16);
        else return -1;
#undef KCPP_D6
        if (variant == 6) {
            switch (NS) {
            case 8: hipLaunchKernelGGL((k_fa_comb4<0, 8>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, H, (unsigned long long *)nullptr, (unsigned *)nullptr); break;
            case 16: hipLaunchKernelGGL((k_fa_comb4<0, 16>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, H, (unsigned long long *)nullptr, (unsigned *)nullptr); break;
            case 32: hipLaunchKernelGGL((k_fa_comb4<0, 32>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, H, (unsigned long long *)nullptr, (unsigned *)nullptr); break;
            default: return -1;
            }
        }
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (variant != 0) return -1;
    const int nch = (nkv + FA_CHUNK - 1) / FA_CHUNK;
    if (nch > FA_MAX_CHUNKS) return -4;
    float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
    float2 *pml = (float2 *)(po + (int64_t)H * nch * 128);
    const dim3 grid(nch, HKV, 1);
#define KCPP_FA_CASE(GG)                                                                                         \
    case GG:                                                                                                     \
        hipLaunchKernelGGL((k_fa_decode<128, GG>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, 1, H, HKV, n_past, \
                           n_past_dev, nch, scale, nullptr, -1, kv_ld, kv_hs);                                   \
        break;
    switch (G) { KCPP_FA_CASE(1) KCPP_FA_CASE(2) KCPP_FA_CASE(4) KCPP_FA_CASE(8) }
#undef KCPP_FA_CASE
    KCPP_CHECK(hipGetLastError());
    if (qout) hipLaunchKernelGGL(k_fa_combine<true>, dim3(H / 2, 1), dim3(1024), 0, s, po, pml, out, (uint8_t *)qout, 1, H, 128, n_past, n_past_dev, nch, 0);
    else hipLaunchKernelGGL(k_fa_combine<false>, dim3(H / 2, 1), dim3(1024), 0, s, po, pml, out, (uint8_t *)nullptr, 1, H, 128, n_past, n_past_dev, nch, 0);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// one query of GGML_OP_FLASH_ATTN_EXT in the graph form (the b1 backend's decode): k_fa_dec5<GRAPH> over the views
// (key j of kv head h at kc + j k_ld + h k_hs elements), the f16 mask row (may be null), q f32 [H][D] with head
// stride q_nb2 bytes rounded to f16 in the kernel, then k_fa_comb4 into out [H][D].  -3: shape not covered.
int kcpp_flash_attn_ext_dec(const float *q, int64_t q_nb2, const uint16_t *kc, const uint16_t *vc, int64_t k_ld,
                            int64_t k_hs, const uint16_t *mask, float *out, void *ws, int H, int HKV, int D, int n_kv,
                            float scale, void *stream) {
    if (D != 128 || H % HKV || H % 2 || n_kv < 1 || q_nb2 % 16 || ((uintptr_t)q & 15)) return -3;
    const int G = H / HKV, NS = fa4_splits(HKV);
    if (!(G == 1 || G == 2 || G == 4 || G == 8)) return -3;
    hipStream_t s = (hipStream_t)stream;
    float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
    float2 *pml = (float2 *)(po + (int64_t)H * NS * 128);
    if (!mask) return -3;                         // (llama.cpp always passes the KQ mask)
#define KCPP_FAD(GG)                                                                                                \
    hipLaunchKernelGGL((k_fa_dec5<GG, true, 4, true>), dim3(NS, HKV), dim3(256), 0, s, (const uint16_t *)nullptr, kc, vc, \
                       po, pml, H, n_kv - 1, (const int32_t *)nullptr, NS, scale, k_ld, k_hs, n_kv, q, q_nb2 / 4, mask)
    switch (G) {
    case 1: KCPP_FAD(1); break;
    case 2: KCPP_FAD(2); break;
    case 4: KCPP_FAD(4); break;
    default: KCPP_FAD(8); break;
    }
#undef KCPP_FAD
    KCPP_CHECK(hipGetLastError());
    switch (NS) {
#define KCPP_FAC(N_) case N_: hipLaunchKernelGGL((k_fa_comb4<0, N_>), dim3(H / 2), dim3(256), 0, s, po, pml, out, (uint8_t *)nullptr, \
                                                 H, (unsigned long long *)nullptr, (unsigned *)nullptr); break;
    KCPP_FAC(4) KCPP_FAC(8) KCPP_FAC(16) KCPP_FAC(32) KCPP_FAC(64)
#undef KCPP_FAC
    default: return -3;
    }
    KCPP_CHECK(hipGetLastError());
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
    if ((D != 128 && D != 64) || H % HKV || H / HKV > FA_MAXG || (H % 2) || n_kv < 1) return -1;
    uint16_t *q16 = (uint16_t *)((uint8_t *)ws + ((kcpp_fa_workspace_bytes(T, H, n_kv) + 255) & ~(int64_t)255));
    hipLaunchKernelGGL(k_q_to_f16, dim3(T, H), dim3(128), 0, s, (const char *)q, q_nb1, q_nb2, T, H, D, q16);
    KCPP_CHECK(hipGetLastError());
    if (mask_ld < 0) mask_ld = 0;
    if (D == 64) {      // 64-dim heads (TinyLlama class): the tiled kernel for every T, under the explicit mask
        hipLaunchKernelGGL(k_fa_prefill<64>, dim3((T + FP_BQ - 1) / FP_BQ, H), dim3(256), 0, s, q16, kc, vc, out, T, H, HKV,
                           0, scale, mask, mask_ld, n_kv, (const int32_t *)nullptr);
        KCPP_CHECK(hipGetLastError());
        return 0;
    }
    if (T <= 16) {
        const int nch = (n_kv + FA_CHUNK - 1) / FA_CHUNK;
        if (nch > FA_MAX_CHUNKS) return -4;
        float *po = (float *)((uint8_t *)ws + FA_WS_TICKETS);
        float2 *pml = (float2 *)(po + (int64_t)T * H * nch * 128);
        const dim3 grid(nch, HKV, T);
#define KCPP_FA_CASE(GG)                                                                                          \
    case GG:                                                                                                      \
        hipLaunchKernelGGL((k_fa_decode<128, GG>), grid, dim3(256), 0, s, q16, kc, vc, po, pml, T, H, HKV, n_kv,   \
                           nullptr, nch, scale, mask, mask_ld, (int64_t)HKV * 128, (int64_t)128);                 \
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
