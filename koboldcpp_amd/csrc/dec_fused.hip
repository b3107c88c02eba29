// dec_fused.hip -- single-token decode: attn_norm -> q|k|v (+RoPE, K/V cache store) and the split-KV attention in
// ONE launch (the graph's ggml_rms_norm / mul_mat x3 / rope x2 / cpy x2 / flash_attn_ext nodes of build_llama,
// src/llama.cpp:10479-10529, up to the attention partials; the combine stays a launch of its own).
//
// Why: the stand-alone attention kernel (k_fa_dec4) spends most of its time waiting for its first K/V bytes
// (3.5 us at 4k context) after a launch boundary, and the q|k|v mat-vec before it moves only 14 MB.  Here the
// attention workgroups start with the q|k|v workgroups and stream the cached keys [0, n_past) into registers at
// once -- they do not depend on this token -- then wait for the q|k|v workgroups and only read q and the new key
// (position n_past) after them.
//
// Roles by block index: [0, nq) run the q|k|v mat-vec (k_gemv_rs_qkv's body: Q4_K_RS rows, optional Q6_K_RS v
// rows, rms_norm -> Q8_K prologue, RoPE + f16 stores), [nq, nq + NS * HKV) the attention split (sp, hk) of
// k_fa_dec4 (attn_dec.h).  Every result is computed exactly as the two stand-alone kernels compute it.
//
// Hand-off (MI355X_MICROARCH.md, handoff-1to1: data-tagged granules): every q|k|v result pair the attention needs --
// the RoPE'd q pairs, and the new key's K and V pairs -- is also stored as one 8-byte granule {two f16, tag} by a
// single write-through (sc1) store, tag = the launch's epoch (a per-token counter the decode step advances on the
// device, x 128 + the layer).  An attention workgroup's wave 0 polls its head group's q granules (wave 1 the new
// key's, in the split that holds it) with 8-byte sc1 loads until every tag matches, parks the data in LDS, and a
// barrier releases the other waves: one memory round trip after the data lands, no counters, no fences.  No deadlock by
// construction: the host launches only when the occupancy query admits every workgroup at once, and every poll is
// bounded (a timeout sets the error word of the granule buffer).
#include "attn_dec.h"
#include "gemv_rs.h"

#include <algorithm>

using namespace rs;

namespace {

#ifndef KCPP_FUSED_PROBE
#define KCPP_FUSED_PROBE 0
#endif
constexpr unsigned kSpinMax = 1u << 22;
#if KCPP_FUSED_PROBE == 5           // timing probe: s_memrealtime stamps of layer 5 (tools/dec_stamps.py, never the product)
__device__ unsigned long long *g_dec_stamps;
#define DEC_STAMP(il, idx)                                                                                        \
    if (threadIdx.x == 0 && (il) == 5 && g_dec_stamps)                                                            \
        __hip_atomic_store(g_dec_stamps + (idx), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,             \
                           __HIP_MEMORY_SCOPE_AGENT);
#else
#define DEC_STAMP(il, idx)
#endif        // x ~0.1 us per poll: a dead producer ends the wait after ~0.4 s

// granule buffer (kcpp_dec_gran_bytes): q pairs [H * 64], then k pairs [HKV * 64], v pairs [HKV * 64] ({f16 pair,
// tag} each), then the timeout word
struct AttArgs {
    const uint16_t *kc, *vc;
    float *part_o;
    float2 *part_ml;
    uint64_t *gran;
    unsigned *err;
    int nq, NS, wph;        // q|k|v workgroups, attention splits, q|k|v workgroups per kv head
    int H, HKV, il;         // heads, kv heads, layer (tag = epoch * 128 + il)
    float scale;
    int64_t kv_ld, kv_hs;
};
__device__ __forceinline__ void st_gran(uint64_t *p, uint32_t data, uint32_t tag) {
    __hip_atomic_store(p, (uint64_t)data | ((uint64_t)tag << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the q|k|v role's epilogue: lean::store_group<2, 2> (RoPE pairs; v rows in pairs too) plus the granules.
// (The DecArgs fields are read into scalars first: a select between fields of the by-value kernel argument would be
// folded into a dynamically indexed load, which places the whole argument in scratch memory.)
__device__ __forceinline__ void store_qkv_wt(const DecArgs &a, const AttArgs &t, uint32_t tag, int role, int row0,
                                             const float (&slot)[2]) {
    const int p = a.pos[0];
    const int H = t.H, HKV = t.HKV;
    if (role == 2) {
        const uint32_t pk = (uint32_t)f2h(slot[0]) | ((uint32_t)f2h(slot[1]) << 16);
        *(uint32_t *)(a.vc + (int64_t)p * a.ekv + row0) = pk;
        st_gran(t.gran + (int64_t)(H + HKV) * 64 + row0 / 2, pk, tag);
    } else {
        const int hd = a.D / 2;
        const float2 cs = a.rope_tab[(int64_t)p * hd + (row0 % a.D) / 2];
        const float x0 = slot[0], x1 = slot[1];
        const float o0 = __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
        const float o1 = __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x));
        const uint32_t pk = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
        if (role == 0) {
            st_gran(t.gran + row0 / 2, pk, tag);
        } else {
            *(uint32_t *)(a.kc + (int64_t)p * a.ekv + row0) = pk;
            st_gran(t.gran + (int64_t)H * 64 + row0 / 2, pk, tag);
        }
    }
}

// rows g * 2, g * 2 + 1 of the concatenated q|k|v rows: segment and first row in it
struct GRows { int seg, row0; };
__device__ __forceinline__ GRows group_rows3(int g, int N0, int N1) {
    const int r = g * 2;
    GRows o;
    o.seg = r < N0 ? 0 : (r < N0 + N1 ? 1 : 2);
    o.row0 = o.seg == 0 ? r : (o.seg == 1 ? r - N0 : r - N0 - N1);
    return o;
}
template <typename T, int NI>
__device__ __forceinline__ void issue_rows(const uint8_t *W, int row0, int RB, int nsb, int np, int lane,
                                           typename T::W (&w)[NI][2]) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < NI; ++i) T::load(W + (int64_t)(row0 + r) * RB, nsb, min(lane + 64 * i, np - 1), w[i][r]);
}

// segments 0, 1 (q, k) in Q4_K_RS; segment 2 (v) in Q6_K_RS when MIX, else Q4_K_RS.  R = 2 rows per group.
// Head-major work split: the wph workgroups [wph hk, wph (hk + 1)) produce exactly the rows kv head hk's attention
// needs -- the G q heads 128 (G hk .. G hk + G), k rows and v rows 128 hk .. -- and arrive on that head's counter,
// so that the head's granules are complete once these wph workgroups are done.
template <int NIA, int NIB, int MIX>
__device__ __forceinline__ void qkv_role(const DecArgs &a, const AttArgs &t, uint32_t tag, int blk, uint8_t *lds) {
    const int wph = t.wph;
    using TA = RS<KT_Q4_K_RS>;
    using TB = RS<KT_Q6_K_RS>;
    constexpr int R = 2;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = (int)a.K, nsb = K / 256;
    const int RBA = nsb * TA::BYTES, RBB = nsb * TB::BYTES;
    const int npA = nsb * TA::PIECES_PER_SB, npB = nsb * TB::PIECES_PER_SB;
    const int G = (int)(a.N[0] / a.N[1]);
    const int hk = blk / wph;
    const int gq = G * 64, ng = gq + 128;          // groups of this head: q, then 64 of k, then 64 of v
    const int nw = wph * 4;
    const int wid = (blk % wph) * 4 + wave;
    const typename TA::Lane lca = TA::lane_consts(lane);
    const typename TB::Lane lcb = TB::lane_consts(lane);
    const uint8_t *const W0 = a.W[0], *const W1 = a.W[1], *const W2 = a.W[2];
    const int role0 = a.role[0], role1 = a.role[1], role2 = a.role[2];
    auto rows_of = [=](int lg) {
        GRows o;
        o.seg = lg < gq ? 0 : (lg < gq + 64 ? 1 : 2);
        o.row0 = o.seg == 0 ? hk * G * 128 + 2 * lg : hk * 128 + 2 * (o.seg == 1 ? lg - gq : lg - gq - 64);
        return o;
    };
    DEC_STAMP(t.il, blk * 4 + 0)
    typename TA::W ba[NIA][R];
    typename TB::W bb[NIB][R];
    const int g0 = min(wid, ng - 1);
    lean::ActPro<1, (NIA + 1) / 2> pro;
    pro.load(a);
    {
        const GRows gr = rows_of(g0);
        if (!MIX || gr.seg < 2) issue_rows<TA, NIA>(gr.seg == 0 ? W0 : (gr.seg == 1 ? W1 : W2), gr.row0, RBA, nsb, npA, lane, ba);
        else issue_rows<TB, NIB>(W2, gr.row0, RBB, nsb, npB, lane, bb);
    }
    pro.compute(a, lds);
    DEC_STAMP(t.il, blk * 4 + 1)
    typename TA::Act xa[NIA];
    typename TB::Act xb[MIX ? NIB : 1];
#pragma unroll
    for (int i = 0; i < NIA; ++i) TA::act(lds, K, min(TA::sb_of(lane, i), nsb - 1), lca, xa[i]);
    if constexpr (MIX) {
#pragma unroll
        for (int i = 0; i < NIB; ++i) TB::act(lds, K, min(TB::sb_of(lane, i), nsb - 1), lcb, xb[i]);
    }
    float slot0 = 0.0f, slot1 = 0.0f;
    int slot_g = -1;
    int k = 0;
    for (int g = wid; g < ng; g += nw, ++k) {
        float acc[R] = {0.0f, 0.0f};
        const GRows gr = rows_of(g);
        if (!MIX || gr.seg < 2) {
            if (k) issue_rows<TA, NIA>(gr.seg == 0 ? W0 : (gr.seg == 1 ? W1 : W2), gr.row0, RBA, nsb, npA, lane, ba);
#pragma unroll
            for (int i = 0; i < NIA; ++i) {
                const bool ok = (NIA * 64 == npA) || lane + 64 * i < npA;
#pragma unroll
                for (int r = 0; r < R; ++r) { const float p = TA::dot(ba[i][r], xa[i], lca); acc[r] += ok ? p : 0.0f; }
            }
        } else if constexpr (MIX) {
            if (k) issue_rows<TB, NIB>(W2, gr.row0, RBB, nsb, npB, lane, bb);
#pragma unroll
            for (int i = 0; i < NIB; ++i) {
                const bool ok = (NIB * 64 == npB) || lane + 64 * i < npB;
#pragma unroll
                for (int r = 0; r < R; ++r) { const float p = TB::dot(bb[i][r], xb[i], lcb); acc[r] += ok ? p : 0.0f; }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_f(acc[r]))));
        const bool mine = lane == k;
        slot0 = mine ? acc[0] : slot0;
        slot1 = mine ? acc[1] : slot1;
        slot_g = mine ? g : slot_g;
    }
    DEC_STAMP(t.il, blk * 4 + 2)
    if (slot_g >= 0) {
        const GRows gr = rows_of(slot_g);
        const float slot[2] = {slot0, slot1};
        store_qkv_wt(a, t, tag, gr.seg == 0 ? role0 : (gr.seg == 1 ? role1 : role2), gr.row0, slot);
    }
#if KCPP_FUSED_PROBE == 5
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    DEC_STAMP(t.il, blk * 4 + 3)
#endif
}

// the attention role: split sp of kv head hk (k_fa_dec4 with the cached keys loaded before the wait)
template <int G>
__device__ __forceinline__ void att_role(const AttArgs &t, const int32_t *pos, uint32_t tag, int blk2) {
    constexpr int D = fadec::D;
    const int NS = t.NS;
    const int sp = blk2 % NS, hk = blk2 / NS;
    const int np = pos[0];                         // the new token's key: written by this launch's q|k|v role
    const int nkv = np + 1;
    const int per = (nkv + NS - 1) / NS;
    const int p0 = sp * per, p1 = min(p0 + per, nkv);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane & 15, kq = lane >> 4;
    __shared__ fadec::Smem<G> sm;
    const float sc2 = t.scale * 1.4426950408889634f;
    const uint16_t *kb = t.kc + (int64_t)hk * t.kv_hs + sub * 8, *vb = t.vc + (int64_t)hk * t.kv_hs + sub * 8;
    uint4 ka[4], va[4], kn[4], vn[4];
    // cached keys by plain loads (the new key np is left zero: it is not written yet when the first groups are issued)
    auto issue = [&](int base, uint4 *kk, uint4 *vv) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = base + 4 * i + kq;
            const bool ok = p < p1 && p != np;
            kk[i] = ok ? *(const uint4 *)(kb + (int64_t)p * t.kv_ld) : make_uint4(0, 0, 0, 0);
            vv[i] = ok ? *(const uint4 *)(vb + (int64_t)p * t.kv_ld) : make_uint4(0, 0, 0, 0);
        }
    };
    DEC_STAMP(t.il, 4096 + blk2 * 4 + 0)
    const int base0 = p0 + 16 * wave;
#if KCPP_FUSED_PROBE == 4           // timing probe (tools/dec_ab.py, never the product): no attention work at all
    return;
#endif
    if (base0 < p1) issue(base0, ka, va);
    if (base0 + 64 < p1) issue(base0 + 64, kn, vn);
#if KCPP_FUSED_PROBE == 1           // probe: the cached-key loads only
    if (ka[0].x == 0x12345 && kn[0].y == 0x777) t.err[1] = 1;
    return;
#endif
    // wave 0: this head group's q granules (G * 64 pairs, G per lane); wave 1 of the split holding the new key: its K
    // and V granules; polled until every tag is this launch's, parked in LDS
    __shared__ uint32_t s_q[G * 64], s_k[64], s_v[64];
    const bool has_new = np >= p0 && np < p1;
    if (wave == 0 || (wave == 1 && has_new)) {
        constexpr int NQ = G;                        // granules per lane
        uint64_t v[NQ];
        const uint64_t *src = t.gran + (wave == 0 ? (int64_t)hk * G * 64 : (int64_t)t.H * 64 + (int64_t)hk * 64);
        const int64_t vof = (int64_t)t.HKV * 64;      // v granules after k
        for (unsigned it = 0;; ++it) {
            bool ok = true;
            if (wave == 0) {
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    v[j] = __hip_atomic_load(src + lane + 64 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok &= (uint32_t)(v[j] >> 32) == tag;
                }
            } else {
                v[0] = __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[1] = __hip_atomic_load(src + vof + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = (uint32_t)(v[0] >> 32) == tag && (uint32_t)(v[1] >> 32) == tag;
            }
            if (__all(ok) || KCPP_FUSED_PROBE == 2) break;       // (probe 2: no wait)
            if (it > kSpinMax) {
                if (lane == 0) __hip_atomic_fetch_or(t.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (wave == 0) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) s_q[lane + 64 * j] = (uint32_t)v[j];
        } else {
            s_k[lane] = (uint32_t)v[0];
            s_v[lane] = (uint32_t)v[1];
        }
    }
    __syncthreads();
    DEC_STAMP(t.il, 4096 + blk2 * 4 + 2)
    fadec::State<G> st;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint32_t *qq = s_q + g * 64 + sub * 4;
        fadec::set_q(st, g, make_uint4(qq[0], qq[1], qq[2], qq[3]));
    }
    fadec::init(st);
    // the new key into the group that holds it (prefetched groups now; streamed groups as they are issued)
    auto patch = [&](int base, uint4 *kk, uint4 *vv) __attribute__((always_inline)) {
        if (has_new && np >= base && np < base + 16) {           // wave-uniform, rare
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (base + 4 * i + kq == np) {
                    kk[i] = make_uint4(s_k[sub * 4], s_k[sub * 4 + 1], s_k[sub * 4 + 2], s_k[sub * 4 + 3]);
                    vv[i] = make_uint4(s_v[sub * 4], s_v[sub * 4 + 1], s_v[sub * 4 + 2], s_v[sub * 4 + 3]);
                }
        }
    };
    patch(base0, ka, va);
    patch(base0 + 64, kn, vn);
    for (int base = base0; base < p1; base += 128) {
        fadec::consume(st, base, p1, kq, sc2, ka, va);
        const int b1 = base + 64;
        if (b1 >= p1) break;
        if (base + 128 < p1) { issue(base + 128, ka, va); patch(base + 128, ka, va); }
        fadec::consume(st, b1, p1, kq, sc2, kn, vn);
        if (b1 + 128 < p1) { issue(b1 + 128, kn, vn); patch(b1 + 128, kn, vn); }
    }
    DEC_STAMP(t.il, 4096 + blk2 * 4 + 1)
    fadec::finish(st, sm, hk, sp, NS, t.part_o, t.part_ml);
#if KCPP_FUSED_PROBE == 5
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    DEC_STAMP(t.il, 4096 + blk2 * 4 + 3)
#endif
}

template <int NIA, int NIB, int MIX, int G>
__global__ void __launch_bounds__(256, 2) k_qkv_att(const DecArgs a, const AttArgs t) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t tag = (uint32_t)a.pos[1] * 128u + (uint32_t)t.il;     // epoch of this launch
    if ((int)blockIdx.x < t.nq) qkv_role<NIA, NIB, MIX>(a, t, tag, blockIdx.x, lds);
    else att_role<G>(t, a.pos, tag, (int)blockIdx.x - t.nq);
}

template <int NIA, int NIB, int MIX, int G>
int launch_qkv_att(const DecArgs &a, AttArgs &t, hipStream_t s) {
    static int cap = -1;                           // workgroups the device holds at once (occupancy x CUs)
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    const size_t lds = (size_t)abytes + 16;
    if (cap < 0) {
        int per_cu = 0, dev = 0, ncu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_qkv_att<NIA, NIB, MIX, G>, 256, lds) != hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -3;
        cap = per_cu * ncu;
    }
    // every workgroup resident at once (the attention role waits on the q|k|v role): the q|k|v role gets the slots
    // the attention splits leave (<= 64 groups per wave: the per-lane result slots)
    const int64_t HKV = a.N[1] / 128, groups_h = (a.N[0] / HKV + 256) / 2;   // q|k|v row pairs per kv head
    const int64_t natt = (int64_t)t.NS * HKV;
    const int64_t wph = std::min<int64_t>((groups_h + 3) / 4, (cap - natt) / HKV);
    if (wph < 1 || wph * 4 * 64 < groups_h) return -3;        // the unfused path
    t.wph = (int)wph;
    t.nq = (int)(wph * HKV);
    const int64_t grid = t.nq + natt;
    hipLaunchKernelGGL((k_qkv_att<NIA, NIB, MIX, G>), dim3((unsigned)grid), dim3(256), lds, s, a, t);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" int kcpp_fa_dec_splits(int HKV);
extern "C" int kcpp_fa_comb_fused(void *ws, float *out, int H, int HKV, void *stream);

// bytes of the granule buffer of kcpp_dec_qkv_att (zeroed once by the caller)
extern "C" int64_t kcpp_dec_gran_bytes(int H, int HKV) { return (int64_t)(H + 2 * HKV) * 64 * 8 + 256; }

// attn_norm -> q|k|v (+RoPE, K/V store at pos[0]) -> attention partials (one launch) -> combine into attn_out.
// a: the mode-2 DecArgs of the q|k|v mat-vec (segments q, k, v; all Q4_K_RS, or v in Q6_K_RS with mixed = 1;
// the K/V cache [n_ctx][HKV][128] f16 in a->kc / a->vc; a->pos = {position, epoch >= 1}, the epoch advanced by every
// decode step).  ws: the flash-attention workspace; gran: the granule buffer; il: the layer (< 128).
// -3: shape / occupancy not covered (the caller runs the two-kernel path).
extern "C" int kcpp_dec_qkv_att(int mixed, const void *args, void *ws, void *gran, int il, int H, int HKV, float scale,
                                float *attn_out, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    if (a.nseg != 3 || a.D != 128 || a.K % 256 || il < 0 || il >= 128 || a.N[0] != (int64_t)H * 128 ||
        a.N[1] != (int64_t)HKV * 128 || a.N[2] != a.N[1] || a.role[0] != 0 || a.role[1] != 1 || a.role[2] != 2 ||
        H % HKV || a.ekv != a.N[1])
        return -3;
    if (!kcpp_rs_supported(KT_Q4_K_RS, a.K) || (mixed && !kcpp_rs_supported(KT_Q6_K_RS, a.K))) return -3;
    const int G = H / HKV, NS = kcpp_fa_dec_splits(HKV);
    const int nsb = (int)(a.K / 256);
    const int nia = (nsb * 8 + 63) / 64, nib = (nsb * 4 + 63) / 64;
    AttArgs t;
    t.kc = a.kc; t.vc = a.vc;
    t.part_o = (float *)((uint8_t *)ws + KCPP_FA_WS_HEADER);
    t.part_ml = (float2 *)(t.part_o + (int64_t)H * NS * 128);
    t.gran = (uint64_t *)gran;
    t.err = (unsigned *)(t.gran + (int64_t)(H + 2 * HKV) * 64);
    t.NS = NS;
    t.H = H; t.HKV = HKV; t.il = il;
    t.scale = scale;
    t.kv_ld = a.ekv;
    t.kv_hs = 128;
    int rc = -3;
#define KCPP_QA(A_, B_, M_, G_)                                                                                        \
    if (nia == A_ && nib == B_ && (mixed != 0) == (M_ != 0) && G == G_) rc = launch_qkv_att<A_, B_, M_, G_>(a, t, s);
    // Llama-3-8B (n_embd 4096, GQA 4), more-bits and plain layers.  (GQA 8, Llama-3-70B, does not fit two waves per
    // SIMD without spills: the unfused path.)
    KCPP_QA(2, 1, 1, 4)
    else KCPP_QA(2, 1, 0, 4)
#undef KCPP_QA
    if (rc) return rc;
    return kcpp_fa_comb_fused(ws, attn_out, H, HKV, stream);
}

#if KCPP_FUSED_PROBE == 5
extern "C" int kcpp_dec_set_stamps(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dec_stamps), &p, sizeof p) == hipSuccess ? 0 : -1;
}
#endif

// the fused launch's timeout flag in the granule buffer (0 = every poll completed since it was cleared)
extern "C" int kcpp_dec_fused_error(void *gran, int H, int HKV) {
    unsigned e = 0;
    if (hipMemcpy(&e, (uint64_t *)gran + (int64_t)(H + 2 * HKV) * 64, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int)e;
}
