// gemv_rs.hip -- single-token mat-vec (decode) over the row-major decode layouts KT_Q4_K_RS / KT_Q5_K_RS / KT_Q6_K_RS.
//
// Why a layout of its own: in the ggml block order (block_q4_K, ggml-common.h:286: 16-B header + 128 B
// of nibbles, repeated) a lane that owns a 64-element unit reads three 16-B pieces at a 144-B stride,
// so every wave-wide load instruction touches ~18 cache lines for 1 KiB of data -- the address
// pattern alone capped a 66 MB gate|up read at 15 us against 11.3 us for a contiguous stream
// (tools/stream_probe.py).  The RS layouts keep each row's bytes together but split them into planes
// (kcpp_common.h):
//   Q4_K_RS row: [nsb][16] headers ++ [nsb][128] nibbles
//   Q5_K_RS row: [nsb][16] headers ++ [nsb][128] nibbles ++ [nsb][32] qh
//   Q6_K_RS row: [4 nsb][16] ql-lo ++ [4 nsb][16] ql-hi ++ [4 nsb][16] qh ++ [4 nsb][4] scales ++ [nsb] f16 d
// so lane l's data piece i is the 16 B at plane + 16 (l + 64 i): one wave load = 1 KiB contiguous.
//
// Work split: lane l owns the same piece positions of every row, so its Q8_K activation slices (from
// the LDS prologue: rms_norm * w -> Q8_K, quantize only, or a copy) live in registers for the whole
// launch; a wave owns R rows per group (x2 for gate|up), groups stride over a persistent grid, the
// next group's loads are in flight while the current one is reduced (PF), and the per-row results are
// parked per lane and stored once after the streaming loop (lean::store_group: residual, SiLU-GLU,
// RoPE + f16 K/V cache stores).
//
// Integer parts are exact (v_dot4_i32_i8 on the 4/6-bit weights and the Q8_K int8 activation, bsums
// for the min / -32 offsets) as in ggml_vec_dot_q4_K_q8_K / ggml_vec_dot_q6_K_q8_K
// (ggml-quants.c:7714, 8919); only the fp32 combination order differs (per 32/64 elements).
#include "gemv_lean.h"

#include <algorithm>
#include <cstdlib>

#ifdef KCPP_STAMPS
// phase stamps (tools/rs_stamps.py; instrumented A/B build only): per workgroup 8 words -- entry, activation
// ready, first group reduced, streaming done, results stored, (grid << 32 | block), K | mode << 24, rows
__device__ unsigned long long *g_rs_stamps;
__device__ unsigned g_rs_slot;
#define RS_STAMP(ph)                                                                                                  \
    if (threadIdx.x == 0 && st_) __hip_atomic_store(&st_[(ph)], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,   \
                                                     __HIP_MEMORY_SCOPE_AGENT);
extern "C" int kcpp_rs_set_stamps(void *p) {
    unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rs_stamps), &p, sizeof p) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rs_slot), &z, sizeof z) == hipSuccess ? 0 : -1;
}
#else
#define RS_STAMP(ph)
#endif

#include "gemv_rs.h"
#include "gemv_dec_impl.h"
using namespace rs;


// NI = pieces per lane per row (ceil(nsb * PIECES_PER_SB / 64)); R rows per group (x2 for gate|up);
// PRO 0: act copy, 1: rms_norm * w -> Q8_K, 2: quantize only; MC = ceil(K / 4096) prologue chunks;
// PF: issue the next group's loads before reducing the current one.
// NWV waves per workgroup (4, or 8: one activation prologue shared by twice the waves)
// XL (long K: 70B ffn_down K = 28672, MoE n_ff > 14336): the lane's activation slices are read from the LDS image per
// piece instead of living in registers for the launch (NI up to 16 pieces per row would not fit beside the weights);
// NI is then a ceiling, pieces past the row are masked (their loads clamped to the row's last piece)
// ROUTE (MoE two-slot GLU, PRO 1, K <= 4096): the router runs in every workgroup on the prologue's normalised row
// (k_moe_route<WT, true>'s thread -> element map, fma order and wave / workgroup sums, so the ids and weights are
// bit-identical), then the expert weights are issued; one launch per layer less
// MODE 3 (MoE, both top-2 slots' down projections in one launch, NWV = 8, PRO 2): waves 0-3 stream expert eid's rows
// against slot 0's h (x), waves 4-7 the same rows of expert eid1 against slot 1's h (x + K); the halves meet in LDS and
// the row is ((w0 o0) + (w1 o1)) + res -- the two chained MODE 0 launches' result bit for bit
template <int TYPE, int NI, int R, int MODE, int PRO, int MC, int PF, int NWV = 4, bool XL = false, bool ROUTE = false>
__global__ void __launch_bounds__(64 * NWV) k_gemv_rs(const DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int KB_BID = (int)blockIdx.x, KB_NBLK = (int)gridDim.x;
    constexpr bool AUX = false;
    float *const aux0 = nullptr, *const aux1 = nullptr, *const aux2 = nullptr;
    uint16_t *const auxh = nullptr;
    const RopeP rp{};
    float *const auxrn = nullptr, *const auxyn = nullptr;
#include "gemv_rs_body.inc"
}
// the ggml plugin's fused nodes (AuxOut): the same body storing the intermediate nodes' tensors too -- MODE 0 the
// product before the residual, MODE 1 gate, silu(gate) and up beside the GLU product
template <int TYPE, int NI, int R, int MODE, int PRO, int MC, int PF, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_gemv_rs_aux(const DecArgs a, const AuxOut o) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int KB_BID = (int)blockIdx.x, KB_NBLK = (int)gridDim.x;
    constexpr bool XL = false, ROUTE = false, AUX = true;
    float *const aux0 = o.p0, *const aux1 = o.p1, *const aux2 = o.p2;
    uint16_t *const auxh = o.h0;
    const RopeP rp = o.rope;
    float *const auxrn = o.rn, *const auxyn = o.yn;
#include "gemv_rs_body.inc"
}

namespace {
// the ggml plugin's AuxOut for the launches below (kcpp_gemv_rs_aux; null: the runtime's plain launches)
thread_local const AuxOut *g_rs_aux = nullptr;

template <int TYPE, int NI, int R, int MODE, int PRO, int MC, int PF, int NWV = 4, bool XL = false, bool ROUTE = false,
          bool AUX = false>
int launch_rs(const DecArgs &a, int max_blocks, hipStream_t s) {
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % R) return -5;
        ntot += a.N[i];
    }
    const int64_t groups = ntot / R;
    constexpr int WPG = MODE == 3 ? NWV / 2 : NWV;
    int64_t nblk = std::min<int64_t>((groups + WPG - 1) / WPG, max_blocks);
    nblk = std::max<int64_t>(nblk, (groups + 64 * WPG - 1) / (64 * WPG));    // <= 64 groups per wave (result slots)
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    const int64_t lbytes = MODE == 3 ? 2 * ((abytes + 15) & ~(int64_t)15) : abytes;
    if constexpr (AUX) {
        static_assert(!XL && !ROUTE, "AUX instances: plain single-token launches");
        hipLaunchKernelGGL((k_gemv_rs_aux<TYPE, NI, R, MODE, PRO, MC, PF, NWV>), dim3((unsigned)nblk), dim3(64 * NWV),
                           (size_t)lbytes + 16, s, a, *g_rs_aux);
    } else {
        hipLaunchKernelGGL((k_gemv_rs<TYPE, NI, R, MODE, PRO, MC, PF, NWV, XL, ROUTE>), dim3((unsigned)nblk), dim3(64 * NWV),
                           (size_t)lbytes + 16, s, a);
    }
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// rows per group, prefetch and grid per shape, from the launch sweep (tools/sweep_rs.sh, MI355X):
//   gate|up (mode 1)  : R 1, PF, 512 workgroups     14.8 us / 66 MB
//   q|k|v (mode 2)    : R 2, 512                     7.0 us / 14 MB
//   head (N > 16384)  : R 2, 512                    69.4 us / 431 MB (6.2 TB/s)
//   down (K > 8192)   : R 1, PF, 256 (Q4_K) / 512 (Q6_K)   12.5 / 15.0 us
//   wo (quantize prologue, PRO 2): R 1, 512          (1024: every workgroup quantizes, more of them cost more)
//   other             : R 1, 1024                    4.9 us / 9.4 MB
template <int TYPE, int NI, int MC>
int pick_rs(const DecArgs &a, int mode, int pro, hipStream_t s) {
    const int64_t ntot = a.N[0] + (a.nseg > 1 ? a.N[1] : 0) + (a.nseg > 2 ? a.N[2] : 0);
    int R = 1, PF = 0, B = 1024;
    if (mode == 1) { PF = 1; B = 512; }
    else if (mode == 2) { R = 2; B = 512; }
    else if (ntot > 16384) { R = 2; B = 512; }
    else if (a.K > 8192) { PF = TYPE == KT_Q4_K_RS; B = TYPE == KT_Q4_K_RS ? 256 : 512; }
    else if (pro == 2) B = 512;          // wo with its quantize prologue (every workgroup quantizes the input)
    // 8-wave workgroups, one per CU (one activation prologue shared by 8 waves instead of 4), measured per kernel in
    // isolation (tools/stream_probe.py dec, weights rotated past the Infinity Cache): GLU 14.8 -> 14.1 us (PF),
    // down Q4_K 11.3 -> 9.7 and Q6_K 13.6 -> 12.2 (no PF: two rows per wave, both in flight), wo 5.4 -> 4.7; in the
    // bench's token graph down 12.0 / 13.7 -> 10.0 / 12.4 us, wo 5.3 -> 5.1, GLU unchanged: 577 -> 600 tok/s.  The
    // q|k|v launches stay at 4 waves (8: 6.8 -> 7.4 us, 592 tok/s).
    // the ggml plugin's fused nodes (aux: the intermediate nodes' tensors stored too), separate instances so the
    // runtime's launches carry none of it: MUL_MAT -> ADD as the plain single-token launch below (quantize prologue,
    // 8 waves), the SiLU GLU as KCPP_RS_P(2)'s mode 1
    if (g_rs_aux) {
        // with a ROPE behind the product: two rows per group (a rope pair in one lane), as the runtime's q|k|v launch
        if (g_rs_aux->rope.out) {
            if (mode != 0 || ntot > 16384 || ntot % 2) return -3;
            if (pro == 2) return launch_rs<TYPE, NI, 2, 0, 2, MC, 0, 4, false, false, true>(a, 512, s);
            if (pro == 1 && MC == 1) return launch_rs<TYPE, NI, 2, 0, 1, MC, 0, 4, false, false, true>(a, 512, s);
            return -3;
        }
        if (mode == 0 && pro == 2 && ntot <= 16384) return launch_rs<TYPE, NI, 1, 0, 2, MC, 0, 8, false, false, true>(a, 256, s);
        if (mode == 1 && a.nseg == 1 && !a.eid && !a.route_w) {
            if (pro == 2) return launch_rs<TYPE, NI, 1, 1, 2, MC, 1, 4, false, false, true>(a, 512, s);
            // the norm in the prologue (the runtime's GLU shape: 8 waves, group prefetch)
            if (pro == 1 && MC == 1) return launch_rs<TYPE, NI, 1, 1, 1, MC, 1, 8, false, false, true>(a, 256, s);
        }
        return -3;
    }
    if (mode == 1 && pro == 1 && R == 1) {
        if (a.route_w) {                  // routed two-slot GLU (MoE decode): K <= 4096 (one prologue chunk), NE <= 8
            if constexpr (MC == 1) {
                if (a.nseg == 2 && a.route_ne >= 2 && a.route_ne <= 8 && a.K <= 4096 && a.route_ids && a.route_wts &&
                    (a.route_wt == KT_F32 || a.route_wt == KT_F16))
                    return launch_rs<TYPE, NI, 1, 1, 1, MC, 1, 8, false, true>(a, 256, s);
            }
            return -3;
        }
        return launch_rs<TYPE, NI, 1, 1, 1, MC, 1, 8>(a, 256, s);
    }
    if (mode == 0 && pro == 2 && R == 1 && ntot <= 16384) return launch_rs<TYPE, NI, 1, 0, 2, MC, 0, 8>(a, 256, s);
#define KCPP_RS_P(PRO_)                                                                                             \
    if (pro == PRO_) {                                                                                              \
        if (mode == 1) return PF ? launch_rs<TYPE, NI, 1, 1, PRO_, MC, 1>(a, B, s) : launch_rs<TYPE, NI, 1, 1, PRO_, MC, 0>(a, B, s); \
        if (mode == 2) return launch_rs<TYPE, NI, 2, 2, PRO_, MC, 0>(a, B, s);                                                \
        if (R == 2) return PF ? launch_rs<TYPE, NI, 2, 0, PRO_, MC, 1>(a, B, s) : launch_rs<TYPE, NI, 2, 0, PRO_, MC, 0>(a, B, s); \
        return PF ? launch_rs<TYPE, NI, 1, 0, PRO_, MC, 1>(a, B, s) : launch_rs<TYPE, NI, 1, 0, PRO_, MC, 0>(a, B, s);             \
    }
    KCPP_RS_P(0)
    KCPP_RS_P(1)
    KCPP_RS_P(2)
#undef KCPP_RS_P
    return -3;
}
// long K (XL): the down projection of Llama-3-70B (K = 28672) and MoE experts with n_ff past 14336 (mode 0, quantize
// or norm prologue), the same tensors read column by column from a quantized activation (pro 0: the M <= 8 prefill
// tail and the ggml plugin's few-row MUL_MAT, gemv_cols), and the projections of models with n_embd past 14336 (GLU
// mode 1, q|k|v mode 2 with the norm prologue).  One row per group (two for mode 2), 8-wave workgroups, no group
// prefetch: a row's NI pieces are already 16 KB (Q4_K, K = 28672) in flight per wave, 128 KB per CU.  NI = the ceiling
// the shape rounds up to.
template <int TYPE, int NI>
int pick_rs_xl(const DecArgs &a, int mode, int pro, hipStream_t s) {
    if (g_rs_aux) return -3;
    constexpr int MC = TYPE == KT_Q6_K_RS ? NI : NI / 2;        // ceil(K / 4096) at the ceiling
    if (mode == 0) {
        if (pro == 2) return launch_rs<TYPE, NI, 1, 0, 2, MC, 0, 8, true>(a, 256, s);
        if (pro == 1) return launch_rs<TYPE, NI, 1, 0, 1, MC, 0, 8, true>(a, 256, s);
        if (pro == 0) return launch_rs<TYPE, NI, 1, 0, 0, MC, 0, 8, true>(a, 256, s);
    } else if (mode == 1) {
        if (a.route_w || (a.nseg != 1 && !a.eid1)) return -3;
        if (pro == 1) return launch_rs<TYPE, NI, 1, 1, 1, MC, 0, 8, true>(a, 256, s);
        if (pro == 0) return launch_rs<TYPE, NI, 1, 1, 0, MC, 0, 8, true>(a, 256, s);
    } else if (mode == 2) {
        if (pro == 1) return launch_rs<TYPE, NI, 2, 2, 1, MC, 0, 8, true>(a, 256, s);
    }
    return -3;
}
template <int TYPE>
int dispatch_rs_xl(const DecArgs &a, int ni, int mode, int pro, hipStream_t s) {
    if constexpr (TYPE == KT_Q6_K_RS) {
        if (ni <= 6) return pick_rs_xl<TYPE, 6>(a, mode, pro, s);
        return pick_rs_xl<TYPE, 8>(a, mode, pro, s);
    } else if constexpr (TYPE == KT_Q5_K_RS) {         // 12 VGPRs per piece: spills past 10 pieces
        return ni <= 10 ? pick_rs_xl<TYPE, 10>(a, mode, pro, s) : -3;
    } else {
        if (ni <= 10) return pick_rs_xl<TYPE, 10>(a, mode, pro, s);
        if (ni <= 12) return pick_rs_xl<TYPE, 12>(a, mode, pro, s);
        return ni <= 14 ? pick_rs_xl<TYPE, 14>(a, mode, pro, s) : -3;
    }
}
}  // namespace

// ---------------------------------------------------------------- q|k (Q4_K_RS) + v (Q6_K_RS) in one launch
// The Q4_K_M "more bits" layers keep attn_v in Q6_K: instead of a second launch for its 1024 rows (a latency-bound
// kernel of its own: prologue, one group per wave, epilogue), segments 0 / 1 (q, k) run the Q4_K_RS path and
// segment 2 (v) the Q6_K_RS path of one grid over the same LDS activation (rms_norm -> Q8_K prologue, both types'
// vec_dot_type); groups are wave-uniform in type.  Mode 2 epilogue (RoPE + f16 q / K / V stores), R = 2.
template <int NIA, int NIB, int MC>
__global__ void __launch_bounds__(256) k_gemv_rs_qkv(const DecArgs a) {
    using TA = RS<KT_Q4_K_RS>;
    using TB = RS<KT_Q6_K_RS>;
    constexpr int R = 2;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = (int)a.K, nsb = K / 256;
    const int RBA = nsb * TA::BYTES, RBB = nsb * TB::BYTES;
    const int npA = nsb * TA::PIECES_PER_SB, npB = nsb * TB::PIECES_PER_SB;
    const int N0 = (int)a.N[0], N1 = (int)a.N[1], N2 = (int)a.N[2];
    const int ngA = (N0 + N1) / R, ngroups = ngA + N2 / R;
    const int nw = (int)gridDim.x * 4;
    const int wid = (int)blockIdx.x * 4 + wave;
    const typename TA::Lane lca = TA::lane_consts(lane);
    const typename TB::Lane lcb = TB::lane_consts(lane);
    auto group_rows = [&](int g, int &seg, int &row0) {
        if (g < ngA) {
            const int r = g * R;
            seg = r < N0 ? 0 : 1;
            row0 = seg == 0 ? r : r - N0;
        } else {
            seg = 2;
            row0 = (g - ngA) * R;
        }
    };
    struct BufA { typename TA::W w[NIA][R]; };
    struct BufB { typename TB::W w[NIB][R]; };
    auto issueA = [&](int g, BufA &b) {
        int seg, row0;
        group_rows(g, seg, row0);
        const uint8_t *W = seg == 0 ? a.W[0] : a.W[1];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < NIA; ++i) TA::load(W + (int64_t)(row0 + r) * RBA, nsb, min(lane + 64 * i, npA - 1), b.w[i][r]);
    };
    auto issueB = [&](int g, BufB &b) {
        const int row0 = (g - ngA) * R;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < NIB; ++i) TB::load(a.W[2] + (int64_t)(row0 + r) * RBB, nsb, min(lane + 64 * i, npB - 1), b.w[i][r]);
    };
    BufA ba;
    BufB bb;
    const int g0 = min(wid, ngroups - 1);
    lean::ActPro<1, MC> pro;
    pro.load(a);
    if (g0 < ngA) issueA(g0, ba);
    else issueB(g0, bb);
    pro.compute(a, lds);
    typename TA::Act xa[NIA];
    typename TB::Act xb[NIB];
#pragma unroll
    for (int i = 0; i < NIA; ++i) TA::act(lds, K, min(TA::sb_of(lane, i), nsb - 1), lca, xa[i]);
#pragma unroll
    for (int i = 0; i < NIB; ++i) TB::act(lds, K, min(TB::sb_of(lane, i), nsb - 1), lcb, xb[i]);
    float slot[R] = {0.0f, 0.0f};
    int slot_g = -1;
    int k = 0;
    for (int g = wid; g < ngroups; g += nw, ++k) {
        float acc[R] = {0.0f, 0.0f};
        if (g < ngA) {
            if (k) issueA(g, ba);
#pragma unroll
            for (int i = 0; i < NIA; ++i) {
                const bool ok = (NIA * 64 == npA) || lane + 64 * i < npA;
#pragma unroll
                for (int r = 0; r < R; ++r) { const float p = TA::dot(ba.w[i][r], xa[i], lca); acc[r] += ok ? p : 0.0f; }
            }
        } else {
            if (k) issueB(g, bb);
#pragma unroll
            for (int i = 0; i < NIB; ++i) {
                const bool ok = (NIB * 64 == npB) || lane + 64 * i < npB;
#pragma unroll
                for (int r = 0; r < R; ++r) { const float p = TB::dot(bb.w[i][r], xb[i], lcb); acc[r] += ok ? p : 0.0f; }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_f(acc[r]))));
        const bool mine = lane == k;
#pragma unroll
        for (int r = 0; r < R; ++r) slot[r] = mine ? acc[r] : slot[r];
        slot_g = mine ? g : slot_g;
    }
    if (slot_g < 0) return;
    int seg, row0;
    group_rows(slot_g, seg, row0);
    lean::store_group<R, 2>(a, seg, row0, slot);
}

// q|k|v decode projection with q, k in Q4_K_RS and v in Q6_K_RS (segments 0, 1, 2): one launch.  -3 when not covered.
extern "C" int kcpp_gemv_rs_qkv_mixed(const void *args, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    if (a.nseg != 3 || a.K % 256 || !kcpp_rs_supported(KT_Q4_K_RS, a.K) || !kcpp_rs_supported(KT_Q6_K_RS, a.K)) return -3;
    if (a.N[0] % 2 || a.N[1] % 2 || a.N[2] % 2) return -5;
    const int nsb = (int)(a.K / 256);
    const int nia = (nsb * 8 + 63) / 64, nib = (nsb * 4 + 63) / 64, mc = (int)((a.K + 4095) / 4096);
    const int64_t groups = (a.N[0] + a.N[1] + a.N[2]) / 2;
    int64_t nblk = std::min<int64_t>((groups + 3) / 4, 512);
    nblk = std::max<int64_t>(nblk, (groups + 255) / 256);
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    hipStream_t s = (hipStream_t)stream;
#define KCPP_QKVM(A_, B_, M_) hipLaunchKernelGGL((k_gemv_rs_qkv<A_, B_, M_>), dim3((unsigned)nblk), dim3(256), (size_t)abytes + 16, s, a)
    if (nia == 2 && nib == 1 && mc == 1) KCPP_QKVM(2, 1, 1);          // n_embd 4096 (Llama-3-8B)
    else if (nia == 4 && nib == 2 && mc == 2) KCPP_QKVM(4, 2, 2);     // n_embd 8192 (Llama-3-70B)
    else if (nia == 1 && nib == 1 && mc == 1) KCPP_QKVM(1, 1, 1);
    else return -3;
#undef KCPP_QKVM
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------- q (RS layout) + k|v (Q8_0) in one launch
// Mixtral's Q5_K_M policy keeps attn_k / attn_v in Q8_0 (n_expert == 8) and attn_q in Q5_K, so its q|k|v decode step
// was two dependent launches of short latency-bound kernels.  Here one grid runs both unchanged: workgroups [0, nA) are
// the RS q launch (k_gemv_rs's body, mode 2: RoPE + f16 q), [nA, nA + nB) the Q8_0 k|v launch (k_gemv_dec's body,
// mode 2: RoPE of k + the f16 K / V cache stores), each with its own prologue (Q8_K / Q8_0 activation of the same
// normalised row) and its own grid size, so every row's arithmetic -- and result -- is the separate launches'.  The
// bodies are included textually (gemv_rs_body.inc, gemv_dec_body.inc) so that each reads its DecArgs kernel parameter
// directly (through a reference the parameter is copied to scratch memory and every load goes through it).
template <int TA, int NIA, int MCA, int ITB>
__global__ void __launch_bounds__(256) k_gemv_qkv_dual(const DecArgs a, const DecArgs b, int nA) {
    if ((int)blockIdx.x < nA) {
        constexpr int TYPE = TA, NI = NIA, R = 2, MODE = 2, PRO = 1, MC = MCA, PF = 0, NWV = 4;
        constexpr bool XL = false, ROUTE = false, AUX = false;
        float *const aux0 = nullptr, *const aux1 = nullptr, *const aux2 = nullptr;
        uint16_t *const auxh = nullptr;
        const RopeP rp{};
        float *const auxrn = nullptr, *const auxyn = nullptr;
        extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
        const int KB_BID = (int)blockIdx.x, KB_NBLK = nA;
#include "gemv_rs_body.inc"
    } else {
        constexpr int TYPE = KT_Q8_0, R = 2, MODE = 2, PRO = 1, MC = 1, IT = ITB;
        extern __shared__ __attribute__((aligned(16))) uint8_t lds_act[];
        const int KB_BID = (int)blockIdx.x - nA, KB_NBLK = (int)gridDim.x - nA;
#define KB_ARGS b
#include "gemv_dec_body.inc"
#undef KB_ARGS
    }
}

// qa: the RS-layout segments (mode 2, rms_norm prologue) -- pick_rs's launch for them; kv: Q8_0 segments (mode 2) --
// dispatch_mode<KT_Q8_0>'s.  -3 when the pair is not covered (the caller launches them separately).
extern "C" int kcpp_gemv_qkv_dual(const void *qargs, int qtype, const void *kvargs, void *stream) {
    const DecArgs &a = *(const DecArgs *)qargs;
    const DecArgs &b = *(const DecArgs *)kvargs;
    if (qtype != KT_Q4_K_RS && qtype != KT_Q5_K_RS && qtype != KT_Q6_K_RS) return -3;
    if (a.K != b.K || a.K % 256 || a.K > 4096 || !kcpp_rs_supported(qtype, a.K) || a.route_w) return -3;
    int64_t na_rows = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % 2) return -5;
        na_rows += a.N[i];
    }
    for (int i = 0; i < b.nseg; ++i)
        if (b.N[i] % 2) return -5;
    // RS side: launch_rs<.., R 2, mode 2, PRO 1, .., NWV 4>(a, 512)
    const int64_t groups = na_rows / 2;
    int64_t nA = std::min<int64_t>((groups + 3) / 4, 512);
    nA = std::max<int64_t>(nA, (groups + 255) / 256);
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    // Q8_0 side: launch_dec_it<KT_Q8_0, 2, 2, 1, 1, IT>
    size_t ldsB = 0;
    const int64_t nB = dec_grid<KT_Q8_0, 2, 1>(b, ldsB);
    const int64_t upr = b.K / Unit<KT_Q8_0>::ELEMS, itb = (upr + 63) / 64;
    const size_t lds = std::max<size_t>((size_t)abytes + 16, ldsB);
    const int nsb = (int)(a.K / 256);
    const int ppsb = qtype == KT_Q6_K_RS ? 4 : 8;
    const int nia = (nsb * ppsb + 63) / 64;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)(nA + nB));
#define KCPP_DUAL(TA_, NIA_, ITB_) hipLaunchKernelGGL((k_gemv_qkv_dual<TA_, NIA_, 1, ITB_>), grid, dim3(256), lds, s, a, b, (int)nA)
    if (itb == 2 && nia == 2 && qtype == KT_Q5_K_RS) KCPP_DUAL(KT_Q5_K_RS, 2, 2);      // Mixtral: K 4096
    else if (itb == 2 && nia == 2 && qtype == KT_Q4_K_RS) KCPP_DUAL(KT_Q4_K_RS, 2, 2);
    else if (itb == 2 && nia == 1 && qtype == KT_Q6_K_RS) KCPP_DUAL(KT_Q6_K_RS, 1, 2);
    else return -3;
#undef KCPP_DUAL
    KCPP_CHECK(hipGetLastError());
    return 0;
}

// K coverage of the RS kernels (the runtime picks an RS layout only where this holds): activation slices in registers
// up to 56 (Q4_K / Q5_K) / 64 (Q6_K) super-blocks; read from LDS (XL, one row's pieces in flight per wave) up to the
// register budget of a row: 112 (Q4_K: K 28672, Llama-3-70B's n_ff), 80 (Q5_K), 128 (Q6_K) super-blocks
extern "C" int kcpp_rs_supported(int type, int64_t K) {
    if (K % 256 || K < 256) return 0;
    const int64_t nsb = K / 256;
    if (type == KT_Q4_K_RS || type == KT_Q4_K) return nsb <= 112;
    if (type == KT_Q5_K_RS || type == KT_Q5_K) return nsb <= 80;
    if (type == KT_Q6_K_RS || type == KT_Q6_K) return nsb % 8 == 0 && nsb <= 128;
    return 0;
}

#ifndef Q_PF
#define Q_PF 0               // MODE 3 group prefetch: measured no faster (23.2 / 21.7 vs 23.2 / 21.0 us), more registers
#endif
#ifndef Q_XL
#define Q_XL false
#endif
// MODE 3 (both MoE slots' down projections): the shapes of the Mixtral class (n_ff 14336: 56 super-blocks)
static int pick_rs_pair(int type, const DecArgs &a, hipStream_t s) {
    if (a.nseg != 1 || !a.eid || !a.eid1 || !a.escale || a.K != 14336) return -3;
    if (type == KT_Q4_K_RS) return launch_rs<KT_Q4_K_RS, 7, 1, 3, 2, 4, Q_PF, 8, Q_XL>(a, 256, s);
    if (type == KT_Q5_K_RS) return launch_rs<KT_Q5_K_RS, 7, 1, 3, 2, 4, Q_PF, 8, Q_XL>(a, 256, s);
    if (type == KT_Q6_K_RS) return launch_rs<KT_Q6_K_RS, 4, 1, 3, 2, 4, Q_PF, 8, Q_XL>(a, 256, s);
    return -3;
}

// -3 = not covered
extern "C" int kcpp_gemv_rs(int type, const void *args, int mode, int pro, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    if (mode == 3) return pro == 2 && kcpp_rs_supported(type, a.K) ? pick_rs_pair(type, a, s) : -3;
    if (a.nseg < 1 || a.nseg > 3 || !kcpp_rs_supported(type, a.K)) return -3;
    if (mode == 1 && a.nseg != 1 && !(a.nseg == 2 && (a.eid1 || a.route_w))) return -3;   // GLU: one segment, or two MoE slots
    const int nsb = (int)(a.K / 256);
    if (type == KT_Q4_K_RS) {
        const int ni = (nsb * 8 + 63) / 64, mc = (int)((a.K + 4095) / 4096);
        switch (ni) {
        case 1: return pick_rs<KT_Q4_K_RS, 1, 1>(a, mode, pro, s);
        case 2: return pick_rs<KT_Q4_K_RS, 2, 1>(a, mode, pro, s);
        case 3: return pick_rs<KT_Q4_K_RS, 3, 2>(a, mode, pro, s);
        case 4: return pick_rs<KT_Q4_K_RS, 4, 2>(a, mode, pro, s);
        case 5: return pick_rs<KT_Q4_K_RS, 5, 3>(a, mode, pro, s);
        case 6: return pick_rs<KT_Q4_K_RS, 6, 3>(a, mode, pro, s);
        case 7: return pick_rs<KT_Q4_K_RS, 7, 4>(a, mode, pro, s);
        default: return dispatch_rs_xl<KT_Q4_K_RS>(a, ni, mode, pro, s);
        }
    }
    if (type == KT_Q5_K_RS) {
        const int ni = (nsb * 8 + 63) / 64, mc = (int)((a.K + 4095) / 4096);
        switch (ni) {
        case 1: return pick_rs<KT_Q5_K_RS, 1, 1>(a, mode, pro, s);
        case 2: return pick_rs<KT_Q5_K_RS, 2, 1>(a, mode, pro, s);
        case 3: return pick_rs<KT_Q5_K_RS, 3, 2>(a, mode, pro, s);
        case 4: return pick_rs<KT_Q5_K_RS, 4, 2>(a, mode, pro, s);
        case 5: return pick_rs<KT_Q5_K_RS, 5, 3>(a, mode, pro, s);
        case 6: return pick_rs<KT_Q5_K_RS, 6, 3>(a, mode, pro, s);
        case 7: return pick_rs<KT_Q5_K_RS, 7, 4>(a, mode, pro, s);
        default: return dispatch_rs_xl<KT_Q5_K_RS>(a, ni, mode, pro, s);
        }
    }
    if (type == KT_Q6_K_RS) {
        const int ni = (nsb * 4 + 63) / 64;
        switch (ni) {
        case 1: return pick_rs<KT_Q6_K_RS, 1, 1>(a, mode, pro, s);
        case 2: return pick_rs<KT_Q6_K_RS, 2, 2>(a, mode, pro, s);
        case 3: return pick_rs<KT_Q6_K_RS, 3, 3>(a, mode, pro, s);
        case 4: return pick_rs<KT_Q6_K_RS, 4, 4>(a, mode, pro, s);
        default: return dispatch_rs_xl<KT_Q6_K_RS>(a, ni, mode, pro, s);
        }
    }
    return -3;
}

// the ggml plugin's fused nodes: kcpp_gemv_rs's launch (modes 0 and 1, quantize prologue, one segment) through the AUX
// instances, which also store the intermediate nodes' tensors (AuxOut); -3 where no AUX instance covers the shape
extern "C" int kcpp_gemv_rs_aux(int type, const void *args, int mode, const AuxOut *aux, void *stream) {
    if (!aux || (mode == 0 && !aux->p0 && !aux->h0 && !aux->rope.out) || (mode == 1 && (!aux->p0 || !aux->p1 || !aux->p2)) ||
        (mode != 0 && mode != 1) || (aux->rope.out && (mode != 0 || !aux->rope.pos || aux->rope.D < 2 || aux->rope.D % 2)))
        return -3;
    // the norm prologue (rn / yn given): x = the norm's input, nw = the MUL's weight, K <= 4096 (one chunk per thread,
    // so the prologue's sum order is the plugin's norm kernels' -- ggml_ops.hip row_sumsq16)
    const DecArgs &da = *(const DecArgs *)args;
    const bool pro1 = da.nw != nullptr;       // (only the plugin's norm-in launches set nw here)
    if (pro1 && (da.K > 4096 || da.K % 256)) return -3;
    g_rs_aux = aux;
    const int rc = kcpp_gemv_rs(type, args, mode, pro1 ? 1 : 2, stream);
    g_rs_aux = nullptr;
    return rc;
}
