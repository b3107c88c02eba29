// gemv_q4k.hip -- lean single-token Q4_K mat-vec (decode), VALU-budgeted.
//
// PMC counters on the unit-per-lane kernel (gemv_dec_impl.h) showed ~2.2 VALU instructions per
// weight element for the gate|up mat-vec -- 8x the essential work (3 ops to split 8 nibbles + 2
// dot4) -- and at batch 1 that VALU time (~9 us of a 21 us launch) is on the critical path next to
// HBM.  This kernel keeps the same unit decomposition (lane = 64 elements = 32 nibble bytes + the
// 16-B super-block header; ggml-common.h:286 block_q4_K) but budgets every instruction:
//   * j = unit & 3 is a per-lane constant (64 % 4 == 0), so the 6-bit scale/min extraction
//     (get_scale_min_k4, ggml-quants.c:1899) is 2 selects + 4 x (bfe, bfe, lshl_or) with shift
//     amounts precomputed once per lane;
//   * 24-bit integer multiplies (full rate) for the scale products, one float combine per unit;
//   * K = 4096 (one unit per lane per row): the lane's Q8_K activation unit lives in registers for
//     the whole launch; K > 4096: read from LDS per unit;
//   * rows of one group stream together (R rows, x2 for gate|up), the next group's loads are
//     issued before the current group is computed (PF = 1), results parked per lane and stored
//     after the loop (no stores in flight while weights stream).
// The float accumulation order differs from the CPU (per 64-element unit instead of per
// super-block); parity is the same tolerance class as every GPU mat-vec here.
#include "gemv_lean.h"

#include <algorithm>
#include <cstdlib>

namespace {

struct ScaleSel {            // per-lane constants for the (sc, m) pairs of sub-blocks 2j, 2j+1
    bool hi;                 // j >= 2
    int sh, offh;            // byte shift of pair j, offset of the 2 high bits (4 or 6)
    int shm;                 // low-4 shift for m when hi (sh + 4), else sh
};
__device__ __forceinline__ ScaleSel scale_sel(int j) {
    ScaleSel s;
    s.hi = j >= 2;
    s.sh = 16 * (j & 1);
    s.offh = s.hi ? 6 : 4;
    s.shm = s.hi ? s.sh + 4 : s.sh;
    return s;
}
// bytes s[0..11] = hdr.y | hdr.z | hdr.w (ggml-quants.c:1899):
//   j < 2 : sc = s[2j(+1)] & 63,                       m = s[2j(+1)+4] & 63
//   j >= 2: sc = s[2j(+1)+4] & 15 | (s[2j(+1)-4] >> 6) << 4,   m = s[2j(+1)+4] >> 4 | (s[2j(+1)] >> 6) << 4
__device__ __forceinline__ void q4k_scales(const uint4 &h, const ScaleSel &s, int &sc0, int &m0, int &sc1, int &m1) {
    const uint32_t lo_sc = s.hi ? h.w : h.y, lo_m = s.hi ? h.w : h.z;
    sc0 = (int)(__builtin_amdgcn_ubfe(lo_sc, s.sh, 4) | (__builtin_amdgcn_ubfe(h.y, s.sh + s.offh, 2) << 4));
    sc1 = (int)(__builtin_amdgcn_ubfe(lo_sc, s.sh + 8, 4) | (__builtin_amdgcn_ubfe(h.y, s.sh + 8 + s.offh, 2) << 4));
    m0 = (int)(__builtin_amdgcn_ubfe(lo_m, s.shm, 4) | (__builtin_amdgcn_ubfe(h.z, s.sh + s.offh, 2) << 4));
    m1 = (int)(__builtin_amdgcn_ubfe(lo_m, s.shm + 8, 4) | (__builtin_amdgcn_ubfe(h.z, s.sh + 8 + s.offh, 2) << 4));
}

struct ActU {                 // one Q8_K activation unit: 64 int8, super-block d, two 32-sums of bsums
    int4 a[4];
    float d;
    int bsA, bsB;
};
__device__ __forceinline__ void act_unit(const uint8_t *lds, int K, int u, ActU &x) {
    const int e0 = 64 * u;
    const int4 *p = (const int4 *)(lds + e0);
    x.a[0] = p[0]; x.a[1] = p[1]; x.a[2] = p[2]; x.a[3] = p[3];
    x.d = ((const float *)(lds + K))[e0 >> 8];
    const int2 b = *(const int2 *)(lds + K + (K / 256) * 4 + 2 * (e0 >> 4));
    x.bsA = (int)(int16_t)(b.x & 0xFFFF) + (int)(int16_t)(b.x >> 16);
    x.bsB = (int)(int16_t)(b.y & 0xFFFF) + (int)(int16_t)(b.y >> 16);
}

__device__ __forceinline__ float q4k_unit(const uint4 &hdr, const uint4 &q0, const uint4 &q1, const ActU &x,
                                          const ScaleSel &ss) {
    int sc0, m0, sc1, m1;
    q4k_scales(hdr, ss, sc0, m0, sc1, m1);
    const uint32_t q[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const int av[16] = {x.a[0].x, x.a[0].y, x.a[0].z, x.a[0].w, x.a[1].x, x.a[1].y, x.a[1].z, x.a[1].w,
                        x.a[2].x, x.a[2].y, x.a[2].z, x.a[2].w, x.a[3].x, x.a[3].y, x.a[3].z, x.a[3].w};
    int dlo = 0, dhi = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        dlo = sdot4((int)(q[i] & 0x0F0F0F0Fu), av[i], dlo);
        dhi = sdot4((int)((q[i] >> 4) & 0x0F0F0F0Fu), av[8 + i], dhi);
    }
    const int sumi = __mul24(sc0, dlo) + __mul24(sc1, dhi);
    const int summ = __mul24(m0, x.bsA) + __mul24(m1, x.bsB);
    const float dw = h2f((uint16_t)(hdr.x & 0xFFFF)), dmw = h2f((uint16_t)(hdr.x >> 16));
    return x.d * fmaf(dw, (float)sumi, -dmw * (float)summ);
}

}  // namespace

// PF: prefetch the next group's weights while computing this one (two register buffers); only worth
// its registers when a wave streams several groups (gate|up, output head), not at one group per wave.
template <int IT, int R, int MODE, int PRO, int MC, int PF>
__global__ void __launch_bounds__(256) k_gemv_q4k(const DecArgs a) {
    constexpr int RR = MODE == 1 ? 2 * R : R;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = (int)a.K, upr = K / 64, RB = K / 256 * 144;
    const int N0 = (int)a.N[0], N1 = a.nseg > 1 ? (int)a.N[1] : 0, N2 = a.nseg > 2 ? (int)a.N[2] : 0;
    const int ngroups = (N0 + N1 + N2) / R;
    const int nw = (int)gridDim.x * 4;
    const int wid = (int)blockIdx.x * 4 + wave;
    const int64_t eoff = dec_expert_offset(a);   // MoE slice
    const int abytes = K + K / 256 * 4 + K / 16 * 2;
    const ScaleSel ss = scale_sel(lane & 3);
    // per-lane byte offsets of the unit (it) inside a row: super-block (u >> 2), chunk j = lane & 3
    auto unit_off = [&](int it) {
        const int u = min(lane + 64 * it, upr - 1);
        return (uint32_t)((u >> 2) * 144);
    };
    const uint32_t jq = 16u + 32u * (uint32_t)(lane & 3);

    auto group_rows = [&](int g, int &seg, int &row0) {
        const int r = g * R;
        seg = r < N0 ? 0 : (r < N0 + N1 ? 1 : 2);
        row0 = seg == 0 ? r : (seg == 1 ? r - N0 : r - N0 - N1);
    };
    struct Buf { uint4 h[IT][RR], q0[IT][RR], q1[IT][RR]; };
    auto issue = [&](int g, Buf &b) {
        int seg, row0;
        group_rows(g, seg, row0);
        const uint8_t *W = (seg == 0 ? a.W[0] : (seg == 1 ? a.W[1] : a.W[2])) + eoff;
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint8_t *rp = (MODE == 1 && r >= R ? a.W2 + eoff : W) + (int64_t)(row0 + (r % R)) * RB;
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const uint32_t o = unit_off(it);
                b.h[it][r] = ld_nt(rp + o);
                b.q0[it][r] = ld_nt(rp + o + jq);
                b.q1[it][r] = ld_nt(rp + o + jq + 16u);
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
    // the lane's activation units (u = lane + 64 it) are the same for every row: held in registers for the
    // whole launch (LDS re-reads at a 64-B lane stride were bank-conflict bound at K = 14336)
    ActU xr[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) act_unit(lds, K, min(lane + 64 * it, upr - 1), xr[it]);

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
#pragma unroll
            for (int r = 0; r < RR; ++r) {
                const float p = q4k_unit(b.h[it][r], b.q0[it][r], b.q1[it][r], xr[it], ss);
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
    // epilogue stores (one group per lane)
    if (slot_g < 0) return;
    int seg, row0;
    group_rows(slot_g, seg, row0);
    lean::store_group<R, MODE>(a, seg, row0, slot);
}

namespace {
template <int IT, int R, int MODE, int PRO, int MC, int PF>
int launch_q4k(const DecArgs &a, hipStream_t s) {
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % R) return -5;
        ntot += a.N[i];
    }
    const int64_t groups = ntot / R;
    // measured (tools/stream_probe.py sweep): 512 workgroups (2 per CU) for every shape, 256 for gate|up with
    // R = 2 -- fewer prologues (each workgroup re-derives the activation) and less queueing than 1024
    const int max_blocks = MODE == 1 && R == 2 ? 256 : 512;
    int64_t nblk = std::min<int64_t>((groups + 3) / 4, max_blocks);
    nblk = std::max<int64_t>(nblk, (groups + 255) / 256);    // <= 64 groups per wave (result slots)
    const int64_t abytes = a.K + a.K / 256 * 4 + a.K / 16 * 2;
    hipLaunchKernelGGL((k_gemv_q4k<IT, R, MODE, PRO, MC, PF>), dim3((unsigned)nblk), dim3(256), (size_t)abytes + 16, s, a);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
}  // namespace

// -3 = not covered (caller falls back)
extern "C" int kcpp_gemv_q4k(const void *args, int mode, int pro, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    if (a.nseg < 1 || a.nseg > 3) return -3;
    // gate|up: R = 2 with prefetch at 256 workgroups (17.5 us vs 21.1 us for gemv_dec_impl.h)
    if (a.K == 4096) {
        if (mode == 1 && pro == 1) return launch_q4k<1, 2, 1, 1, 1, 1>(a, s);
        if (mode == 2 && pro == 1) return launch_q4k<1, 2, 2, 1, 1, 0>(a, s);
        if (mode == 0 && pro == 0) return launch_q4k<1, 1, 0, 0, 1, 0>(a, s);
        if (mode == 0 && pro == 1) return launch_q4k<1, 2, 0, 1, 1, 1>(a, s);
        return -3;
    }
    // ffn_down (K = 14336): R = 1 without prefetch (tools/probe_down sweep: R 2 / prefetch variants no faster)
    if (a.K == 14336 && mode == 0 && pro == 2) return launch_q4k<4, 1, 0, 2, 4, 0>(a, s);
    if (a.K == 14336 && mode == 0 && pro == 0) return launch_q4k<4, 1, 0, 0, 4, 0>(a, s);
    return -3;
}
