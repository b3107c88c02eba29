// gemv_stream.hip -- single-token Q4_K mat-vec with fully coalesced weight streaming.
//
// Why a second decode mat-vec: the unit-per-lane loader of gemv_dec_impl.h reads each 144-B Q4_K
// super-block as three 16-B pieces per lane (header + 2 x nibbles) at a 144-B lane stride, so one
// wave-instruction touches ~18 cache lines for 1 KB of data.  Measured on MI355X (tools/
// stream_probe.py) that access pattern alone caps a 66 MB read at 4.4 TB/s versus 5.9 TB/s for a
// contiguous stream.  Here every wave-instruction reads whole contiguous 256-B..1-KB pieces:
//
//   * a wave owns G = 64/LPR rows (a "tile"); LPR lanes stream one row: lane l reads 16-B chunk
//     c = l + LPR*i of the row (i = 0 .. NI-1), so each instruction covers G contiguous runs of
//     16*LPR bytes.  A Q4_K super-block is 9 chunks: chunk 0 = {d, dmin, 12 scale bytes},
//     chunks 1..8 = 128 nibble bytes (ggml-common.h:286-297 block_q4_K).
//   * header chunks are parked in a per-wave LDS table (one 16-B slot per super-block), then every
//     nibble chunk reads its super-block's header from LDS -- no second global read of headers.
//   * the dot product is the CPU vec_dot_q4_K_q8_K split per 32 nibbles (ggml-quants.c:7714):
//     chunk k of a super-block holds elements 64j+16h+[0,16) (low nibbles, sub-block 2j) and
//     64j+32+16h+[0,16) (high nibbles, sub-block 2j+1), j = (k-1)/2, h = (k-1)%2; exact int8 dots
//     against the Q8_K activation in LDS, then d*sc*dot - dmin*m*bsum in fp32.
//   * activation prologue as gemv_dec_impl.h (rms_norm * w -> Q8_K in LDS), its global loads
//     issued before the first weight loads.
//   * results are reduced per row (DPP), parked in lane k of the row's lanes for the wave's k-th
//     tile, and stored after the loop, so no store is in flight while weights stream.
#include "gemv_units.h"
#include "kcpp_internal.h"

#include <algorithm>
#include <cstdlib>

namespace {

template <int LPR>
__device__ __forceinline__ float row_sum(float v) {          // sum over the LPR lanes of a row
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    if constexpr (LPR >= 32) v += __shfl_xor(v, 16, 64);
    if constexpr (LPR >= 64) v += __shfl_xor(v, 32, 64);
    return v;
}

// Activation prologue (see gemv_dec_impl.h); split so its loads precede the weight loads.
template <int PRO, int MAXC>
struct ActPro {
    float v[MAXC][16];
    float w[PRO == 1 ? MAXC : 1][16];
    __device__ __forceinline__ void load(const DecArgs &a) {
        const int tid = threadIdx.x, nchunk = (int)(a.K / 16);
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = min(tid + 256 * i, nchunk - 1);
            const float4 *p = (const float4 *)(a.x + 16 * (int64_t)c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 f = p[k];
                v[i][4 * k] = f.x; v[i][4 * k + 1] = f.y; v[i][4 * k + 2] = f.z; v[i][4 * k + 3] = f.w;
            }
            if constexpr (PRO == 1) {
                const float4 *q = (const float4 *)(a.nw + 16 * (int64_t)c);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 f = q[k];
                    w[i][4 * k] = f.x; w[i][4 * k + 1] = f.y; w[i][4 * k + 2] = f.z; w[i][4 * k + 3] = f.w;
                }
            }
        }
    }
    __device__ __forceinline__ void compute(const DecArgs &a, uint8_t *lds) {
        const int tid = threadIdx.x;
        const int64_t K = a.K;
        const int nchunk = (int)(K / 16);
        if constexpr (PRO == 1) {
            double ss = 0.0;
#pragma unroll
            for (int i = 0; i < MAXC; ++i)
                if (tid + 256 * i < nchunk) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) ss += (double)__fmul_rn(v[i][e], v[i][e]);
                }
            ss = wave_sum_d(ss);
            __shared__ double red[4];
            if ((tid & 63) == 0) red[tid >> 6] = ss;
            __syncthreads();
            const double sum = red[0] + red[1] + red[2] + red[3];
            const float scale = 1.0f / sqrtf((float)(sum / (double)K) + a.eps);   // ggml.c:12089
#pragma unroll
            for (int i = 0; i < MAXC; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) v[i][e] = __fmul_rn(__fmul_rn(v[i][e], scale), w[i][e]);
        }
        int8_t *qs = (int8_t *)lds;
        float *d = (float *)(lds + K);
        int16_t *bs = (int16_t *)(lds + K + K / 256 * 4);
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = tid + 256 * i;
            if (c < nchunk) q8k_quant16(v[i], c & 15, qs + (c >> 4) * 256, d + (c >> 4), bs + (c >> 4) * 16);
        }
        __syncthreads();
    }
};

// Header parking: the lane holding a super-block's first chunk {d, dmin, scales[12]} decodes the eight
// 6-bit (scale, min) pairs (get_scale_min_k4, ggml-quants.c:1899) once, into
//   dtab[sb] = d | dmin << 16 (fp16 pair, as stored)       stab[sb].word[j] = sc2j | m2j<<8 | sc2j+1<<16 | m2j+1<<24
__device__ __forceinline__ uint4 q4k_decode_scales(const uint4 &hdr) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int s0, m0, s1, m1;
        k4_scale_min(hdr, 2 * j, s0, m0);
        k4_scale_min(hdr, 2 * j + 1, s1, m1);
        w[j] = (uint32_t)s0 | ((uint32_t)m0 << 8) | ((uint32_t)s1 << 16) | ((uint32_t)m1 << 24);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// one Q4_K nibble chunk (k = 1..8 of its super-block) against the Q8_K activation in LDS
__device__ __forceinline__ float q4k_chunk_dot(const uint4 &q, uint32_t dd, uint32_t scw, int sb, int k,
                                               const int8_t *aqs, const float *ad, const int16_t *abs) {
    const int j = (k - 1) >> 1, h = (k - 1) & 1;
    const int sc0 = scw & 0xFF, m0 = (scw >> 8) & 0xFF, sc1 = (scw >> 16) & 0xFF, m1 = scw >> 24;
    const int e = sb * 256 + 64 * j + 16 * h;
    const int4 alo = *(const int4 *)(aqs + e);
    const int4 ahi = *(const int4 *)(aqs + e + 32);
    const int blo = abs[(e >> 4)], bhi = abs[(e >> 4) + 2];
    int dlo = 0, dhi = 0;
    dlo = sdot4((int)(q.x & 0x0F0F0F0Fu), alo.x, dlo);
    dlo = sdot4((int)(q.y & 0x0F0F0F0Fu), alo.y, dlo);
    dlo = sdot4((int)(q.z & 0x0F0F0F0Fu), alo.z, dlo);
    dlo = sdot4((int)(q.w & 0x0F0F0F0Fu), alo.w, dlo);
    dhi = sdot4((int)((q.x >> 4) & 0x0F0F0F0Fu), ahi.x, dhi);
    dhi = sdot4((int)((q.y >> 4) & 0x0F0F0F0Fu), ahi.y, dhi);
    dhi = sdot4((int)((q.z >> 4) & 0x0F0F0F0Fu), ahi.z, dhi);
    dhi = sdot4((int)((q.w >> 4) & 0x0F0F0F0Fu), ahi.w, dhi);
    const float xd = ad[sb];
    const float d = __fmul_rn(xd, h2f((uint16_t)(dd & 0xFFFF)));
    const float dmin = __fmul_rn(xd, h2f((uint16_t)(dd >> 16)));
    return __fsub_rn(__fmul_rn(d, (float)(sc0 * dlo + sc1 * dhi)), __fmul_rn(dmin, (float)(m0 * blo + m1 * bhi)));
}

}  // namespace

// NI = iterations (16-B chunks per lane) per row, a compile-time bound; rows must have <= 64*NI...
template <int LPR, int NI, int MODE, int PRO, int MC>
__global__ void __launch_bounds__(256) k_gemv_stream(const DecArgs a) {
    constexpr int G = 64 / LPR;                       // rows per tile (per wave)
    constexpr int NM = MODE == 1 ? 2 : 1;             // weight matrices (gate, up)
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63, l = lane % LPR, gi = lane / LPR;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = (int)a.K, nsb = K / 256, NC = nsb * 9, RB = nsb * 144;
    const int N0 = (int)a.N[0], N1 = a.nseg > 1 ? (int)a.N[1] : 0, N2 = a.nseg > 2 ? (int)a.N[2] : 0;
    const int ntiles = (N0 + N1 + N2) / G;
    const int nw = (int)gridDim.x * 4;
    const int wid = (int)blockIdx.x * 4 + wave;
    // LDS: activation (Q8_K, M = 1) | per-wave header tables [4 waves][NM][G][nsb] x 16 B
    const int abytes = K + nsb * 4 + (K / 16) * 2;
    const int8_t *aqs = (const int8_t *)lds;
    const float *ad = (const float *)(lds + K);
    const int16_t *abs = (const int16_t *)(lds + K + nsb * 4);
    uint4 *stab = (uint4 *)(lds + ((abytes + 15) & ~15)) + (size_t)wave * NM * G * nsb;
    uint32_t *dtab = (uint32_t *)((uint4 *)(lds + ((abytes + 15) & ~15)) + (size_t)4 * NM * G * nsb) +
                     (size_t)wave * NM * G * nsb;

    auto tile_rows = [&](int t, int &seg, int &row0) {  // all G rows of a tile share a segment
        const int r = t * G;
        seg = r < N0 ? 0 : (r < N0 + N1 ? 1 : 2);
        row0 = seg == 0 ? r : (seg == 1 ? r - N0 : r - N0 - N1);
    };
    uint4 wq[NM][NI];
    auto issue = [&](int t) {
        int seg, row0;
        tile_rows(t, seg, row0);
        const uint8_t *W = seg == 0 ? a.W[0] : (seg == 1 ? a.W[1] : a.W[2]);
        const uint8_t *base0 = W + (int64_t)(row0 + gi) * RB;
        const uint8_t *base1 = MODE == 1 ? a.W2 + (int64_t)(row0 + gi) * RB : base0;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const uint32_t c = (uint32_t)min(l + LPR * i, NC - 1);
            wq[0][i] = ld_nt(base0 + 16u * c);
            if constexpr (NM == 2) wq[1][i] = ld_nt(base1 + 16u * c);
        }
    };

    // prologue: activation loads, first tile's weights, activation quantization
    const int t0 = wid < ntiles ? wid : ntiles - 1;
    if constexpr (PRO != 0) {
        ActPro<PRO, MC> pro;
        pro.load(a);
        issue(t0);
        pro.compute(a, lds);
    } else {
        uint4 r[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = min(((int)threadIdx.x + 256 * i) * 16, abytes - 16);
            r[i] = *(const uint4 *)(a.act + o);
        }
        issue(t0);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int o = ((int)threadIdx.x + 256 * i) * 16;
            if (o < abytes) *(uint4 *)(lds + o) = r[i];
        }
        __syncthreads();
    }

    float slot = 0.0f;
    int slot_t = -1;
    int k = 0;
    for (int t = wid; t < ntiles; t += nw, ++k) {
        if (k > 0) issue(t);
        // the per-chunk index math depends only on (lane, i): kept opaque per tile so the compiler
        // recomputes it instead of hoisting NI sets of indices out of the loop (VGPR pressure)
        int lx = l;
        asm volatile("" : "+v"(lx));
        // 1. park the header chunks of this tile
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = lx + LPR * i;
            if (c < NC && c % 9 == 0) {
#pragma unroll
                for (int m = 0; m < NM; ++m) {
                    stab[(m * G + gi) * nsb + c / 9] = q4k_decode_scales(wq[m][i]);
                    dtab[(m * G + gi) * nsb + c / 9] = wq[m][i].x;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // 2. nibble chunks
        float acc[NM];
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m] = 0.0f;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = lx + LPR * i;
            const int cc = min(c, NC - 1);
            const int sb = cc / 9, kr = cc - 9 * sb, kk = max(kr, 1);
            const bool valid = c < NC && kr != 0;          // branch-free: invalid chunks weigh 0
            const int j = (kk - 1) >> 1;
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const int ti = (m * G + gi) * nsb + sb;
                const uint32_t scw = ((const uint32_t *)(stab + ti))[j];
                const float p = q4k_chunk_dot(wq[m][i], dtab[ti], scw, sb, kk, aqs, ad, abs);
                acc[m] += valid ? p : 0.0f;
            }
            // one chunk at a time: hoisting all NI chunks' LDS reads would multiply live VGPRs
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m] = row_sum<LPR>(acc[m]);
        float v;
        if constexpr (MODE == 1) v = (acc[0] / (1.0f + expf(-acc[0]))) * acc[1];
        else v = acc[0];
        const bool mine = l == k;
        slot = mine ? v : slot;
        slot_t = mine ? t : slot_t;
        __builtin_amdgcn_wave_barrier();              // header table reuse by the next tile
    }
    // store (row = tile row gi of tile slot_t)
    if constexpr (MODE == 2) {
        // RoPE pairs are rows (2i, 2i+1) = adjacent row groups (G even); all lanes join the exchange
        const float other = __shfl_xor(slot, LPR, 64);
        if (slot_t >= 0) {
            int seg, row0;
            tile_rows(slot_t, seg, row0);
            const int row = row0 + gi;
            const int role = seg == 0 ? a.role[0] : (seg == 1 ? a.role[1] : a.role[2]);
            const int p = a.pos[0];
            if (role == 2) {
                a.vc[(int64_t)p * a.ekv + row] = f2h(slot);
            } else {
                const float2 cs = a.rope_tab[(int64_t)p * (a.D / 2) + (row % a.D) / 2];
                const bool odd = row & 1;
                const float x0 = odd ? other : slot, x1 = odd ? slot : other;
                const float o = odd ? __fadd_rn(__fmul_rn(x0, cs.y), __fmul_rn(x1, cs.x))
                                    : __fsub_rn(__fmul_rn(x0, cs.x), __fmul_rn(x1, cs.y));
                if (role == 0) a.q16[row] = f2h(o);
                else a.kc[(int64_t)p * a.ekv + row] = f2h(o);
            }
        }
    } else {
        if (slot_t >= 0) {
            int seg, row0;
            tile_rows(slot_t, seg, row0);
            const int row = row0 + gi;
            float *Y = seg == 0 ? a.Y[0] : (seg == 1 ? a.Y[1] : a.Y[2]);
            Y[row] = (MODE == 0 && a.res) ? __fadd_rn(slot, a.res[row]) : slot;
        }
    }
}

namespace {

template <int LPR, int NI, int MODE, int PRO, int MC>
int launch_stream(const DecArgs &a, hipStream_t s) {
    constexpr int G = 64 / LPR;
    const int64_t K = a.K, nsb = K / 256;
    int64_t ntot = 0;
    for (int i = 0; i < a.nseg; ++i) {
        if (a.N[i] % G) return -5;
        ntot += a.N[i];
    }
    const int64_t tiles = ntot / G;
    int64_t nblk = std::min<int64_t>((tiles + 3) / 4, 1024);
    nblk = std::max<int64_t>(nblk, (tiles + 4 * LPR - 1) / (4 * LPR));   // <= LPR tiles per wave (slots)
    const int64_t abytes = K + nsb * 4 + (K / 16) * 2;
    const size_t lds = (size_t)((abytes + 15) & ~15) + (size_t)4 * (MODE == 1 ? 2 : 1) * G * nsb * (16 + 4);
    hipLaunchKernelGGL((k_gemv_stream<LPR, NI, MODE, PRO, MC>), dim3((unsigned)nblk), dim3(256), lds, s, a);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace

// Returns -3 when the shape/type is not covered (the caller falls back to kcpp_gemv_dec).
extern "C" int kcpp_gemv_stream(int type, const void *args, int mode, int pro, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    if (type != KT_Q4_K || a.K % 256 || a.nseg < 1 || a.nseg > 3 || a.eid) return -3;
    // measured (tools/stream_probe.py): only the K = 14336 quantize-prologue shape (ffn_down in the kcpp Q4_K
    // layout) beats the unit-per-lane kernel (20.3 vs 24.6 us); at K = 4096 it loses on VALU work per byte
    if (a.K == 14336 && mode == 0 && pro == 2) return launch_stream<64, 8, 0, 2, 4>(a, s);   // one row per wave
    return -3;
}
