// q80_pattern_probe.hip -- what HBM rate can a batch-32 Q8_0 GEMM reach when every wave streams its own 32-row tile
// straight into MFMA B-operand registers?  (tools only; BASELINE config 3 design probe)
// Weights [N][K] int8 (the SoA qs plane of KT_Q8_0), 8 copies rotated past the Infinity Cache.
//   P0 "frag": lane l reads row (l % 32), bytes 32 b + 16 (l / 32) of block b -- the v_mfma_i32_32x32x32_i8 B operand
//              straight from the ggml-order rows: one wave instruction = 32 rows x 32 B (32 cache lines, each line
//              read by 4 consecutive block instructions)
//   P1 "contig": the same bytes as if stored fragment-major (1 KiB contiguous per wave instruction)
// Each block: one i8 MFMA against a register A operand and a 16-value f32 epilogue (the real kernel's work).
// build: hipcc --offload-arch=gfx950 -O3 tools/q80_pattern_probe.hip -o tools/q80_pattern_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                                 \
    do {                                                                                                      \
        hipError_t e_ = (x);                                                                                  \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(1); }     \
    } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 ldw(const uint8_t *p) {
    const v4u x = __builtin_nontemporal_load((const v4u *)p);
    return i32x4{(int)x[0], (int)x[1], (int)x[2], (int)x[3]};
}

// grid (N / 32 / W, S), W waves: wave w owns tile 4 blockIdx.x + w, blocks [b0, b1) of its K split; U blocks per
// batch, two batches in flight
template <int P, int U, int W>
__global__ void __launch_bounds__(64 * W) k_probe(const uint8_t *__restrict__ qs, int64_t K, int64_t N, float *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nb = K / 32, S = gridDim.y;
    const int64_t tile = (int64_t)blockIdx.x * W + wave;
    const int64_t bps = nb / S, b0 = blockIdx.y * bps, b1 = b0 + bps;
    const uint8_t *base;
    int64_t step;                      // bytes between consecutive blocks of this lane
    if (P == 0) { base = qs + (tile * 32 + (lane & 31)) * K + 16 * (lane >> 5); step = 32; }
    else { base = qs + tile * 32 * K + lane * 16; step = 1024; }
    const i32x4 a = {lane, 3 * lane, 5, 7};
    float tot[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) tot[r] = 0.0f;
    i32x4 wa[U], wb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw(base + (b0 + u) * step);
    for (int64_t b = b0; b < b1; b += 2 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) wb[u] = ldw(base + (b + U + u < b1 ? b + U + u : b1 - 1) * step);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            i32x16 acc = {};
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, wa[u], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) tot[r] = __fadd_rn(tot[r], __fmul_rn((float)acc[r], 0.001f * (float)(u + 1)));
        }
        if (b + U >= b1) break;
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = ldw(base + (b + 2 * U + u < b1 ? b + 2 * U + u : b1 - 1) * step);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            i32x16 acc = {};
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, wb[u], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) tot[r] = __fadd_rn(tot[r], __fmul_rn((float)acc[r], 0.001f * (float)(u + 1)));
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += tot[r];
    if (s == 1234.5f) out[tile] = s;
}

template <int P, int U, int W>
static void run(const char *name, uint8_t **bufs, int nbuf, int64_t K, int64_t N, int S, float *out) {
    const dim3 grid((unsigned)(N / 32 / W), (unsigned)S);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < nbuf; ++i) hipLaunchKernelGGL((k_probe<P, U, W>), grid, dim3(64 * W), 0, 0, bufs[i], K, N, out);
    CK(hipDeviceSynchronize());
    const int it = 64;
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_probe<P, U, W>), grid, dim3(64 * W), 0, 0, bufs[i % nbuf], K, N, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / it, bytes = (double)K * N;
    printf("%-8s U=%d W=%d S=%-2d K=%-6lld N=%-6lld wgs=%-5d %8.2f us  %7.1f GB/s\n", name, U, W, S, (long long)K,
           (long long)N, (int)(grid.x * grid.y), us, bytes / us * 1e-3);
}

int main() {
    const int nbuf = 8;
    uint8_t *bufs[nbuf];
    float *out;
    const int64_t maxb = 14336LL * 4096;
    for (int i = 0; i < nbuf; ++i) { CK(hipMalloc(&bufs[i], maxb)); CK(hipMemset(bufs[i], i + 1, maxb)); }
    CK(hipMalloc(&out, 1 << 20));
    struct Shape { int64_t K, N; } shapes[] = {{4096, 14336}, {14336, 4096}, {4096, 4096}, {4096, 6144}};
    for (auto sh : shapes) {
        for (int S : {1, 2, 4, 8}) {
            if ((sh.K / 32) % S) continue;
            run<0, 8, 4>("frag", bufs, nbuf, sh.K, sh.N, S, out);
            run<1, 8, 4>("contig", bufs, nbuf, sh.K, sh.N, S, out);
        }
        run<0, 4, 4>("frag", bufs, nbuf, sh.K, sh.N, 4, out);
        run<0, 16, 4>("frag", bufs, nbuf, sh.K, sh.N, 2, out);
        run<0, 8, 8>("frag", bufs, nbuf, sh.K, sh.N, 4, out);
    }
    return 0;
}
