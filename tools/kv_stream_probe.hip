// kv_stream_probe.hip -- how fast can a decode step read one layer's f16 KV cache? (tools only)
// Llama-3-8B shapes: 8 kv heads x 128 dims, pos-major cache [pos][hk][D], 3851 positions = 15.8 MB (K+V).
// 32 layers' caches (548 MB, past the Infinity Cache) read by a hipGraph chain of 32 launches, one per layer,
// each launch only loading and summing (the minimal work of flash attention's streaming phase).
// Variants: grid / block shapes and access orders of the split-KV kernels.
// build: hipcc --offload-arch=gfx950 -O3 tools/kv_stream_probe.hip -o tools/kv_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(1); } \
    } while (0)

constexpr int HKV = 8, D = 128, NCTX = 4176, NKV = 3851, L = 32;
constexpr long long EKV = HKV * D;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4 *p) {
    const v4u x = __builtin_nontemporal_load((const v4u *)p);
    return make_uint4(x[0], x[1], x[2], x[3]);
}
__device__ __forceinline__ float f4(uint4 v) {
    return __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
}

// split-KV per kv head: grid (NS, HKV), W waves; 16 lanes per row, 4 rows per wave instruction; each wave
// owns 16 consecutive keys per step
template <int W, bool NT>
__global__ void __launch_bounds__(64 * W) k_head_split(const uint16_t *kc, const uint16_t *vc, float *out) {
    const int sp = blockIdx.x, NS = gridDim.x, hk = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15, kq = lane >> 4;
    const int per = (NKV + NS - 1) / NS;
    const int p0 = sp * per, p1 = min(p0 + per, NKV);
    float acc = 0.0f;
    for (int c0 = p0; c0 < p1; c0 += 16 * W) {
        uint4 k[4], v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = c0 + 16 * wave + 4 * i + kq;
            const uint4 *pk = (const uint4 *)(kc + p * EKV + hk * D + sub * 8);
            const uint4 *pv = (const uint4 *)(vc + p * EKV + hk * D + sub * 8);
            if (p < p1) {
                if (NT) { k[i] = ntl(pk); v[i] = ntl(pv); }
                else { k[i] = *pk; v[i] = *pv; }
            } else {
                k[i] = v[i] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += f4(k[i]) + f4(v[i]);
    }
    if (acc == 1234.5f) out[blockIdx.y * NS + sp] = acc;
}

// all kv heads of a position range per workgroup: the rows of consecutive positions are one contiguous
// run of 2 KB each (K) and (V); grid NB, 256 threads, lane = 16 B
template <bool NT>
__global__ void __launch_bounds__(256) k_pos_split(const uint16_t *kc, const uint16_t *vc, float *out) {
    const int b = blockIdx.x, NB = gridDim.x;
    const int per = (NKV + NB - 1) / NB;
    const int p0 = b * per, p1 = min(p0 + per, NKV);
    const long long e0 = (long long)p0 * EKV / 8, e1 = (long long)p1 * EKV / 8;   // uint4 units
    const uint4 *K = (const uint4 *)kc, *V = (const uint4 *)vc;
    float acc = 0.0f;
    for (long long e = e0 + threadIdx.x; e < e1; e += 256 * 4) {
        uint4 k[4], v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const long long x = e + 256 * i;
            if (x < e1) {
                if (NT) { k[i] = ntl(K + x); v[i] = ntl(V + x); }
                else { k[i] = K[x]; v[i] = V[x]; }
            } else {
                k[i] = v[i] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += f4(k[i]) + f4(v[i]);
    }
    if (acc == 1234.5f) out[b] = acc;
}

template <typename F>
static void time_chain(const char *name, hipStream_t s, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 0; l < L; ++l) launch(l);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    const int R = 20;
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / R / L;
    const double bytes = 2.0 * NKV * EKV * 2;
    printf("{\"variant\": \"%s\", \"us_per_layer\": %.3f, \"GBps\": %.0f}\n", name, us, bytes / us / 1e3);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t per_layer = (size_t)NCTX * EKV * 2;
    uint16_t *kc, *vc;
    float *out;
    CK(hipMalloc(&kc, per_layer * L));
    CK(hipMalloc(&vc, per_layer * L));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(kc, 0x11, per_layer * L));
    CK(hipMemset(vc, 0x22, per_layer * L));
    auto K = [&](int l) { return kc + (size_t)l * per_layer / 2; };
    auto V = [&](int l) { return vc + (size_t)l * per_layer / 2; };
    time_chain("head_split ns32 w8", s, [&](int l) { hipLaunchKernelGGL((k_head_split<8, false>), dim3(32, HKV), dim3(512), 0, s, K(l), V(l), out); });
    time_chain("head_split ns32 w8 nt", s, [&](int l) { hipLaunchKernelGGL((k_head_split<8, true>), dim3(32, HKV), dim3(512), 0, s, K(l), V(l), out); });
    time_chain("head_split ns32 w4", s, [&](int l) { hipLaunchKernelGGL((k_head_split<4, false>), dim3(32, HKV), dim3(256), 0, s, K(l), V(l), out); });
    time_chain("head_split ns64 w4", s, [&](int l) { hipLaunchKernelGGL((k_head_split<4, false>), dim3(64, HKV), dim3(256), 0, s, K(l), V(l), out); });
    time_chain("head_split ns64 w2", s, [&](int l) { hipLaunchKernelGGL((k_head_split<2, false>), dim3(64, HKV), dim3(128), 0, s, K(l), V(l), out); });
    time_chain("head_split ns128 w2", s, [&](int l) { hipLaunchKernelGGL((k_head_split<2, false>), dim3(128, HKV), dim3(128), 0, s, K(l), V(l), out); });
    time_chain("head_split ns16 w8", s, [&](int l) { hipLaunchKernelGGL((k_head_split<8, false>), dim3(16, HKV), dim3(512), 0, s, K(l), V(l), out); });
    for (int nb : {128, 256, 512, 1024}) {
        char nm[64];
        snprintf(nm, sizeof nm, "pos_split nb%d", nb);
        time_chain(nm, s, [&](int l) { hipLaunchKernelGGL((k_pos_split<false>), dim3(nb), dim3(256), 0, s, K(l), V(l), out); });
        snprintf(nm, sizeof nm, "pos_split nb%d nt", nb);
        time_chain(nm, s, [&](int l) { hipLaunchKernelGGL((k_pos_split<true>), dim3(nb), dim3(256), 0, s, K(l), V(l), out); });
    }
    return 0;
}
