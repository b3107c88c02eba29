// handoff_probe.hip -- the decode engine's edge primitive alone (dec_engine.hip arrive / poll): 256 workgroups of 512
// threads, the control wave (7) of every workgroup arrives on an 8-way sharded counter and polls the sum, `rounds`
// times (one all-to-all edge per round); prints whether every edge completed and the time per edge.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/handoff_probe tools/handoff_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ void arrive(unsigned *c, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int poll(const unsigned *c0, int n, unsigned target, int lane) {
    for (unsigned it = 0; it < (1u << 20); ++it) {
        unsigned v = lane < n ? __hip_atomic_load(c0 + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        v = __builtin_amdgcn_readfirstlane(v);
        if ((int)(v - target) >= 0) return 0;
        __builtin_amdgcn_s_sleep(1);
    }
    return 1;
}
__global__ void __launch_bounds__(512, 1) k(unsigned *c, unsigned *err, int rounds, int mode) {
    extern __shared__ unsigned char lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, b = blockIdx.x;
    for (int r = 0; r < rounds; ++r) {
        if (wave == 7) {
            if (mode == 0) {          // all-to-all: every workgroup arrives on shard b % 8, waits for all of them
                arrive(c + (r * 8 + (b & 7)) * 32, lane);
                if (poll(c + r * 8 * 32, 8, gridDim.x, lane) && lane == 0) atomicAdd(err, 1u);
            } else {                  // 32 -> 32: one counter per group b % 8
                arrive(c + (r * 8 + (b & 7)) * 32, lane);
                if (poll(c + (r * 8 + (b & 7)) * 32, 1, gridDim.x / 8, lane) && lane == 0) atomicAdd(err, 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) lds[0] = (unsigned char)r;
    }
}
int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int rounds = 200;
    unsigned *c, *err;
    hipMalloc(&c, rounds * 8 * 128);
    hipMalloc(&err, 4);
    hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 132 * 1024);
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(c, 0, rounds * 8 * 128);
            hipMemset(err, 0, 4);
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(ncu), dim3(512), 132 * 1024, 0, c, err, rounds, mode);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned e = 0;
            hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
            std::vector<unsigned> h(rounds * 8 * 32);
            hipMemcpy(h.data(), c, h.size() * 4, hipMemcpyDeviceToHost);
            unsigned s0 = 0;
            for (int i = 0; i < 8; ++i) s0 += h[i * 32];
            printf("mode %d ncu %d: timeouts %u, round-0 sum %u, %.2f us per edge (%s)\n", mode, ncu, e, s0,
                   ms * 1e3 / rounds, hipGetErrorString(hipGetLastError()));
        }
    }
    return 0;
}
