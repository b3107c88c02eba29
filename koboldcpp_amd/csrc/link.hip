// link.hip -- the single-token stage hand-off of the layer-split pipeline, done by the stages' own kernels.
//
// The reference moves a split's input between backends with an async peer copy ordered by events
// (ggml_backend_cuda_cpy_tensor_async + cudaEventRecord / cudaStreamWaitEvent, ggml-cuda.cu:2392-2445, driven by
// ggml_backend_sched_compute_splits, ggml-backend.cpp:2108-2201).  On MI355X that costs ~70 us per boundary on one
// GPU (tools/handoff_trace.py): an event wait is resolved by the command processor of the waiting queue, ~20 us
// after the producer's last kernel, then a blit kernel and another dispatch gap.  Here each stage's single-token
// graph is bracketed by two one-workgroup kernels instead, and no host call or event sits between stages:
//
//   k_link_wait    (first node): step = ++stepctr; poll ready_in >= step - in_lag and copied_out >= step - out_lag
//                  (the consumer has pulled this stage's previous output, so it may be overwritten); acquire; pull
//                  the producer's residual row (x of stage s-1, n floats, peer memory on another GPU) -- or, on
//                  stage 0, the last stage's greedy token -- into this stage's input; report copied = step to the
//                  producer.
//   k_link_publish (last node): ready_out = step (the consumer's ready_in); the stage's results were written back
//                  by the end of its previous kernel.
//
// Every wait is on a word that an EARLIER enqueued kernel sets (the host enqueues stages in pipeline order), so
// in-order queues never hold a waiter in front of what it waits for.  Flags are polled with system-scope relaxed
// loads (cross-device words over xGMI) with s_sleep between polls, by one lane; the flag blocks are fine-grained
// device memory (expose.cpp init_links), so a peer's stores are seen without waiting for a kernel boundary.  A wait
// gives up after ~2 s (LINK_POLL_MAX polls), sets the stage's error word and lets the step run: a lost flag then
// costs a wrong step the host reports (expose.cpp link_errors), never a GPU that spins forever.
#include "kcpp_common.h"
#include "kcpp_internal.h"

#define LINK_POLL_MAX (1u << 24)     // x s_sleep(2) (~128 clocks): ~1-2 s

__global__ void __launch_bounds__(256) k_link_wait(const KLink L) {
    __shared__ unsigned s_step;
    const int tid = threadIdx.x;
    if (tid == 0) {
        const unsigned step = __hip_atomic_load(L.stepctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        __hip_atomic_store(L.stepctr, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned polls = 0;
        while (__hip_atomic_load(L.ready_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + (unsigned)L.in_lag < step &&
               ++polls < LINK_POLL_MAX)
            __builtin_amdgcn_s_sleep(2);
        while (__hip_atomic_load(L.copied_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + (unsigned)L.out_lag < step &&
               ++polls < LINK_POLL_MAX)
            __builtin_amdgcn_s_sleep(2);
        if (polls >= LINK_POLL_MAX && L.err) __hip_atomic_store(L.err, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        s_step = step;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (L.src_x) {           // all of a thread's loads in flight before its stores (one round trip per 32 KB)
        const float4 *src = (const float4 *)L.src_x;
        float4 *dst = (float4 *)L.dst_x;
        const int n4 = L.n / 4;
        for (int i0 = 0; i0 < n4; i0 += 8 * 256) {
            float4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + tid + 256 * k;
                if (i < n4) v[k] = src[i];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + tid + 256 * k;
                if (i < n4) dst[i] = v[k];
            }
        }
    }
    if (L.src_tok && tid == 0) *L.dst_tok = *L.src_tok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(L.copied_report, s_step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) k_link_publish(const KLink L) {
    if (threadIdx.x == 0) {
        const unsigned step = __hip_atomic_load(L.stepctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(L.ready_out, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int kcpp_link_wait(const KLink &L, hipStream_t s) {
    if (!L.stepctr || !L.ready_in || !L.copied_out || !L.copied_report || (L.src_x && (!L.dst_x || L.n % 4)) ||
        (L.src_tok && !L.dst_tok))
        return -1;
    hipLaunchKernelGGL(k_link_wait, dim3(1), dim3(256), 0, s, L);
    KCPP_CHECK(hipGetLastError());
    return 0;
}

int kcpp_link_publish(const KLink &L, hipStream_t s) {
    if (!L.stepctr || !L.ready_out) return -1;
    hipLaunchKernelGGL(k_link_publish, dim3(1), dim3(64), 0, s, L);
    KCPP_CHECK(hipGetLastError());
    return 0;
}
