// launch_probe.hip -- per-launch cost of dependent kernels replayed from a hipGraph (tools only).
// Chains of N launches of: empty 1-WG kernel, empty 256-WG kernel, 256-WG kernel with a 256-B by-value
// argument struct (like DecArgs), and a 256-WG kernel that loads one dword from the previous kernel's output.
// Prints wall time per launch (HIP events around graph replays).
// build: hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorName(e_), __LINE__); exit(1); } \
    } while (0)

struct Big { long long v[32]; };

__global__ void k_empty(int *p) { if (p && threadIdx.x == 1023) p[0] = 1; }
__global__ void k_big(Big b, int *p) { if (threadIdx.x == 1023) p[0] = (int)b.v[31]; }
template <int NB> struct Arg { long long v[NB / 8]; };
// a 256-WG kernel reading its first and last argument words (the kernarg size sweep: DecArgs is 296 B)
template <int NB>
__global__ void k_arg(Arg<NB> b, int *p) {
    if (threadIdx.x == 1023) p[0] = (int)(b.v[0] + b.v[NB / 8 - 1]);
}
__global__ void k_dep(const int *in, int *out) {
    const int v = in[blockIdx.x & 255];
    if (threadIdx.x == 0) out[blockIdx.x & 255] = v + 1;
}

template <typename F>
static double time_chain(const char *name, int n, hipStream_t s, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) launch(i);
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
    const double us = ms * 1e3 / R / n;
    printf("{\"chain\": \"%s\", \"n\": %d, \"us_per_launch\": %.3f}\n", name, n, us);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return us;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *buf;
    CK(hipMalloc(&buf, 1 << 20));
    CK(hipMemset(buf, 0, 1 << 20));
    Big big{};
    for (int n : {64, 256}) {
        time_chain("empty_1wg_64thr", n, s, [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, buf); });
        time_chain("empty_256wg_256thr", n, s, [&](int) { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, buf); });
        time_chain("empty_1024wg_256thr", n, s, [&](int) { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, buf); });
        time_chain("bigarg_256wg_256thr", n, s, [&](int) { hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, buf); });
        time_chain("dep_256wg_256thr", n, s, [&](int i) {
            hipLaunchKernelGGL(k_dep, dim3(256), dim3(256), 0, s, buf + (i & 1) * 4096, buf + ((i + 1) & 1) * 4096);
        });
    }
    // kernarg size sweep, 256-launch chains
#define KA(NB) { Arg<NB> a{}; time_chain("arg" #NB, 256, s, [&](int) { hipLaunchKernelGGL(k_arg<NB>, dim3(256), dim3(256), 0, s, a, buf); }); }
    KA(16) KA(64) KA(128) KA(192) KA(248) KA(256) KA(264) KA(296) KA(320) KA(384) KA(512) KA(1024)
    KA(16) KA(296) KA(320)
#undef KA
    // eager (no graph) for comparison
    {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, buf);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, buf);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"chain\": \"eager_empty_256wg\", \"n\": 2000, \"us_per_launch\": %.3f}\n", ms * 1e3 / 2000);
    }
    return 0;
}
