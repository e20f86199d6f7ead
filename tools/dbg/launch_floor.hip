// launch_floor: per-call latency floor of the pieces a per-frame decode call
// is made of, on one MI355X (kernel enqueue, stream sync, mapped-memory flag
// wait, dependent reads of mapped host memory).  Diagnostic only.
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/dbg/launch_floor tools/dbg/launch_floor.hip
// Run:   tools/dbg/launch_floor [spin]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                          \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) {                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
            return 1;                                                                                  \
        }                                                                                              \
    } while (0)

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1000) p[0] = 1;
}
// completion flag in mapped host memory, written after a system-scope fence
__global__ void k_flag(unsigned *flag, unsigned v) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// n dependent reads of mapped host memory (a pointer chase over 4 slots)
__global__ void k_chase(const unsigned *h, int n, unsigned *out) {
    unsigned i = 0;
    for (int k = 0; k < n; k++) i = __hip_atomic_load(h + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 0) out[0] = i;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *hflag, *dflag, *hch, *dch, *dout;
    CK(hipHostMalloc((void **)&hflag, 64));
    CK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
    CK(hipHostMalloc((void **)&hch, 64));
    CK(hipHostGetDevicePointer((void **)&dch, hch, 0));
    hch[0] = 1; hch[1] = 2; hch[2] = 3; hch[3] = 0;
    CK(hipMalloc((void **)&dout, 64));
    const int N = 2000;
    std::vector<double> t;
    auto report = [&](const char *name) { printf("%-44s median %7.2f us\n", name, med(t)); t.clear(); };
    for (int w = 0; w < 200; w++) hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
    CK(hipStreamSynchronize(s));

    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        CK(hipStreamSynchronize(s));
        t.push_back(us(a, clk::now()));
    }
    report("sync of an idle stream");
    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        t.push_back(us(a, clk::now()));
        CK(hipStreamSynchronize(s));
    }
    report("enqueue of one kernel (host side)");
    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        CK(hipStreamSynchronize(s));
        t.push_back(us(a, clk::now()));
    }
    report("1 empty kernel + stream sync");
    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        for (int k = 0; k < 3; k++) hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        CK(hipStreamSynchronize(s));
        t.push_back(us(a, clk::now()));
    }
    report("3 empty kernels + stream sync");
    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_flag, 1, 256, 0, s, dflag, (unsigned)(i + 1));
        while (__atomic_load_n((volatile unsigned *)hflag, __ATOMIC_ACQUIRE) != (unsigned)(i + 1)) {
        }
        t.push_back(us(a, clk::now()));
    }
    CK(hipStreamSynchronize(s));
    report("1 flag kernel + host spin on mapped flag");
    for (int i = 0; i < N; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        hipLaunchKernelGGL(k_flag, 1, 256, 0, s, dflag, (unsigned)(N + i + 1));
        while (__atomic_load_n((volatile unsigned *)hflag, __ATOMIC_ACQUIRE) != (unsigned)(N + i + 1)) {
        }
        t.push_back(us(a, clk::now()));
    }
    CK(hipStreamSynchronize(s));
    report("2 empty + 1 flag kernel + host spin");
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < 3; k++) hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < N; i++) {
            auto a = clk::now();
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            t.push_back(us(a, clk::now()));
        }
        report("graph of 3 empty kernels + stream sync");
    }
    for (int n : {1, 10}) {
        for (int i = 0; i < 400; i++) {
            auto a = clk::now();
            hipLaunchKernelGGL(k_chase, 1, 64, 0, s, (const unsigned *)dch, n, dout);
            CK(hipStreamSynchronize(s));
            t.push_back(us(a, clk::now()));
        }
        char name[64];
        snprintf(name, sizeof name, "chase %d mapped host reads + sync", n);
        report(name);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int n : {1, 10}) {
        for (int i = 0; i < 200; i++) {
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_chase, 1, 64, 0, s, (const unsigned *)dch, n, dout);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1000.0);
        }
        char name[64];
        snprintf(name, sizeof name, "chase %d mapped host reads (events)", n);
        report(name);
    }
    return 0;
}
