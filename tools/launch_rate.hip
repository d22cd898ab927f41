// tools/launch_rate.hip — host cadence of back-to-back launches (not shipped): how much of the
// N=1 sweep's small-bucket time is the HIP launch itself, how much the engine's C-ABI entry,
// and how much the Python / ctypes loop of bench.py (measured there).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_rate.hip -o tools/bin/launch_rate \
//       -Iinclude -Lexperiment-distributed-deep-learning_amd/lib -lddl_amd \
//       -Wl,-rpath,$PWD/experiment-distributed-deep-learning_amd/lib
//   ./launch_rate
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "ddl_amd_testing.h"

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e = (x);                                                                           \
        if (e != hipSuccess) {                                                                        \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                             \
        }                                                                                             \
    } while (0)

__global__ void k_empty(float *p) {
    if (p && threadIdx.x == 1000000) p[0] = 0.f;  // never true: keeps the argument live
}

int main() {
    const int N = 20000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *a = nullptr, *b = nullptr;
    CK(hipMalloc(&a, 64 << 20));
    CK(hipMalloc(&b, 64 << 20));
    CK(hipMemset(a, 0, 64 << 20));
    CK(hipMemset(b, 0, 64 << 20));
    using clk = std::chrono::steady_clock;
    auto per_call_us = [&](auto &&fn) {
        for (int i = 0; i < 200; ++i) fn();
        CK(hipStreamSynchronize(s));
        const auto t0 = clk::now();
        for (int i = 0; i < N; ++i) fn();
        const auto t1 = clk::now();  // host cadence: enqueue only
        CK(hipStreamSynchronize(s));
        const auto t2 = clk::now();
        return std::make_pair(std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                              std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
    };
    auto e = per_call_us([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, a); });
    std::printf("empty kernel, 1 workgroup:            host %.2f us/launch, with device %.2f us\n", e.first, e.second);
    auto e2 = per_call_us([&] { hipLaunchKernelGGL(k_empty, dim3(8), dim3(128), 0, s, a); });
    std::printf("empty kernel, 8 workgroups x 128:     host %.2f us/launch, with device %.2f us\n", e2.first, e2.second);
    for (size_t bytes : {(size_t)4096, (size_t)65536, (size_t)1 << 20, (size_t)4 << 20}) {
        auto r = per_call_us([&] {
            if (ddl_reduce_local(a, b, bytes / 4, DDL_FLOAT, s) != 0) std::exit(2);
        });
        std::printf("ddl_reduce_local %8zu B (C-ABI):   host %.2f us/call,   with device %.2f us\n", bytes, r.first,
                    r.second);
    }
    return 0;
}
