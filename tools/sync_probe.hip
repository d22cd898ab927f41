// tools/sync_probe.hip — which HIP host calls wait for device work they are not ordered after
// (not shipped). A kernel that runs ~400 ms (a bounded clock64 loop on one wave) is
// launched on stream A; then, from the host, each call below runs on unrelated memory / another
// stream and is timed. A call that returns in microseconds does not synchronise the device; one
// that takes ~400 ms waited for the kernel — on a thread that posts RCCL work while another
// communicator's RCCL kernels are in flight, such a call can deadlock the ranks (r06 s6).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sync_probe.hip -o tools/bin/sync_probe
//   ./tools/bin/sync_probe          (one JSON line per call)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e = (x);                                                                           \
        if (e != hipSuccess) {                                                                        \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                             \
        }                                                                                             \
    } while (0)

// one wave spins on its own clock for `cycles` (bounded: every launch ends), then writes a flag
__global__ void k_busy(long long cycles, int *flag) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) flag[0] = 1;
}

using clk = std::chrono::steady_clock;

int main() {
    CK(hipSetDevice(0));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    int *flag = nullptr;
    CK(hipMalloc(&flag, sizeof(int)));
    // calibrate: the clock64 rate, from a short run
    long long cycles = 100000000;  // 100 M cycles
    {
        const clk::time_point t0 = clk::now();
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, a, cycles, flag);
        CK(hipStreamSynchronize(a));
        const double s = std::chrono::duration<double>(clk::now() - t0).count();
        cycles = (long long)(cycles * (0.4 / s));  // ~400 ms
    }
    const size_t big = 64 << 20;
    std::vector<std::pair<std::string, std::function<void()>>> calls;
    void *d = nullptr, *h = nullptr;
    char *reg = static_cast<char *>(std::aligned_alloc(4096, big));
    std::memset(reg, 0, big);
    calls.push_back({"hipMalloc", [&] { CK(hipMalloc(&d, big)); }});
    calls.push_back({"hipFree", [&] { CK(hipFree(d)); }});
    calls.push_back({"hipHostMalloc", [&] { CK(hipHostMalloc(&h, big, hipHostMallocDefault)); }});
    calls.push_back({"hipHostFree", [&] { CK(hipHostFree(h)); }});
    calls.push_back({"hipHostRegister", [&] { CK(hipHostRegister(reg, big, hipHostRegisterDefault)); }});
    calls.push_back({"hipHostUnregister", [&] { CK(hipHostUnregister(reg)); }});
    hipStream_t s2 = nullptr;
    calls.push_back({"hipStreamCreateWithFlags", [&] { CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking)); }});
    calls.push_back({"hipStreamDestroy(other stream)", [&] { CK(hipStreamDestroy(s2)); }});
    hipEvent_t ev = nullptr;
    calls.push_back({"hipEventCreate", [&] { CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming)); }});
    calls.push_back({"hipEventDestroy", [&] { CK(hipEventDestroy(ev)); }});
    void *d2 = nullptr;
    CK(hipMalloc(&d2, big));
    calls.push_back({"hipMemsetAsync(other stream)", [&] { CK(hipMemsetAsync(d2, 0, big, b)); CK(hipStreamSynchronize(b)); }});
    calls.push_back({"hipMallocAsync+hipFreeAsync(other stream)", [&] {
                         void *p = nullptr;
                         CK(hipMallocAsync(&p, big, b));
                         CK(hipFreeAsync(p, b));
                         CK(hipStreamSynchronize(b));
                     }});
    for (auto &c : calls) {
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, a, cycles, flag);
        CK(hipGetLastError());
        // let the kernel start
        const clk::time_point t_launch = clk::now();
        while (std::chrono::duration<double>(clk::now() - t_launch).count() < 0.02) {
        }
        const clk::time_point t0 = clk::now();
        c.second();
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        const bool kernel_done = hipStreamQuery(a) == hipSuccess;
        CK(hipStreamSynchronize(a));
        std::printf("{\"call\": \"%s\", \"ms\": %.3f, \"kernel_done_after\": %s, \"waited_for_kernel\": %s}\n",
                    c.first.c_str(), ms, kernel_done ? "true" : "false", ms > 200.0 ? "true" : "false");
        std::fflush(stdout);
    }
    CK(hipFree(d2));
    CK(hipFree(flag));
    std::free(reg);
    return 0;
}
