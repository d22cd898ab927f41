// tools/queue_probe.hip — which HIP streams share an in-order hardware queue with a given one
// (not shipped). A bounded ~300 ms kernel (one wave spinning on its own clock) runs
// on stream 0; then a short kernel is launched on each other stream in turn, and whether it
// finishes while the long one still runs tells whether the two streams sit on different hardware
// queues (an in-order queue runs its packets one after another). Streams: 8 ordinary non-blocking
// ones (HIP pools a process's streams onto GPU_MAX_HW_QUEUES queues), then non-blocking streams at
// the greatest and least priority, then a full-CU-mask stream; then, within each priority's own
// pool of 8 streams, which share the pool's first stream's queue.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/queue_probe.hip -o tools/bin/queue_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
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

__global__ void k_busy(long long cycles, int *flag) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) flag[0] = 1;
}

using clk = std::chrono::steady_clock;

int main() {
    CK(hipSetDevice(0));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    int *flag = nullptr;
    CK(hipMalloc(&flag, 2 * sizeof(int)));
    std::vector<std::pair<std::string, hipStream_t>> s;
    for (int i = 0; i < 8; ++i) {
        hipStream_t x;
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        s.push_back({"pooled_" + std::to_string(i), x});
    }
    std::vector<hipStream_t> hi, lo;  // the priority pools' own sizes: 8 streams each (second pass)
    for (int i = 0; i < 8; ++i) {
        hipStream_t x;
        CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, greatest));
        if (i < 2) s.push_back({"greatest_priority_" + std::to_string(i), x});
        hi.push_back(x);
    }
    for (int i = 0; i < 8; ++i) {
        hipStream_t x;
        CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, least));
        if (i < 2) s.push_back({"least_priority_" + std::to_string(i), x});
        lo.push_back(x);
    }
    {
        int ncu = 0;
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
        hipStream_t x;
        CK(hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data()));
        s.push_back({"full_cu_mask", x});
    }
    long long cycles = 100000000;
    {
        const clk::time_point t0 = clk::now();
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s[0].second, cycles, flag);
        CK(hipStreamSynchronize(s[0].second));
        cycles = (long long)(cycles * (0.3 / std::chrono::duration<double>(clk::now() - t0).count()));
    }
    std::printf("{\"priority_range\": {\"least\": %d, \"greatest\": %d}}\n", least, greatest);
    for (size_t i = 1; i < s.size(); ++i) {
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s[0].second, cycles, flag);  // ~300 ms on stream 0
        const clk::time_point t0 = clk::now();
        while (std::chrono::duration<double>(clk::now() - t0).count() < 0.02) {
        }
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s[i].second, 1000LL, flag + 1);  // short
        const clk::time_point t1 = clk::now();
        CK(hipStreamSynchronize(s[i].second));
        const double short_ms = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
        CK(hipStreamSynchronize(s[0].second));
        std::printf("{\"stream\": \"%s\", \"short_kernel_ms\": %.3f, \"shares_queue_with_pooled_0\": %s}\n",
                    s[i].first.c_str(), short_ms, short_ms > 150.0 ? "true" : "false");
        std::fflush(stdout);
    }
    // second pass: within each priority pool, which streams share the pool's first stream's queue
    for (auto *pool : {&hi, &lo}) {
        const char *name = pool == &hi ? "greatest" : "least";
        for (size_t i = 1; i < pool->size(); ++i) {
            hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, (*pool)[0], cycles, flag);
            const clk::time_point t0 = clk::now();
            while (std::chrono::duration<double>(clk::now() - t0).count() < 0.02) {
            }
            hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, (*pool)[i], 1000LL, flag + 1);
            const clk::time_point t1 = clk::now();
            CK(hipStreamSynchronize((*pool)[i]));
            const double short_ms = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
            CK(hipStreamSynchronize((*pool)[0]));
            std::printf("{\"pool\": \"%s\", \"stream\": %zu, \"short_kernel_ms\": %.3f, \"shares_queue_with_pool_0\": %s}\n",
                        name, i, short_ms, short_ms > 150.0 ? "true" : "false");
            std::fflush(stdout);
        }
    }
    CK(hipFree(flag));
    return 0;
}
