// tools/lane_copy_probe.hip — the keyed host path's unpack lane in isolation (not shipped;
// VERDICT r5 next #4): per pinned-slot allocation kind, the D2H DMA rate into a
// 32 MiB slot, and the host memcpy rate from that slot into a warm pageable destination with
// 1..16 threads — the two phases the engine's lane job runs per staged chunk (handler.cpp
// unpack_async: wait for the D2H event, then CopyPool::run of the chunk's pieces). Each copy
// reads a slot right after the DMA wrote it, as the lane does.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread tools/lane_copy_probe.hip -o tools/bin/lane_copy_probe
//   ./tools/bin/lane_copy_probe            (one JSON line per (kind, threads))
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e = (x);                                                                           \
        if (e != hipSuccess) {                                                                        \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                             \
        }                                                                                             \
    } while (0)

using clk = std::chrono::steady_clock;
static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// T persistent workers; run() splits [src, src + n) into T contiguous parts and copies them.
struct Pool {
    std::vector<std::thread> th;
    std::atomic<int> gen{0}, done{0};
    std::atomic<bool> stop{false};
    char *dst = nullptr;
    const char *src = nullptr;
    size_t n = 0;
    int T;
    explicit Pool(int t) : T(t) {
        for (int i = 1; i < T; ++i)
            th.emplace_back([this, i] {
                int seen = 0;
                for (;;) {
                    while (gen.load(std::memory_order_acquire) == seen && !stop.load()) std::this_thread::yield();
                    if (stop.load()) return;
                    seen = gen.load();
                    part(i);
                    done.fetch_add(1, std::memory_order_release);
                }
            });
    }
    void part(int i) {
        const size_t per = (n / T + 4095) & ~size_t(4095);
        const size_t lo = std::min(n, per * i), hi = std::min(n, lo + per);
        if (hi > lo) std::memcpy(dst + lo, src + lo, hi - lo);
    }
    void run(char *d, const char *s, size_t bytes) {
        dst = d;
        src = s;
        n = bytes;
        done.store(0);
        gen.fetch_add(1, std::memory_order_release);
        part(0);
        while (done.load(std::memory_order_acquire) < T - 1) std::this_thread::yield();
    }
    ~Pool() {
        stop = true;
        for (auto &t : th) t.join();
    }
};

int main() {
    const size_t chunk = 32ull << 20, total = 2ull << 30;
    const int slots = 4, chunks = (int)(total / chunk);
    CK(hipSetDevice(0));
    void *dev = nullptr;
    CK(hipMalloc(&dev, chunk));
    CK(hipMemset(dev, 0x3c, chunk));
    char *dst = static_cast<char *>(std::malloc(total));
    std::memset(dst, 1, total);  // warm pageable destination (the tensors were written before)
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct Kind {
        const char *name;
        unsigned flags;
        int how;  // 0 hipHostMalloc(flags), 1 malloc + hipHostRegister, 2 malloc (pageable: D2H staged by HIP)
    } kinds[] = {{"hipHostMallocDefault", hipHostMallocDefault, 0},
                 {"hipHostMallocNonCoherent", hipHostMallocNonCoherent, 0},
                 {"hipHostMallocCoherent", hipHostMallocCoherent, 0},
                 {"hipHostMallocNumaUser", hipHostMallocNumaUser, 0},
                 {"malloc+hipHostRegister", hipHostRegisterDefault, 1},
                 {"malloc_pageable", 0, 2}};
    const int threads[] = {1, 4, 7, 8, 16};
    for (const Kind &k : kinds) {
        std::vector<char *> slot(slots, nullptr);
        bool ok = true;
        for (int j = 0; j < slots; ++j) {
            if (k.how == 0) {
                if (hipHostMalloc(reinterpret_cast<void **>(&slot[j]), chunk, k.flags) != hipSuccess) ok = false;
            } else {
                slot[j] = static_cast<char *>(std::aligned_alloc(4096, chunk));
                std::memset(slot[j], 0, chunk);
                if (k.how == 1 && hipHostRegister(slot[j], chunk, k.flags) != hipSuccess) ok = false;
            }
        }
        if (!ok) {
            (void)hipGetLastError();
            std::printf("{\"kind\": \"%s\", \"error\": \"allocation failed\"}\n", k.name);
            continue;
        }
        for (int T : threads) {
            Pool pool(T);
            double dma_s = 0, copy_s = 0;
            for (int rep = 0; rep < chunks; ++rep) {
                char *sl = slot[rep % slots];
                const clk::time_point t0 = clk::now();
                CK(hipMemcpyAsync(sl, dev, chunk, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                const clk::time_point t1 = clk::now();
                pool.run(dst + (size_t)rep * chunk, sl, chunk);
                const clk::time_point t2 = clk::now();
                if (rep >= slots) {  // the first lap warms the slots
                    dma_s += secs(t0, t1);
                    copy_s += secs(t1, t2);
                }
            }
            const double bytes = (double)chunk * (chunks - slots);
            std::printf("{\"kind\": \"%s\", \"threads\": %d, \"d2h_GBs\": %.2f, \"copy_GBs\": %.2f, "
                        "\"d2h_ms_per_GiB\": %.3f, \"copy_ms_per_GiB\": %.3f}\n",
                        k.name, T, bytes / dma_s / 1e9, bytes / copy_s / 1e9, dma_s * 1e3 / (bytes / (1 << 30)),
                        copy_s * 1e3 / (bytes / (1 << 30)));
            std::fflush(stdout);
        }
        for (int j = 0; j < slots; ++j) {
            if (k.how == 0) CK(hipHostFree(slot[j]));
            else {
                if (k.how == 1) CK(hipHostUnregister(slot[j]));
                std::free(slot[j]);
            }
        }
    }
    std::free(dst);
    CK(hipFree(dev));
    return 0;
}
