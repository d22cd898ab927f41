// tools/copy_tune.hip — the 1-read + 1-write ceiling on MI355X (measurement tool, not shipped):
// what the fusion pack / unpack kernels (csrc/pack.hip) can reach at best. Copies S bytes
// between rotating buffer pairs (3 pairs, so no pass re-reads Infinity-Cache-resident data)
// with one-tile-per-workgroup mappings (U chunks of 16 B per lane, NT lanes per workgroup,
// non-temporal loads/stores) next to hipMemcpyAsync. Interleaved rounds, best and median.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/copy_tune.hip -o tools/bin/copy_tune
//   tools/bin/copy_tune [MiB=512] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

using u4 = unsigned int __attribute__((ext_vector_type(4)));

template <int U, int NT, bool NTL, bool NTS>
__global__ void __launch_bounds__(NT) k_copy_tile(u4 *o, const u4 *a, size_t nv) {
    const size_t base = (size_t)blockIdx.x * NT * U + threadIdx.x;
    u4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * NT;
        if (i < nv) x[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * NT;
        if (i < nv) {
            if (NTS) __builtin_nontemporal_store(x[u], o + i);
            else o[i] = x[u];
        }
    }
}

struct Case {
    std::string name;
    std::function<void(hipStream_t, int)> run;
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::atol(argv[1]) : 512;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t S = mib << 20, nv = S / 16;
    constexpr int kPairs = 3;
    u4 *src[kPairs], *dst[kPairs];
    for (int p = 0; p < kPairs; ++p) {
        CK(hipMalloc(&src[p], S));
        CK(hipMalloc(&dst[p], S));
        CK(hipMemset(src[p], p + 1, S));
        CK(hipMemset(dst[p], 0, S));
    }
    std::vector<Case> cases;
#define TILE(U, NT, L, St)                                                                                       \
    cases.push_back({"tile U" #U " lanes" #NT " ntl" #L " nts" #St, [=](hipStream_t s, int p) {                    \
                         hipLaunchKernelGGL((k_copy_tile<U, NT, L, St>), dim3((unsigned)((nv + U * NT - 1) / (U * NT))), \
                                            dim3(NT), 0, s, dst[p], src[p], nv);                                  \
                     }, {}});
    TILE(1, 64, true, true)
    TILE(1, 128, true, true)
    TILE(1, 256, true, true)
    TILE(2, 128, true, true)
    TILE(4, 128, true, true)
    TILE(4, 256, true, true)
    TILE(16, 256, true, true)
    TILE(1, 128, false, false)
    TILE(1, 128, true, false)
    TILE(1, 256, false, false)
    TILE(16, 256, false, false)
    TILE(16, 256, false, true)
    cases.push_back({"hipMemcpyAsync D2D", [=](hipStream_t s, int p) {
                         CK(hipMemcpyAsync(dst[p], src[p], S, hipMemcpyDeviceToDevice, s));
                     }, {}});
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = std::max(6, (int)(3072 / mib));
    for (auto &c : cases)
        for (int p = 0; p < kPairs; ++p) c.run(s, p);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r)
        for (auto &c : cases) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) c.run(s, k % kPairs);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            c.ms.push_back(ms / reps);
        }
    std::printf("# copy of %zu MiB, %d rotating pairs, %d rounds x %d reps; GB/s (read + write bytes)\n", mib, kPairs,
                rounds, reps);
    for (auto &c : cases) {
        std::vector<float> m = c.ms;
        std::sort(m.begin(), m.end());
        std::printf("%-32s best %7.1f GB/s  median %7.1f GB/s\n", c.name.c_str(), 2.0 * S / (m[0] * 1e-3) / 1e9,
                    2.0 * S / (m[m.size() / 2] * 1e-3) / 1e9);
    }
    return 0;
}
