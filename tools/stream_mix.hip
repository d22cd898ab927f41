// tools/stream_mix.hip — measurement harness, not shipped: the HBM ceiling of a streaming kernel
// as a function of its read:write mix, in the shipped kernels' form (one 128-lane workgroup per
// 2 KiB tile of every stream, one buffer_load_dwordx4 per lane and input stream with the
// non-temporal bit, one write-through buffer_store_dwordx4 per lane). R input streams and W
// (0 or 1) output streams of C bytes each; 3 rotating buffer sets keep everything out of the
// 256 MiB Infinity Cache. The question it answers: is the 8-input fold
// (R = 8, W = 1) below the two-input reduce (R = 2, W = 1) because of its kernel, or because a
// read-heavy stream mix tops out lower on this HBM?
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_mix.hip -o tools/bin/stream_mix
//   ./stream_mix [total MiB per launch = 288] [rounds = 5] [occ: occupancy-cap sweep instead]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

using u4 = unsigned int __attribute__((ext_vector_type(4)));
using f4 = float __attribute__((ext_vector_type(4)));
constexpr int kMaxR = 8;
constexpr int kT = 128;  // lanes per workgroup = 16-byte vectors per tile
constexpr int kAuxNt = 2, kAuxWt = 1 | 16;
constexpr int kWord3 = 0x00020000;

struct Streams {
    u4 *x[kMaxR];
    u4 *o;
};

// R reads + W writes per 16-byte lane vector; W = 0 keeps the sum live with a store that never
// fires (the inputs are finite, the test is for a NaN pattern)
template <int R, int W, int LOADAUX>
__global__ void __launch_bounds__(kT) k_mix(Streams s, unsigned long long nv) {
    const unsigned long long base = (unsigned long long)blockIdx.x * kT;
    if (base >= nv) return;
    const int bytes = (int)((nv - base < kT ? nv - base : kT) * 16);
    const int off = (int)threadIdx.x * 16;
    u4 raw[R];
#pragma unroll
    for (int k = 0; k < R; ++k)
        raw[k] = __builtin_amdgcn_raw_buffer_load_b128(__builtin_amdgcn_make_buffer_rsrc(s.x[k] + base, 0, bytes, kWord3),
                                                       off, 0, LOADAUX);
    f4 acc = __builtin_bit_cast(f4, raw[0]);
#pragma unroll
    for (int k = 1; k < R; ++k) acc += __builtin_bit_cast(f4, raw[k]);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(s.o + base, 0, bytes, kWord3);
    if constexpr (W == 1) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc), ro, off, 0, kAuxWt);
    } else {
        if (__builtin_bit_cast(unsigned, acc.x) == 0x7fc01234u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc), ro, off, 0, kAuxWt);
    }
}

// Blocked form: a workgroup owns U consecutive tiles of the output and streams them input by
// input — U loads per lane from input k in flight, accumulated, then input k + 1 — so each
// workgroup reads one stream at a time in U * 2 KiB runs instead of 1 tile from all R streams.
template <int R, int U, int T = kT, bool INPLACE = false>
__global__ void __launch_bounds__(T) k_mix_blocked(Streams s, unsigned long long nv) {
    const unsigned long long base = (unsigned long long)blockIdx.x * T * U;
    if (base >= nv) return;
    const int bytes = (int)((nv - base < (unsigned long long)T * U ? nv - base : (unsigned long long)T * U) * 16);
    const int off = (int)threadIdx.x * 16;
    f4 acc[U];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(s.x[k] + base, 0, bytes, kWord3);
        u4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) raw[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + u * T * 16, 0, kAuxNt);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = k == 0 ? __builtin_bit_cast(f4, raw[u]) : acc[u] + __builtin_bit_cast(f4, raw[u]);
    }
    const auto ro = __builtin_amdgcn_make_buffer_rsrc((INPLACE ? s.x[0] : s.o) + base, 0, bytes, kWord3);
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[u]), ro, off + u * T * 16, 0, kAuxWt);
}

__global__ void k_init(u4 *p, unsigned long long nv, unsigned seed) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < nv;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        float f = (float)(h & 0xffff) / 65536.0f - 0.5f;
        p[i] = __builtin_bit_cast(u4, f4{f, f, f, f});
    }
}

struct Case {
    std::string name;
    int r, w;
    std::function<void(const Streams &, unsigned long long, hipStream_t)> launch;
};

// lds_kib > 0 reserves that much (unused) dynamic LDS per workgroup: 160 KiB per CU / lds_kib caps
// the workgroups resident on a CU, so fewer tiles of every stream are in flight at once
template <int R, int W, int AUX>
Case mk(const char *pol, int lds_kib = 0) {
    char nm[96];
    if (lds_kib)
        std::snprintf(nm, sizeof nm, "R%d W%d (%d:%d) %s, <= %d WG/CU", R, W, R, W, pol, 160 / lds_kib);
    else
        std::snprintf(nm, sizeof nm, "R%d W%d (%d:%d) %s", R, W, R, W, pol);
    return Case{nm, R, W, [lds_kib](const Streams &s, unsigned long long nv, hipStream_t st) {
                    const unsigned tiles = (unsigned)((nv + kT - 1) / kT);
                    hipLaunchKernelGGL((k_mix<R, W, AUX>), dim3(tiles), dim3(kT), (size_t)lds_kib << 10, st, s, nv);
                }};
}

template <int R, int U, int T = kT, bool INPLACE = false>
Case mk_blocked() {
    char nm[96];
    std::snprintf(nm, sizeof nm, "R%d W1 (%d:1) blocked%s, %d lanes x %d vectors (%d KiB runs)", R, R,
                  INPLACE ? " in place" : "", T, U, T * U * 16 / 1024);
    return Case{nm, R, 1, [](const Streams &s, unsigned long long nv, hipStream_t st) {
                    const unsigned wgs = (unsigned)((nv + (unsigned long long)T * U - 1) / ((unsigned long long)T * U));
                    hipLaunchKernelGGL((k_mix_blocked<R, U, T, INPLACE>), dim3(wgs), dim3(T), 0, st, s, nv);
                }};
}

int main(int argc, char **argv) {
    const size_t total_mib = argc > 1 ? std::atoi(argv[1]) : 288;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const int reps = 8, sets = 3;
    const bool occ = argc > 3 && std::string(argv[3]) == "occ";
    std::vector<Case> cases = {
        mk<1, 0, kAuxNt>("nt loads"),           mk<2, 0, kAuxNt>("nt loads"),
        mk<4, 0, kAuxNt>("nt loads"),           mk<8, 0, kAuxNt>("nt loads"),
        mk<1, 1, kAuxNt>("nt loads, wt store"), mk<2, 1, kAuxNt>("nt loads, wt store"),
        mk<4, 1, kAuxNt>("nt loads, wt store"), mk<8, 1, kAuxNt>("nt loads, wt store"),
        mk<8, 0, 0>("plain loads"),             mk<8, 1, 0>("plain loads, wt store"),
    };
    if (argc > 3 && std::string(argv[3]) == "blocked") {  // one stream at a time per workgroup
        cases = {mk<8, 1, kAuxNt>("nt loads, wt store"), mk_blocked<8, 4>(), mk_blocked<8, 8>(), mk_blocked<8, 16>(),
                 mk_blocked<8, 32>(), mk_blocked<8, 4, 256>(), mk_blocked<8, 8, 256>(), mk_blocked<8, 2, 512>(),
                 mk_blocked<8, 4, 512>(), mk_blocked<8, 8, 64>(), mk_blocked<8, 16, 64>(),
                 mk<4, 1, kAuxNt>("nt loads, wt store"), mk_blocked<4, 8>(), mk_blocked<4, 16>(),
                 mk<2, 1, kAuxNt>("nt loads, wt store"), mk_blocked<2, 4>(), mk_blocked<2, 8>(), mk_blocked<2, 16>(),
                 mk_blocked<2, 4, 256>(), mk_blocked<2, 8, 256>(), mk_blocked<2, 4, kT, true>(),
                 mk_blocked<2, 8, kT, true>(), mk_blocked<2, 16, kT, true>()};
    }
    if (argc > 3 && std::string(argv[3]) == "rform") {  // tile vs run form for every fold width
        cases = {mk<2, 1, kAuxNt>("nt loads, wt store"), mk_blocked<2, 8>(),
                 mk<3, 1, kAuxNt>("nt loads, wt store"), mk_blocked<3, 8>(),
                 mk<4, 1, kAuxNt>("nt loads, wt store"), mk_blocked<4, 8>(),
                 mk<5, 1, kAuxNt>("nt loads, wt store"), mk_blocked<5, 8>(),
                 mk<6, 1, kAuxNt>("nt loads, wt store"), mk_blocked<6, 8>(),
                 mk<7, 1, kAuxNt>("nt loads, wt store"), mk_blocked<7, 8>(),
                 mk<8, 1, kAuxNt>("nt loads, wt store"), mk_blocked<8, 8>(),
                 mk_blocked<2, 2>(), mk_blocked<2, 2, kT, true>(), mk_blocked<2, 4, 64>(), mk_blocked<2, 4, 64, true>()};
    }
    if (occ) {  // occupancy caps: does a smaller in-flight window per stream lift the many-stream mixes?
        cases.clear();
        for (int lds : {0, 10, 20, 27, 32, 40, 64}) {
            cases.push_back(mk<8, 1, kAuxNt>("nt loads, wt store", lds));
            cases.push_back(mk<2, 1, kAuxNt>("nt loads, wt store", lds));
            cases.push_back(mk<8, 0, kAuxNt>("nt loads", lds));
        }
    }
    // every case moves the same total: stream bytes C = total / (R + W)
    const size_t max_stream = (total_mib << 20) / 1;  // R = 1, W = 0 needs one stream of the total
    std::vector<std::vector<u4 *>> bufs(sets, std::vector<u4 *>(kMaxR + 1));
    for (auto &set : bufs)
        for (auto &p : set) {
            // each slot sized for the largest stream any case uses (R + W = 1: the total)
            CK(hipMalloc(&p, max_stream));
            hipLaunchKernelGGL(k_init, dim3(1024), dim3(256), 0, 0, p, max_stream / 16, (unsigned)(size_t)p);
        }
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> ms(cases.size());
    for (int round = 0; round < rounds; ++round)
        for (size_t c = 0; c < cases.size(); ++c) {
            const Case &cs = cases[c];
            const size_t stream_bytes = ((total_mib << 20) / (cs.r + cs.w)) & ~size_t(2047);
            const unsigned long long nv = stream_bytes / 16;
            auto streams = [&](int set) {
                Streams s{};
                for (int k = 0; k < kMaxR; ++k) s.x[k] = bufs[set][k];
                s.o = bufs[set][kMaxR];
                return s;
            };
            cs.launch(streams(0), nv, 0);  // warm
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) cs.launch(streams(i % sets), nv, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[c].push_back(t / reps);
        }
    std::printf("# stream mix, %zu MiB moved per launch (R reads + W writes of total/(R+W) each), %d rounds x %d reps, "
                "%d rotating sets; GB/s = moved bytes / kernel time\n",
                total_mib, rounds, reps, sets);
    for (size_t c = 0; c < cases.size(); ++c) {
        std::vector<double> v = ms[c];
        std::sort(v.begin(), v.end());
        const size_t stream_bytes = ((total_mib << 20) / (cases[c].r + cases[c].w)) & ~size_t(2047);
        const double moved = (double)stream_bytes * (cases[c].r + cases[c].w);
        std::printf("%-32s best %7.1f GB/s  median %7.1f GB/s  (%.4f ms)\n", cases[c].name.c_str(),
                    moved / (v.front() * 1e-3) / 1e9, moved / (v[v.size() / 2] * 1e-3) / 1e9, v.front());
    }
    return 0;
}
