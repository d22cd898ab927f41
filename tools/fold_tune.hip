// tools/fold_tune.hip — standalone tuning harness for the N-input fold (k_sumN_tile), not shipped.
// out = x_0 + ... + x_{K-1} (fp32, left fold, 16 B per lane access) over K = 8 inputs of one
// chunk, under several tile shapes: lanes per workgroup (T) x 16-byte vectors per lane and input
// (U; a workgroup covers T*U*16 contiguous bytes of every input), and cache policies. 3 rotating
// buffer sets (9 streams each) keep the operands out of the 256 MiB Infinity Cache; rounds are
// interleaved (guide: known-good references next to the variants).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fold_tune.hip -o tools/bin/fold_tune
//   ./fold_tune [chunk MiB=32] [rounds=5]
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

using f4 = float __attribute__((ext_vector_type(4)));
using u4 = unsigned int __attribute__((ext_vector_type(4)));
constexpr int K = 8;  // inputs (P = 8: own + 7 received)

struct Ins {
    const f4 *x[K];
};

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// POL bit 0: non-temporal loads, bit 1: non-temporal store, bit 2: write-through store. Vector u
// of lane l at u*T + l; the loads of every input issued before the first add.
template <int T, int U, int POL>
__global__ void __launch_bounds__(T) k_fold(f4 *o, Ins in, size_t nv) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    f4 r[K][U];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * T;
            r[k][u] = i < nv ? ld<(POL & 1) != 0>(in.x[k] + i) : f4{0, 0, 0, 0};
        }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * T;
        if (i >= nv) continue;
        f4 s = r[0][u];
#pragma unroll
        for (int k = 1; k < K; ++k) s += r[k][u];
        if constexpr ((POL & 4) != 0) {  // write-through (sc0 sc1) raw buffer store
            // one descriptor per workgroup (a per-lane base would make hipcc loop over lanes)
            const size_t wg = (size_t)blockIdx.x * T * U;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(o + wg, 0, 0x7fffffff, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, s), rs, (int)((i - wg) * 16), 0, 17);
        } else if constexpr ((POL & 2) != 0) {
            __builtin_nontemporal_store(s, o + i);
        } else {
            o[i] = s;
        }
    }
}

// running-sum variant: the compiler may issue the K loads back to back or interleave the adds;
// a reference point for the "all loads first" rule of the shipped kernel
template <int T, int POL>
__global__ void __launch_bounds__(T) k_fold_serial(f4 *o, Ins in, size_t nv) {
    const size_t i = (size_t)blockIdx.x * T + threadIdx.x;
    if (i >= nv) return;
    f4 s = ld<(POL & 1) != 0>(in.x[0] + i);
#pragma unroll
    for (int k = 1; k < K; ++k) {
        const f4 v = ld<(POL & 1) != 0>(in.x[k] + i);
        s += v;
    }
    if constexpr ((POL & 2) != 0) __builtin_nontemporal_store(s, o + i);
    else o[i] = s;
}

// Buffer form (the two-input reduce's mapping): one descriptor per input tile, 32-bit lane
// offsets, the cache bits in each access's aux word. AUXL: loads' aux (2 = nt), AUXS: store's
// aux (2 = nt, 17 = sc0 sc1 write-through, 0 plain).
template <int T, int AUXL, int AUXS>
__global__ void __launch_bounds__(T) k_fold_buf(f4 *o, Ins in, size_t nv) {
    const size_t base = (size_t)blockIdx.x * T;
    if (base >= nv) return;
    const int bytes = (int)((nv - base < (size_t)T ? nv - base : (size_t)T) * 16);
    const int off = (int)threadIdx.x * 16;
    u4 r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(in.x[k] + base), 0, bytes, 0x00020000);
        r[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUXL);
    }
    f4 s = __builtin_bit_cast(f4, r[0]);
#pragma unroll
    for (int k = 1; k < K; ++k) s += __builtin_bit_cast(f4, r[k]);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(o + base, 0, bytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, s), ro, off, 0, AUXS);
}

struct Variant {
    std::string name;
    std::function<void(f4 *, Ins, size_t, hipStream_t)> run;
};

template <int T, int U, int POL>
Variant make(const char *tag) {
    char buf[96];
    std::snprintf(buf, sizeof buf, "fold T%d U%d pol%d %s", T, U, POL, tag);
    return Variant{buf, [](f4 *o, Ins in, size_t nv, hipStream_t s) {
                       const size_t per = (size_t)T * U;
                       hipLaunchKernelGGL((k_fold<T, U, POL>), dim3((unsigned)((nv + per - 1) / per)), dim3(T), 0, s,
                                          o, in, nv);
                   }};
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::atol(argv[1]) : 32;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const int reps = 8, sets = 3;
    const size_t bytes = mib << 20, nv = bytes / 16;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // argv[3]: skew in bytes between the inputs' bases (input k starts k * skew bytes into its
    // allocation): tests whether 8 streams at the same offsets alias the same HBM channels
    const size_t skew = argc > 3 ? std::atol(argv[3]) : 0;
    std::vector<f4 *> bufs((K + 1) * sets);
    for (size_t j = 0; j < bufs.size(); ++j) {
        char *b;
        CK(hipMalloc(&b, bytes + K * skew));
        CK(hipMemset(b, 0, bytes + K * skew));
        bufs[j] = reinterpret_cast<f4 *>(b + (j % (K + 1)) * skew);
    }
    std::vector<Variant> vs = {
        make<128, 1, 3>("(shipped: 128 lanes, 1 vector, all NT)"),
        make<128, 1, 0>("plain"),
        make<128, 1, 1>("NT loads"),
        make<64, 1, 3>(""),
        make<256, 1, 3>(""),
        make<64, 2, 3>(""),
        make<128, 2, 3>(""),
        make<256, 2, 3>(""),
        make<64, 4, 3>(""),
        make<128, 4, 3>(""),
        make<256, 4, 1>("NT loads"),
        make<128, 2, 1>("NT loads"),
        make<128, 1, 5>("NT loads, write-through store"),
        Variant{"fold_buf T128 nt loads, nt store", [](f4 *o, Ins in, size_t nv, hipStream_t st) {
                    hipLaunchKernelGGL((k_fold_buf<128, 2, 2>), dim3((unsigned)((nv + 127) / 128)), dim3(128), 0, st, o, in, nv);
                }},
        Variant{"fold_buf T128 nt loads, wt store", [](f4 *o, Ins in, size_t nv, hipStream_t st) {
                    hipLaunchKernelGGL((k_fold_buf<128, 2, 17>), dim3((unsigned)((nv + 127) / 128)), dim3(128), 0, st, o, in, nv);
                }},
        Variant{"fold_buf T64 nt loads, nt store", [](f4 *o, Ins in, size_t nv, hipStream_t st) {
                    hipLaunchKernelGGL((k_fold_buf<64, 2, 2>), dim3((unsigned)((nv + 63) / 64)), dim3(64), 0, st, o, in, nv);
                }},
        Variant{"fold_buf T128 plain loads, wt store", [](f4 *o, Ins in, size_t nv, hipStream_t st) {
                    hipLaunchKernelGGL((k_fold_buf<128, 0, 17>), dim3((unsigned)((nv + 127) / 128)), dim3(128), 0, st, o, in, nv);
                }},
        make<128, 1, 4>("plain loads, write-through store"),
        Variant{"fold_serial T128 pol3",
                [](f4 *o, Ins in, size_t nv, hipStream_t st) {
                    hipLaunchKernelGGL((k_fold_serial<128, 3>), dim3((unsigned)((nv + 127) / 128)), dim3(128), 0, st, o,
                                       in, nv);
                }},
        Variant{"hipMemcpyAsync D2D (1R+1W, bytes counted 2x chunk)",
                [bytes](f4 *o, Ins in, size_t, hipStream_t st) { CK(hipMemcpyAsync(o, in.x[0], bytes, hipMemcpyDeviceToDevice, st)); }},
    };
    std::vector<std::vector<float>> ms(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto ins_of = [&](int set) {
        Ins in;
        for (int k = 0; k < K; ++k) in.x[k] = bufs[set * (K + 1) + k];
        return in;
    };
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int w = 0; w < 3; ++w) vs[v].run(bufs[w * (K + 1) + K], ins_of(w), nv, s);
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) {
                const int set = i % sets;
                vs[v].run(bufs[set * (K + 1) + K], ins_of(set), nv, s);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / reps);
        }
    }
    std::printf("# fp32 fold of %d inputs, %zu MiB chunk, %d rounds x %d reps, %d rotating sets, input skew %zu B; GB/s = (K+1)*chunk / t\n",
                K, mib, rounds, reps, sets, skew);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = ms[v];
        std::sort(x.begin(), x.end());
        const double moved = vs[v].name.rfind("hipMemcpy", 0) == 0 ? 2.0 * bytes : (double)(K + 1) * bytes;
        std::printf("%-52s best %7.1f GB/s  median %7.1f GB/s  (%.4f ms)\n", vs[v].name.c_str(), moved / (x[0] * 1e6),
                    moved / (x[x.size() / 2] * 1e6), x[0]);
    }
    return 0;
}
