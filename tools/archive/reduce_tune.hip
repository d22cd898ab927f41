// tools/reduce_tune.hip — standalone tuning harness for the per-hop reduce kernel (not shipped).
// Times out = a + b (fp32, 16 B per lane access) under several workgroup->data mappings,
// unroll depths and occupancies, next to copy / read-only / hipMemcpy baselines measured on the
// same device (guide §5.4 rules 10 and 24: known-good references, interleaved rounds).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/reduce_tune.hip -o reduce_tune
//   ./reduce_tune [MiB=256] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

using f4 = float __attribute__((ext_vector_type(4)));

// MAP 0: grid-stride, UNROLL accesses strided by the grid
template <int UNROLL, int NT>
__global__ void __launch_bounds__(NT) k_gridstride(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    const size_t stride = (size_t)gridDim.x * NT;
    size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < nv; i += UNROLL * stride) {
        f4 x[UNROLL], y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) { x[u] = a[i + u * stride]; y[u] = b[i + u * stride]; }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) o[i + u * stride] = x[u] + y[u];
    }
    for (; i < nv; i += stride) o[i] = a[i] + b[i];
}

// MAP 1: tiles of NT*UNROLL contiguous vectors, tiles dealt grid-stride
template <int UNROLL, int NT>
__global__ void __launch_bounds__(NT) k_tiles(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    const size_t tile = (size_t)NT * UNROLL;
    const size_t ntiles = nv / tile;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const size_t base = t * tile + threadIdx.x;
        f4 x[UNROLL], y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) { x[u] = a[base + u * NT]; y[u] = b[base + u * NT]; }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) o[base + u * NT] = x[u] + y[u];
    }
    for (size_t i = ntiles * tile + (size_t)blockIdx.x * NT + threadIdx.x; i < nv; i += (size_t)gridDim.x * NT)
        o[i] = a[i] + b[i];
}

// MAP 1 with one tile per workgroup and optional non-temporal loads / stores and XCD remap:
// XCD=1 deals consecutive tiles to the same XCD (blocks b and b+8 share an XCD).
template <int UNROLL, int NT, int NTL, int NTS, int XCD>
__global__ void __launch_bounds__(NT) k_tile1(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    size_t t = blockIdx.x;
    if (XCD) {
        const size_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = t % 8, k = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    }
    const size_t base = t * (size_t)NT * UNROLL + threadIdx.x;
    f4 x[UNROLL], y[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const size_t i = base + (size_t)u * NT;
        if (i < nv) {
            if (NTL) { x[u] = __builtin_nontemporal_load(a + i); y[u] = __builtin_nontemporal_load(b + i); }
            else { x[u] = a[i]; y[u] = b[i]; }
        }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        const size_t i = base + (size_t)u * NT;
        if (i < nv) {
            if (NTS) __builtin_nontemporal_store(x[u] + y[u], o + i);
            else o[i] = x[u] + y[u];
        }
    }
}

typedef __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;
// one tile per workgroup, b staged through LDS by global_load_lds_dwordx4
template <int NT>
__global__ void __launch_bounds__(NT) k_tile1_lds(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    __shared__ __attribute__((aligned(16))) f4 st[NT];
    const size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
    const int wave = threadIdx.x >> 6;
    if (i < nv) __builtin_amdgcn_global_load_lds((gptr_t)(b + i), (lptr_t)(st + wave * 64), 16, 0, 0);
    f4 x = i < nv ? a[i] : f4{0, 0, 0, 0};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (i < nv) o[i] = x + st[threadIdx.x];
}

// MAP 2: each workgroup streams one contiguous range
template <int UNROLL, int NT>
__global__ void __launch_bounds__(NT) k_ranges(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    const size_t per = (nv + gridDim.x - 1) / gridDim.x;
    const size_t beg = (size_t)blockIdx.x * per;
    const size_t end = beg + per < nv ? beg + per : nv;
    size_t i = beg + threadIdx.x;
    for (; i + (UNROLL - 1) * NT < end; i += (size_t)UNROLL * NT) {
        f4 x[UNROLL], y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) { x[u] = a[i + u * NT]; y[u] = b[i + u * NT]; }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) o[i + u * NT] = x[u] + y[u];
    }
    for (; i < end; i += NT) o[i] = a[i] + b[i];
}

template <int UNROLL, int NT>
__global__ void __launch_bounds__(NT) k_copy(f4 *o, const f4 *a, size_t nv) {
    const size_t stride = (size_t)gridDim.x * NT;
    size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < nv; i += UNROLL * stride) {
        f4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) o[i + u * stride] = x[u];
    }
    for (; i < nv; i += stride) o[i] = a[i];
}

template <int UNROLL, int NT>
__global__ void __launch_bounds__(NT) k_read2(float *sink, const f4 *a, const f4 *b, size_t nv) {
    const size_t stride = (size_t)gridDim.x * NT;
    size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    for (; i + (UNROLL - 1) * stride < nv; i += UNROLL * stride) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += a[i + u * stride] + b[i + u * stride];
    }
    for (; i < nv; i += stride) acc += a[i] + b[i];
    if (acc.x + acc.y + acc.z + acc.w == 12345.678f) sink[0] = 1.f;
}

__global__ void k_fill(float *p, size_t n, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (float)(x & 0xffffff) / 16777216.0f * 2.f - 1.f;
    }
}

struct Case {
    std::string name;
    double bytes_per_call;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::atol(argv[1]) : 256;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t S = mib << 20, n = S / 4, nv = n / 4;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float *a, *b, *o, *sink;
    CK(hipMalloc(&a, S));
    CK(hipMalloc(&b, S));
    CK(hipMalloc(&o, S));
    CK(hipMalloc(&sink, 64));
    k_fill<<<2048, 256>>>(a, n, 1);
    k_fill<<<2048, 256>>>(b, n, 2);
    k_fill<<<2048, 256>>>(o, n, 3);
    CK(hipDeviceSynchronize());
    f4 *A = (f4 *)a, *B = (f4 *)b, *O = (f4 *)o;
    std::vector<Case> cases;
    auto add3 = [&](std::string nm, std::function<void(hipStream_t)> f) { cases.push_back({nm, 3.0 * S, f, {}}); };

#define GRID_CASES(U, NT, BPC)                                                                                         \
    add3("gridstride U" #U " NT" #NT " bpc" #BPC, [=](hipStream_t s) { hipLaunchKernelGGL((k_gridstride<U, NT>), dim3(cus * BPC), dim3(NT), 0, s, O, A, B, nv); }); \
    add3("tiles      U" #U " NT" #NT " bpc" #BPC, [=](hipStream_t s) { hipLaunchKernelGGL((k_tiles<U, NT>), dim3(cus * BPC), dim3(NT), 0, s, O, A, B, nv); }); \
    add3("ranges     U" #U " NT" #NT " bpc" #BPC, [=](hipStream_t s) { hipLaunchKernelGGL((k_ranges<U, NT>), dim3(cus * BPC), dim3(NT), 0, s, O, A, B, nv); });

    GRID_CASES(4, 256, 8)
    GRID_CASES(8, 256, 8)
#define TILE1(U, NT, NTL, NTS, XCD)                                                                                 \
    add3("tile1 U" #U " NT" #NT " ntl" #NTL " nts" #NTS " xcd" #XCD, [=](hipStream_t s) {                          \
        hipLaunchKernelGGL((k_tile1<U, NT, NTL, NTS, XCD>), dim3((unsigned)((nv + U * NT - 1) / (U * NT))), dim3(NT), 0, s, O, A, B, nv); });
    TILE1(1, 64, 0, 0, 0)
    TILE1(1, 128, 0, 0, 0)
    TILE1(1, 256, 0, 0, 0)
    TILE1(1, 512, 0, 0, 0)
    TILE1(1, 1024, 0, 0, 0)
    TILE1(2, 256, 0, 0, 0)
    TILE1(2, 128, 0, 0, 0)
    TILE1(4, 256, 0, 0, 0)
    TILE1(4, 64, 0, 0, 0)
    TILE1(1, 256, 1, 0, 0)
    TILE1(1, 256, 0, 1, 0)
    TILE1(1, 256, 1, 1, 0)
    TILE1(1, 256, 0, 0, 1)
    TILE1(2, 256, 0, 0, 1)
    TILE1(4, 256, 0, 0, 1)
    TILE1(2, 256, 1, 0, 0)
    TILE1(2, 256, 1, 1, 0)
    TILE1(4, 256, 1, 1, 0)
    TILE1(1, 512, 1, 1, 0)
    TILE1(2, 128, 1, 1, 0)
    TILE1(1, 128, 1, 1, 0)
    TILE1(4, 64, 1, 1, 0)
    add3("tile1_lds NT256", [=](hipStream_t s) { hipLaunchKernelGGL((k_tile1_lds<256>), dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, O, A, B, nv); });
    add3("tile1 inplace U1 NT256", [=](hipStream_t s) { hipLaunchKernelGGL((k_tile1<1, 256, 0, 0, 0>), dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, A, A, B, nv); });
    add3("tiles U1 NT256 grid=all tiles", [=](hipStream_t s) { hipLaunchKernelGGL((k_tiles<1, 256>), dim3((unsigned)(nv / 256)), dim3(256), 0, s, O, A, B, nv); });
    add3("tiles U2 NT256 grid=tiles/4", [=](hipStream_t s) { hipLaunchKernelGGL((k_tiles<2, 256>), dim3((unsigned)(nv / 2048)), dim3(256), 0, s, O, A, B, nv); });
    add3("tiles U1 NT256 bpc32", [=](hipStream_t s) { hipLaunchKernelGGL((k_tiles<1, 256>), dim3(cus * 32), dim3(256), 0, s, O, A, B, nv); });
    add3("tiles U2 NT256 bpc32", [=](hipStream_t s) { hipLaunchKernelGGL((k_tiles<2, 256>), dim3(cus * 32), dim3(256), 0, s, O, A, B, nv); });
    cases.push_back({"copy U4 NT256 bpc8 (1R+1W)", 2.0 * S, [=](hipStream_t s) { hipLaunchKernelGGL((k_copy<4, 256>), dim3(cus * 8), dim3(256), 0, s, O, A, nv); }, {}});
    cases.push_back({"read2 U4 NT256 bpc8 (2R)", 2.0 * S, [=](hipStream_t s) { hipLaunchKernelGGL((k_read2<4, 256>), dim3(cus * 8), dim3(256), 0, s, sink, A, B, nv); }, {}});
    cases.push_back({"hipMemcpyAsync D2D (1R+1W)", 2.0 * S, [=](hipStream_t s) { CK(hipMemcpyAsync(o, a, S, hipMemcpyDeviceToDevice, s)); }, {}});

    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = std::max(3, (int)(2048 / mib));
    // warm: ~1 s of traffic to settle clocks
    for (int w = 0; w < 3; ++w)
        for (auto &c : cases) c.run(s);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r) {
        for (auto &c : cases) {
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) c.run(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            c.ms.push_back(ms / reps);
        }
    }
    std::printf("# %zu MiB fp32 buckets, %d CUs, %d rounds x %d reps; GB/s by min and median time\n", mib, cus, rounds, reps);
    std::sort(cases.begin(), cases.end(), [](const Case &x, const Case &y) {
        return x.bytes_per_call / *std::min_element(x.ms.begin(), x.ms.end()) >
               y.bytes_per_call / *std::min_element(y.ms.begin(), y.ms.end());
    });
    for (auto &c : cases) {
        std::vector<float> m = c.ms;
        std::sort(m.begin(), m.end());
        std::printf("%-40s best %7.1f GB/s  median %7.1f GB/s  (%.4f ms)\n", c.name.c_str(),
                    c.bytes_per_call / (m[0] * 1e-3) / 1e9, c.bytes_per_call / (m[m.size() / 2] * 1e-3) / 1e9, m[0]);
    }
    return 0;
}
