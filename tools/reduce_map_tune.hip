// tools/reduce_map_tune.hip — workgroup -> tile mappings of the two-input reduce (not shipped).
// acc = acc + in (fp32, in place, as the N=1 bench and the ring step run it) over 256 MiB with
// the shipped cache policy (non-temporal loads and stores, raw buffer accesses), varying only
// which bytes a workgroup moves:
//   shipped      one 2 KiB tile per 128-lane workgroup, tile = blockIdx (dispatch order)
//   xcd-R        workgroups are dealt round-robin to the 8 XCDs; tile remapped so each XCD
//                sweeps runs of R consecutive tiles (R = 1: XCD x takes x, x+8, ...: identity)
//   u2-near      two neighbouring tiles per workgroup (4 loads in flight per lane, then 2 stores)
//   u2-far       tiles b and b + T/2 per workgroup (two DRAM regions per workgroup)
//   lanes64      one 1 KiB tile per 64-lane workgroup
//   outofplace   the shipped mapping writing a third buffer
// 3 rotating buffer sets (beyond the 256 MiB Infinity Cache), interleaved rounds.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/reduce_map_tune.hip -o tools/bin/reduce_map_tune
//   ./reduce_map_tune [MiB=256] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
constexpr int kRsrcWord3 = 0x00020000;
constexpr int kNt = 2;

template <int LANES>
__device__ __forceinline__ void tile_op(f4 *o, const f4 *a, const f4 *b, size_t nv, size_t tile) {
    const size_t base = tile * LANES;
    if (base >= nv) return;
    const int bytes = (int)((nv - base < (size_t)LANES ? nv - base : (size_t)LANES) * 16);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(a + base), 0, bytes, kRsrcWord3);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(b + base), 0, bytes, kRsrcWord3);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(o + base, 0, bytes, kRsrcWord3);
    const int off = threadIdx.x * 16;
    const u4 x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, kNt);
    const u4 y = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kNt);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, __builtin_bit_cast(f4, x) + __builtin_bit_cast(f4, y)),
                                           ro, off, 0, kNt);
}

template <int LANES>
__global__ void __launch_bounds__(LANES) k_shipped(f4 *o, const f4 *a, const f4 *b, size_t nv, size_t) {
    tile_op<LANES>(o, a, b, nv, blockIdx.x);
}

// XCD-aware: blockIdx b runs on XCD b % 8; its j-th workgroup (j = b / 8) takes tile
// (j / R) * 8R + xcd * R + j % R, i.e. runs of R consecutive tiles per XCD
template <int R>
__global__ void __launch_bounds__(128) k_xcd(f4 *o, const f4 *a, const f4 *b, size_t nv, size_t ntiles) {
    const size_t bidx = blockIdx.x, x = bidx % 8, j = bidx / 8;
    size_t tile = (j / R) * 8 * R + x * R + j % R;
    if (ntiles % (8 * R) && bidx >= ntiles / (8 * R) * (8 * R)) tile = bidx;  // ragged tail: identity
    tile_op<128>(o, a, b, nv, tile);
}

template <bool FAR>
__global__ void __launch_bounds__(128) k_u2(f4 *o, const f4 *a, const f4 *b, size_t nv, size_t ntiles) {
    const size_t half = (ntiles + 1) / 2;
    const size_t t0 = FAR ? blockIdx.x : 2 * (size_t)blockIdx.x, t1 = FAR ? blockIdx.x + half : t0 + 1;
    u4 x[2], y[2];
    int bytes[2];
    __amdgpu_buffer_rsrc_t ro[2];
    const int off = threadIdx.x * 16;
    const size_t ts[2] = {t0, t1};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const size_t base = ts[u] * 128;
        bytes[u] = base >= nv ? 0 : (int)((nv - base < 128 ? nv - base : 128) * 16);
        const size_t bb = base >= nv ? 0 : base;
        const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(a + bb), 0, bytes[u], kRsrcWord3);
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(b + bb), 0, bytes[u], kRsrcWord3);
        ro[u] = __builtin_amdgcn_make_buffer_rsrc(o + bb, 0, bytes[u], kRsrcWord3);
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, kNt);
        y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kNt);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u4, __builtin_bit_cast(f4, x[u]) + __builtin_bit_cast(f4, y[u])), ro[u], off, 0, kNt);
}

struct Variant {
    std::string name;
    void (*launch)(f4 *, const f4 *, const f4 *, size_t, hipStream_t);
    bool inplace;
};

template <int LANES>
void l_shipped(f4 *o, const f4 *a, const f4 *b, size_t nv, hipStream_t s) {
    const size_t nt = (nv + LANES - 1) / LANES;
    hipLaunchKernelGGL(k_shipped<LANES>, dim3((unsigned)nt), dim3(LANES), 0, s, o, a, b, nv, nt);
}
template <int R>
void l_xcd(f4 *o, const f4 *a, const f4 *b, size_t nv, hipStream_t s) {
    const size_t nt = (nv + 127) / 128;
    hipLaunchKernelGGL(k_xcd<R>, dim3((unsigned)nt), dim3(128), 0, s, o, a, b, nv, nt);
}
template <bool FAR>
void l_u2(f4 *o, const f4 *a, const f4 *b, size_t nv, hipStream_t s) {
    const size_t nt = (nv + 127) / 128;
    hipLaunchKernelGGL(k_u2<FAR>, dim3((unsigned)((nt + 1) / 2)), dim3(128), 0, s, o, a, b, nv, nt);
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::atol(argv[1]) : 256;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const int reps = 8, sets = 3;
    const size_t bytes = mib << 20, nv = bytes / 16;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<f4 *> bufs(3 * sets);
    for (auto &p : bufs) {
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 0, bytes));
    }
    const std::vector<Variant> vs = {
        {"shipped (128 lanes, tile = blockIdx)", l_shipped<128>, true},
        {"xcd-1 (identity check)", l_xcd<1>, true},
        {"xcd-4 (8 KiB runs per XCD)", l_xcd<4>, true},
        {"xcd-16 (32 KiB runs per XCD)", l_xcd<16>, true},
        {"xcd-256 (512 KiB runs per XCD)", l_xcd<256>, true},
        {"u2-near", l_u2<false>, true},
        {"u2-far", l_u2<true>, true},
        {"lanes64 (1 KiB tiles)", l_shipped<64>, true},
        {"shipped, out of place", l_shipped<128>, false},
    };
    // correctness of every mapping against the shipped one (ragged size)
    {
        const size_t tn = 4096 * 64 + 77;
        std::vector<float> ha(tn * 4), hb(tn * 4), ref(tn * 4), got(tn * 4);
        for (size_t i = 0; i < ha.size(); ++i) {
            ha[i] = (float)((i * 2654435761u) % 1000) * 0.37f;
            hb[i] = (float)((i * 40503u) % 777) * -1.1f;
        }
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipMemcpy(bufs[0], ha.data(), tn * 16, hipMemcpyHostToDevice));
            CK(hipMemcpy(bufs[1], hb.data(), tn * 16, hipMemcpyHostToDevice));
            CK(hipMemset(bufs[2], 0xff, tn * 16));
            f4 *out = vs[v].inplace ? bufs[0] : bufs[2];
            vs[v].launch(out, bufs[0], bufs[1], tn, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(v == 0 ? ref.data() : got.data(), out, tn * 16, hipMemcpyDeviceToHost));
            if (v && std::memcmp(ref.data(), got.data(), tn * 16) != 0) {
                std::printf("MISMATCH: %s\n", vs[v].name.c_str());
                return 1;
            }
        }
    }
    std::vector<std::vector<float>> ms(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const Variant &v, int set) {
        f4 *a = bufs[3 * set], *b = bufs[3 * set + 1];
        v.launch(v.inplace ? a : bufs[3 * set + 2], a, b, nv, s);
    };
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int w = 0; w < 3; ++w) run(vs[v], w);
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) run(vs[v], i % sets);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / reps);
        }
    }
    std::printf("# fp32 acc = acc + in, %zu MiB, nt loads + nt stores, %d rounds x %d reps, %d rotating sets; GB/s = 3 x bytes / t\n",
                mib, rounds, reps, sets);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = ms[v];
        std::sort(x.begin(), x.end());
        std::printf("%-40s best %7.1f GB/s  median %7.1f GB/s  (%.4f ms)\n", vs[v].name.c_str(), 3.0 * bytes / (x[0] * 1e6),
                    3.0 * bytes / (x[x.size() / 2] * 1e6), x[0]);
    }
    return 0;
}
