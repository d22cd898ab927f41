// tools/reduce_policy_tune.hip — cache-policy bits of the two-input reduce (not shipped).
// out = a + b (fp32) with the shipped mapping (128 lanes = one 2 KiB tile per workgroup, one
// 16-byte vector per lane and operand), loads and stores issued as raw buffer operations whose
// aux word sets the gfx950 cache bits per access (bit 0 sc0, bit 1 nt, bit 4 sc1; the guide's
// store table: plain / sc0 / nt keep the line in the XCD's L2, sc1 / sc0 sc1 drop it). Compared
// with the shipped kernel's __builtin_nontemporal_* accesses. 3 rotating buffer sets (beyond the
// 256 MiB Infinity Cache), interleaved rounds.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/reduce_policy_tune.hip -o tools/bin/reduce_policy_tune
//   ./reduce_policy_tune [MiB=256] [rounds=5]
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
constexpr int T = 128;
constexpr int kRsrcWord3 = 0x00020000;  // raw 32-bit buffer (CK's gfx9 third dword)

// the shipped form: builtin non-temporal loads and store
__global__ void __launch_bounds__(T) k_builtin_nt(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    const size_t i = (size_t)blockIdx.x * T + threadIdx.x;
    if (i < nv) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), o + i);
}

// buffer form: one resource per tile (scalar base = the tile), 16-byte lane offsets
template <int LA, int LB, int ST>
__global__ void __launch_bounds__(T) k_buffer(f4 *o, const f4 *a, const f4 *b, size_t nv) {
    const size_t base = (size_t)blockIdx.x * T;
    const int bytes = (int)((nv - base < (size_t)T ? nv - base : (size_t)T) * 16);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(a + base), 0, bytes, kRsrcWord3);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(b + base), 0, bytes, kRsrcWord3);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(o + base, 0, bytes, kRsrcWord3);
    const int off = threadIdx.x * 16;  // out of range lanes read 0 and drop their store
    const u4 x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, LA);
    const u4 y = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, LB);
    const u4 r = __builtin_bit_cast(u4, __builtin_bit_cast(f4, x) + __builtin_bit_cast(f4, y));
    __builtin_amdgcn_raw_buffer_store_b128(r, ro, off, 0, ST);
}

struct Variant {
    std::string name;
    void (*launch)(f4 *, const f4 *, const f4 *, size_t, hipStream_t);
};

template <int LA, int LB, int ST>
void launch_buffer(f4 *o, const f4 *a, const f4 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL((k_buffer<LA, LB, ST>), dim3((unsigned)((nv + T - 1) / T)), dim3(T), 0, s, o, a, b, nv);
}

void launch_builtin(f4 *o, const f4 *a, const f4 *b, size_t nv, hipStream_t s) {
    hipLaunchKernelGGL(k_builtin_nt, dim3((unsigned)((nv + T - 1) / T)), dim3(T), 0, s, o, a, b, nv);
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
    // aux: 1 = sc0, 2 = nt, 16 = sc1
    const std::vector<Variant> vs = {
        {"builtin nt loads + nt store (shipped)", launch_builtin},
        {"buffer ld nt,nt st nt", launch_buffer<2, 2, 2>},
        {"buffer ld nt,nt st plain", launch_buffer<2, 2, 0>},
        {"buffer ld nt,nt st sc1", launch_buffer<2, 2, 16>},
        {"buffer ld nt,nt st sc0 sc1", launch_buffer<2, 2, 17>},
        {"buffer ld nt,nt st nt sc1", launch_buffer<2, 2, 18>},
        {"buffer ld nt,nt st nt sc0 sc1", launch_buffer<2, 2, 19>},
        {"buffer ld nt,nt st sc0", launch_buffer<2, 2, 1>},
        {"buffer ld sc0 sc1 x2, st nt", launch_buffer<17, 17, 2>},
        {"buffer ld nt sc1 x2, st nt", launch_buffer<18, 18, 2>},
        {"buffer ld nt sc1 x2, st nt sc1", launch_buffer<18, 18, 18>},
        {"buffer ld plain x2, st sc1", launch_buffer<0, 0, 16>},
        {"buffer ld plain x2, st plain", launch_buffer<0, 0, 0>},
        {"buffer ld plain x2, st sc0 sc1", launch_buffer<0, 0, 17>},
    };
    std::vector<std::vector<float>> ms(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const Variant &v, int set) { v.launch(bufs[3 * set + 2], bufs[3 * set], bufs[3 * set + 1], nv, s); };
    // correctness of every variant against the shipped one on small random data
    {
        const size_t tn = 4096 * 16 + 3;  // vectors (ragged last tile)
        std::vector<float> ha(tn * 4), hb(tn * 4), ref(tn * 4), got(tn * 4);
        for (size_t i = 0; i < ha.size(); ++i) {
            ha[i] = (float)((i * 2654435761u) % 1000) * 0.37f;
            hb[i] = (float)((i * 40503u) % 777) * -1.1f;
        }
        CK(hipMemcpy(bufs[0], ha.data(), tn * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(bufs[1], hb.data(), tn * 16, hipMemcpyHostToDevice));
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipMemset(bufs[2], 0xff, (tn + T) * 16));
            vs[v].launch(bufs[2], bufs[0], bufs[1], tn, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(v == 0 ? ref.data() : got.data(), bufs[2], tn * 16, hipMemcpyDeviceToHost));
            if (v && std::memcmp(ref.data(), got.data(), tn * 16) != 0) {
                std::printf("MISMATCH: %s\n", vs[v].name.c_str());
                return 1;
            }
        }
    }
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
    std::printf("# fp32 out = a + b, %zu MiB per operand, 128-lane tiles, %d rounds x %d reps, %d rotating sets; GB/s = 3 x bytes / t\n",
                mib, rounds, reps, sets);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = ms[v];
        std::sort(x.begin(), x.end());
        std::printf("%-40s best %7.1f GB/s  median %7.1f GB/s  (%.4f ms)\n", vs[v].name.c_str(), 3.0 * bytes / (x[0] * 1e6),
                    3.0 * bytes / (x[x.size() / 2] * 1e6), x[0]);
    }
    return 0;
}
