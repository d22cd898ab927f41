// reduce_kernels.hip — the per-hop reduce of the gradient-bucket ring on CDNA4 (gfx950).
//
// Replaces the elementwise MPI_SUM that MPICH applies inside MPI_Allreduce at the
// reference's data-plane call (src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28).
// Memory-bound vector add: no MFMA. Algorithmic HBM bytes per element = 3 * sizeof(T)
// (two reads, one write).
//
// Layout / mapping:
//   * one launch covers up to kMaxSegments independent (out, a, b, n) problems — the ring
//     issues one segment per concurrent ring — with blockIdx.y = segment;
//   * 256-thread workgroups (4 waves of 64), every lane moves 16 B per access
//     (global_load_dwordx4), UNROLL independent accesses per operand in flight per lane;
//   * grid-stride over 16-byte vectors, the grid capped at 8 workgroups per CU so the launch
//     fills all 256 CUs / 8 XCDs without a tail of tiny workgroups;
//   * the n mod V tail is done by the first lanes of the grid (one element each), so there is
//     no separate epilogue launch; misaligned buffers take a scalar grid-stride kernel.
//   * fp16 adds with v_pk_add_f16 (IEEE, round-to-nearest-even, denormals kept) — identical to
//     round_f16(float(a) + float(b)) because fp32 has >= 2*11+2 significand bits; bf16 adds in
//     fp32 and rounds once (v_cvt_pk_bf16_f32).
#include <hip/hip_runtime.h>

#include "common.h"

namespace ddl {
namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using f64x2 = double __attribute__((ext_vector_type(2)));
using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));
using h16x8 = _Float16 __attribute__((ext_vector_type(8)));
using f32x2 = float __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;

template <int DT>
struct Add;

template <>
struct Add<DDL_FLOAT> {
    using S = float;
    __device__ static u32x4 vec(u32x4 a, u32x4 b) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b));
    }
    __device__ static S one(S a, S b) { return a + b; }
};
template <>
struct Add<DDL_DOUBLE> {
    using S = double;
    __device__ static u32x4 vec(u32x4 a, u32x4 b) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(f64x2, a) + __builtin_bit_cast(f64x2, b));
    }
    __device__ static S one(S a, S b) { return a + b; }
};
template <>
struct Add<DDL_INT32> {  // two's-complement wrap-around
    using S = unsigned int;
    __device__ static u32x4 vec(u32x4 a, u32x4 b) { return a + b; }
    __device__ static S one(S a, S b) { return a + b; }
};
template <>
struct Add<DDL_INT64> {
    using S = unsigned long long;
    __device__ static u32x4 vec(u32x4 a, u32x4 b) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(u64x2, a) + __builtin_bit_cast(u64x2, b));
    }
    __device__ static S one(S a, S b) { return a + b; }
};
template <>
struct Add<DDL_UINT64> : Add<DDL_INT64> {};
template <>
struct Add<DDL_HALF> {
    using S = _Float16;
    __device__ static u32x4 vec(u32x4 a, u32x4 b) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(h16x8, a) + __builtin_bit_cast(h16x8, b));
    }
    __device__ static S one(S a, S b) { return a + b; }
};
template <>
struct Add<DDL_BFLOAT16> {
    using S = __bf16;
    __device__ static unsigned int add_pair(unsigned int a, unsigned int b) {
        // two bf16 per dword: widen exactly to fp32, add, round once to bf16 (RNE)
        float alo = __builtin_bit_cast(float, a << 16), ahi = __builtin_bit_cast(float, a & 0xffff0000u);
        float blo = __builtin_bit_cast(float, b << 16), bhi = __builtin_bit_cast(float, b & 0xffff0000u);
        __bf16 lo = (__bf16)(alo + blo), hi = (__bf16)(ahi + bhi);
        return (unsigned int)__builtin_bit_cast(unsigned short, lo) |
               ((unsigned int)__builtin_bit_cast(unsigned short, hi) << 16);
    }
    __device__ static u32x4 vec(u32x4 a, u32x4 b) {
        u32x4 r;
        r.x = add_pair(a.x, b.x);
        r.y = add_pair(a.y, b.y);
        r.z = add_pair(a.z, b.z);
        r.w = add_pair(a.w, b.w);
        return r;
    }
    __device__ static S one(S a, S b) { return (__bf16)((float)a + (float)b); }
};

typedef __attribute__((address_space(1))) void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

template <int VARIANT>
__device__ __forceinline__ u32x4 load_v(const u32x4 *p) {
    if constexpr (VARIANT == kNonTemporal) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int VARIANT>
__device__ __forceinline__ void store_v(u32x4 *p, u32x4 v) {
    if constexpr (VARIANT == kNonTemporal) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// out = a + b on 16-byte vectors. out may alias a or b (no __restrict__): every access of
// a lane touches only its own vectors, loads of an unrolled group precede its stores.
template <int DT, int VARIANT, int UNROLL>
__global__ void __launch_bounds__(kThreads) k_sum2_vec(SegTable t) {
    using A = Add<DT>;
    using S = typename A::S;
    constexpr int V = 16 / sizeof(S);
    const int seg = blockIdx.y;
    const u32x4 *a = static_cast<const u32x4 *>(t.a[seg]);
    const u32x4 *b = static_cast<const u32x4 *>(t.b[seg]);
    u32x4 *o = static_cast<u32x4 *>(t.out[seg]);
    const uint64_t n = t.n[seg];
    const uint64_t nv = n / V;
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    const uint64_t gid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    uint64_t i = gid;

    if constexpr (VARIANT == kLdsStage) {
        // Incoming operand b staged through LDS by LDS-DMA (global_load_lds_dwordx4): each wave
        // owns a private 1 KiB slot per unrolled access, lane l lands at slot + 16*l.
        __shared__ __attribute__((aligned(16))) u32x4 stage[UNROLL * kThreads];
        const int wave = threadIdx.x >> 6;
        for (; i + (uint64_t)(UNROLL - 1) * stride < nv; i += (uint64_t)UNROLL * stride) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                __builtin_amdgcn_global_load_lds((gptr_t)(b + i + (uint64_t)u * stride),
                                                 (lptr_t)(stage + u * kThreads + wave * 64), 16, 0, 0);
            u32x4 x[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) x[u] = a[i + (uint64_t)u * stride];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                o[i + (uint64_t)u * stride] = A::vec(x[u], stage[u * kThreads + threadIdx.x]);
        }
    } else {
        for (; i + (uint64_t)(UNROLL - 1) * stride < nv; i += (uint64_t)UNROLL * stride) {
            u32x4 x[UNROLL], y[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                x[u] = load_v<VARIANT>(a + i + (uint64_t)u * stride);
                y[u] = load_v<VARIANT>(b + i + (uint64_t)u * stride);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) store_v<VARIANT>(o + i + (uint64_t)u * stride, A::vec(x[u], y[u]));
        }
    }
    for (; i < nv; i += stride) o[i] = A::vec(a[i], b[i]);

    // tail: n mod V elements, one per lane of the first wave(s) of the grid
    const uint64_t rem = n - nv * V;
    if (gid < rem) {
        const uint64_t e = nv * V + gid;
        const S *as = reinterpret_cast<const S *>(t.a[seg]);
        const S *bs = reinterpret_cast<const S *>(t.b[seg]);
        S *os = reinterpret_cast<S *>(t.out[seg]);
        os[e] = A::one(as[e], bs[e]);
    }
}

// Misaligned buffers: element-granular grid-stride (correct for any alignment of T).
template <int DT>
__global__ void __launch_bounds__(kThreads) k_sum2_scalar(SegTable t) {
    using A = Add<DT>;
    using S = typename A::S;
    const int seg = blockIdx.y;
    const S *a = static_cast<const S *>(t.a[seg]);
    const S *b = static_cast<const S *>(t.b[seg]);
    S *o = static_cast<S *>(t.out[seg]);
    const uint64_t n = t.n[seg];
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
        o[i] = A::one(a[i], b[i]);
}

constexpr int kUnroll = 4;

template <int DT>
void launch_dt(const SegTable &t, hipStream_t stream, int variant, bool aligned, int blocks_x) {
    dim3 grid(blocks_x, t.count), block(kThreads);
    if (!aligned) {
        hipLaunchKernelGGL(k_sum2_scalar<DT>, grid, block, 0, stream, t);
        return;
    }
    switch (variant) {
        case kLdsStage:
            hipLaunchKernelGGL((k_sum2_vec<DT, kLdsStage, kUnroll>), grid, block, 0, stream, t);
            break;
        case kNonTemporal:
            hipLaunchKernelGGL((k_sum2_vec<DT, kNonTemporal, kUnroll>), grid, block, 0, stream, t);
            break;
        default:
            hipLaunchKernelGGL((k_sum2_vec<DT, kRegStream, kUnroll>), grid, block, 0, stream, t);
            break;
    }
}

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---- fusion pack / unpack --------------------------------------------------------------
constexpr int kPackBatch = 64;

struct PackTable {
    const char *src[kPackBatch];
    char *dst[kPackBatch];
    uint64_t start[kPackBatch + 1];  // byte offset of each segment's slot in the flat space
    uint64_t len[kPackBatch];        // bytes to move
    int count;
    int vec_ok;                      // every pointer/offset/length is 16-byte aligned
};

// Flat byte space [0, start[count]) covers all segments back to back; each thread moves
// 16-byte units (or single bytes when some segment is not 16-byte aligned) and finds its
// segment by binary search over start[].
__global__ void __launch_bounds__(kThreads) k_copy_segments(PackTable t) {
    const uint64_t total = t.start[t.count];
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    const uint64_t gid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t unit = t.vec_ok ? 16 : 1;
    for (uint64_t u = gid; u * unit < total; u += stride) {
        const uint64_t off = u * unit;
        int lo = 0, hi = t.count - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (t.start[mid] <= off) lo = mid; else hi = mid - 1;
        }
        const uint64_t local = off - t.start[lo];
        if (local >= t.len[lo]) continue;
        if (t.vec_ok) {
            *reinterpret_cast<u32x4 *>(t.dst[lo] + local) =
                *reinterpret_cast<const u32x4 *>(t.src[lo] + local);
        } else {
            t.dst[lo][local] = t.src[lo][local];
        }
    }
}

int g_cu_count = 0;

}  // namespace

int device_cu_count() {
    if (g_cu_count == 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            g_cu_count = cus;
        else
            g_cu_count = 256;
    }
    return g_cu_count;
}

void launch_sum2(const SegTable &t, int dtype, hipStream_t stream, int variant) {
    DDL_REQUIRE(t.count >= 1 && t.count <= kMaxSegments, DDL_STATUS_INVALID_ARGUMENT,
                "segment count " << t.count << " outside [1, " << kMaxSegments << "]");
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    uint64_t max_n = 0;
    bool aligned = true;
    for (int s = 0; s < t.count; ++s) {
        if (t.n[s] == 0) continue;
        DDL_REQUIRE(t.a[s] && t.b[s] && t.out[s], DDL_STATUS_INVALID_ARGUMENT, "null buffer in segment " << s);
        max_n = t.n[s] > max_n ? t.n[s] : max_n;
        aligned = aligned && aligned16(t.a[s]) && aligned16(t.b[s]) && aligned16(t.out[s]);
    }
    if (max_n == 0) return;
    const uint64_t per_block = aligned ? (uint64_t)kThreads * kUnroll * (16 / es) : (uint64_t)kThreads * 4;
    const uint64_t cap = (uint64_t)device_cu_count() * 8 / (uint64_t)t.count;
    uint64_t blocks = (max_n + per_block - 1) / per_block;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    switch (dtype) {
        case DDL_FLOAT: launch_dt<DDL_FLOAT>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_DOUBLE: launch_dt<DDL_DOUBLE>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_INT32: launch_dt<DDL_INT32>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_INT64: launch_dt<DDL_INT64>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_UINT64: launch_dt<DDL_UINT64>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_HALF: launch_dt<DDL_HALF>(t, stream, variant, aligned, (int)blocks); break;
        case DDL_BFLOAT16: launch_dt<DDL_BFLOAT16>(t, stream, variant, aligned, (int)blocks); break;
        default: fail(DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype");
    }
    DDL_HIP(hipGetLastError());
}

namespace {
void launch_copy(const char *const *srcs, char *const *dsts, const size_t *bytes, int count,
                 hipStream_t stream, bool to_flat_dst, char *flat) {
    (void)to_flat_dst;
    (void)flat;
    for (int base = 0; base < count; base += kPackBatch) {
        PackTable t;
        t.count = count - base < kPackBatch ? count - base : kPackBatch;
        uint64_t off = 0;
        bool vec_ok = true;
        for (int i = 0; i < t.count; ++i) {
            t.src[i] = srcs[base + i];
            t.dst[i] = dsts[base + i];
            t.len[i] = bytes[base + i];
            t.start[i] = off;
            off += (bytes[base + i] + 15) & ~uint64_t(15);
            vec_ok = vec_ok && aligned16(t.src[i]) && aligned16(t.dst[i]) && (t.len[i] % 16 == 0);
        }
        t.start[t.count] = off;
        t.vec_ok = vec_ok ? 1 : 0;
        if (off == 0) continue;
        const uint64_t units = vec_ok ? off / 16 : off;
        uint64_t blocks = (units + kThreads - 1) / kThreads;
        const uint64_t cap = (uint64_t)device_cu_count() * 8;
        if (blocks > cap) blocks = cap;
        hipLaunchKernelGGL(k_copy_segments, dim3((unsigned)blocks), dim3(kThreads), 0, stream, t);
        DDL_HIP(hipGetLastError());
    }
}
}  // namespace

// Fused layout: segment i occupies [off_i, off_i + bytes_i) of dst with off_i the running sum
// of the 256-byte-rounded sizes of the segments before it (FusionLayout in engine.cpp).
void launch_pack(void *dst, const void *const *srcs, const size_t *bytes, int count, hipStream_t stream) {
    if (count <= 0) return;
    const char **s = new const char *[count];
    char **d = new char *[count];
    uint64_t off = 0;
    for (int i = 0; i < count; ++i) {
        s[i] = static_cast<const char *>(srcs[i]);
        d[i] = static_cast<char *>(dst) + off;
        off += (bytes[i] + 255) & ~uint64_t(255);
    }
    try {
        launch_copy(s, d, bytes, count, stream, true, static_cast<char *>(dst));
    } catch (...) {
        delete[] s;
        delete[] d;
        throw;
    }
    delete[] s;
    delete[] d;
}

void launch_unpack(void *const *dsts, const void *src, const size_t *bytes, int count, hipStream_t stream) {
    if (count <= 0) return;
    const char **s = new const char *[count];
    char **d = new char *[count];
    uint64_t off = 0;
    for (int i = 0; i < count; ++i) {
        s[i] = static_cast<const char *>(src) + off;
        d[i] = static_cast<char *>(dsts[i]);
        off += (bytes[i] + 255) & ~uint64_t(255);
    }
    try {
        launch_copy(s, d, bytes, count, stream, false, nullptr);
    } catch (...) {
        delete[] s;
        delete[] d;
        throw;
    }
    delete[] s;
    delete[] d;
}

}  // namespace ddl
