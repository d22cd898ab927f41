// reduce_kernels.hip — the per-hop reduce of the gradient-bucket ring on CDNA4 (gfx950).
//
// Replaces the elementwise MPI_SUM that MPICH applies inside MPI_Allreduce at the
// reference's data-plane call (src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28).
// Memory-bound vector add: no MFMA. Algorithmic HBM bytes per element = 3 * sizeof(T)
// (two reads, one write).
//
// Layout / mapping (measured in profiles/r01/reduce_tune_*.txt and
// profiles/r02/reduce_policy/):
//   * one workgroup = 128 lanes = one 2 KiB tile of each operand (DDL_REDUCE_THREADS): lane l
//     moves bytes [16l, 16l+16) of the tile with one buffer_load_dwordx4 per operand and one
//     buffer_store_dwordx4 (one descriptor per operand tile). The grid has one workgroup per
//     tile (no grid-stride loop): the dispatcher hands out workgroups in order, so the tiles in
//     flight form one compact address window and every HBM page opened is drained by
//     neighbouring workgroups. This measured 5.9-6.1 TB/s vs 4.6 for an 8-workgroups-per-CU
//     grid-stride loop.
//   * up to kMaxSegments independent (out, a, b, n) problems per launch (one per ring):
//     blockIdx.y = segment, workgroups past a segment's last tile exit at once.
//   * cache bits per access (default_variant by bucket size): non-temporal loads of the
//     once-read operands, and write-through (sc0 sc1) stores of out below 256 MiB — the line
//     leaves the XCD's L2 at once instead of waiting there to be written back (+3-14 % at
//     32-128 MiB); non-temporal stores from 256 MiB.
//   * the n mod V tail (V = elements per 16 B) is done by the lanes of the last tile, one
//     element each: no epilogue launch. Misaligned buffers take a scalar grid-stride kernel.
//   * fp16 adds with v_pk_add_f16 (IEEE, round-to-nearest-even, denormals kept) — identical to
//     round_f16(float(a) + float(b)) because fp32 has >= 2*11+2 significand bits; bf16 adds in
//     fp32 and rounds once (v_cvt_pk_bf16_f32).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace ddl {
namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using f64x2 = double __attribute__((ext_vector_type(2)));
using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));
using h16x8 = _Float16 __attribute__((ext_vector_type(8)));

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

template <bool NT>
__device__ __forceinline__ u32x4 load_v(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// gfx950 buffer-access cache bits (the aux operand of the raw buffer builtins) and the third
// descriptor dword of a raw 32-bit buffer
constexpr int kAuxSc0 = 1, kAuxNt = 2, kAuxSc1 = 16;
constexpr int kRsrcWord3 = 0x00020000;
constexpr int store_aux(int variant) {
    return ((variant & kNtStore) ? kAuxNt : 0) | ((variant & kWtStore) ? (kAuxSc0 | kAuxSc1) : 0);
}

// out = a + b, one tile per workgroup. out may alias a or b (no __restrict__): each lane
// reads its own 16 bytes of a and b before it writes the same 16 bytes of out.
template <int DT, int VARIANT, int THREADS>
__global__ void __launch_bounds__(THREADS) k_sum2_tile(SegTable t) {
    using A = Add<DT>;
    using S = typename A::S;
    constexpr uint64_t V = 16 / sizeof(S);
    constexpr uint64_t kTileVec = THREADS;  // 16-byte vectors per tile
    const int seg = blockIdx.y;
    const uint64_t n = t.n[seg];
    const uint64_t nv = n / V;
    const uint64_t tile = blockIdx.x;
    const uint64_t i = tile * kTileVec + threadIdx.x;
    const u32x4 *a = static_cast<const u32x4 *>(t.a[seg]);
    const u32x4 *b = static_cast<const u32x4 *>(t.b[seg]);
    u32x4 *o = static_cast<u32x4 *>(t.out[seg]);

    if constexpr ((VARIANT & kLdsStageB) != 0) {
        // operand b through LDS by LDS-DMA: each wave owns a 1 KiB slot, lane l lands at 16*l
        __shared__ __attribute__((aligned(16))) u32x4 stage[THREADS];
        if (tile * kTileVec > nv) return;  // (uniform) past this segment's tiles
        const int wave = threadIdx.x >> 6;
        if (i < nv)
            __builtin_amdgcn_global_load_lds((gptr_t)(b + i), (lptr_t)(stage + wave * 64), 16, 0, 0);
        u32x4 x = i < nv ? load_v<(VARIANT & kNtLoadA) != 0>(a + i) : u32x4{0, 0, 0, 0};
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (i < nv) {
            u32x4 r = A::vec(x, stage[threadIdx.x]);
            if constexpr ((VARIANT & kNtStore) != 0) __builtin_nontemporal_store(r, o + i);
            else o[i] = r;
        }
    } else {
        // raw buffer accesses, one descriptor per operand tile: the aux word carries the cache
        // bits per access (nt / sc0 sc1 write-through), lanes past the tile's last vector read 0
        // and drop their store (num_records), and each lane's address is a 32-bit offset
        const uint64_t base = tile * kTileVec;
        if (base < nv) {
            const int bytes = (int)((nv - base < kTileVec ? nv - base : kTileVec) * 16);
            const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(a + base), 0, bytes, kRsrcWord3);
            const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(b + base), 0, bytes, kRsrcWord3);
            const auto ro = __builtin_amdgcn_make_buffer_rsrc(o + base, 0, bytes, kRsrcWord3);
            const int off = (int)threadIdx.x * 16;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, (VARIANT & kNtLoadA) ? kAuxNt : 0);
            const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, (VARIANT & kNtLoadB) ? kAuxNt : 0);
            __builtin_amdgcn_raw_buffer_store_b128(A::vec(x, y), ro, off, 0, store_aux(VARIANT));
        }
    }
    // tail: the n mod V elements past the last full vector, one per lane of the tile holding nv
    const uint64_t rem = n - nv * V;
    if (rem && tile == nv / kTileVec && threadIdx.x < rem) {
        const uint64_t e = nv * V + threadIdx.x;
        const S *as = reinterpret_cast<const S *>(t.a[seg]);
        const S *bs = reinterpret_cast<const S *>(t.b[seg]);
        S *os = reinterpret_cast<S *>(t.out[seg]);
        os[e] = A::one(as[e], bs[e]);
    }
}

// Run form of the two-input reduce (measurement variant kRunForm, r05): a 128-lane workgroup owns
// U consecutive 2 KiB tiles; each lane loads its U vectors of a, then its U vectors of b, then
// stores the U sums — so a workgroup streams one operand at a time in U * 2 KiB runs (the fold's
// run form, §5.2). Tail elements as k_sum2_tile's (the lanes of the run holding nv).
template <int DT, int VARIANT, int U>
__global__ void __launch_bounds__(128) k_sum2_run(SegTable t) {
    using A = Add<DT>;
    using S = typename A::S;
    constexpr uint64_t V = 16 / sizeof(S);
    constexpr uint64_t kRun = 128ull * U;  // 16-byte vectors per run
    const int seg = blockIdx.y;
    const uint64_t n = t.n[seg];
    const uint64_t nv = n / V;
    const uint64_t base = (uint64_t)blockIdx.x * kRun;
    const u32x4 *a = static_cast<const u32x4 *>(t.a[seg]);
    const u32x4 *b = static_cast<const u32x4 *>(t.b[seg]);
    u32x4 *o = static_cast<u32x4 *>(t.out[seg]);
    if (base < nv) {
        const int bytes = (int)((nv - base < kRun ? nv - base : kRun) * 16);
        const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(a + base), 0, bytes, kRsrcWord3);
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(b + base), 0, bytes, kRsrcWord3);
        const auto ro = __builtin_amdgcn_make_buffer_rsrc(o + base, 0, bytes, kRsrcWord3);
        const int off = (int)threadIdx.x * 16;
        u32x4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, off + u * 2048, 0, (VARIANT & kNtLoadA) ? kAuxNt : 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, off + u * 2048, 0, (VARIANT & kNtLoadB) ? kAuxNt : 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(A::vec(x[u], y[u]), ro, off + u * 2048, 0, store_aux(VARIANT));
    }
    const uint64_t rem = n - nv * V;
    if (rem && blockIdx.x == nv / kRun && threadIdx.x < rem) {
        const uint64_t e = nv * V + threadIdx.x;
        const S *as = reinterpret_cast<const S *>(t.a[seg]);
        const S *bs = reinterpret_cast<const S *>(t.b[seg]);
        S *os = reinterpret_cast<S *>(t.out[seg]);
        os[e] = A::one(as[e], bs[e]);
    }
}

// ---- N-input fold (direct schedule) --------------------------------------------------------
// Accumulator type: fp32 for fp16/bf16 (one rounding at the end), the element type otherwise.
template <int DT>
struct Acc {
    using S = typename Add<DT>::S;
    using T = S;
    __device__ static T widen(S x) { return x; }
    __device__ static S narrow(T x) { return x; }
    __device__ static T add(T a, T b) { return Add<DT>::one(a, b); }
};
template <>
struct Acc<DDL_HALF> {
    using T = float;
    __device__ static T widen(_Float16 x) { return (float)x; }
    __device__ static _Float16 narrow(T x) { return (_Float16)x; }
    __device__ static T add(T a, T b) { return a + b; }
};
template <>
struct Acc<DDL_BFLOAT16> {
    using T = float;
    __device__ static T widen(__bf16 x) { return (float)x; }
    __device__ static __bf16 narrow(T x) { return (__bf16)x; }
    __device__ static T add(T a, T b) { return a + b; }
};

// Sum of the K values w[0..K-1] (inputs in order x_0..x_{K-1}) in FoldOrder ORDER; every index
// is a compile-time constant after unrolling. Half types always fold left in fp32 (one rounding
// at the end), so ORDER only changes fp32 / fp64 (integers wrap: any order is the same sum).
template <int DT, int K, int ORDER>
__device__ __forceinline__ typename Acc<DT>::T fold_values(typename Acc<DT>::T *w) {
    using A = Acc<DT>;
    if constexpr (ORDER == kFoldBinomial) {
#pragma unroll
        for (int m = 1; m < K; m *= 2)
#pragma unroll
            for (int t = 0; t + m < K; t += 2 * m) w[t] = A::add(w[t], w[t + m]);
        return w[0];
    } else if constexpr (ORDER == kFoldMpichTree) {
        constexpr int pof2 = K >= 16 ? 16 : K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
        constexpr int rem = K - pof2;
        typename A::T leaf[pof2];
#pragma unroll
        for (int t = 0; t < pof2; ++t) leaf[t] = t < rem ? A::add(w[2 * t], w[2 * t + 1]) : w[t + rem];
#pragma unroll
        for (int m = 1; m < pof2; m *= 2)
#pragma unroll
            for (int t = 0; t < pof2; t += 2 * m) leaf[t] = A::add(leaf[t], leaf[t + m]);
        return leaf[0];
    } else {
#pragma unroll
        for (int k = 1; k < K; ++k) w[0] = A::add(w[0], w[k]);
        return w[0];
    }
}

// Lanes per workgroup (one tile of kReduceThreads x 16 B) of the two-input reduce: 128 (2 KiB
// tiles) measured 6.72-6.77 TB/s vs 6.37-6.55 with 256 lanes on the N=1 bench (256 MiB fp32, 3
// rotating sets, interleaved rounds); 64 lanes were slower too.
constexpr int kReduceThreads = 128;

// Fold cache policy (FV bits): 1 non-temporal loads, 2 non-temporal store, 4 write-through
// (sc0 sc1) store. Launches of more than 4 MiB per input stream every input once: non-temporal
// loads, and the output written through (it leaves the XCD's L2 at once; r03 tools/fold_tune.hip
// at 32 MiB, 8 inputs: 6.48-6.51 TB/s vs 6.35-6.36 all-nt, the r02 policy). Up to 4 MiB per input
// (the operands of a 2 MiB slice, where RCCL has just written the received data) read through the
// caches. r05 interleaved A/B of plain (4) vs non-temporal (5) loads, P = 8, one fold per launch,
// operands cache-resident / HBM-resident (tools/fold_batch_policy_ab.py, profiles/r05/s5/):
// 2 MiB fp16 3.7 / 5.7 us (4) vs 4.8 / 5.4 (5); 3 MiB fp32 4.0 / 7.3 vs 5.6 / 7.0; 4 MiB 4.8 / 8.8
// vs 5.7 / 8.1 — and from 5 MiB on the non-temporal loads win both ways (5 MiB 9.5 / 12.0 vs
// 8.6 / 10.9; 8 MiB 12.8 / 15.5 vs 12.0 / 14.0; 12 MiB 18.3 / 23.2 vs 16.8 / 20.8). r02-r04 split at
// 8 MiB. A batched launch (FoldBatch) goes by its summed bytes per input: 8 chunks of 2 MiB read
// non-temporally (26.2 vs 28.9 us from HBM, 23.3 vs 23.9 cache-resident).
int fold_variant(size_t chunk_bytes) { return chunk_bytes <= (4u << 20) ? 4 : 5; }
// ddl_testing_fold_variant: forces the policy (4 or 5; -1 = fold_variant's rule) for A/Bs
std::atomic<int> g_fold_variant{-1};

// One 2 KiB tile of the output per 128-lane workgroup: each lane folds its 16 bytes across a
// and the nb received inputs, one buffer_load_dwordx4 per input through one descriptor per input
// tile (32-bit lane offsets, the cache bits in each access's aux word; lanes past the tile's last
// vector read 0 and drop their store) — the two-input reduce's mapping. All NB + 1 loads are in
// flight before the first add. HBM bytes per element: (nb + 2) * sizeof(T).
// NB (received inputs) is a template parameter: every load is unconditional (a runtime "load or
// skip" per input makes hipcc wait vmcnt(0) per input).
constexpr int kFoldThreads = 128;
template <int DT, int NB, int FV, int ORDER>
__global__ void __launch_bounds__(kFoldThreads) k_sumN_tile(FoldBatch fb) {
    const SegTableN &t = fb.t[blockIdx.y];  // (uniform: the problem's table stays in the kernarg segment)
    constexpr uint64_t kTileVec = kFoldThreads;
    using A = Acc<DT>;
    using S = typename Add<DT>::S;
    using T = typename A::T;
    constexpr int V = 16 / sizeof(S);
    constexpr int kLoadAux = (FV & 1) ? kAuxNt : 0;
    constexpr int kStoreAux = ((FV & 2) ? kAuxNt : 0) | ((FV & 4) ? (kAuxSc0 | kAuxSc1) : 0);
    const uint64_t nv = t.n / V;
    const uint64_t base = (uint64_t)blockIdx.x * kTileVec;
    if (base < nv) {
        const int bytes = (int)((nv - base < kTileVec ? nv - base : kTileVec) * 16);
        const int off = (int)threadIdx.x * 16;
        u32x4 raw[NB + 1];
        raw[0] = __builtin_amdgcn_raw_buffer_load_b128(
            __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(static_cast<const u32x4 *>(t.a) + base), 0, bytes,
                                              kRsrcWord3),
            off, 0, kLoadAux);
#pragma unroll
        for (int k = 0; k < NB; ++k)
            raw[k + 1] = __builtin_amdgcn_raw_buffer_load_b128(
                __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(static_cast<const u32x4 *>(t.b[k]) + base), 0,
                                                  bytes, kRsrcWord3),
                off, 0, kLoadAux);
        u32x4 res;
        S *rs = reinterpret_cast<S *>(&res);
#pragma unroll
        for (int e = 0; e < V; ++e) {
            T w[NB + 1];
#pragma unroll
            for (int k = 0; k <= NB; ++k) w[k] = A::widen(reinterpret_cast<const S *>(&raw[k])[e]);
            rs[e] = A::narrow(fold_values<DT, NB + 1, ORDER>(w));
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            res, __builtin_amdgcn_make_buffer_rsrc(static_cast<u32x4 *>(t.out) + base, 0, bytes, kRsrcWord3), off, 0,
            kStoreAux);
    }
    const uint64_t rem = t.n - nv * V;
    if (rem && blockIdx.x == nv / kTileVec && threadIdx.x < rem) {
        const uint64_t e = nv * V + threadIdx.x;
        T w[NB + 1];
        w[0] = A::widen(static_cast<const S *>(t.a)[e]);
#pragma unroll
        for (int k = 0; k < NB; ++k) w[k + 1] = A::widen(static_cast<const S *>(t.b[k])[e]);
        static_cast<S *>(t.out)[e] = A::narrow(fold_values<DT, NB + 1, ORDER>(w));
    }
}

// ---- run form of the fold (large chunks) ----------------------------------------------------
// The tile form above has every workgroup read one 2 KiB tile of all NB + 1 inputs at once, so
// the chip streams NB + 2 address streams in lock step — and HBM delivers less the more streams
// are live (tools/stream_mix.hip, DESIGN §5.2: 6.1 TB/s for a 9-stream 8:1 mix). Here a
// workgroup owns kRunTiles consecutive tiles (a 16 KiB run of every input) and walks the inputs
// one at a time: kRunTiles loads per lane from input k in flight, folded in, then input k + 1 —
// each workgroup streams one input at a time in 16 KiB runs (6.6-6.7 TB/s for the same mix in the
// harness). The addition order is the same as fold_values': the MPICH tree is evaluated depth
// first over its leaves (left subtree, right subtree, left + right), so at most log2(pof2) + 1
// partial sums are live; the left fold (and every half type, in fp32) is one running sum.
constexpr int kRunTiles = 8;
constexpr uint64_t kRunVec = (uint64_t)kFoldThreads * kRunTiles;  // 16-byte vectors per run

template <int DT>
struct RunVec {  // one lane's kRunTiles vectors of one input, widened to the accumulator type
    using A = Acc<DT>;
    using S = typename Add<DT>::S;
    static constexpr int V = 16 / sizeof(S);
    typename A::T e[kRunTiles][V];
};

// loads input j (0: t.a, j: t.b[j - 1]) of this workgroup's run into x
template <int DT, int AUX>
__device__ __forceinline__ void run_load(RunVec<DT> &x, const SegTableN &t, int j, uint64_t base, int bytes, int off) {
    using S = typename Add<DT>::S;
    constexpr int V = RunVec<DT>::V;
    const u32x4 *src = static_cast<const u32x4 *>(j == 0 ? t.a : t.b[j - 1]) + base;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(src), 0, bytes, kRsrcWord3);
    u32x4 raw[kRunTiles];
#pragma unroll
    for (int u = 0; u < kRunTiles; ++u)
        raw[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + u * kFoldThreads * 16, 0, AUX);
#pragma unroll
    for (int u = 0; u < kRunTiles; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) x.e[u][e] = Acc<DT>::widen(reinterpret_cast<const S *>(&raw[u])[e]);
}

template <int DT>
__device__ __forceinline__ void run_add(RunVec<DT> &a, const RunVec<DT> &b) {  // a = a + b
#pragma unroll
    for (int u = 0; u < kRunTiles; ++u)
#pragma unroll
        for (int e = 0; e < RunVec<DT>::V; ++e) a.e[u][e] = Acc<DT>::add(a.e[u][e], b.e[u][e]);
}

// MPICH's tree over leaves [LO, HI) of K inputs (pof2 leaves; leaf l < rem is x_2l + x_2l+1,
// leaf l >= rem is x_l+rem), evaluated depth first into `out`
template <int DT, int K, int LO, int HI, int AUX>
__device__ __forceinline__ void run_tree(RunVec<DT> &out, const SegTableN &t, uint64_t base, int bytes, int off) {
    constexpr int pof2 = K >= 16 ? 16 : K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
    constexpr int rem = K - pof2;
    if constexpr (HI - LO == 1) {
        if constexpr (LO < rem) {
            run_load<DT, AUX>(out, t, 2 * LO, base, bytes, off);
            RunVec<DT> y;
            run_load<DT, AUX>(y, t, 2 * LO + 1, base, bytes, off);
            run_add<DT>(out, y);
        } else {
            run_load<DT, AUX>(out, t, LO + rem, base, bytes, off);
        }
    } else {
        constexpr int MID = (LO + HI) / 2;
        run_tree<DT, K, LO, MID, AUX>(out, t, base, bytes, off);
        RunVec<DT> right;
        run_tree<DT, K, MID, HI, AUX>(right, t, base, bytes, off);
        run_add<DT>(out, right);
    }
}

template <int DT, int NB, int FV, int ORDER>
__global__ void __launch_bounds__(kFoldThreads) k_sumN_run(FoldBatch fb) {
    const SegTableN &t = fb.t[blockIdx.y];
    using A = Acc<DT>;
    using S = typename Add<DT>::S;
    using T = typename A::T;
    constexpr int V = RunVec<DT>::V;
    constexpr int K = NB + 1;
    constexpr int kLoadAux = (FV & 1) ? kAuxNt : 0;
    constexpr int kStoreAux = ((FV & 2) ? kAuxNt : 0) | ((FV & 4) ? (kAuxSc0 | kAuxSc1) : 0);
    const uint64_t nv = t.n / V;
    const uint64_t base = (uint64_t)blockIdx.x * kRunVec;
    if (base < nv) {
        const int bytes = (int)((nv - base < kRunVec ? nv - base : kRunVec) * 16);
        const int off = (int)threadIdx.x * 16;
        RunVec<DT> acc;
        if constexpr (ORDER == kFoldMpichTree) {
            constexpr int pof2 = K >= 16 ? 16 : K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
            run_tree<DT, K, 0, pof2, kLoadAux>(acc, t, base, bytes, off);
        } else {  // left fold (and the half types' fp32 running sum)
            run_load<DT, kLoadAux>(acc, t, 0, base, bytes, off);
#pragma unroll
            for (int j = 1; j < K; ++j) {
                RunVec<DT> x;
                run_load<DT, kLoadAux>(x, t, j, base, bytes, off);
                run_add<DT>(acc, x);
            }
        }
        const auto ro = __builtin_amdgcn_make_buffer_rsrc(static_cast<u32x4 *>(t.out) + base, 0, bytes, kRsrcWord3);
#pragma unroll
        for (int u = 0; u < kRunTiles; ++u) {
            u32x4 res;
            S *rs = reinterpret_cast<S *>(&res);
#pragma unroll
            for (int e = 0; e < V; ++e) rs[e] = A::narrow(acc.e[u][e]);
            __builtin_amdgcn_raw_buffer_store_b128(res, ro, off + u * kFoldThreads * 16, 0, kStoreAux);
        }
    }
    const uint64_t rem = t.n - nv * V;
    if (rem && blockIdx.x == nv / kRunVec && threadIdx.x < rem) {
        const uint64_t e = nv * V + threadIdx.x;
        T w[NB + 1];
        w[0] = A::widen(static_cast<const S *>(t.a)[e]);
#pragma unroll
        for (int k = 0; k < NB; ++k) w[k + 1] = A::widen(static_cast<const S *>(t.b[k])[e]);
        static_cast<S *>(t.out)[e] = A::narrow(fold_values<DT, NB + 1, ORDER>(w));
    }
}

// Fold form (config "fold_form", set_fold_form): the run form for chunks of at least
// kFoldRunMinBytes with at least kFoldRunMinInputs inputs in the left or MPICH-tree order, the
// tile form otherwise. P = 8 fp32 (tools/fold_form_sizes.py): run 7.0 vs tile 8.1-8.5 us at 4 MiB,
// 12.1-12.3 vs 12.8 at 8 MiB, 22.7 vs 24.8-25.4 at 16 MiB, but 4.0 vs 3.2 at 2 MiB, where 128
// workgroups cannot cover one memory round trip the way 1025 do. The binomial order is for
// <= 2 KiB; and below 7 inputs the run form measured no better or worse than the tile form
// (tools/stream_mix.hip rform, two boxes: 8:1 +2.5 to +10 %, 7:1 0 to +2 %, 2:1 to 6:1 -3 to
// +1 %; profiles/r03/stream_mix/).
constexpr size_t kFoldRunMinBytes = 4u << 20;
constexpr int kFoldRunMinInputs = 7;
std::atomic<int> g_fold_form{0};
bool fold_run_form(size_t chunk_bytes, int order, int inputs) {
    if (order == kFoldBinomial) return false;
    const int f = g_fold_form.load(std::memory_order_relaxed);
    if (f != 0) return f == 2;
    return chunk_bytes >= kFoldRunMinBytes && inputs >= kFoldRunMinInputs;
}

// Half types fold left in fp32 whatever the order: only kFoldLeft is instantiated for them.
template <int DT>
constexpr bool kHalfType = DT == DDL_HALF || DT == DDL_BFLOAT16;

template <int DT, int NB, int FV>
void launch_sumN_order(const FoldBatch &b, hipStream_t stream) {
    constexpr uint64_t V = 16 / sizeof(typename Add<DT>::S);
    const SegTableN &t = b.t[0];  // nb and order are the batch's; the form and grid follow its largest problem
    uint64_t max_n = 0;
    for (int i = 0; i < b.count; ++i) max_n = b.t[i].n > max_n ? b.t[i].n : max_n;
    if (fold_run_form((size_t)max_n * sizeof(typename Add<DT>::S), t.order, NB + 1)) {
        const dim3 grid((unsigned)((max_n / V + kRunVec) / kRunVec), (unsigned)b.count);  // +1 vector for the tail
        if constexpr (!kHalfType<DT>) {
            if (t.order == kFoldMpichTree) {
                hipLaunchKernelGGL((k_sumN_run<DT, NB, FV, kFoldMpichTree>), grid, dim3(kFoldThreads), 0, stream, b);
                return;
            }
        }
        hipLaunchKernelGGL((k_sumN_run<DT, NB, FV, kFoldLeft>), grid, dim3(kFoldThreads), 0, stream, b);
        return;
    }
    const uint64_t tiles = (max_n / V + kFoldThreads) / kFoldThreads;
    DDL_REQUIRE(tiles < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "segment too large: " << max_n << " elements");
    const dim3 grid((unsigned)tiles, (unsigned)b.count);
    if constexpr (!kHalfType<DT>) {
        if (t.order == kFoldMpichTree) {
            hipLaunchKernelGGL((k_sumN_tile<DT, NB, FV, kFoldMpichTree>), grid, dim3(kFoldThreads), 0, stream, b);
            return;
        }
        if (t.order == kFoldBinomial) {
            hipLaunchKernelGGL((k_sumN_tile<DT, NB, FV, kFoldBinomial>), grid, dim3(kFoldThreads), 0, stream, b);
            return;
        }
    }
    hipLaunchKernelGGL((k_sumN_tile<DT, NB, FV, kFoldLeft>), grid, dim3(kFoldThreads), 0, stream, b);
}

template <int DT, int NB>
void launch_sumN_nb(const FoldBatch &b, hipStream_t stream) {
    if constexpr (NB > kMaxInputs) {
        fail(DDL_STATUS_INVALID_ARGUMENT, "too many reduce inputs");
    } else {
        if (b.t[0].nb == NB) {
            // cache policy (fold_variant, by the batch's bytes per input): 5 = non-temporal loads +
            // write-through store (large chunks), 4 = plain loads + write-through store (up to
            // 8 MiB, in cache)
            uint64_t elems = 0;
            for (int i = 0; i < b.count; ++i) elems += b.t[i].n;
            const int forced = g_fold_variant.load(std::memory_order_relaxed);
            const int fv = forced >= 0 ? forced : fold_variant((size_t)elems * sizeof(typename Add<DT>::S));
            if (fv == 4) launch_sumN_order<DT, NB, 4>(b, stream);
            else launch_sumN_order<DT, NB, 5>(b, stream);
        } else {
            launch_sumN_nb<DT, NB + 1>(b, stream);
        }
    }
}

// Misaligned buffers for the N-input fold: element-granular grid-stride, in the same order.
template <int DT, int NB, int ORDER>
__global__ void __launch_bounds__(kThreads) k_sumN_scalar(SegTableN t) {
    using A = Acc<DT>;
    using S = typename Add<DT>::S;
    using T = typename A::T;
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t e = (uint64_t)blockIdx.x * kThreads + threadIdx.x; e < t.n; e += stride) {
        T w[NB + 1];
        w[0] = A::widen(static_cast<const S *>(t.a)[e]);
#pragma unroll
        for (int k = 0; k < NB; ++k) w[k + 1] = A::widen(static_cast<const S *>(t.b[k])[e]);
        static_cast<S *>(t.out)[e] = A::narrow(fold_values<DT, NB + 1, ORDER>(w));
    }
}

template <int DT, int NB>
void launch_sumN_scalar_nb(const SegTableN &t, hipStream_t stream, unsigned blocks) {
    if constexpr (NB > kMaxInputs) {
        fail(DDL_STATUS_INVALID_ARGUMENT, "too many reduce inputs");
    } else {
        if (t.nb != NB) {
            launch_sumN_scalar_nb<DT, NB + 1>(t, stream, blocks);
            return;
        }
        if constexpr (!kHalfType<DT>) {
            if (t.order == kFoldMpichTree) {
                hipLaunchKernelGGL((k_sumN_scalar<DT, NB, kFoldMpichTree>), dim3(blocks), dim3(kThreads), 0, stream, t);
                return;
            }
            if (t.order == kFoldBinomial) {
                hipLaunchKernelGGL((k_sumN_scalar<DT, NB, kFoldBinomial>), dim3(blocks), dim3(kThreads), 0, stream, t);
                return;
            }
        }
        hipLaunchKernelGGL((k_sumN_scalar<DT, NB, kFoldLeft>), dim3(blocks), dim3(kThreads), 0, stream, t);
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

template <int DT, int V>
void launch_variant(const SegTable &t, hipStream_t stream, int variant, dim3 grid) {
    if constexpr (V > kVariantMask) {
        fail(DDL_STATUS_INVALID_ARGUMENT, "bad reduce variant");
    } else {
        if (variant == V) {
            hipLaunchKernelGGL((k_sum2_tile<DT, V, kReduceThreads>), grid, dim3(kReduceThreads), 0, stream, t);
        } else {
            launch_variant<DT, V + 1>(t, stream, variant, grid);
        }
    }
}

template <int DT, int U>
void launch_run(const SegTable &t, hipStream_t stream, int policy, uint64_t max_n) {
    constexpr uint64_t V = 16 / sizeof(typename Add<DT>::S);
    const uint64_t runs = (max_n / V + 128ull * U) / (128ull * U);  // +1 vector of room for the tail
    DDL_REQUIRE(runs < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "segment too large: " << max_n << " elements");
    const dim3 grid((unsigned)runs, t.count);
    switch (policy) {  // the cache-bit combinations the N = 1 bench compares
        case 0: hipLaunchKernelGGL((k_sum2_run<DT, 0, U>), grid, dim3(128), 0, stream, t); break;
        case kWtStore: hipLaunchKernelGGL((k_sum2_run<DT, kWtStore, U>), grid, dim3(128), 0, stream, t); break;
        case kNtLoadA | kNtLoadB | kWtStore:
            hipLaunchKernelGGL((k_sum2_run<DT, kNtLoadA | kNtLoadB | kWtStore, U>), grid, dim3(128), 0, stream, t);
            break;
        case kNtLoadA | kNtLoadB | kNtStore:
            hipLaunchKernelGGL((k_sum2_run<DT, kNtLoadA | kNtLoadB | kNtStore, U>), grid, dim3(128), 0, stream, t);
            break;
        default: fail(DDL_STATUS_INVALID_ARGUMENT, "run-form reduce: cache policy " + std::to_string(policy));
    }
}

template <int DT>
void launch_dt(const SegTable &t, hipStream_t stream, int variant, bool aligned, uint64_t max_n) {
    if (aligned && (variant & kRunForm)) {
        if (variant & kRun4) launch_run<DT, 4>(t, stream, variant & kVariantMask, max_n);
        else launch_run<DT, 8>(t, stream, variant & kVariantMask, max_n);
        return;
    }
    if (!aligned) {
        uint64_t blocks = (max_n + kThreads * 4 - 1) / (kThreads * 4);
        const uint64_t cap = (uint64_t)device_cu_count() * 8;
        blocks = blocks > cap ? cap : (blocks < 1 ? 1 : blocks);
        hipLaunchKernelGGL(k_sum2_scalar<DT>, dim3((unsigned)blocks, t.count), dim3(kThreads), 0, stream, t);
        return;
    }
    constexpr uint64_t V = 16 / sizeof(typename Add<DT>::S);
    constexpr uint64_t tv = kReduceThreads;
    const uint64_t tiles = (max_n / V + tv) / tv;  // +1 vector of room for the tail
    DDL_REQUIRE(tiles < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "segment too large: " << max_n << " elements");
    launch_variant<DT, 0>(t, stream, variant, dim3((unsigned)tiles, t.count));
}

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int g_cu_count = 0;

}  // namespace

void set_fold_form(int form) { g_fold_form.store(form, std::memory_order_relaxed); }
void set_testing_fold_variant(int v) { g_fold_variant.store(v, std::memory_order_relaxed); }
int get_fold_form() { return g_fold_form.load(std::memory_order_relaxed); }

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

namespace {
bool fold_aligned(const SegTableN &t) {
    bool aligned = aligned16(t.a) && aligned16(t.out);
    for (int k = 0; k < t.nb; ++k) aligned = aligned && aligned16(t.b[k]);
    return aligned;
}

template <int DT>
void launch_sumN_scalar_dt(const SegTableN &t, hipStream_t stream) {
    uint64_t blocks = (t.n + kThreads * 4 - 1) / (kThreads * 4);
    const uint64_t cap = (uint64_t)device_cu_count() * 8;
    blocks = blocks > cap ? cap : (blocks < 1 ? 1 : blocks);
    launch_sumN_scalar_nb<DT, 1>(t, stream, (unsigned)blocks);
}

template <int DT>
void launch_sumN_dt(const FoldBatch &b, hipStream_t stream) {
    bool aligned = true;
    for (int i = 0; i < b.count; ++i) aligned = aligned && fold_aligned(b.t[i]);
    if (!aligned) {  // misaligned buffers: element-granular, one problem at a time
        for (int i = 0; i < b.count; ++i) launch_sumN_scalar_dt<DT>(b.t[i], stream);
        return;
    }
    launch_sumN_nb<DT, 1>(b, stream);
}

void check_fold(const SegTableN &t) {
    DDL_REQUIRE(t.nb >= 1 && t.nb <= kMaxInputs, DDL_STATUS_INVALID_ARGUMENT, "reduce inputs " << t.nb);
    DDL_REQUIRE(t.order >= kFoldLeft && t.order <= kFoldBinomial, DDL_STATUS_INVALID_ARGUMENT, "fold order " << t.order);
    DDL_REQUIRE(t.a && t.out, DDL_STATUS_INVALID_ARGUMENT, "null reduce buffer");
    for (int k = 0; k < t.nb; ++k) DDL_REQUIRE(t.b[k], DDL_STATUS_INVALID_ARGUMENT, "null reduce input " << k);
}
}  // namespace

void launch_sumN_batch(const SegTableN *t, int count, int dtype, hipStream_t stream) {
    DDL_REQUIRE(count >= 0 && count <= kMaxFoldBatch, DDL_STATUS_INVALID_ARGUMENT, "fold batch of " << count);
    FoldBatch b;
    b.count = 0;
    for (int i = 0; i < count; ++i) {
        if (t[i].n == 0) continue;
        check_fold(t[i]);
        DDL_REQUIRE(b.count == 0 || (t[i].nb == b.t[0].nb && t[i].order == b.t[0].order), DDL_STATUS_INVALID_ARGUMENT,
                    "a fold batch needs one input count and one order");
        b.t[b.count++] = t[i];
    }
    if (b.count == 0) return;
    switch (dtype) {
        case DDL_FLOAT: launch_sumN_dt<DDL_FLOAT>(b, stream); break;
        case DDL_DOUBLE: launch_sumN_dt<DDL_DOUBLE>(b, stream); break;
        case DDL_INT32: launch_sumN_dt<DDL_INT32>(b, stream); break;
        case DDL_INT64: launch_sumN_dt<DDL_INT64>(b, stream); break;
        case DDL_UINT64: launch_sumN_dt<DDL_UINT64>(b, stream); break;
        case DDL_HALF: launch_sumN_dt<DDL_HALF>(b, stream); break;
        case DDL_BFLOAT16: launch_sumN_dt<DDL_BFLOAT16>(b, stream); break;
        default: fail(DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype");
    }
    DDL_HIP(hipGetLastError());
}

void launch_sumN(const SegTableN &t, int dtype, hipStream_t stream) { launch_sumN_batch(&t, 1, dtype, stream); }

// Standalone reduce (acc += in over whole buckets) of `bytes` per operand, by bucket size
// (3 rotating buffer sets per size, interleaved A/Bs: profiles/r02/reduce_policy/, profiles/r05/s6/,
// profiles/r05/s15/):
//   * from 256 MiB every access is non-temporal: the bucket streams through once (6.7-6.8 TB/s at
//     256 MiB; write-through stores 0.5-0.8 % slower there; the run form 6.27 vs 6.70);
//   * 96-256 MiB: the tile form, non-temporal loads, write-through stores (96 / 112 / 128 MiB: 6.32-6.46 /
//     6.37-6.45 / 6.51-6.60 TB/s vs 6.27-6.31 / 6.30-6.32 / 6.27-6.35 for the run form);
//   * 12-96 MiB: the run form with 4-tile runs (a workgroup streams one operand at a time) and
//     write-through stores, where part of the operand sets stays in the Infinity Cache; its loads
//     non-temporal except from 22 to 42 MiB, where plain loads measured faster on three boxes
//     (24 / 28 / 32 / 36 MiB: 6.39-6.47 / 6.49-6.60 / 6.57-6.66 / 6.65-6.69 TB/s vs 6.15-6.25 /
//     6.26-6.27 / 6.31-6.41 / 6.44-6.45 non-temporal); non-temporal wins at 12-20 MiB (16 MiB:
//     6.04-6.46 vs 5.78-6.03) and from 44 MiB (64 MiB 6.87-6.89, 80 MiB 6.91-6.99 vs 5.5-5.8
//     plain); against the tile form with plain loads, r05's rule below 32 MiB: 16 MiB 6.04-6.46 vs
//     5.78-5.89, 32 MiB 6.57-6.66 vs 6.39-6.66;
//   * below 12 MiB: the tile form, plain loads — the operands of a small bucket are likely still
//     in the Infinity Cache from whoever produced them — and write-through stores (8 MiB: 5.93-5.95
//     TB/s vs 4.7-6.3 for the run forms).
struct VariantBand {
    size_t below;  // bytes per operand
    int variant;
};
constexpr VariantBand kReduceBands[] = {
    {12u << 20, kWtStore},
    {22u << 20, kRunForm | kRun4 | kNtLoadA | kNtLoadB | kWtStore},
    {42u << 20, kRunForm | kRun4 | kWtStore},
    {96u << 20, kRunForm | kRun4 | kNtLoadA | kNtLoadB | kWtStore},
    {256u << 20, kNtLoadA | kNtLoadB | kWtStore},
};
int default_variant(size_t bytes) {
    for (const VariantBand &b : kReduceBands)
        if (bytes < b.below) return b.variant;
    return kNtLoadA | kNtLoadB | kNtStore;
}

// Ring reduce-scatter step: a = the rank's own gradient (read once: non-temporal), b = the slice
// RCCL just received (likely still in the Infinity Cache: plain), out = forwarded by the next
// step's send (keep it cache-resident: plain store).
int ring_variant() { return kNtLoadA; }

void launch_sum2(const SegTable &t, int dtype, hipStream_t stream, int variant) {
    DDL_REQUIRE(t.count >= 1 && t.count <= kMaxSegments, DDL_STATUS_INVALID_ARGUMENT,
                "segment count " << t.count << " outside [1, " << kMaxSegments << "]");
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    uint64_t max_n = 0, total_n = 0;
    bool aligned = true;
    for (int s = 0; s < t.count; ++s) {
        if (t.n[s] == 0) continue;
        DDL_REQUIRE(t.a[s] && t.b[s] && t.out[s], DDL_STATUS_INVALID_ARGUMENT, "null buffer in segment " << s);
        max_n = t.n[s] > max_n ? t.n[s] : max_n;
        total_n += t.n[s];
        aligned = aligned && aligned16(t.a[s]) && aligned16(t.b[s]) && aligned16(t.out[s]);
    }
    if (max_n == 0) return;
    if (variant < 0) variant = default_variant((size_t)total_n * es);
    DDL_REQUIRE(variant <= (kVariantMask | kRunForm | kRun4), DDL_STATUS_INVALID_ARGUMENT, "bad reduce variant " << variant);
    switch (dtype) {
        case DDL_FLOAT: launch_dt<DDL_FLOAT>(t, stream, variant, aligned, max_n); break;
        case DDL_DOUBLE: launch_dt<DDL_DOUBLE>(t, stream, variant, aligned, max_n); break;
        case DDL_INT32: launch_dt<DDL_INT32>(t, stream, variant, aligned, max_n); break;
        case DDL_INT64: launch_dt<DDL_INT64>(t, stream, variant, aligned, max_n); break;
        case DDL_UINT64: launch_dt<DDL_UINT64>(t, stream, variant, aligned, max_n); break;
        case DDL_HALF: launch_dt<DDL_HALF>(t, stream, variant, aligned, max_n); break;
        case DDL_BFLOAT16: launch_dt<DDL_BFLOAT16>(t, stream, variant, aligned, max_n); break;
        default: fail(DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype");
    }
    DDL_HIP(hipGetLastError());
}

}  // namespace ddl
