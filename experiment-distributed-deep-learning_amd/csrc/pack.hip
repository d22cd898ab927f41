// pack.hip — fusion gather/scatter between many gradient tensors and one HBM fusion buffer.
//
// Replaces the per-tensor memcpy loops of MPIRingTokenCommunication::executeCommunicatePlan_
// (MPIRingTokenCommunication.cc:548-733: memcpy in -> MPI_Allreduce -> memcpy out) with one
// launch per direction for any number of segments. HBM-bound copy: 2 bytes moved per byte.
//
// Fused layout: segment i occupies [off_i, off_i + len_i) of the flat buffer, off_i = running
// sum of the 256-byte-rounded lengths before it (every segment starts 256-byte aligned, so a
// fused bucket keeps the ring's 16-byte vector alignment). The segment table lives in device
// memory (uploaded with one async copy from a pinned staging table); each 256-lane workgroup
// copies a 64 KiB span of the flat space (see k_segments).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace ddl {

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;
constexpr uint64_t kTileBytes = kThreads * 16;

struct SegDesc {
    uint64_t ptr;   // segment address (tensor side)
    uint64_t off;   // offset in the flat buffer (256-byte aligned)
    uint64_t len;   // bytes
    uint64_t vec;   // 1 if ptr is 16-byte aligned (16-byte units), else byte copies
};

constexpr int kLdsSegs = 64;  // descriptors staged in LDS per workgroup

// Misaligned or partial chunk: byte copy (rare; kept out of line so the unrolled main loop
// stays small).
__device__ inline void copy_bytes(char *dst, const char *src, uint32_t m) {
    for (uint32_t k = 0; k < m; ++k) dst[k] = src[k];
}

// Last segment with off <= x: wave-parallel search, 64 samples per round (2 rounds for 4096
// segments instead of 12 dependent loads of a binary search). Called by all 64 lanes of a wave.
__device__ int find_segment(const SegDesc *__restrict__ d, int count, uint64_t x) {
    const int lane = threadIdx.x & 63;
    int lo = 0, hi = count;  // answer in [lo, hi)
    while (hi - lo > 1) {
        const int step = (hi - lo + 63) / 64;
        const int idx = lo + lane * step;
        const bool ok = idx < hi && d[idx].off <= x;
        const unsigned long long m = __ballot(ok);  // d[lo].off <= x, so lane 0 is always set
        const int last = 63 - __builtin_clzll(m);
        lo += last * step;
        hi = min(lo + step, hi);
    }
    return lo;
}

// dir 0: gather segments -> flat; dir 1: scatter flat -> segments. One workgroup per 64 KiB
// span of the flat buffer: wave 0 finds the span's first segment and stages the next 64
// descriptors in LDS; every lane then resolves its 16 chunks from LDS, issues all 16 loads,
// then all 16 stores (no dependent descriptor loads between data accesses). Spans holding more
// than 64 segments (segments under 1 KiB) resolve the rest from global memory.
template <int DIR, int kIters, bool NT_STORE>
__global__ void __launch_bounds__(kThreads) k_segments(char *flat, const SegDesc *__restrict__ d, int count,
                                                       uint64_t total) {
    constexpr uint64_t kSpanBytes = kTileBytes * kIters;
    __shared__ uint64_t s_off[kLdsSegs + 1], s_len[kLdsSegs], s_ptr[kLdsSegs];
    __shared__ int s_vec[kLdsSegs];
    __shared__ int s_seg0;
    const uint64_t span0 = (uint64_t)blockIdx.x * kSpanBytes;
    if (threadIdx.x < 64) {
        const int seg0 = find_segment(d, count, span0);
        const int i = seg0 + (int)threadIdx.x;
        if (i < count) {
            s_off[threadIdx.x] = d[i].off;
            s_len[threadIdx.x] = d[i].len;
            s_ptr[threadIdx.x] = d[i].ptr;
            s_vec[threadIdx.x] = (int)d[i].vec;
        } else {
            s_off[threadIdx.x] = ~0ull;
            s_len[threadIdx.x] = 0;
        }
        if (threadIdx.x == 0) {
            s_off[kLdsSegs] = seg0 + kLdsSegs < count ? d[seg0 + kLdsSegs].off : ~0ull;
            s_seg0 = seg0;
        }
    }
    __syncthreads();
    // resolve: the tensor-side address of each of this lane's 16-byte chunks (0 = padding or
    // already copied by the byte path, which handles misaligned and partial chunks at once)
    uint64_t addr[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        const uint64_t o = span0 + (uint64_t)it * kTileBytes + (uint64_t)threadIdx.x * 16;
        addr[it] = 0;
        if (o >= total) continue;
        // branchless binary search of the LDS offsets (s_off[0] <= span0 <= o; entries past
        // the table are ~0): s = last staged segment starting at or before o, 64 = beyond
        int s = 0;
#pragma unroll
        for (int step = kLdsSegs / 2; step > 0; step >>= 1) s = s_off[s + step] <= o ? s + step : s;
        if (s == kLdsSegs - 1 && s_off[kLdsSegs] <= o) s = kLdsSegs;
        uint64_t off, len, ptr;
        int vec;
        if (s < kLdsSegs) {
            off = s_off[s];
            len = s_len[s];
            ptr = s_ptr[s];
            vec = s_vec[s];
        } else {  // dense span: keep walking in global memory
            int g = s_seg0 + kLdsSegs;
            while (g + 1 < count && d[g + 1].off <= o) ++g;
            off = d[g].off;
            len = d[g].len;
            ptr = d[g].ptr;
            vec = (int)d[g].vec;
        }
        const uint64_t local = o - off;
        if (local >= len) continue;  // padding between segments
        if (vec && local + 16 <= len) {
            addr[it] = ptr + local;
        } else {
            const uint32_t m = (uint32_t)(len - local < 16 ? len - local : 16);
            if (DIR == 0) copy_bytes(flat + o, reinterpret_cast<const char *>(ptr + local), m);
            else copy_bytes(reinterpret_cast<char *>(ptr + local), flat + o, m);
        }
    }
    u32x4 v[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        if (!addr[it]) continue;
        const char *src = DIR == 0 ? reinterpret_cast<const char *>(addr[it])
                                   : flat + span0 + (uint64_t)it * kTileBytes + threadIdx.x * 16;
        // every byte is read once: non-temporal loads (and stores, by default: the consumer —
        // the collective or the optimizer — comes after the whole bucket is copied)
        v[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src));
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        if (!addr[it]) continue;
        char *fl = flat + span0 + (uint64_t)it * kTileBytes + threadIdx.x * 16;
        u32x4 *dst = reinterpret_cast<u32x4 *>(DIR == 0 ? fl : reinterpret_cast<char *>(addr[it]));
        if (NT_STORE) __builtin_nontemporal_store(v[it], dst);
        else *dst = v[it];
    }
}

}  // namespace

SegmentCopier::~SegmentCopier() {
    for (Slot &sl : slots_) {
        if (sl.ready) (void)hipEventSynchronize(sl.ready);
        if (sl.ready) (void)hipEventDestroy(sl.ready);
        if (sl.host) (void)hipHostFree(sl.host);
        if (sl.dev) (void)hipFree(sl.dev);
    }
}

// Table slots rotate; a slot is rewritten only after the copy that read it has run (its event).
// A slot still in use is skipped and the pool grows, so a pipeline of pack / unpack launches
// queued behind allreduces never blocks the host; at kMaxSlots the oldest slot is waited for.
SegmentCopier::Slot &SegmentCopier::free_slot_() {
    for (size_t k = 0; k < slots_.size(); ++k) {
        Slot &sl = slots_[(next_ + k) % slots_.size()];
        if (!sl.ready) continue;
        const hipError_t q = hipEventQuery(sl.ready);
        if (q == hipErrorNotReady) continue;
        DDL_HIP(q);
        next_ = (next_ + k + 1) % slots_.size();
        return sl;
    }
    if (slots_.size() < kMaxSlots) {
        slots_.emplace_back();
        Slot &sl = slots_.back();
        DDL_HIP(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
        next_ = 0;
        return sl;
    }
    Slot &sl = slots_[next_];
    next_ = (next_ + 1) % slots_.size();
    DDL_HIP(hipEventSynchronize(sl.ready));
    return sl;
}

size_t SegmentCopier::flat_bytes(const size_t *bytes, int count) {
    size_t off = 0;
    for (int i = 0; i < count; ++i) off += (bytes[i] + 255) & ~size_t(255);
    return off;
}

void SegmentCopier::run(int dir, void *flat, void *const *segs, const size_t *bytes, int count,
                        hipStream_t stream) {
    if (count <= 0) return;
    DDL_REQUIRE(flat && segs && bytes, DDL_STATUS_INVALID_ARGUMENT, "null pack arguments");
    const size_t need = (size_t)count * sizeof(SegDesc);
    Slot &sl = free_slot_();
    if (need > sl.cap) {
        if (sl.host) DDL_HIP(hipHostFree(sl.host));
        if (sl.dev) DDL_HIP(hipFree(sl.dev));
        sl.host = sl.dev = nullptr;
        sl.cap = need + need / 2;
        DDL_HIP(hipHostMalloc(&sl.host, sl.cap, hipHostMallocDefault));
        DDL_HIP(hipMalloc(&sl.dev, sl.cap));
    }
    SegDesc *t = static_cast<SegDesc *>(sl.host);
    uint64_t off = 0;
    for (int i = 0; i < count; ++i) {
        DDL_REQUIRE(bytes[i] == 0 || segs[i], DDL_STATUS_INVALID_ARGUMENT, "null segment " << i);
        t[i].ptr = reinterpret_cast<uint64_t>(segs[i]);
        t[i].off = off;
        t[i].len = bytes[i];
        t[i].vec = (reinterpret_cast<uintptr_t>(segs[i]) & 15u) == 0;
        off += (bytes[i] + 255) & ~uint64_t(255);
    }
    if (off == 0) return;
    DDL_HIP(hipMemcpyAsync(sl.dev, sl.host, need, hipMemcpyHostToDevice, stream));
    // DDL_PACK_VARIANT (measurement only): bit 0 non-temporal stores, bit 1 32 chunks per lane
    // instead of 16. Default 1: 16 chunks, NT stores — 5.5 / 5.6 TB/s pack / unpack on the C5
    // bucket set vs 5.3 / 5.6 (cacheable stores) and 5.3 / 5.1 (32 chunks); tools/pack_tune.py.
    static const int variant = [] {
        const char *e = std::getenv("DDL_PACK_VARIANT");
        return e ? std::atoi(e) : 1;
    }();
    const int iters = (variant & 2) ? 32 : 16;
    const uint64_t spans = (off + kTileBytes * iters - 1) / (kTileBytes * iters);
    DDL_REQUIRE(spans < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "fusion buffer too large");
    char *fl = static_cast<char *>(flat);
    const SegDesc *dd = static_cast<const SegDesc *>(sl.dev);
#define DDL_PACK_LAUNCH(D, I, N) \
    hipLaunchKernelGGL((k_segments<D, I, N>), dim3((unsigned)spans), dim3(kThreads), 0, stream, fl, dd, count, (uint64_t)off)
    const bool nt = variant & 1;
    if (dir == 0) {
        if (iters == 16) { if (nt) DDL_PACK_LAUNCH(0, 16, true); else DDL_PACK_LAUNCH(0, 16, false); }
        else { if (nt) DDL_PACK_LAUNCH(0, 32, true); else DDL_PACK_LAUNCH(0, 32, false); }
    } else {
        if (iters == 16) { if (nt) DDL_PACK_LAUNCH(1, 16, true); else DDL_PACK_LAUNCH(1, 16, false); }
        else { if (nt) DDL_PACK_LAUNCH(1, 32, true); else DDL_PACK_LAUNCH(1, 32, false); }
    }
#undef DDL_PACK_LAUNCH
    DDL_HIP(hipGetLastError());
    DDL_HIP(hipEventRecord(sl.ready, stream));
}

}  // namespace ddl
