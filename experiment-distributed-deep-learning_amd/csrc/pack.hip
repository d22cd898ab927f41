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
// copies one 4 KiB tile of the flat space — the tile mapping of the reduce kernel — after one
// lane binary-searches the segment holding the tile start (LDS broadcast); lanes then walk
// forward at most a few segments (segments are >= 256 B apart, a tile spans <= 16).
#include <hip/hip_runtime.h>

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

// dir 0: gather segments -> flat; dir 1: scatter flat -> segments
template <int DIR>
__global__ void __launch_bounds__(kThreads) k_segments(char *flat, const SegDesc *__restrict__ d, int count) {
    __shared__ int seg0;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kTileBytes;
    if (threadIdx.x == 0) {
        int lo = 0, hi = count - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (d[mid].off <= tile0) lo = mid; else hi = mid - 1;
        }
        seg0 = lo;
    }
    __syncthreads();
    const uint64_t off = tile0 + (uint64_t)threadIdx.x * 16;
    int s = seg0;
    while (s + 1 < count && d[s + 1].off <= off) ++s;
    const uint64_t local = off - d[s].off;
    const uint64_t len = d[s].len;
    if (local >= len) return;  // padding between segments
    char *seg = reinterpret_cast<char *>(d[s].ptr) + local;
    char *fl = flat + off;
    if (d[s].vec && local + 16 <= len) {
        // the source is read once (non-temporal load); the destination is read next (the ring
        // sends the fused bucket; the optimizer reads the gradient): plain, cacheable store
        if (DIR == 0)
            *reinterpret_cast<u32x4 *>(fl) = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(seg));
        else
            *reinterpret_cast<u32x4 *>(seg) = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fl));
    } else {
        const uint64_t m = len - local < 16 ? len - local : 16;
        for (uint64_t k = 0; k < m; ++k) {
            if (DIR == 0) fl[k] = seg[k];
            else seg[k] = fl[k];
        }
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
    // table slots rotate; a slot is rewritten only after the kernel that read it has finished
    // (its event), so consecutive pack / unpack launches never wait on each other on the host
    Slot &sl = slots_[next_];
    next_ = (next_ + 1) % kSlots;
    if (sl.ready) DDL_HIP(hipEventSynchronize(sl.ready));
    else DDL_HIP(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
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
    const uint64_t tiles = (off + kTileBytes - 1) / kTileBytes;
    DDL_REQUIRE(tiles < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "fusion buffer too large");
    if (dir == 0)
        hipLaunchKernelGGL(k_segments<0>, dim3((unsigned)tiles), dim3(kThreads), 0, stream, static_cast<char *>(flat),
                           static_cast<const SegDesc *>(sl.dev), count);
    else
        hipLaunchKernelGGL(k_segments<1>, dim3((unsigned)tiles), dim3(kThreads), 0, stream, static_cast<char *>(flat),
                           static_cast<const SegDesc *>(sl.dev), count);
    DDL_HIP(hipGetLastError());
    DDL_HIP(hipEventRecord(sl.ready, stream));
}

}  // namespace ddl
