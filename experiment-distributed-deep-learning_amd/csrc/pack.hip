// pack.hip — fusion gather/scatter between many gradient tensors and one HBM fusion buffer.
//
// Replaces the per-tensor memcpy loops of MPIRingTokenCommunication::executeCommunicatePlan_
// (MPIRingTokenCommunication.cc:548-733: memcpy in -> MPI_Allreduce -> memcpy out) with one
// launch per direction for any number of segments. HBM-bound copy: 2 bytes moved per byte.
//
// Fused layout: segment i occupies [off_i, off_i + len_i) of the flat buffer, off_i = running
// sum of the 256-byte-rounded lengths before it (every segment starts 256-byte aligned, so a
// fused bucket keeps the ring's 16-byte vector alignment). The segment table lives in device
// memory (uploaded with one async copy from a pinned staging table). Default mapping: every
// segment is cut into 1 KiB tiles that restart at the segment start, one 64-lane workgroup per
// tile, the tile's segment from a per-tile index built on the device (k_tile_index, k_seg_tiles).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace ddl {

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

struct SegDesc {
    uint64_t ptr;   // segment address (tensor side)
    uint64_t off;   // offset in the flat buffer (256-byte aligned)
    uint64_t len;   // bytes
    uint32_t vec;   // 1 if ptr is 16-byte aligned (16-byte units), else byte copies
    uint32_t tile0; // segment-aligned tiling: index of the segment's first tile
};

// Misaligned or partial chunk: byte copy (rare; kept out of line so the unrolled main loop
// stays small).
__device__ inline void copy_bytes(char *dst, const char *src, uint32_t m) {
    for (uint32_t k = 0; k < m; ++k) dst[k] = src[k];
}

// dir 0: gather segments -> flat; dir 1: scatter flat -> segments.
// Segment-aligned tiling: every segment is cut into tiles of THREADS * 16 * kIters bytes that
// restart at the segment start, so a tile never crosses a segment and its workgroup needs no
// per-chunk search: tile_seg[t] (k_tile_index: one thread per tile, binary search of the
// tile0 column) names the segment, one scalar descriptor load gives ptr / off / len, and lane l
// moves bytes [16 l + it * THREADS * 16, ...) of the tile. Small tiles (1 KiB per 64-lane
// workgroup) keep the chunks in flight a compact window of each stream (tools/copy_tune.hip:
// 1R+1W copies reach 6.5 TB/s with 1-2 KiB per workgroup vs 5.3 TB/s with 64 KiB).
// XCD grouping: the dispatcher deals workgroups round-robin over the 8 XCDs, each with its own
// L2, so with tile = blockIdx every XCD would fetch every 64-byte line of tile_seg (16 tiles)
// and the descriptor it points at: 8x the index bytes from HBM (+3 % traffic on the C5 set,
// r01 PMC). Inside each run of 128 workgroups, XCD x takes 16 consecutive tiles — one
// tile_seg line — so each line is fetched once, and the window stays 128 tiles wide.
__global__ void __launch_bounds__(256) k_tile_index(const SegDesc *__restrict__ d, int count, uint64_t tiles,
                                                    int *__restrict__ tile_seg) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= tiles) return;
    int lo = 0, hi = count;  // last segment with tile0 <= t (segments without tiles share tile0)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (d[mid].tile0 <= t) lo = mid;
        else hi = mid;
    }
    tile_seg[t] = lo;
}

template <int DIR, int kIters, int THREADS>
__global__ void __launch_bounds__(THREADS) k_seg_tiles(char *flat, const SegDesc *__restrict__ d,
                                                       const int *__restrict__ tile_seg, int xcd_group) {
    constexpr uint64_t kTile = (uint64_t)THREADS * 16 * kIters;
    constexpr unsigned kXcds = 8, kLine = 16, kRun = kXcds * kLine;
    const unsigned bid = blockIdx.x;
    const unsigned full = xcd_group ? gridDim.x - gridDim.x % kRun : 0;  // the tail keeps tile = blockIdx
    const unsigned r = bid % kRun;
    const unsigned tile = bid < full ? bid - r + (r % kXcds) * kLine + r / kXcds : bid;
    const SegDesc sd = d[tile_seg[tile]];
    const uint64_t base = (uint64_t)(tile - sd.tile0) * kTile;  // tile start inside the segment
    char *fl = flat + sd.off;
    char *tp = reinterpret_cast<char *>(sd.ptr);
    if (!sd.vec) {  // misaligned tensor: bytes
        for (uint64_t b = base + threadIdx.x; b < sd.len && b < base + kTile; b += THREADS) {
            if (DIR == 0) fl[b] = tp[b];
            else tp[b] = fl[b];
        }
        return;
    }
    u32x4 v[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        const uint64_t b = base + (uint64_t)it * THREADS * 16 + threadIdx.x * 16;
        if (b + 16 <= sd.len)
            v[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>((DIR == 0 ? tp : fl) + b));
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        const uint64_t b = base + (uint64_t)it * THREADS * 16 + threadIdx.x * 16;
        if (b + 16 <= sd.len) {
            __builtin_nontemporal_store(v[it], reinterpret_cast<u32x4 *>((DIR == 0 ? fl : tp) + b));
        } else if (b < sd.len) {  // the segment's last partial 16 bytes
            const uint32_t m = (uint32_t)(sd.len - b);
            if (DIR == 0) copy_bytes(fl + b, tp + b, m);
            else copy_bytes(tp + b, fl + b, m);
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
        if (sl.idx) (void)hipFree(sl.idx);
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
    // DDL_PACK_VARIANT (measurement only; tools/pack_tune.py, C5 bucket set, pack / unpack, r01):
    //   1: segment tiles of 1 KiB, 64 lanes (default)                                     6.10 / 6.37 TB/s
    //   2: segment tiles of 2 KiB, 128 lanes                                              6.09 / 6.29
    //   3: segment tiles of 4 KiB, 128 lanes x 2 chunks                                   5.74 / 6.30
    // (the r01 span kernel — 64 KiB spans with an in-kernel segment search — measured 5.56 / 5.61
    // and is gone; spans of 2-8 KiB with the search measured 4.5-6.0.)
    static const int variant = [] {
        const char *e = std::getenv("DDL_PACK_VARIANT");
        const int v = e ? std::atoi(e) : 1;
        return v >= 1 && v <= 3 ? v : 1;
    }();
    // DDL_PACK_XCD=0 turns the XCD grouping of tiles off (measurement)
    static const int xcd = [] {
        const char *e = std::getenv("DDL_PACK_XCD");
        return e ? (std::atoi(e) != 0) : 1;
    }();
    if (need > sl.cap) {
        if (sl.host) DDL_HIP(hipHostFree(sl.host));
        if (sl.dev) DDL_HIP(hipFree(sl.dev));
        sl.host = sl.dev = nullptr;
        sl.cap = need + need / 2;
        DDL_HIP(hipHostMalloc(&sl.host, sl.cap, hipHostMallocDefault));
        DDL_HIP(hipMalloc(&sl.dev, sl.cap));
    }
    // segment-aligned tiles (variants 1..3): tile bytes per workgroup; tile0 = running tile count
    const uint64_t seg_tile = variant == 2 ? 2048 : variant == 3 ? 4096 : 1024;
    SegDesc *t = static_cast<SegDesc *>(sl.host);
    uint64_t off = 0, tiles = 0;
    for (int i = 0; i < count; ++i) {
        DDL_REQUIRE(bytes[i] == 0 || segs[i], DDL_STATUS_INVALID_ARGUMENT, "null segment " << i);
        t[i].ptr = reinterpret_cast<uint64_t>(segs[i]);
        t[i].off = off;
        t[i].len = bytes[i];
        t[i].vec = (reinterpret_cast<uintptr_t>(segs[i]) & 15u) == 0;
        t[i].tile0 = (uint32_t)tiles;
        off += (bytes[i] + 255) & ~uint64_t(255);
        tiles += (bytes[i] + seg_tile - 1) / seg_tile;
    }
    DDL_REQUIRE(tiles < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "fusion buffer too large");
    if (off == 0) return;
    DDL_HIP(hipMemcpyAsync(sl.dev, sl.host, need, hipMemcpyHostToDevice, stream));
    char *fl = static_cast<char *>(flat);
    const SegDesc *dd = static_cast<const SegDesc *>(sl.dev);
    if (tiles > 0) {
        const size_t ib = tiles * sizeof(int);
        if (ib > sl.idx_cap) {
            if (sl.idx) DDL_HIP(hipFree(sl.idx));
            sl.idx = nullptr;
            sl.idx_cap = ib + ib / 2;
            DDL_HIP(hipMalloc(&sl.idx, sl.idx_cap));
        }
        int *ts = static_cast<int *>(sl.idx);
        hipLaunchKernelGGL(k_tile_index, dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, stream, dd, count,
                           (uint64_t)tiles, ts);
        const dim3 g((unsigned)tiles);
        if (dir == 0) {
            if (variant == 2) hipLaunchKernelGGL((k_seg_tiles<0, 1, 128>), g, dim3(128), 0, stream, fl, dd, ts, xcd);
            else if (variant == 3) hipLaunchKernelGGL((k_seg_tiles<0, 2, 128>), g, dim3(128), 0, stream, fl, dd, ts, xcd);
            else hipLaunchKernelGGL((k_seg_tiles<0, 1, 64>), g, dim3(64), 0, stream, fl, dd, ts, xcd);
        } else {
            if (variant == 2) hipLaunchKernelGGL((k_seg_tiles<1, 1, 128>), g, dim3(128), 0, stream, fl, dd, ts, xcd);
            else if (variant == 3) hipLaunchKernelGGL((k_seg_tiles<1, 2, 128>), g, dim3(128), 0, stream, fl, dd, ts, xcd);
            else hipLaunchKernelGGL((k_seg_tiles<1, 1, 64>), g, dim3(64), 0, stream, fl, dd, ts, xcd);
        }
    }
    DDL_HIP(hipGetLastError());
    DDL_HIP(hipEventRecord(sl.ready, stream));
}

}  // namespace ddl
