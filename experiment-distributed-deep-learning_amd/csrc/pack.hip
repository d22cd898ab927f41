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

// dir 0: gather segments -> flat; dir 1: scatter flat -> segments. One workgroup of THREADS
// lanes per span of THREADS * 16 * kIters bytes of the flat buffer: wave 0 finds the span's first
// segment and stages the next kSegs descriptors in LDS; every lane then resolves its kIters
// chunks from LDS, issues all kIters loads, then all kIters stores (no dependent descriptor
// loads between data accesses). Spans holding more than kSegs segments resolve the rest from
// global memory. Small spans (2 chunks per lane, 4 KiB per 128-lane workgroup) keep the chunks
// in flight a compact, interleaved window of each stream, as the reduce kernel's one-tile-per-
// workgroup mapping does; tools/copy_tune.hip: 1R+1W copies reach 6.5 TB/s with 2-4 KiB tiles
// per workgroup vs 5.3 TB/s with 64 KiB.
// Segment-aligned tiling: every segment is cut into tiles of THREADS * 16 * kIters bytes that
// restart at the segment start, so a tile never crosses a segment and its workgroup needs no
// per-chunk search: tile_seg[t] (k_tile_index: one thread per tile, binary search of the
// tile0 column) names the segment, one scalar descriptor load gives ptr / off / len, and lane l
// moves bytes [16 l + it * THREADS * 16, ...) of the tile.
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
                                                       const int *__restrict__ tile_seg) {
    constexpr uint64_t kTile = (uint64_t)THREADS * 16 * kIters;
    const SegDesc sd = d[tile_seg[blockIdx.x]];
    const uint64_t base = (uint64_t)(blockIdx.x - sd.tile0) * kTile;  // tile start inside the segment
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

template <int DIR, int kIters, bool NT_STORE, int THREADS, int kSegs>
__global__ void __launch_bounds__(THREADS) k_segments(char *flat, const SegDesc *__restrict__ d, int count,
                                                      uint64_t total) {
    constexpr uint64_t kTileBytes = (uint64_t)THREADS * 16;
    constexpr uint64_t kSpanBytes = kTileBytes * kIters;
    static_assert(kSegs <= 64 && (kSegs & (kSegs - 1)) == 0, "LDS descriptor table: power of two <= 64");
    __shared__ uint64_t s_off[kSegs + 1], s_len[kSegs], s_ptr[kSegs];
    __shared__ int s_vec[kSegs];
    __shared__ int s_seg0;
    const uint64_t span0 = (uint64_t)blockIdx.x * kSpanBytes;
    if (threadIdx.x < 64) {
        const int seg0 = find_segment(d, count, span0);
        const int i = seg0 + (int)threadIdx.x;
        if (threadIdx.x < kSegs) {
            if (i < count) {
                s_off[threadIdx.x] = d[i].off;
                s_len[threadIdx.x] = d[i].len;
                s_ptr[threadIdx.x] = d[i].ptr;
                s_vec[threadIdx.x] = (int)d[i].vec;
            } else {
                s_off[threadIdx.x] = ~0ull;
                s_len[threadIdx.x] = 0;
            }
        }
        if (threadIdx.x == 0) {
            s_off[kSegs] = seg0 + kSegs < count ? d[seg0 + kSegs].off : ~0ull;
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
        for (int step = kSegs / 2; step > 0; step >>= 1) s = s_off[s + step] <= o ? s + step : s;
        if (s == kSegs - 1 && s_off[kSegs] <= o) s = kSegs;
        uint64_t off, len, ptr;
        int vec;
        if (s < kSegs) {
            off = s_off[s];
            len = s_len[s];
            ptr = s_ptr[s];
            vec = s_vec[s];
        } else {  // dense span: keep walking in global memory
            int g = s_seg0 + kSegs;
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
    // DDL_PACK_VARIANT (measurement only; tools/pack_tune.py, C5 bucket set, pack / unpack):
    //   0: span kernel, 256 lanes x 16 chunks per 64 KiB span, in-kernel segment search  5.56 / 5.61 TB/s
    //   1: segment tiles of 1 KiB, 64 lanes (default)                                     6.10 / 6.37
    //   2: segment tiles of 2 KiB, 128 lanes                                              6.09 / 6.29
    //   3: segment tiles of 4 KiB, 128 lanes x 2 chunks                                   5.74 / 6.30
    // (spans of 2-8 KiB with the in-kernel search, with or without a precomputed first segment
    // per span, measured 4.5-6.0: the per-chunk search and the LDS round trip cost more than
    // the smaller window saves.)
    static const int variant = [] {
        const char *e = std::getenv("DDL_PACK_VARIANT");
        const int v = e ? std::atoi(e) : 1;
        return v >= 0 && v <= 3 ? v : 1;
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
    if (variant == 0) {
        const uint64_t spans = (off + 65535) / 65536;
        DDL_REQUIRE(spans < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "fusion buffer too large");
        if (dir == 0) hipLaunchKernelGGL((k_segments<0, 16, true, 256, 64>), dim3((unsigned)spans), dim3(256), 0, stream, fl, dd, count, (uint64_t)off);
        else hipLaunchKernelGGL((k_segments<1, 16, true, 256, 64>), dim3((unsigned)spans), dim3(256), 0, stream, fl, dd, count, (uint64_t)off);
    } else if (tiles > 0) {
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
            if (variant == 2) hipLaunchKernelGGL((k_seg_tiles<0, 1, 128>), g, dim3(128), 0, stream, fl, dd, ts);
            else if (variant == 3) hipLaunchKernelGGL((k_seg_tiles<0, 2, 128>), g, dim3(128), 0, stream, fl, dd, ts);
            else hipLaunchKernelGGL((k_seg_tiles<0, 1, 64>), g, dim3(64), 0, stream, fl, dd, ts);
        } else {
            if (variant == 2) hipLaunchKernelGGL((k_seg_tiles<1, 1, 128>), g, dim3(128), 0, stream, fl, dd, ts);
            else if (variant == 3) hipLaunchKernelGGL((k_seg_tiles<1, 2, 128>), g, dim3(128), 0, stream, fl, dd, ts);
            else hipLaunchKernelGGL((k_seg_tiles<1, 1, 64>), g, dim3(64), 0, stream, fl, dd, ts);
        }
    }
    DDL_HIP(hipGetLastError());
    DDL_HIP(hipEventRecord(sl.ready, stream));
}

}  // namespace ddl
