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
// tile, the tile's segment from a one-byte-per-tile index built on the device (k_tile_index,
// k_seg_tiles).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "deptrace.h"

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
// Tile -> segment map, compact: the dispatcher deals workgroups round-robin over the 8 XCDs,
// each with its own L2, so every 128-byte line of a per-tile index is fetched by all 8 (r01: an
// int32 per tile cost +3.2 % HBM traffic on the C5 set). The map is therefore one byte per tile,
// the segment's distance from a per-128-tile base (kIdxBlock), so a line covers 128 tiles:
// seg = base[tile / 128] + delta[tile]. When some block spans more than 255 segments (runs of
// empty segments) the host falls back to an int32 per tile. Remapping tiles to XCDs instead cut
// the traffic too but slowed the copy 4-5 % (profiles/r02/pack/pack_xcd_ab.txt).
constexpr uint32_t kIdxBlock = 128;

template <bool NARROW>
__global__ void __launch_bounds__(256) k_tile_index(const SegDesc *__restrict__ d, int count, uint64_t tiles,
                                                    const uint32_t *__restrict__ base, void *__restrict__ map) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= tiles) return;
    int lo = 0, hi = count;  // last segment with tile0 <= t (segments without tiles share tile0)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (d[mid].tile0 <= t) lo = mid;
        else hi = mid;
    }
    if (NARROW) static_cast<uint8_t *>(map)[t] = (uint8_t)(lo - (int)base[t / kIdxBlock]);
    else static_cast<int *>(map)[t] = lo;
}

template <int DIR, int kIters, int THREADS, bool NARROW>
__global__ void __launch_bounds__(THREADS) k_seg_tiles(char *flat, const SegDesc *__restrict__ d,
                                                       const uint32_t *__restrict__ blk_base,
                                                       const void *__restrict__ map) {
    constexpr uint64_t kTile = (uint64_t)THREADS * 16 * kIters;
    const unsigned tile = blockIdx.x;
    // the byte is read as its aligned dword (a scalar load; a byte load would go through the
    // vector memory path and delay the whole tile)
    const int seg = NARROW ? (int)(blk_base[tile / kIdxBlock] +
                                   ((static_cast<const uint32_t *>(map)[tile / 4] >> (8 * (tile % 4))) & 0xffu))
                           : static_cast<const int *>(map)[tile];
    const SegDesc sd = d[seg];
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

// one 1 KiB tile per 64-lane workgroup (kSegTile): the r01 tile-shape measurement (C5 bucket
// set, pack / unpack) had 6.10 / 6.37 TB/s for it against 6.09 / 6.29 for 2 KiB tiles of 128 lanes
// and 5.74 / 6.30 for 4 KiB tiles of 128 lanes x 2 chunks; the span kernel with an in-kernel
// segment search (2-64 KiB spans) 4.5-6.0
constexpr uint64_t kSegTile = 1024;
template <int DIR, bool NARROW>
void launch_dir(dim3 g, hipStream_t stream, char *fl, const SegDesc *dd, const uint32_t *db, const void *map) {
    hipLaunchKernelGGL((k_seg_tiles<DIR, 1, 64, NARROW>), g, dim3(64), 0, stream, fl, dd, db, map);
}

void launch_tiles(int dir, bool narrow, dim3 g, hipStream_t stream, char *fl, const SegDesc *dd, const uint32_t *db,
                  const void *map) {
    if (dir == 0) {
        if (narrow) launch_dir<0, true>(g, stream, fl, dd, db, map);
        else launch_dir<0, false>(g, stream, fl, dd, db, map);
    } else {
        if (narrow) launch_dir<1, true>(g, stream, fl, dd, db, map);
        else launch_dir<1, false>(g, stream, fl, dd, db, map);
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
    Slot &sl = free_slot_();
    // segment-aligned tiles of kSegTile bytes per workgroup; tile0 = running tile count
    const uint64_t seg_tile = kSegTile;
    uint64_t tiles = 0;
    for (int i = 0; i < count; ++i) tiles += (bytes[i] + seg_tile - 1) / seg_tile;
    DDL_REQUIRE(tiles < (1ull << 31), DDL_STATUS_INVALID_ARGUMENT, "fusion buffer too large");
    const uint64_t nblk = (tiles + kIdxBlock - 1) / kIdxBlock;
    const size_t table = (size_t)count * sizeof(SegDesc);
    const size_t need = table + nblk * sizeof(uint32_t);  // descriptors, then the block bases
    if (need > sl.cap) {  // outgrown tables kept until ddl_finalize: no hipFree on a data path (engine.h)
        retire_host(sl.host);
        retire_device(sl.dev);
        sl.host = sl.dev = nullptr;
        sl.cap = need + need / 2;
        DDL_HIP(hipHostMalloc(&sl.host, sl.cap, hipHostMallocDefault));
        DDL_HIP(hipMalloc(&sl.dev, sl.cap));
    }
    SegDesc *t = static_cast<SegDesc *>(sl.host);
    uint32_t *bases = reinterpret_cast<uint32_t *>(static_cast<char *>(sl.host) + table);
    uint64_t off = 0, tl = 0;
    for (int i = 0; i < count; ++i) {
        DDL_REQUIRE(bytes[i] == 0 || segs[i], DDL_STATUS_INVALID_ARGUMENT, "null segment " << i);
        t[i].ptr = reinterpret_cast<uint64_t>(segs[i]);
        t[i].off = off;
        t[i].len = bytes[i];
        t[i].vec = (reinterpret_cast<uintptr_t>(segs[i]) & 15u) == 0;
        t[i].tile0 = (uint32_t)tl;
        off += (bytes[i] + 255) & ~uint64_t(255);
        tl += (bytes[i] + seg_tile - 1) / seg_tile;
    }
    if (off == 0) return;
    // block b's base: the segment of tile b * 128 (the last one with tile0 <= it, as
    // k_tile_index resolves); narrow when no block spans more than 255 segments
    bool narrow = true;
    for (uint64_t b = 0, s0 = 0, s1 = 0; b < nblk; ++b) {
        const uint64_t first = b * kIdxBlock, last = std::min(tiles, first + kIdxBlock) - 1;
        while (s0 + 1 < (uint64_t)count && t[s0 + 1].tile0 <= first) ++s0;
        if (s1 < s0) s1 = s0;
        while (s1 + 1 < (uint64_t)count && t[s1 + 1].tile0 <= last) ++s1;
        bases[b] = (uint32_t)s0;
        if (s1 - s0 > 255) narrow = false;
    }
    DDL_HIP(hipMemcpyAsync(sl.dev, sl.host, need, hipMemcpyHostToDevice, stream));
    char *fl = static_cast<char *>(flat);
    const SegDesc *dd = static_cast<const SegDesc *>(sl.dev);
    const uint32_t *db = reinterpret_cast<const uint32_t *>(static_cast<char *>(sl.dev) + table);
    if (tiles > 0) {
        const size_t ib = narrow ? (tiles + 3) & ~uint64_t(3) : tiles * sizeof(int);
        if (ib > sl.idx_cap) {
            retire_device(sl.idx);
            sl.idx = nullptr;
            sl.idx_cap = ib + ib / 2;
            DDL_HIP(hipMalloc(&sl.idx, sl.idx_cap));
        }
        const dim3 ig((unsigned)((tiles + 255) / 256)), g((unsigned)tiles);
        if (narrow) hipLaunchKernelGGL(k_tile_index<true>, ig, dim3(256), 0, stream, dd, count, (uint64_t)tiles, db, sl.idx);
        else hipLaunchKernelGGL(k_tile_index<false>, ig, dim3(256), 0, stream, dd, count, (uint64_t)tiles, db, sl.idx);
        launch_tiles(dir, narrow, g, stream, fl, dd, db, sl.idx);
    }
    DDL_HIP(hipGetLastError());
    DDL_HIP(hipEventRecord(sl.ready, stream));
    if (dep::on()) {  // happens-before trace (deptrace.h): the segments and the flat buffer
        std::vector<dep::Access> acc;
        acc.push_back(dir == 0 ? dep::wr(flat, off) : dep::rd(flat, off));
        for (int i = 0; i < count; ++i)
            if (bytes[i]) acc.push_back(dir == 0 ? dep::rd(segs[i], bytes[i]) : dep::wr(segs[i], bytes[i]));
        dep::op(stream, dir == 0 ? "pack" : "unpack", std::move(acc));
    }
}

}  // namespace ddl
