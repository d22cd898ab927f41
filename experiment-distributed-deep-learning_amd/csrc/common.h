// common.h — shared definitions of the MI355X allreduce engine (host side).
//
// dtype numbers and status codes follow the C-ABI (include/ddl_amd.h), which mirrors the
// reference's tensorflow::DataType use (src/cpp/def.h:10) and StatusCode (def.h:70-74).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <string>
#include <sstream>
#include <vector>

#include "ddl_amd_testing.h"

namespace ddl {

inline size_t dtype_size(int dt) {
    switch (dt) {
        case DDL_FLOAT: case DDL_INT32: return 4;
        case DDL_DOUBLE: case DDL_INT64: case DDL_UINT64: return 8;
        case DDL_HALF: case DDL_BFLOAT16: return 2;
        default: return 0;
    }
}

inline const char *dtype_name(int dt) {
    switch (dt) {
        case DDL_FLOAT: return "float32";
        case DDL_DOUBLE: return "float64";
        case DDL_INT32: return "int32";
        case DDL_INT64: return "int64";
        case DDL_UINT64: return "uint64";
        case DDL_HALF: return "float16";
        case DDL_BFLOAT16: return "bfloat16";
        default: return "unsupported";
    }
}

// Thread-local description of the last failure (ddl_last_error).
void set_error(const std::string &msg);
const char *last_error();

// Error carried inside the library; converted to a status at the C-ABI (no exception
// crosses the boundary).
struct Error {
    int status;
    std::string msg;
};

[[noreturn]] inline void fail(int status, const std::string &msg) { throw Error{status, msg}; }

#define DDL_HIP(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            std::ostringstream _os;                                                         \
            _os << #expr << " failed: " << hipGetErrorString(_e) << " (" << __FILE__ << ":" \
                << __LINE__ << ")";                                                         \
            ::ddl::fail(DDL_STATUS_HIP_ERROR, _os.str());                                   \
        }                                                                                   \
    } while (0)

#define DDL_REQUIRE(cond, status, msg)                    \
    do {                                                  \
        if (!(cond)) {                                    \
            std::ostringstream _os;                       \
            _os << msg;                                   \
            ::ddl::fail((status), _os.str());             \
        }                                                 \
    } while (0)

// Logging (the reference logs per rank to log-<rank>.txt, GlobalLog.cc:17-49; here
// stderr, gated by the "log_level" config: 0 errors, 1 info, 2 debug).
int log_level();
void log_line(int level, const std::string &msg);

#define DDL_LOG(level, msg)                                     \
    do {                                                        \
        if (::ddl::log_level() >= (level)) {                    \
            std::ostringstream _os;                             \
            _os << msg;                                         \
            ::ddl::log_line((level), _os.str());                \
        }                                                       \
    } while (0)

// Step-by-step trace of the program posting (log_level >= 4): every HIP call of run_, flushed
// before the call, so a crash inside the runtime names the call it was in.
#define DDL_TRACE(msg)                                                                          \
    do {                                                                                        \
        if (::ddl::log_level() >= 4) {                                                          \
            std::ostringstream _os;                                                             \
            _os << msg;                                                                         \
            std::fprintf(stderr, "[ddl trace] %s\n", _os.str().c_str());                         \
            std::fflush(stderr);                                                                \
        }                                                                                       \
    } while (0)

// ---- kernels (reduce_kernels.hip) ----------------------------------------------------
constexpr int kMaxSegments = 8;

// Up to kMaxSegments independent out = a + b problems in one launch (one per ring).
struct SegTable {
    const void *a[kMaxSegments];
    const void *b[kMaxSegments];
    void *out[kMaxSegments];
    uint64_t n[kMaxSegments];
    int count;
};

// One N-input problem over the inputs x_0 = a, x_1 = b[0], ..., x_nb = b[nb-1]: the direct and
// one-shot schedules' reduce of a chunk with its P-1 received copies.
constexpr int kMaxInputs = 15;
// Addition order of an N-input fold (fp32 / fp64; integers wrap, so any order is the same):
enum FoldOrder : int {
    kFoldLeft = 0,      // ((x_0 + x_1) + x_2) + ...: the ring-0 order of the direct schedule
    kFoldMpichTree = 1, // MPICH 3.3.2 MPI_Allreduce above 2048 bytes (x in rank order): the first
                        // 2*rem inputs folded in pairs, then a pairwise tree over pof2 leaves
    kFoldBinomial = 2,  // MPICH 3.3.2 MPI_Allreduce up to 2048 bytes: binomial tree over ranks
};
// MPICH's order for an allreduce of `message_bytes` of `esize`-byte elements over P ranks
// (MPICH 3.3.2 MPIR_Allreduce_intra_auto): recursive doubling — the binomial order — when the
// message is at most MPIR_CVAR_ALLREDUCE_SHORT_MSG_SIZE = 2048 bytes or its element count is
// below pof2 (largest power of two <= P; above 2048 bytes that takes P >= 512), else
// reduce-scatter + allgather (pre-fold + pairwise tree). Pinned by live MPICH runs up to P = 520
// on one host (tests/golden, tests/test_live_mpich.py).
inline int mpich_fold_order(size_t message_bytes, size_t esize, int P) {
    size_t pof2 = 1;
    while (pof2 * 2 <= (size_t)P) pof2 *= 2;
    return message_bytes <= 2048 || message_bytes / esize < pof2 ? kFoldBinomial : kFoldMpichTree;
}
struct SegTableN {
    const void *a;
    const void *b[kMaxInputs];
    void *out;
    uint64_t n;
    int nb;
    int order = kFoldLeft;  // FoldOrder
};
// fp32/fp64/int: one rounding per add in `order`; fp16/bf16 (no reference order: the reference
// rejects them): accumulate in fp32 and round once at the end, whatever the order.
void launch_sumN(const SegTableN &t, int dtype, hipStream_t stream);
// Up to kMaxFoldBatch independent folds with the same input count and order in ONE launch
// (blockIdx.y = problem): the grouped allreduce folds every bucket's slice of a tick together, so
// 64 back-to-back 2 MiB fp16 chunks (C4) become 8 launches of 8 chunks instead of 64 latency-bound
// ones. No problem may read what another writes. Misaligned problems are launched one by one.
constexpr int kMaxFoldBatch = 8;
struct FoldBatch {
    SegTableN t[kMaxFoldBatch];
    int count;
};
void launch_sumN_batch(const SegTableN *t, int count, int dtype, hipStream_t stream);

// Reduce-kernel cache-policy / staging flags (bit set). kVariantDefault is what the engine uses;
// the others exist for measurement (ddl_reduce_sum2_variant, bench.py, tools/reduce_tune.hip).
enum ReduceVariant : int {
    kNtLoadA = 1,   // non-temporal loads of operand a (the rank's own gradient: read once)
    kNtLoadB = 2,   // non-temporal loads of operand b (the received chunk)
    kNtStore = 4,   // non-temporal stores of out
    kLdsStageB = 8, // operand b staged through LDS by global_load_lds_dwordx4
    kWtStore = 16,  // write-through stores of out (sc0 sc1: the line leaves the XCD's L2)
    kVariantMask = 31,
    // run form (r05): one workgroup per run of 8 tiles (kRun4: 4 tiles), a's run loaded, then
    // b's, then the stores — each workgroup on one stream at a time, as the fold's run form (cache
    // bits from the low bits; the LDS staging bit is not combined with it). default_variant takes
    // it with 4-tile runs from 32 to 128 MiB.
    kRunForm = 32,
    kRun4 = 64,
};
int default_variant(size_t bytes);  // standalone reduce (ddl_reduce_local / ddl_reduce_sum2), by bucket size
int ring_variant();     // reduce-scatter step of the ring
// Form of the N-input fold (config "fold_form"): 0 auto (the run form for chunks of at least 4 MiB
// and at least 7 inputs), 1 the tile form always, 2 the run form always (the binomial order is
// always tiled). Local: it changes no collective's program, only the kernel (the same sums either
// way).
void set_fold_form(int form);
void set_testing_fold_variant(int v);  // ddl_testing_fold_variant: 4 / 5 forced, -1 the size rule
int get_fold_form();

// out = a + b for each segment; dtype-generic. Returns via fail() on bad arguments.
// variant < 0 selects default_variant().
void launch_sum2(const SegTable &t, int dtype, hipStream_t stream, int variant = -1);
int device_cu_count();

// Chunk boundaries [cut[i], cut[i + 1]) of a host-staged transfer of `total` bytes through
// `chunk`-byte slots (chunk a multiple of 256): whole chunks, the last one short. They depend
// only on (total, chunk) — host_chunk_bytes is a shared tunable — so every rank cuts the same
// chunks (the per-chunk collectives must match). (r03 measured quarter chunks at the ends of a
// transfer — a shorter fill and drain — against whole chunks on two boxes: never faster, DESIGN §7;
// that option is gone.)
inline std::vector<size_t> host_chunk_cuts(size_t total, size_t chunk) {
    std::vector<size_t> cut{0};
    while (cut.back() < total) cut.push_back(cut.back() + std::min(chunk, total - cut.back()));
    return cut;
}

// Gather (dir 0: segments -> flat) / scatter (dir 1: flat -> segments) between tensors and a
// fusion buffer in one launch (pack.hip). Segment i sits at the running sum of the 256-byte-
// rounded lengths before it. Not thread-safe: one copier per engine thread.
class SegmentCopier {
public:
    SegmentCopier() = default;
    ~SegmentCopier();
    SegmentCopier(const SegmentCopier &) = delete;
    SegmentCopier &operator=(const SegmentCopier &) = delete;
    void run(int dir, void *flat, void *const *segs, const size_t *bytes, int count, hipStream_t stream);
    static size_t flat_bytes(const size_t *bytes, int count);

private:
    struct Slot {
        void *host = nullptr, *dev = nullptr;
        size_t cap = 0;
        void *idx = nullptr;  // first segment per span (k_span_index)
        size_t idx_cap = 0;
        hipEvent_t ready = nullptr;
    };
    Slot &free_slot_();  // a slot whose last table copy has been consumed (grows the pool)
    static constexpr size_t kMaxSlots = 64;
    std::vector<Slot> slots_;
    size_t next_ = 0;
};

// Memory a data path outgrew (r06). hipFree / hipHostFree synchronise the whole device, and on a
// thread that posts RCCL work that can deadlock the ranks once two communicators are in flight:
// rank A's handler of communicator X blocks in hipFree until its in-flight kernel of communicator
// Y finishes, which waits for rank B's Y kernel, which B's handler of Y has not posted because it
// is blocked the same way behind its X kernel, which waits for A's X work (found with multi-rank
// RCCL communicators on one GPU, tests/test_multiproc_rccl_gpu.py). So buffers that grow during
// operation (staging, fusion buffers, pinned slots, tuning scratch) hand their old allocation here
// instead of freeing it; ddl_finalize frees the lot once every communicator is gone. Growth is
// geometric, so what waits here is less than twice the final sizes.
void retire_device(void *p);
void retire_host(void *p);
void free_retired();
// Device scratch of at least `bytes` for the calling thread on the current device (the control
// collectives: config agreement, the tuner's max, split records) — no allocation per call.
void *thread_scratch(size_t bytes);

// Hardware-queue class of an engine stream (executor.h create_engine_stream).
enum class QueueClass { kPooled, kHigh, kLow };

}  // namespace ddl
