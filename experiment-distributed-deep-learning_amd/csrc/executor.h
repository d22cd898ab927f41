// executor.h — runs a ring program on HIP streams: recv -> reduce -> send overlap.
//
// Per rank two non-blocking streams: `comm` posts the send/recv groups of each tick (RCCL
// kernels), `compute` runs the reduce kernel of each reduce-scatter tick. Events chain them:
// reduce(s,k) waits for group(s,k); group(s+1,k) waits for reduce(s,k) (it forwards what that
// reduce produced). With K slices per chunk the group of slice k+1 overlaps the reduce of
// slice k. The caller's stream is forked into both and joined back — no host
// synchronisation anywhere on the path.
#pragma once

#include <atomic>
#include <functional>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "deptrace.h"
#include "fusion.h"
#include "rccl_api.h"
#include "schedule.h"

namespace ddl {

class Transport {
public:
    virtual ~Transport() = default;
    // Post one tick's sends and recvs as one group on `stream`.
    virtual void group(const std::vector<P2POp> &ops, hipStream_t stream) = 0;
    // Allgather of `bytes` per rank into recv (rank q's block at q * bytes) on `stream`.
    virtual void allgather(const GatherOp &g, hipStream_t stream) = 0;
    // Whether group() / allgather() only enqueue stream work (so they can be captured into a
    // hipGraph); a transport that synchronises the host cannot.
    virtual bool capturable() const = 0;
    // One group of host-buffer operations (the test transport's config agreement and tuner max;
    // RCCL communicators use collectives instead): refused by every other transport.
    virtual void host_group(std::vector<ddl_p2p_op> &ops);
};

// True while `s` is being captured into a hipGraph (hipStreamBeginCapture, torch.cuda.graph).
// The engine then enqueues graph-safe work only: no allocation, no host synchronisation, no
// autotuning — the calls that need those must run once outside the capture first (the same
// warm-up rule as for any captured workload).
bool stream_capturing(hipStream_t s);
// Config "capture_mode": how a program is posted inside a capture — 0 serially on the captured
// stream, 2 as a single-stream DAG (Poster).
int config_capture_mode();
// Config "compute_cu_mask" (0 off, 2 / 4 / 8): the compute streams of multi-rank executors leave
// every n-th CU to RCCL (read when an executor is created).
int config_compute_cu_mask();
// A non-blocking stream whose kernels avoid every `every`-th CU (every >= 2; otherwise, or where
// the runtime refuses CU masks, an ordinary non-blocking stream).
hipStream_t create_compute_stream(int every);
// Hardware-queue isolation of the engine's streams (r06). HIP maps a process's
// streams of one priority onto a small pool of in-order hardware queues (tools/queue_probe.hip:
// the 8th ordinary stream shares the 1st one's queue, profiles/r06/s24), so two communicators'
// RCCL kernels — or their stream waits — can land on one queue and run in posting order; ranks
// that posted them in different orders then wait for each other forever (three communicators
// running keyed rounds at once over real RCCL, profiles/r06/s23). Each priority has a pool of
// its own (s24), so the engine spreads its communicators over the three:
//  kPooled  the default priority: the world's own executor (the user's direct collectives,
//           ordered by the user and, against keyed rounds, by §6) and the test harness;
//  kHigh    the greatest priority: the world's keyed data plane (handler, fusion pipe, its
//           private communicator) — apart from the user's streams, and communication first;
//  kLow     the least priority: every stream of a split communicator and of its keyed path.
// Splits still share the least priority's pool with each other: keyed rounds on two splits that
// share ranks are not isolated. All three are non-blocking streams (a CU-masked
// stream would get a queue of its own but is ordered with the legacy NULL stream).
// Config "queue_isolation" 0 (the default) makes every stream kPooled.
// (enum QueueClass { kPooled, kHigh, kLow } lives in common.h)
hipStream_t create_engine_stream(QueueClass qc, int cu_mask_every = 0);

// Posts a program's ops on its logical streams (each rank's comm / compute stream, a transport
// stream) with event records and waits between them, in one of three ways:
//  * kStreams — on the real streams: record / wait are hipEventRecord / hipStreamWaitEvent (eager
//    calls; r03's capture_mode 1 posted captures this way too, and HIP 7.0's hipStreamEndCapture
//    crashed on it — removed in r04);
//  * kSerial — every op on the caller's stream in posting order, records and waits dropped
//    (stream order implies every dependency: they all point backwards; capture_mode 0, the
//    default: the chain replays fastest in HIP 7.0's graph executor);
//  * kDag — inside a capture: every op on the captured stream, whose capture dependency set is
//    replaced right before the op by the op's logical stream's node set
//    (hipStreamUpdateCaptureDependencies) and read back right after it (the op's terminal nodes,
//    hipStreamGetCaptureInfo_v2); records copy a logical stream's node set, waits union one in.
//    The graph gets exactly the forked program's DAG — recv / reduce / send overlap included —
//    with no forked stream, which sidesteps the runtime's capture defect with three or more
//    cross-waiting forked streams (capture_mode 2).
// Use: `X(..., p.on(s)); p.posted(s);` around every op posted on logical stream s.
class Poster {
public:
    enum Mode { kStreams, kSerial, kDag };
    Poster(Mode m, hipStream_t user);
    // the mode run_ uses for a call on `user`: kStreams unless `user` is being captured
    static Mode mode_for(hipStream_t user);
    Mode mode() const { return m_; }
    hipStream_t on(hipStream_t s);  // the real stream to post logical stream s's next op on
    void posted(hipStream_t s);     // after that op (kDag: s's node set = the op's terminal nodes)
    void record(hipEvent_t e, hipStream_t s);
    void wait(hipStream_t s, hipEvent_t e);
    // kDag: leave the captured stream depending on the caller's logical node set (after the
    // program's joins, every branch); a no-op otherwise
    void finish();

private:
    Mode m_;
    hipStream_t user_;
    std::map<hipStream_t, std::vector<hipGraphNode_t>> tail_;
    std::map<hipEvent_t, std::vector<hipGraphNode_t>> ev_;
};

class RcclTransport : public Transport {
public:
    explicit RcclTransport(ncclComm_t comm) : comm_(comm) {}
    void group(const std::vector<P2POp> &ops, hipStream_t stream) override;
    void allgather(const GatherOp &g, hipStream_t stream) override;  // ncclAllGather
    bool capturable() const override { return true; }

private:
    ncclComm_t comm_;
};

// Test harness only (ddl_init_test_transport, testing library): groups and the tuner's
// max-reduce go through host callbacks, so several processes can run the whole engine on one GPU
// without RCCL. The transport itself (CallbackTransport, test_worlds.h) is built by
// `make_transport`, which the testing library sets; the deployment library has no way to create
// hooks.
struct TestHooks {
    ddl_test_group_fn group = nullptr;
    ddl_test_max_fn max = nullptr;
    void *user = nullptr;
    std::atomic<long long> next_tag{1};  // communicator tags: 0 = world, then splits in order
    std::unique_ptr<Transport> (*make_transport)(const std::shared_ptr<TestHooks> &hooks, long long tag,
                                                 std::vector<int> world_ranks, int rank, int size) = nullptr;
};

// Mutation knob for the executor's ordering tests (ddl_testing_drop_wait): RingExecutor::run_
// skips the wait_reduce wait of this tick (-1: none).
void set_testing_drop_wait(int tick);

// Streams, events and staging memory of one rank (reused across calls).
class RankResources {
public:
    // cu_mask_every >= 2: the compute stream (reduce / fold kernels) is created with every
    // cu_mask_every-th CU masked off (config "compute_cu_mask"), leaving those to RCCL's kernels
    RankResources(int device, int cu_mask_every = 0, QueueClass qc = QueueClass::kPooled);
    ~RankResources();
    RankResources(const RankResources &) = delete;
    RankResources &operator=(const RankResources &) = delete;

    void ensure_events(size_t ticks);
    // Staging of at least `bytes`; growing it is refused while the caller's stream is captured.
    // Once a capture has used the staging buffer, a graph may hold its address for as long as
    // the graph lives: a later (eager) growth retires the buffer instead of freeing it — it stays
    // allocated until these resources are destroyed, so replaying the graph stays valid.
    void *ensure_staging(size_t bytes, bool capturing = false);
    size_t retired_staging() const { return retired_.size(); }

    int device;
    hipStream_t comm = nullptr, compute = nullptr;
    std::vector<hipEvent_t> comm_ev, red_ev, pre_ev, post_ev;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr, join_cp_ev = nullptr;

private:
    void *staging_ = nullptr;
    size_t staging_bytes_ = 0;
    bool staging_captured_ = false;  // a graph capture has used staging_
    std::vector<void *> retired_;    // captured staging buffers replaced by a larger one
};

// Optional timing of the reduce kernels on the compute stream (bench.py's roofline leg):
// timing events bracket every reduce launch while enabled; totals are read on demand.
struct KernelStats {
    long long launches = 0;
    double bytes = 0;  // algorithmic HBM bytes: 3 * n * sizeof(T) per ring step, (nb + 2) * n * sizeof(T) per fold
    double ms = 0;
};

// Single-rank executor over a Transport (RCCL in production).
class RingExecutor {
public:
    RingExecutor(int rank, int size, int device, std::unique_ptr<Transport> transport,
                 QueueClass qc = QueueClass::kPooled);
    ~RingExecutor();
    void allreduce(const void *in, void *out, size_t n, int dtype, hipStream_t user,
                   const RingConfig &cfg);
    // `count` buckets of one dtype as one grouped program (build_batch_program): one group and
    // batched folds per tick instead of a program per bucket
    void allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                         hipStream_t user, const RingConfig &cfg);
    void broadcast(void *buf, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg);
    void allgatherv(const void *send, void *recv, const size_t *counts, const size_t *displs, int dtype,
                    hipStream_t user);
    int rank() const { return rank_; }
    int size() const { return size_; }
    void set_timing(bool on);
    KernelStats collect_stats();  // synchronises the recorded timing events, then resets
    const RankResources &resources() const { return res_; }

private:
    // posts prog_ on the streams, forked from / joined to user (graph-safe when user is captured)
    void run_(int dtype, hipStream_t user);

    int rank_, size_;
    std::unique_ptr<Transport> transport_;
    RankResources res_;
    RingProgram prog_;
    bool timing_ = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timed_;  // recorded, not yet collected
    std::vector<double> timed_bytes_;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> free_pairs_;
};

// Most recent tick <= w that launched a reduce (-1 if none).
int last_reduce_at_or_before(const RingProgram &p, int w);

// Launches a tick's reduce (2-input ring step or N-input direct fold) on `stream`; returns its
// algorithmic HBM bytes.
double launch_tick_reduce(const Tick &tk, int dtype, hipStream_t stream);
// The byte ranges a tick's reduce reads and writes, and a trace label (deptrace.h).
std::vector<dep::Access> tick_reduce_access(const Tick &tk, int dtype);
std::string dep_label(const char *what, int rank, size_t tick);

}  // namespace ddl
