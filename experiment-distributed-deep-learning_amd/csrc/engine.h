// engine.h — communicators, configuration and the process-wide registry.
//
// Mirrors the reference's Global singleton wiring (src/cpp/global/Global.cc:10-34,
// initialize.cc:25-112) and its Communicator (communicate/backend/Communicator.h:18-118),
// MI355X-first: one process per GPU, one RCCL communicator per Communicator, the id is the
// address of the Communicator object (the reference uses the MPI_Comm* address,
// MPICommunicator.cc:107-109).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "control.h"
#include "executor.h"

namespace ddl {

class RequestHandler;  // keyed requests (handler.h)

struct Config {
    std::atomic<long long> algo{kAlgoRing};  // kAlgoRing / kAlgoDirect (schedule.h)
    std::atomic<long long> slice_bytes{2ll << 20};
    std::atomic<long long> rings{kMaxRings};
    std::atomic<long long> max_slices{8};
    // fusion plan cap; the reference uses MAX_MPI_BUFFER_SIZE = 2^31 - 1 (MPIBackend.h:12)
    std::atomic<long long> fusion_threshold_bytes{(1ll << 31) - 1};
    std::atomic<long long> log_level{0};
    // keyed requests: rank 0 waits this long after the first registration before proposing
    // a round (0 = propose at once, as the reference's READY token does)
    std::atomic<long long> cycle_time_us{0};
    // host-resident pipeline chunk (ddl_allreduce_host, keyed host requests)
    std::atomic<long long> host_chunk_bytes{32ll << 20};
    // memcpy workers of the keyed host-staging pipeline (pageable <-> pinned), besides the
    // engine thread itself
    std::atomic<long long> host_copy_threads{7};
    // keyed host allreduce plans whose outputs are all pinned and mapped into the device's
    // address space (torch pin_memory, hipHostMalloc, hipHostRegister): the unpack kernel writes
    // them over PCIe in place of the D2H copy and the host unpack memcpy (1 on, 0 always stage)
    std::atomic<long long> host_zero_copy{1};
    // keyed host requests: pageable tensors are hipHostRegister'ed once and the registration kept
    // (up to this many bytes, least recently used out), so repeated allreduce(cpu_tensor) calls take
    // the pinned paths. 0 (default) = off: a registered range must stay allocated while cached —
    // the caller opts in for tensors that live as long as the training loop (gradients), and
    // setting it back to 0 unregisters every cached range at once (ddl_set_config), before the
    // caller frees them: a freed range left registered poisons later copies from that address.
    std::atomic<long long> host_register_cache_bytes{0};
    // keyed host path: the engine thread and the copy threads bind to the CPUs of the GPU's NUMA
    // node (within the process's affinity) when its handler starts — pinned host memory lives
    // there, and threads on the other socket pack it at half the rate (1 on, 0 leave placement to
    // the OS)
    std::atomic<long long> host_numa_bind{1};
    // read-only statistics of that cache (ddl_get_config): bytes registered now, failed registrations
    std::atomic<long long> host_registered_bytes{0};
    std::atomic<long long> host_register_failures{0};
    std::atomic<long long> host_register_hits{0};  // tensors found inside a cached registration
    std::atomic<long long> host_unregistered_ranges{0};  // cached registrations dropped by ddl_host_unregister
    // read-only statistic (ddl_get_config "host_zero_copy_plans"): keyed host allreduce plans
    // that unpacked on the device in this process
    std::atomic<long long> host_zero_copy_plans{0};
    // read-only statistics of the keyed host plans' timeline (ddl_get_config, microseconds summed
    // over every plan of the process): the engine thread packing chunks into pinned slots (host
    // memcpy, with the copy threads), waiting for a slot whose earlier DMA / device work is still
    // in flight, and unpacking staged results
    std::atomic<long long> host_pack_ns{0};  // read as microseconds (host_pack_us, ...)
    std::atomic<long long> host_wait_ns{0};
    std::atomic<long long> host_unpack_ns{0};
    // keyed host allreduce plans: the pinned-output check before each plan, and the whole of
    // each plan's staging loop (pack, slot waits, posting, unpack; host_plan_us)
    std::atomic<long long> host_check_ns{0};
    std::atomic<long long> host_plan_ns{0};
    // inside the staging loop, besides pack / slot waits / unpack waits: the chunk's allreduce
    // posting (host_coll_us), the D2H enqueue of staged chunks (host_d2h_post_us) and the unpack
    // job's submission (host_unpack_submit_us)
    std::atomic<long long> host_coll_ns{0};
    std::atomic<long long> host_d2h_post_ns{0};
    std::atomic<long long> host_unpack_submit_ns{0};
    // the unpack lane's jobs (staged outputs of keyed host plans), on the lane's thread: polling
    // the chunk's D2H event (host_lane_d2h_wait_us), then the pinned download slot -> output
    // memcpy with the copy threads (host_lane_copy_us, host_lane_copy_bytes), per job
    // (host_lane_jobs)
    std::atomic<long long> host_lane_d2h_wait_ns{0};
    std::atomic<long long> host_lane_copy_ns{0};
    std::atomic<long long> host_lane_copy_bytes{0};
    std::atomic<long long> host_lane_jobs{0};
    // autotune the schedule per bucket-size class on first use (P > 1): 1 on, 0 use the
    // fields above as set
    std::atomic<long long> tune{1};
    // keyed fusion: a multi-request plan larger than this runs as a pipeline of sub-plans of at
    // most this many bytes — pack of sub-plan j+1 and unpack of j-1 overlap the allreduce of j
    // (0 = one pack, one allreduce, one unpack per plan)
    std::atomic<long long> fusion_pipeline_bytes{256ll << 20};
    // a one-rank world skips the keyed data plane (the sum is the input); 0 runs pack ->
    // allreduce -> unpack anyway (tests of the fusion path on one GPU)
    std::atomic<long long> one_rank_shortcut{1};
    // keyed rounds: 1 — a completion thread waits for a round's data plane and fires its done()
    // calls while the engine thread negotiates and enqueues the next round; 0 — the engine
    // thread waits for each round before negotiating the next (as the reference's recv thread
    // blocks in MPI_Allreduce)
    std::atomic<long long> pipeline_rounds{1};
    // 1: every sum equals the reference's MPI_Allreduce (MPICH 3.3.2) bit for bit — direct /
    // one-shot folds in MPICH's order, the ring replaced by the direct schedule at P > 2
    // (RingConfig::ref_order); 0: ring order / left folds (error-bounded against the reference)
    std::atomic<long long> reference_order{1};
    // how a program is posted inside a hipGraph capture: 0 (default) — serially on the
    // captured stream: one dependency chain, which HIP 7.0's graph executor replays fastest
    // (1.7-3x faster than the DAG below in profiles/r03/graph/capture_overlap_*); 2 — as a
    // single-stream DAG: every op on the captured stream with its dependencies set explicitly
    // from its logical stream (comm / compute of each rank), so the graph keeps the recv / reduce /
    // send overlap without forked streams. (r03's mode 1, the forked streams as eagerly, crashed
    // hipStreamEndCapture in this HIP runtime and was removed in r04.)
    std::atomic<long long> capture_mode{0};
    // multi-rank executors' compute streams (the reduce / fold kernels that overlap RCCL's send /
    // recv kernels) run on all CUs but every n-th (n = 2, 4, 8; 0 = all CUs, the default): those
    // stay free for RCCL. The kernels keep their full HBM rate on such masks (tools/cu_mask_probe.py:
    // 6.56-6.59 vs 6.59 TB/s), but a CU-masked stream takes a hardware queue of its own: 8 processes
    // sharing one GPU ran their collectives 2.6x slower with it — off until a node
    // measures it (bench leg compute_cu_mask_ab). Read when an executor is created; local.
    std::atomic<long long> compute_cu_mask{0};
    // RCCL communicator configuration (ncclConfig_t.minCTAs / maxCTAs): the
    // bounds on the channel (CTA) count RCCL gives a communicator, which also caps its p2p
    // channels — whether the direct schedule's 7 concurrent sends and receives per tick fill
    // 7 xGMI links depends on it. 0 = NCCL_CONFIG_UNDEF_INT (RCCL's own choice, the default).
    // Read when a communicator is created (ddl_init, ddl_comm_split, the keyed data plane's
    // private split); shared (in shared_hash): ranks with different channel counts would post
    // mismatched RCCL kernels.
    std::atomic<long long> rccl_min_ctas{0};
    std::atomic<long long> rccl_max_ctas{0};
    // 1: the engine's streams are created in hardware-queue classes (executor.h QueueClass): the
    // world's user streams, its keyed path and the splits each in a priority pool of HIP's
    // hardware queues of their own; 0 (default; env DDL_QUEUE_ISOLATION seeds it): every stream
    // in HIP's default pool. Off by default: the extra queues crawled the 8-rank one-GPU rehearsal
    // (profiles/r06/s29) and no node has measured them yet. Read when a communicator is created;
    // local.
    std::atomic<long long> queue_isolation{0};
    // bumped by every ddl_set_config
    std::atomic<long long> epoch{0};
    // Hash of the tunables every rank of a communicator must share (they shape the collectives'
    // programs, the fusion plans and the host chunks): algo, slice_bytes, rings, max_slices,
    // fusion_threshold_bytes, tune, fusion_pipeline_bytes, reference_order, host_chunk_bytes,
    // rccl_min_ctas, rccl_max_ctas.
    // Never 0 or kCfgMismatch. Local tunables (log_level, cycle_time_us, host_copy_threads,
    // host_zero_copy, pipeline_rounds, one_rank_shortcut) are not in it.
    uint64_t shared_hash() const;
    RingConfig ring() const {
        RingConfig c;
        c.algo = (int)algo.load();
        c.rings = (int)rings.load();
        c.slice_bytes = (size_t)slice_bytes.load();
        c.max_slices = (int)max_slices.load();
        c.ref_order = reference_order.load() ? 1 : 0;
        return c;
    }
};
Config &config();

struct TuneResult {
    std::vector<RingConfig> candidates;  // [0] = the configured schedule
    std::vector<float> ms;               // per candidate, max over ranks
    int chosen = -1;
};

// floor(log2(bytes)): the autotuner's bucket-size class.
int size_class(size_t bytes);

// Times every candidate schedule for a P-rank bucket of `bytes` (`run` launches one allreduce
// on `stream`), combines the per-candidate times across ranks with `agree_max` and picks the
// fastest. Deterministic given the agreed times, so all ranks choose the same schedule.
TuneResult run_tuning(int P, size_t bytes, hipStream_t stream, const RingConfig &base,
                      const std::function<void(const RingConfig &)> &run,
                      const std::function<void(float *, int)> &agree_max);

class Communicator {
public:
    // `hooks` (test harness only, ddl_init_test_transport): groups go to host callbacks, `tag`
    // names this communicator to them, `world_ranks[i]` is the world rank of rank i (empty: the
    // world itself); nullptr = RCCL on `nccl`.
    // `qc`: the hardware-queue class of the communicator's own streams (executor, control, host
    // pipeline; executor.h QueueClass), decided by who creates it: the world kPooled, the world's
    // private keyed communicator kHigh, splits and theirs kLow (RCCL only, config
    // queue_isolation 1).
    Communicator(int rank, int size, int device, ncclComm_t nccl, std::shared_ptr<TestHooks> hooks = nullptr,
                 long long tag = 0, std::vector<int> world_ranks = {}, QueueClass qc = QueueClass::kPooled);
    ~Communicator();

    long long id() const { return reinterpret_cast<long long>(this); }
    int rank() const { return rank_; }
    int size() const { return size_; }
    int device() const { return device_; }
    QueueClass queue_class() const { return qclass_; }
    // the class of the streams of this communicator's keyed path (handler, fusion pipe, private
    // data-plane communicator): apart from the world's user streams (kHigh) for the world, its
    // split's (kLow) for a split; fixed at creation like queue_class()
    QueueClass keyed_queue_class() const { return keyed_qclass_; }
    ncclComm_t nccl() const { return nccl_; }

    // Communicator::allreduce (reference Communicator.h:45-48), device buffers, stream-ordered.
    // `order_bytes`: the size of the reference's MPI_Allreduce message this call is part of (a
    // fused plan's bytes, the whole host buffer), which fixes MPICH's summation order; 0 = n.
    void allreduce(const void *send, void *recv, size_t n, int dtype, int op, hipStream_t stream,
                   size_t order_bytes = 0);
    // Host-resident buckets (the reference's deployment case: framework CPU tensors behind the
    // MPI buffers): chunked pinned H2D -> device ring -> D2H pipeline; returns when recv holds
    // the result.
    // `count` buckets of one dtype in one grouped program (RingExecutor::allreduce_batch); the
    // schedule is the one tuned for the largest bucket's size class
    void allreduce_batch(const void *const *send, void *const *recv, const size_t *n, int count, int dtype, int op,
                         hipStream_t stream);
    void allreduce_host(const void *send, void *recv, size_t n, int dtype, int op);
    // Communicator::broadcast (reference Communicator.h:81-92): root's n elements of `buf` into
    // every rank's `buf`, stream-ordered.
    void broadcast(void *buf, size_t n, int dtype, int root, hipStream_t stream);
    // Communicator::allgather, per-rank counts (Communicator.h:50-66): rank q's counts[q]
    // elements land at recv + displs[q] on every rank; `send` holds counts[rank()] elements.
    void allgatherv(const void *send, void *recv, const size_t *counts, const size_t *displs, int dtype,
                    hipStream_t stream);
    // MPI_Comm_split (MPICommunicator.cc:92-101), collective over this communicator: ranks of one
    // color form a communicator ordered by (key, rank here); color < 0 joins none (fails after
    // taking part). The members exchange (color, key, control endpoint) over this
    // communicator's data plane; with `keyed` a new communicator of more than one rank also gets
    // its own token ring over TCP and its private data-plane communicator for keyed requests, as
    // the reference gives every communicator its own handler and token ring
    // (RingTokenCommunicateController.cc:53-79, MPIRingTokenCommunication.cc:50-57).
    std::shared_ptr<Communicator> split(int color, int key, bool keyed = true);

    // The schedule for an n-element bucket: the tuned choice for its size class (tuning it now,
    // collectively, if this is the class's first bucket), or the configured one.
    RingConfig ring_config(size_t n, int dtype, hipStream_t stream);
    // Tuning result for the size class of `bytes` (chosen = -1 if not tuned yet).
    TuneResult tune_result(size_t bytes);

    // Keyed requests: the handler (created on first use; not collective), this communicator's
    // token ring and the private data-plane communicator its handler reduces on.
    RequestHandler &handler();
    RequestHandler *handler_if_created();
    ControlChannel *control() const { return control_.get(); }
    // Collective over this communicator: adopts `ch` (already connected over these ranks) as the
    // token ring and creates the keyed data-plane communicator (world: ddl_control_connect).
    void enable_keyed(std::shared_ptr<ControlChannel> ch);
    std::shared_ptr<Communicator> keyed_data() const { return keyed_data_; }
    RingExecutor &executor() { return *exec_; }
    std::mutex &mutex() { return mu_; }
    // RCCL's own ncclAllReduce on this communicator (bench comparator), as a user collective.
    void rccl_allreduce(const void *send, void *recv, size_t n, int dtype, hipStream_t stream);
    // How the ranks of this communicator are connected: kind 0 none (one rank), 1 RCCL
    // (*ranks = ncclCommCount), 2 the test transport (*ranks = size).
    void transport(int *kind, int *ranks) const;

    // ---- order between user collectives and keyed rounds (a communicator with a token ring) ----
    // The keyed handler reduces on a private RCCL communicator; the user's collectives run on this
    // one. Two RCCL communicators must see their operations in the same order on every rank
    // (their kernels can share a hardware queue), which the reference gets from
    // MPI_THREAD_MULTIPLE (MPIBackend.cc:77-86). So every keyed round is placed after exactly U*
    // user collectives on every rank: each rank reports how many it has issued when it joins the
    // round (and issues no more until the round's place is known), rank 0 announces the maximum,
    // and each rank enqueues the round's data plane once its user collectives reach U* — never
    // before, never after. With no keyed round under way a user collective only takes a mutex.
    long long round_freeze();            // handler: user collectives entered here; no more enter
    void round_release(long long at);    // handler: the round goes after user collective `at`
    void round_enter(long long at);      // handler: waits until `at` user collectives are enqueued
    void round_unfreeze();               // handler: the round is enqueued (or failed)
    // handler: it stopped on an error (a control link lost mid-round, a token-protocol fault) or is
    // shutting down. Clears the freeze, wakes every gate wait, and from then on every user
    // collective on this communicator fails with `status` instead of blocking behind a round that
    // can no longer be placed (the keyed / user collective order is no longer known).
    void round_abort(int status, const std::string &why);
    long long user_collectives() const;  // issued so far (tests)
    // The round release points this rank used, most recent last (bounded log; tests compare
    // them across ranks).
    std::vector<long long> round_log() const;

    // Shared-config agreement of the direct path (ddl_allreduce & co.): at the first collective,
    // and whenever this rank's shared tunables changed since the last agreement, every rank's
    // Config::shared_hash() is allgathered over the data plane; a mismatch fails the collective on
    // every rank with DDL_STATUS_CONFIG_MISMATCH before any program is built (different slice
    // sizes would otherwise build different programs and hang RCCL). The exchange is collective:
    // it is matched only when every rank changes its values between the same two collectives; a
    // one-sided change after the first collective posts an unmatched exchange (unsupported, see
    // ddl_set_config in ddl_amd.h). Keyed rounds carry the hash in their tokens instead (every
    // round, so they see one-sided changes too).
    void agree_config(hipStream_t stream);

private:
    class UserCollective;  // scope of one user collective (the order gate above)
    std::mutex gate_mu_;
    std::condition_variable gate_cv_;
    long long user_seq_ = 0;    // user collectives entered
    long long user_done_ = 0;   // user collectives enqueued (or failed)
    bool frozen_ = false;       // a keyed round is being placed
    int aborted_ = 0;           // round_abort's status (0: the handler is healthy)
    std::string abort_msg_;
    long long release_ = 0;     // while frozen: user collectives may run while user_seq_ < release_
    std::vector<long long> round_log_;
    uint64_t agreed_hash_ = 0;  // last shared-config hash all ranks agreed on (0: none yet)
    uint64_t tuned_hash_ = 0;   // the shared config the tuned choices were made under
    hipStream_t ctl_stream_ = nullptr;  // the config agreement's exchange
    // elementwise max of host floats over the ranks (the autotuner's agreement)
    void agree_max_(float *values, int count, hipStream_t stream);

    int rank_, size_, device_;
    ncclComm_t nccl_;
    std::shared_ptr<TestHooks> hooks_;
    long long tag_ = 0;
    std::vector<int> world_ranks_;
    Transport *cb_ = nullptr;  // the executor's transport when hooks_ (owned by exec_): host groups
    std::mutex mu_;  // one collective at a time per communicator (RCCL ordering)
    std::unique_ptr<RingExecutor> exec_;
    std::shared_ptr<ControlChannel> control_;
    std::shared_ptr<Communicator> keyed_data_;
    std::unique_ptr<RequestHandler> handler_;
    std::mutex handler_mu_;
    std::map<int, TuneResult> tuned_;  // by floor(log2(bucket bytes)); guarded by mu_
    TuneResult tune_(size_t n, int dtype, hipStream_t stream, const RingConfig &base);
    // host pipeline resources (lazily created)
    hipStream_t h2d_ = nullptr, ring_ = nullptr, d2h_ = nullptr;
    static constexpr int kHostSlots = 4;
    void *slots_[kHostSlots] = {};
    size_t slot_bytes_ = 0;
    // the tuner's scratch buckets (grow-only, retired on growth: no hipFree while others run)
    void *tune_a_ = nullptr, *tune_b_ = nullptr;
    size_t tune_cap_ = 0;
    QueueClass qclass_ = QueueClass::kPooled, keyed_qclass_ = QueueClass::kPooled;
};

// Set on a request handler's engine and completion threads. The last reference to a communicator
// dropped on such a thread (a done() callback that detaches its own communicator, or any C-ABI
// call from a callback racing a detach) must not run the destructor there: ~RequestHandler joins
// those threads. CommunicatorDeleter hands the destruction to a thread of its own instead.
extern thread_local bool t_handler_thread;

struct CommunicatorDeleter {
    void operator()(Communicator *c) const;
};
// Waits up to limit_ms for the communicators being deleted off their handlers' threads; false on
// timeout. ddl_finalize calls it (and an exit hook, 10 s).
bool wait_deferred_deletions(long long limit_ms);


// every Communicator is owned through this (make_shared would bypass the deleter)
template <class... A>
std::shared_ptr<Communicator> new_communicator(A &&...a) {
    return std::shared_ptr<Communicator>(new Communicator(std::forward<A>(a)...), CommunicatorDeleter{});
}

class Registry {
public:
    static Registry &get();
    void add(const std::shared_ptr<Communicator> &c);
    std::shared_ptr<Communicator> find(long long id);  // throws if unknown
    void detach(long long id);
    std::shared_ptr<Communicator> world();              // throws if not initialized
    std::vector<std::shared_ptr<Communicator>> all();   // every registered communicator
    void set_world(const std::shared_ptr<Communicator> &c);
    void clear();
    bool initialized();

private:
    std::mutex mu_;
    std::map<long long, std::shared_ptr<Communicator>> comms_;
    std::shared_ptr<Communicator> world_;
};

// Cleanups ddl_finalize runs once the registry is cleared (the testing library adds its own: its
// control channels and worlds).
void add_finalize_hook(void (*fn)());
void run_finalize_hooks();

// Current-device guard: sets `device` for the scope, restores the previous one.
class DeviceGuard {
public:
    explicit DeviceGuard(int device);
    ~DeviceGuard();

private:
    int prev_ = -1;
};

// ---- RCCL pieces shared by the product path and the one-GPU loopback tests ---------------------
// ncclCommInitRank of `rank` in a `size`-rank communicator from a 128-byte ncclUniqueId.
ncclComm_t rccl_init_rank(int rank, int size, const void *unique_id, size_t len);
// ncclCommSplit (MPI_Comm_split, MPICommunicator.cc:92-101): nullptr when color < 0 (the rank is
// in no communicator); *rank / *size of the new communicator from ncclCommUserRank / Count.
ncclComm_t rccl_split(ncclComm_t parent, int color, int key, int *rank, int *size);
// Elementwise max over the communicator's ranks of `count` host floats (the autotuner's
// agreement step: one ncclAllReduce(MAX) on `stream`, host-synchronising).
void rccl_max_floats(ncclComm_t comm, float *values, int count, hipStream_t stream);
// values[rank] of every rank into values[0 .. size) (one ncclAllGather, host-synchronising).
void rccl_allgather_u64(ncclComm_t comm, uint64_t *values, int size, int rank, hipStream_t stream);
// Fails with DDL_STATUS_CONFIG_MISMATCH (naming every rank's hash) unless all hashes are equal.
void check_config_agreement(int rank, const std::vector<uint64_t> &hashes);

}  // namespace ddl
