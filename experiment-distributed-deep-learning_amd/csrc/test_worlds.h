// test_worlds.h — the engine's test / diagnostic harness, linked into the testing library only
// (libddl_amd_testing.so, include/ddl_amd_testing.h): the host-callback test transport that lets
// several processes run the whole engine on one GPU, P virtual ranks in one process over device
// copies or a one-rank RCCL communicator (LocalWorld, RcclLoopback), and P production
// RingExecutors on threads over an asynchronous fabric (ThreadWorld). The deployment library
// (libddl_amd.so) contains none of it; both link the same engine objects.
#pragma once

#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "engine.h"
#include "executor.h"

namespace ddl {

// Stages the sends in pinned host memory (copies ordered on the group's stream only),
// synchronises that stream, runs the callback, copies the received bytes to the device: the
// group is complete, in stream order, when group() returns.
// Peers are ranks of the communicator; the callback sees world ranks (world_ranks[peer], or the
// peer itself when world_ranks is empty).
class CallbackTransport : public Transport {
public:
    CallbackTransport(std::shared_ptr<TestHooks> hooks, long long tag, std::vector<int> world_ranks, int rank,
                      int size)
        : hooks_(std::move(hooks)), tag_(tag), world_ranks_(std::move(world_ranks)), rank_(rank), size_(size) {}
    void group(const std::vector<P2POp> &ops, hipStream_t stream) override;
    // own block copied on the device, the others as one group of sends / recvs
    void allgather(const GatherOp &g, hipStream_t stream) override;
    bool capturable() const override { return false; }
    // One group of host-buffer operations straight to the callback (no device staging).
    void host_group(std::vector<ddl_p2p_op> &ops) override;
    ~CallbackTransport() override;
    CallbackTransport(const CallbackTransport &) = delete;
    CallbackTransport &operator=(const CallbackTransport &) = delete;

private:
    std::shared_ptr<TestHooks> hooks_;
    long long tag_;
    std::vector<int> world_ranks_;
    int rank_, size_;
    char *pinned_ = nullptr;  // host side of a group's device buffers (pinned: truly async copies)
    size_t pinned_bytes_ = 0;
};

// TestHooks::make_transport of ddl_init_test_transport's hooks
std::unique_ptr<Transport> make_callback_transport(const std::shared_ptr<TestHooks> &hooks, long long tag,
                                                   std::vector<int> world_ranks, int rank, int size);

// In-process thread transport (test / diagnostic, ddl_testing_thread_*): P threads, each driving
// its own RingExecutor — the production executor, asynchronously — exchange through device
// copies with RCCL's contract: group() only rendezvous with the peers on the HOST ENQUEUE (a
// receive waits until the matching send is posted, never until it has run), the k-th send from q
// to r matches r's k-th receive from q (per-pair FIFO, as RCCL), a receive is a
// hipStreamWaitEvent on the sender's "ready" event (recorded where the send was posted) plus a
// D2D copy, and the sender's stream waits for the receiver's "copied" event before anything
// after the group may overwrite the send buffer. No hipStreamSynchronize anywhere: a missing
// event wait inside the executor shows up as wrong data, which the host-synchronising test
// transport (CallbackTransport) would hide.
class ThreadFabric {
public:
    // `loopback` (a one-rank RCCL communicator, optional): each matched send / receive pair moves
    // its bytes through RcclTransport::group as a self send + self receive on the receiver's
    // stream (after the wait on the sender's ready event) instead of a D2D copy — the production
    // executor then runs asynchronously AND hands its data to RCCL (ddl_testing_thread_transport)
    explicit ThreadFabric(int P, ncclComm_t loopback = nullptr);
    ~ThreadFabric();
    ThreadFabric(const ThreadFabric &) = delete;
    ThreadFabric &operator=(const ThreadFabric &) = delete;
    struct Send {
        const void *ptr;
        size_t bytes;
        int tag;
        hipEvent_t ready;
        hipEvent_t copied = nullptr;  // set by the receiver once its copy is enqueued
    };
    int size() const { return P_; }
    void group(int rank, const std::vector<P2POp> &ops, hipStream_t stream);
    void abort();  // wakes every waiter with an error (a rank failed)
    // Between calls (every rank's host enqueue done, so every wait on them has been issued): the
    // events handed out become reusable.
    void recycle();

private:
    hipEvent_t event_();  // an event no pending host wait refers to
    int P_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::deque<std::shared_ptr<Send>>> q_;  // q_[from * P + to]: posted, not yet received
    std::vector<hipEvent_t> events_;
    size_t next_event_ = 0;
    bool aborted_ = false;
    std::unique_ptr<RcclTransport> loop_;  // see the constructor
    std::mutex loop_mu_;                   // one thread at a time inside an RCCL group
public:
    std::atomic<long long> loopback_pairs{0};  // pairs moved through RCCL
};

class ThreadTransport : public Transport {
public:
    ThreadTransport(std::shared_ptr<ThreadFabric> fab, int rank) : fab_(std::move(fab)), rank_(rank) {}
    void group(const std::vector<P2POp> &ops, hipStream_t stream) override { fab_->group(rank_, ops, stream); }
    void allgather(const GatherOp &g, hipStream_t stream) override;
    bool capturable() const override { return false; }

private:
    std::shared_ptr<ThreadFabric> fab_;
    int rank_;
};

// P virtual ranks in one process on one GPU: the same per-rank programs, with
// device-to-device copies standing in for RCCL send/recv (matched by peer and ring tag).
//
// With `loopback` (a one-rank RCCL communicator) the bytes move through RCCL instead: each
// tick's matched send/recv pairs of all P virtual ranks are posted through RcclTransport::group
// as self-send / self-recv pairs in matching order (RCCL pairs the k-th send to a peer with the
// k-th receive from it), on a transport stream that waits for every rank to reach the tick.
// That runs the production transport code on one GPU (test / diagnostic path).
class LocalWorld {
public:
    LocalWorld(int nranks, int device, ncclComm_t loopback = nullptr);
    ~LocalWorld();
    void allreduce(const void *const *in, void *const *out, size_t n, int dtype, hipStream_t user,
                   const RingConfig &cfg);
    // in[r * count + b] / out[r * count + b]: rank r's bucket b (RingExecutor::allreduce_batch)
    void allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                         hipStream_t user, const RingConfig &cfg);
    void broadcast(void *const *bufs, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg);
    void allgatherv(const void *const *sends, void *const *recvs, const size_t *counts, const size_t *displs,
                    int dtype, hipStream_t user);
    // self pairs posted through RCCL since construction (loopback only)
    long long loopback_pairs() const { return loop_pairs_; }

private:
    void run_(int dtype, hipStream_t user);
    // the matching send of rank r's recv `op` at tick t (k-th recv from a (peer, tag) pairs with
    // the peer's k-th send to r with that tag)
    const P2POp &match_(int r, size_t t, const P2POp &op, std::map<std::pair<int, int>, int> &seen) const;

    int P_;
    std::vector<std::unique_ptr<RankResources>> res_;
    std::vector<RingProgram> progs_;
    std::unique_ptr<RcclTransport> loop_;
    hipStream_t loop_stream_ = nullptr;
    std::vector<hipEvent_t> loop_ev_;
    hipEvent_t loop_join_ = nullptr;
    long long loop_pairs_ = 0;
};

// P RingExecutors over one ThreadFabric, each driven by its own thread per call; every rank works
// on its own stream forked from / joined to the caller's (test / diagnostic path).
class ThreadWorld {
public:
    ThreadWorld(int nranks, int device, ncclComm_t loopback = nullptr);
    long long loopback_pairs() const { return fab_->loopback_pairs; }
    ~ThreadWorld();
    void allreduce(const void *const *in, void *const *out, size_t n, int dtype, hipStream_t user,
                   const RingConfig &cfg);
    // in[r * count + b] / out[r * count + b]: rank r's bucket b (RingExecutor::allreduce_batch)
    void allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                         hipStream_t user, const RingConfig &cfg);
    void broadcast(void *const *bufs, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg);
    void allgatherv(const void *const *sends, void *const *recvs, const size_t *counts, const size_t *displs,
                    int dtype, hipStream_t user);
    // The keyed path's multi-request plan on every rank (FusionPipe::run, what the handler runs:
    // pack -> allreduce -> unpack, sub-plans above `cap` bytes), each sub-plan's allreduce through
    // the rank's RingExecutor with the whole plan's message size. srcs[r * count + i] /
    // dsts[r * count + i]: rank r's segment i of bytes[i] bytes. Returns the sub-plans per rank.
    size_t fused_allreduce(const void *const *srcs, void *const *dsts, const size_t *bytes, int count, int dtype,
                           hipStream_t user, const RingConfig &cfg, size_t cap);

private:
    void run_(hipStream_t user, const std::function<void(int, hipStream_t)> &body);
    int P_, device_;
    std::shared_ptr<ThreadFabric> fab_;
    std::vector<std::unique_ptr<RingExecutor>> ex_;
    std::vector<std::unique_ptr<FusionPipe>> pipes_;  // one per rank (fused_allreduce)
    std::vector<hipStream_t> streams_;
    std::vector<hipEvent_t> done_;
    hipEvent_t fork_ = nullptr;
};

LocalWorld &local_world(int nranks);

// One-rank RCCL communicator driving P virtual ranks' programs through RcclTransport (self
// send/recv pairs) — test / diagnostic path (ddl_rccl_loopback_*), never used by ddl_init.
struct RcclLoopback {
    std::mutex mu;
    ncclComm_t comm = nullptr;                  // current (the last split, or the initial comm)
    std::vector<ncclComm_t> owned;              // every communicator created, destroyed at finalize
    std::map<std::pair<int, ncclComm_t>, std::unique_ptr<LocalWorld>> worlds;  // (P, comm)
    LocalWorld &world(int nranks);
};
RcclLoopback &rccl_loopback();

}  // namespace ddl
