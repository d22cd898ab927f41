// handler.h — keyed asynchronous collective requests (allreduce, broadcast, allgather) with
// cross-rank negotiation and fusion.
//
// Replaces the reference's request path below the TF op:
//   TensorAllreduceRequest (collective/request/TensorAllreduceRequest.h:13-41)
//   RingTokenCommunicateHandler (controller/rtc/RingTokenCommunicateHandler.cc:13-410):
//     per-communicator background thread, ring-token negotiation of which keys every rank
//     has registered, communication of the agreed set in lexicographic (type, key) order;
//   MPIRingTokenCommunication::allreduceRequests (rtc/mpi/MPIRingTokenCommunication.cc:105-157,
//     495-749): dtype classification (ascending enum), plans capped at the fusion threshold,
//     memcpy in -> MPI_Allreduce -> memcpy out, done() as each tensor's last element lands.
//
// MI355X-first changes: a round is 3 hops over a star around rank 0 instead of 3 laps of a ring
// (READY+SYNC merged: a member answers the proposal once it has the proposal's first key, with
// its intersection; rank 0 intersects the answers and announces the result); one-request plans
// run the ring directly on the tensor (no staging copy); multi-request plans are packed by
// one gather kernel into an HBM fusion buffer and scattered by one kernel; the data plane
// runs on a private RCCL communicator so user-level ddl_allreduce calls never interleave.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory_resource>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "control.h"
#include "engine.h"
#include "fusion.h"

namespace ddl {

// Input-ready event recorded on the submitter's stream; shared by the requests of one batch.
struct ReadyEvent {
    hipEvent_t e = nullptr;
    explicit ReadyEvent(hipStream_t s);
    ~ReadyEvent();
    ReadyEvent(const ReadyEvent &) = delete;
    ReadyEvent &operator=(const ReadyEvent &) = delete;
};

// Request types, numbered as the reference's Token::RequestType (rtc/Token.h:23-29); the type
// name prefixes the key on the wire and in the pending map ("Allreduce::grad_0", as
// RingTokenCommunicateHandler.cc:140-146 builds its ready keys).
enum RequestType : int { kReqAllreduce = 1, kReqBroadcast = 2, kReqAllgather = 3 };
const char *request_type_name(int type);

struct Request {
    int type = kReqAllreduce;
    std::string key;
    const void *in = nullptr;
    void *out = nullptr;
    size_t n = 0;  // elements of `in`
    int dtype = 0;
    int op = 0;
    int root = 0;                     // broadcast: TensorBroadcastRequest::rootRank()
    size_t first_dim = 0;             // allgather: rows of `in` (n = first_dim * row_elems)
    size_t row_elems = 1;             //   elements per row (the shape without its first dim)
    ddl_alloc_fn alloc = nullptr;     //   output allocation once the gathered first dim is known
    bool host = false;                // in / out are host memory (the reference's CPU tensors)
    int64_t cidx = -1;                // index in the control channel's id table, once agreed before
    std::shared_ptr<ReadyEvent> ready;
    ddl_done_fn done = nullptr;
    void *user = nullptr;
};

// Parallel host memcpy for the host-staging pipeline (pageable <-> pinned): one memcpy thread
// moves ~10 GB/s, less than the PCIe link, so large chunks are split over a few workers.
class CopyPool {
public:
    struct Piece {
        void *dst;
        const void *src;
        size_t bytes;
    };
    // cpus non-empty: every worker binds itself to that CPU set (the GPU's NUMA node)
    explicit CopyPool(int threads, std::vector<int> cpus = {});
    ~CopyPool();
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;
    // Copies every piece; returns when all are done (the caller's thread takes a share).
    void run(const std::vector<Piece> &pieces);
    // fn(lo, hi) over [0, n) cut into one range per thread (the caller's thread takes the first);
    // returns when every range is done
    void parallel(size_t n, const std::function<void(size_t, size_t)> &fn);
    int threads() const { return (int)threads_.size(); }

private:
    void worker_();
    void submit_and_wait_(std::vector<std::function<void()>> &tasks);  // tasks[0] on the caller
    std::vector<int> cpus_;
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::function<void()>> queue_;
    size_t outstanding_ = 0;
    bool stop_ = false;
};

// One worker thread running jobs in submission order: the host unpack of staged chunks, so the
// engine thread packs chunk i (CopyPool) while chunk i - kHostSlots is unpacked (its own CopyPool)
// — the two host memcpys overlap instead of alternating on the engine thread. wait(seq) blocks
// until job `seq` (1-based, from submit) has run; a job's Error is rethrown by the next wait.
class AsyncLane {
public:
    explicit AsyncLane(std::vector<int> cpus = {});
    ~AsyncLane();
    AsyncLane(const AsyncLane &) = delete;
    AsyncLane &operator=(const AsyncLane &) = delete;
    uint64_t submit(std::function<void()> job);
    void wait(uint64_t seq);
    void drain() noexcept;  // every job submitted so far has run (errors dropped)

private:
    void worker_();
    std::vector<int> cpus_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::function<void()>> q_;
    uint64_t submitted_ = 0, done_ = 0;
    bool stop_ = false;
    bool failed_ = false;
    Error err_{0, ""};
    std::thread thread_;
};

// Request identity: (type, key), ordered as the reference's (typeName, key) pairs —
// "Allgather" < "Allreduce" < "Broadcast", then the key bytewise. On the wire it is the string
// "<TypeName>::<key>".
struct ReqId {
    int order;  // type_order(type)
    std::string key;
    bool operator<(const ReqId &o) const { return order != o.order ? order < o.order : key < o.key; }
};
int type_order(int type);
ReqId req_id(const Request &r);
std::string wire_id(const ReqId &id);
ReqId parse_wire_id(const std::string &s);  // throws on an unknown type name

struct Plan {  // makeCollectiveCommunicatePlan's (requestBegin, elementBegin, requestEnd, elementEnd)
    size_t req_begin, elem_begin, req_end, elem_end;
};

// Plans over requests (in order) capped at `limit` bytes. Same walk as the reference
// (MPIRingTokenCommunication.cc:495-546) except that a plan ending exactly on a request
// boundary advances to requestEnd + 1 (the reference advances requestBegin by one, which
// re-plans requests when a multi-request plan ends on a boundary; unreachable with its odd
// 2^31-1 cap and even element sizes, reachable with a configurable cap).
std::vector<Plan> make_plans(const std::vector<size_t> &elements, const std::vector<size_t> &esize,
                             size_t limit);

// The process's listening / standalone control channel: ddl_control_listen opens it,
// ddl_control_connect hands it to the world communicator (replacing it with a fresh one),
// ddl_control_connect_ranked keeps it for ddl_control_negotiate (tools, CPU tests).
std::shared_ptr<ControlChannel> &standalone_control();

// One negotiation round over the star (control.h).
//   root:   SYNC(proposal) to every member; every member's SYNC(intersection) back; the
//           proposal's ids every member kept go out as COMMUNICATE(agreed). (negotiate_root_finish
//           is a no-op kept for the ring's call sites.)
//   member: receives SYNC, intersects with what it holds (may block until the first proposed
//           id is registered), answers rank 0, then receives COMMUNICATE.
// A proposal made only of ids agreed in earlier rounds travels as indices into the channel's
// IdCache (TOKEN_*_CACHED) and is intersected by index; otherwise as "Type::key" strings.
// Every token also carries the sender's Config::shared_hash(): rank 0 compares the members'
// with its own and the COMMUNICATE says whether they all agree (cfg_ok); a round whose ranks
// disagree takes its agreed requests out on every rank and fails them with
// DDL_STATUS_CONFIG_MISMATCH instead of running them. `snapshot` (optional) freezes the rank's
// user collectives and returns how many it has issued (Communicator::round_freeze): members
// call it right before answering, rank 0 once every answer is in; the COMMUNICATE carries the
// maximum (release: the round goes after that many user collectives on every rank, -1 without
// snapshots).
struct Agreed {
    bool cached = false;
    std::vector<uint32_t> idx;      // cached round: indices into ch.cache
    std::vector<std::string> wire;  // string round: ids, sorted (their (type, key) order)
    bool cfg_ok = true;
    long long release = -1;
};
Agreed negotiate_root(ControlChannel &ch, bool cached, const std::vector<uint32_t> &idx,
                      const std::vector<std::string> &strs, int request_type = kReqAllreduce,
                      const std::function<long long()> &snapshot = nullptr);
void negotiate_root_finish(ControlChannel &ch);
Agreed negotiate_member(ControlChannel &ch, const Token &sync,
                        const std::function<std::vector<std::string>(const std::vector<std::string> &)> &by_string,
                        const std::function<std::vector<uint32_t>(const std::vector<uint32_t> &)> &by_index,
                        const std::function<long long()> &snapshot = nullptr);

class RequestHandler {
public:
    explicit RequestHandler(Communicator *owner);
    ~RequestHandler();
    hipStream_t stream() const { return stream_; }  // the engine thread's (pack / unpack)

    void submit(Request r);
    // Unregisters every range of the host registration cache (ddl_set_config
    // "host_register_cache_bytes" 0): waits for the handler's streams first.
    void release_registrations();
    // The host range [ptr, ptr + bytes) is about to be freed (ddl_host_unregister): every cached
    // registration overlapping it goes — now if no host plan is being posted, otherwise before the
    // next lookup of the cache (the engine thread drains the queue first), so a later tensor at the
    // same address is never taken for the old, still-registered pages.
    void unregister_range(const void *ptr, size_t bytes);
    // All-or-nothing registration of several requests under one lock (one wake-up).
    void submit_batch(std::vector<Request> &rs);
    void wait_all();

private:
    void main_();
    void root_round_();
    void member_round_(Token &first);
    // Runs the agreed requests; `forced` != OK takes them out and fails them with that status
    // (a round whose ranks' shared tunables differ) without stopping the handler.
    void execute_(const std::vector<ReqId> &ids, int forced = DDL_STATUS_OK);
    // root_round_ / member_round_ after the agreement: places the round among the user collectives
    // (Communicator::round_release / round_enter), executes it, lifts the freeze
    void run_agreed_(const Agreed &a);
    std::vector<ReqId> agreed_ids_(const Agreed &a);  // learns new ids (string rounds)
    void forget_ids_();                                 // the id table was cleared
    void mark_cached_(const ReqId &id, Request &r);
    struct Done {
        size_t plan;  // index into the round's plan events (kNoPlan: nothing to wait for)
        size_t req;
        int status;
    };
    static constexpr size_t kNoPlan = (size_t)-1;
    // One executed round: its requests, their done() order, the plan events they wait for.
    // The engine thread enqueues the round's data plane and hands it to the completion thread,
    // which waits for each plan's event and fires done() in plan order, rounds in FIFO order;
    // meanwhile the engine thread negotiates the next round (pipeline_rounds = 1). The
    // reference's recv thread blocks in MPI_Allreduce instead (MPIRingTokenCommunication.cc:
    // 548-733); pipeline_rounds = 0 waits the same way.
    struct Round {
        std::vector<Request> reqs;
        std::vector<Done> dones;
        std::vector<hipEvent_t> events;
        int status = 0;
        size_t nplans = 0;
        std::chrono::steady_clock::time_point t0, t1, t2;  // take / enqueue phase bounds (log)
    };
    // a round of at most this many bytes, with no earlier round in flight, completes on the
    // engine thread even when pipelined (its data plane is microseconds: the hand-off costs more)
    static constexpr size_t kInlineRoundBytes = 256u << 10;
    size_t record_plan_(size_t &nplans);  // records the round's next plan event on stream_
    void complete_(Round &rd);            // waits the plan events, fires done(), frees the events
    void completer_();                    // the completion thread
    void wait_inputs_(const Request &r, std::vector<hipEvent_t> &waited);
    void *ensure_(void *&buf, size_t &cap, size_t need);
    void allreduce_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans);
    // Host-resident requests (the reference's deployment case, MPIRingTokenCommunication.cc:
    // 548-733 copies CPU tensors into its MPI buffer): the plan's segments are staged through
    // pinned slots in chunks — host pack (CopyPool) -> H2D -> `coll` on the device slot
    // (stream_) -> D2H -> host unpack — with kHostSlots chunks in flight so the copies overlap
    // the collective. `upload` false: nothing is packed (a broadcast's non-root ranks).
    // `padded`: segment i starts at the 256-byte-rounded running offset (the fusion kernels'
    // layout), so plans with and without `device_unpack` cut the same chunks — and issue the
    // same collectives — on ranks that differ in which outputs are pinned; otherwise back to
    // back (broadcast, as the reference packs).
    // `device_unpack` (every destination pinned and mapped on the device, mapped_host_dsts_): the
    // unpack kernel writes each chunk's result straight into the outputs over PCIe (d2h_), in
    // place of the D2H copy and the host unpack; the host never waits for a chunk to come back
    // (measured 43 GB/s each way with the uploads running, vs 32 when the pack kernel also
    // reads the tensors over PCIe: profiles/r02/host/zero_copy_probe.jsonl).
    struct HostSeg {
        const char *src;
        char *dst;
        size_t bytes;
        char *ddst = nullptr;  // the device's address of dst (device unpack; mapped_host_dsts_)
    };
    void host_staged_(const std::vector<HostSeg> &segs, size_t es, bool upload,
                      const std::function<void(void *dev, size_t elems)> &coll, bool padded = false,
                      bool device_unpack = false);
    void host_pieces_(const std::vector<HostSeg> &segs, const std::vector<size_t> &starts, size_t off, size_t len,
                      char *pinned, bool pack, std::vector<CopyPool::Piece> &out);
    // true when every segment's destination range is 16-byte-aligned pinned host memory that the
    // device reaches at the same address, inside one allocation
    // fills every segment's ddst; false unless all of them are mapped
    // (the queries of a plan's 4096 tensors run on the copy threads: ~3 HIP calls each)
    bool mapped_host_dsts_(std::vector<HostSeg> &segs);
    size_t host_slots_(size_t total);  // chunk size for `total` bytes; (re)allocates the slots
    CopyPool &pool_for_config_();     // the copy threads, rebuilt when host_copy_threads changed
    std::vector<int> local_cpus_;     // the GPU's NUMA node's CPUs (config host_numa_bind; empty: no binding)
    void broadcast_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans);
    void allgather_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans);
    void fail_all_(int status);

    Communicator *owner_;
    ControlChannel *ch_ = nullptr;        // the owner's token ring (size > 1)
    // the data plane: the owner's private keyed communicator at size > 1, the owner itself at
    // size 1. Not owning: the owner holds keyed_data_ and destroys this handler first; an owning
    // pointer to the owner was a cycle that kept a detached size-1 split (and these threads) alive
    Communicator *data_ = nullptr;
    hipStream_t stream_ = nullptr;
    // multi-request plans: pack -> allreduce -> unpack, pipelined in sub-plans above
    // fusion_pipeline_bytes (fusion.h); its buffer 0 also packs broadcast / allgather plans
    FusionPipe fp_;
    void *gather_ = nullptr;  // allgather receive side
    size_t gather_bytes_ = 0;
    void *dims_ = nullptr;    // allgather first-dim exchange
    size_t dims_bytes_ = 0;
    std::vector<hipEvent_t> round_events_;  // plan events of the round being enqueued (engine thread)
    static constexpr int kHostSlots = 4;
    void *pin_[kHostSlots] = {};    // pinned host staging slots (uploads)
    void *pout_[kHostSlots] = {};   // pinned download slots: a chunk's D2H lands here, apart from the
                                    // upload slot, so its host unpack overlaps the next packs
    void *dslot_[kHostSlots] = {};  // device slots
    size_t host_slot_bytes_ = 0;
    hipStream_t h2d_ = nullptr, d2h_ = nullptr;
    hipEvent_t hev_[3 * kHostSlots] = {};  // per slot: input landed, collective done, output landed
    bool slot_used_[kHostSlots] = {};        // hev_[3k + 2] marks the slot's last device use
    std::unique_ptr<CopyPool> pool_;
    // the host unpack of staged chunks (its own copy threads, host_copy_threads of them); the lane
    // is destroyed first (its jobs use out_pool_)
    std::unique_ptr<CopyPool> out_pool_;
    std::unique_ptr<AsyncLane> lane_;
    // opt-in registration cache (config "host_register_cache_bytes"): pageable host tensors of
    // keyed requests are hipHostRegister'ed once and kept (least recently used out past the cap),
    // so a training loop's CPU gradients take the pinned paths (direct DMA in, device unpack out)
    // registers the page ranges of (pointer, bytes) that are not pinned yet: ranges sharing a page
    // are merged (a page cannot be registered twice), overlapping entries join the union
    void register_hosts_(const std::vector<std::pair<const void *, size_t>> &ranges);
    void unregister_all_();  // the cache was switched off (host_register_cache_bytes 0)
    // drops the entries overlapping [lo, hi) (reg_mu_ held); syncs the handler's streams first
    void drop_overlapping_(uintptr_t lo, uintptr_t hi);
    void drain_unregisters_();  // reg_mu_ held: the queued unregister_range calls
    std::mutex unreg_mu_;
    std::vector<std::pair<uintptr_t, uintptr_t>> unreg_q_;
    std::mutex reg_mu_;  // reg_: the engine thread registers, ddl_set_config may release
    std::map<uintptr_t, std::pair<size_t, uint64_t>> reg_;  // page-aligned start -> (bytes, last use)
    size_t reg_bytes_ = 0;
    uint64_t reg_tick_ = 0;
    void *pin_gather_ = nullptr;  // host allgather staging
    size_t pin_gather_bytes_ = 0;

    std::mutex mu_;
    std::condition_variable cv_;       // new registrations / stop
    std::condition_variable idle_cv_;  // completions
    // the pending map's nodes come from a pool, allocated and freed under mu_ only: a 4096-request
    // batch's sorted inserts and its take walk ran 2-3x faster than with the process heap
    // (CPU micro-benchmark; r05 s22 on the box)
    std::pmr::unsynchronized_pool_resource pending_pool_;
    std::pmr::map<ReqId, Request> pending_{&pending_pool_};  // (type name, key) order
    // id table mirror (indices of the ring's cache): parsed ids, key -> index per type,
    // and which indices are pending here — a cached round is intersected by index
    std::vector<ReqId> cache_req_;
    std::unordered_map<std::string, uint32_t> cache_by_key_[3];
    std::vector<uint8_t> pend_flag_;
    size_t inflight_ = 0;
    bool stop_ = false;
    std::atomic<int> failed_{0};  // a completion failed: the engine thread stops with this status
    std::thread thread_;
    // completion thread state (done_mu_): executed rounds waiting for their events, free plan
    // events (returned once waited for, so none is re-recorded while still pending)
    std::mutex done_mu_;
    std::condition_variable done_cv_;
    std::deque<Round> rounds_;
    std::vector<hipEvent_t> event_pool_;
    unsigned long long rounds_queued_ = 0, rounds_done_ = 0;
    bool done_stop_ = false;
    std::thread done_thread_;
};

// Test hook (ddl_testing_control_fault): the next keyed round a member joins closes that member's
// control link right after its snapshot froze the user collectives (a link lost mid-round).
void set_testing_control_fault(int on);
// Test hook (ddl_testing_host_coll_fault): the next host plan's staging loop fails at chunk
// `chunk` (-1: off) — its device collective is not posted — to check that no unpack job of the
// chunks before outlives the plan.
void set_testing_host_coll_fault(long long chunk);

}  // namespace ddl
