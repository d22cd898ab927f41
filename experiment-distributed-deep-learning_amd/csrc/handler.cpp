// handler.cpp — see handler.h.
#include "handler.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <set>
#include <thread>
#include <tuple>

namespace ddl {

std::vector<Plan> make_plans(const std::vector<size_t> &elements, const std::vector<size_t> &esize,
                             size_t limit) {
    std::vector<Plan> plans;
    const size_t nreq = elements.size();
    if (nreq == 0) return plans;
    DDL_REQUIRE(limit > 0, DDL_STATUS_INVALID_ARGUMENT, "fusion threshold must be > 0");
    std::vector<size_t> begins(nreq);
    size_t all = 0;
    for (size_t i = 0; i < nreq; ++i) {
        begins[i] = all;
        all += elements[i] * esize[i];
    }
    size_t byte_size = 0, pb = 0, pbe = 0;
    while (byte_size < all) {
        size_t pe = nreq - 1, pe_elem = elements[nreq - 1];
        byte_size += limit;
        if (byte_size < all) {
            for (size_t i = pb; i < nreq; ++i) {
                if (i == nreq - 1 || (begins[i] < byte_size && byte_size <= begins[i + 1])) {
                    pe = i;
                    pe_elem = (byte_size - begins[i]) / esize[i];
                    break;
                }
            }
        }
        // a plan must make progress: if the cap is below one element, take one element
        if (pe == pb && pe_elem <= pbe) pe_elem = pbe + 1;
        plans.push_back(Plan{pb, pbe, pe, pe_elem});
        if (pe_elem == elements[pe]) {
            pb = pe + 1;
            pbe = 0;
        } else {
            pb = pe;
            pbe = pe_elem;
        }
        byte_size = begins[pe] + esize[pe] * pe_elem;
    }
    return plans;
}

const char *request_type_name(int type) {
    switch (type) {
        case kReqAllreduce: return "Allreduce";  // TensorAllreduceRequest.cc:10
        case kReqBroadcast: return "Broadcast";  // TensorBroadcastRequest.cc:10
        case kReqAllgather: return "Allgather";  // TensorAllgatherRequest.cc:10
        default: return "Unknown";
    }
}

int type_order(int type) {  // rank of the type name in byte order
    switch (type) {
        case kReqAllgather: return 0;
        case kReqAllreduce: return 1;
        case kReqBroadcast: return 2;
        default: return 3;
    }
}

ReqId req_id(const Request &r) { return ReqId{type_order(r.type), r.key}; }

namespace {
const int kTypeByOrder[3] = {kReqAllgather, kReqAllreduce, kReqBroadcast};
}

std::string wire_id(const ReqId &id) {
    DDL_REQUIRE(id.order >= 0 && id.order < 3, DDL_STATUS_ERROR_UNKNOWN, "bad request id");
    return std::string(request_type_name(kTypeByOrder[id.order])) + "::" + id.key;
}

ReqId parse_wire_id(const std::string &s) {
    const size_t sep = s.find("::");
    DDL_REQUIRE(sep != std::string::npos, DDL_STATUS_COMM_ERROR, "token: malformed request id '" << s << "'");
    const std::string name = s.substr(0, sep);
    for (int o = 0; o < 3; ++o)
        if (name == request_type_name(kTypeByOrder[o])) return ReqId{o, s.substr(sep + 2)};
    fail(DDL_STATUS_COMM_ERROR, "token: unknown request type '" + name + "'");
}

ReadyEvent::ReadyEvent(hipStream_t s) {
    DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipError_t r = hipEventRecord(e, s);
    if (r != hipSuccess) {
        (void)hipEventDestroy(e);
        e = nullptr;
        DDL_HIP(r);
    }
}

ReadyEvent::~ReadyEvent() {
    if (e) (void)hipEventDestroy(e);
}

namespace {
// The CPUs of the NUMA node the device's PCI function hangs off, intersected with this thread's
// affinity; empty when unknown, or when binding would not narrow the set. The keyed host path's
// memcpy reads pinned host memory, which the HIP runtime places on the GPU's node: threads on the
// other socket pack the C5 set at half the rate (tools/numa_probe.py).
std::vector<int> gpu_local_cpus(int device) {
    int dom = 0, bus = 0, dev = 0;
    if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess ||
        hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess) {
        (void)hipGetLastError();
        return {};
    }
    char path[128];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node", dom, bus, dev);
    FILE *f = std::fopen(path, "r");
    int node = -1;
    if (f) {
        if (std::fscanf(f, "%d", &node) != 1) node = -1;
        std::fclose(f);
    }
    if (node < 0) return {};
    std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    f = std::fopen(path, "r");
    if (!f) return {};
    char buf[4096] = {};
    const size_t got = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[got] = 0;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return {};
    std::vector<int> cpus;
    for (char *p = buf; *p;) {  // "0-63,128-191"
        char *end = nullptr;
        const long a = std::strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        if (*end == '-') b = std::strtol(end + 1, &end, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET((int)c, &allowed)) cpus.push_back((int)c);
        p = *end == ',' ? end + 1 : end;
        if (*p == '\n') break;
    }
    if (cpus.empty() || (int)cpus.size() == CPU_COUNT(&allowed)) return {};
    return cpus;
}

void bind_this_thread(const std::vector<int> &cpus) {
    if (cpus.empty()) return;
    cpu_set_t s;
    CPU_ZERO(&s);
    for (int c : cpus) CPU_SET(c, &s);
    (void)pthread_setaffinity_np(pthread_self(), sizeof s, &s);
}
}  // namespace

AsyncLane::AsyncLane(std::vector<int> cpus) : cpus_(std::move(cpus)) {
    thread_ = std::thread(&AsyncLane::worker_, this);
}

AsyncLane::~AsyncLane() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
}

uint64_t AsyncLane::submit(std::function<void()> job) {
    uint64_t seq;
    {
        std::lock_guard<std::mutex> g(mu_);
        q_.push_back(std::move(job));
        seq = ++submitted_;
    }
    cv_.notify_one();
    return seq;
}

void AsyncLane::wait(uint64_t seq) {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return done_ >= seq; });
    if (failed_) {
        failed_ = false;
        throw err_;
    }
}

void AsyncLane::drain() noexcept {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return done_ >= submitted_; });
    failed_ = false;
}

void AsyncLane::worker_() {
    bind_this_thread(cpus_);
    for (;;) {
        std::function<void()> job;
        {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;  // stop_, nothing left
            job = std::move(q_.front());
            q_.pop_front();
        }
        bool bad = false;
        Error e{0, ""};
        try {
            job();
        } catch (const Error &x) {
            bad = true;
            e = x;
        } catch (const std::exception &x) {
            bad = true;
            e = Error{DDL_STATUS_ERROR_UNKNOWN, x.what()};
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            if (bad && !failed_) {
                failed_ = true;
                err_ = e;
            }
            ++done_;
        }
        done_cv_.notify_all();
    }
}

CopyPool::CopyPool(int threads, std::vector<int> cpus) : cpus_(std::move(cpus)) {
    for (int i = 0; i < threads; ++i) threads_.emplace_back(&CopyPool::worker_, this);
}

CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (std::thread &t : threads_) t.join();
}

void CopyPool::worker_() {
    bind_this_thread(cpus_);
    for (;;) {
        std::function<void()> task;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
            if (stop_ && queue_.empty()) return;
            task = std::move(queue_.back());
            queue_.pop_back();
        }
        task();
        {
            std::lock_guard<std::mutex> g(mu_);
            --outstanding_;
        }
        done_cv_.notify_all();
    }
}

void CopyPool::submit_and_wait_(std::vector<std::function<void()>> &tasks) {
    if (tasks.empty()) return;
    {
        std::lock_guard<std::mutex> g(mu_);
        for (size_t i = 1; i < tasks.size(); ++i) queue_.push_back(std::move(tasks[i]));
        outstanding_ += tasks.size() - 1;
    }
    cv_.notify_all();
    tasks[0]();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return outstanding_ == 0; });
}

void CopyPool::parallel(size_t n, const std::function<void(size_t, size_t)> &fn) {
    const size_t T = std::min(threads_.size() + 1, n);
    if (T <= 1) {
        if (n) fn(0, n);
        return;
    }
    std::vector<std::function<void()>> tasks;
    for (size_t t = 0; t < T; ++t) {
        const size_t lo = n * t / T, hi = n * (t + 1) / T;
        tasks.push_back([&fn, lo, hi] { fn(lo, hi); });
    }
    submit_and_wait_(tasks);
}

void CopyPool::run(const std::vector<Piece> &pieces) {
    size_t total = 0;
    for (const Piece &p : pieces) total += p.bytes;
    const size_t T = threads_.size() + 1;
    if (threads_.empty() || total < (2u << 20)) {
        for (const Piece &p : pieces) std::memcpy(p.dst, p.src, p.bytes);
        return;
    }
    // T shares of about total / T bytes each, pieces cut where a share ends
    const size_t share = (total + T - 1) / T;
    std::vector<std::vector<Piece>> shares(1);
    size_t room = share;
    for (Piece p : pieces) {
        while (p.bytes) {
            if (room == 0) {
                shares.emplace_back();
                room = share;
            }
            const size_t n = p.bytes < room ? p.bytes : room;
            shares.back().push_back(Piece{p.dst, p.src, n});
            p.dst = static_cast<char *>(p.dst) + n;
            p.src = static_cast<const char *>(p.src) + n;
            p.bytes -= n;
            room -= n;
        }
    }
    std::vector<std::function<void()>> tasks;
    for (auto &sh : shares)
        tasks.push_back([work = std::move(sh)] {
            for (const Piece &p : work) std::memcpy(p.dst, p.src, p.bytes);
        });
    submit_and_wait_(tasks);
}

std::shared_ptr<ControlChannel> &standalone_control() {
    static auto *ch = new std::shared_ptr<ControlChannel>(std::make_shared<ControlChannel>());
    return *ch;
}

RequestHandler::RequestHandler(Communicator *owner) : owner_(owner) {
    DeviceGuard g(owner_->device());
    if (owner_->size() > 1) {
        ch_ = owner_->control();
        DDL_REQUIRE(ch_ && ch_->connected() && ch_->size() == owner_->size() && ch_->rank() == owner_->rank() &&
                        owner_->keyed_data(),
                    DDL_STATUS_NOT_INITIALIZED,
                    "keyed requests at size > 1 need the communicator's token ring (ddl_control_connect for the "
                    "world; split_communicator builds one for every split)");
        // the private data-plane communicator made with the ring (Communicator::enable_keyed)
        data_ = owner_->keyed_data().get();
    } else {
        data_ = owner_;
    }
    // the fusion pack / unpack kernels overlap other plans' RCCL kernels at size > 1: the same CU
    // mask as the executors' compute streams (config compute_cu_mask; pack / unpack keep their
    // rate on it, tools/cu_mask_probe.py)
    // its hardware-queue class (executor.h QueueClass): apart from the user's streams
    stream_ = create_engine_stream(owner_->keyed_queue_class(), owner_->size() > 1 ? config_compute_cu_mask() : 0);
    fp_.qc = owner_->keyed_queue_class();
    done_thread_ = std::thread(&RequestHandler::completer_, this);
    thread_ = std::thread(&RequestHandler::main_, this);
}

RequestHandler::~RequestHandler() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    // a round waiting in round_enter for user collectives that will never be issued now fails
    // (the communicator is going away) instead of blocking the join below
    owner_->round_abort(DDL_STATUS_NOT_INITIALIZED, "the communicator is being destroyed");
    if (thread_.joinable()) thread_.join();
    {  // the rounds already handed over complete (or fail) first, in order
        std::lock_guard<std::mutex> g(done_mu_);
        done_stop_ = true;
    }
    done_cv_.notify_all();
    if (done_thread_.joinable()) done_thread_.join();
    fail_all_(DDL_STATUS_COMM_ERROR);
    if (lane_) lane_->drain();  // unpack jobs read the pinned download slots freed below
    for (hipEvent_t e : event_pool_) (void)hipEventDestroy(e);
    if (gather_) (void)hipFree(gather_);
    if (dims_) (void)hipFree(dims_);
    if (pin_gather_) (void)hipHostFree(pin_gather_);
    for (hipStream_t st : {h2d_, d2h_})
        if (st) (void)hipStreamSynchronize(st);
    for (int k = 0; k < kHostSlots; ++k) {
        if (pin_[k]) (void)hipHostFree(pin_[k]);
        if (pout_[k]) (void)hipHostFree(pout_[k]);
        if (dslot_[k]) (void)hipFree(dslot_[k]);
    }
    for (hipEvent_t e : hev_)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : reg_) (void)hipHostUnregister(reinterpret_cast<void *>(e.first));
    for (hipStream_t st : {h2d_, d2h_})
        if (st) (void)hipStreamDestroy(st);
    if (stream_) (void)hipStreamDestroy(stream_);
}

namespace {
void validate(const Request &r, int size) {
    DDL_REQUIRE(dtype_size(r.dtype) != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << r.dtype);
    switch (r.type) {
        case kReqAllreduce:
            DDL_REQUIRE(r.op == DDL_ALLREDUCE_OP_SUM, DDL_STATUS_INVALID_ARGUMENT, "only SUM is supported");
            DDL_REQUIRE(r.n == 0 || (r.in && r.out), DDL_STATUS_INVALID_ARGUMENT, "null buffer");
            break;
        case kReqBroadcast:
            DDL_REQUIRE(r.root >= 0 && r.root < size, DDL_STATUS_INVALID_ARGUMENT,
                        "root " << r.root << " outside [0, " << size << ")");
            DDL_REQUIRE(r.n == 0 || (r.in && r.out), DDL_STATUS_INVALID_ARGUMENT, "null buffer");
            break;
        case kReqAllgather:
            DDL_REQUIRE(r.alloc != nullptr, DDL_STATUS_INVALID_ARGUMENT, "allgather needs an output allocator");
            DDL_REQUIRE(r.row_elems > 0 && r.n == r.first_dim * r.row_elems, DDL_STATUS_INVALID_ARGUMENT,
                        "allgather: elements " << r.n << " != first_dim " << r.first_dim << " x row " << r.row_elems);
            DDL_REQUIRE(r.n == 0 || r.in, DDL_STATUS_INVALID_ARGUMENT, "null buffer");
            break;
        default: fail(DDL_STATUS_INVALID_ARGUMENT, "unknown request type " + std::to_string(r.type));
    }
}
}  // namespace

// A request whose id was agreed before gets its id-table index (under mu_).
void RequestHandler::mark_cached_(const ReqId &id, Request &r) {
    r.cidx = -1;
    if (id.order < 0 || id.order >= 3 || cache_by_key_[id.order].empty()) return;  // (no hashing at size 1)
    auto it = cache_by_key_[id.order].find(id.key);
    if (it == cache_by_key_[id.order].end()) return;
    r.cidx = it->second;
    pend_flag_[it->second] = 1;
}

void RequestHandler::submit(Request r) {
    validate(r, owner_->size());
    {
        std::lock_guard<std::mutex> g(mu_);
        DDL_REQUIRE(!stop_, DDL_STATUS_NOT_INITIALIZED, "handler is shutting down");
        ReqId id = req_id(r);
        DDL_REQUIRE(pending_.find(id) == pending_.end(), DDL_STATUS_DUPLICATE_KEY,
                    "a request with key '" << r.key << "' is already pending");
        mark_cached_(id, r);
        pending_.emplace(std::move(id), std::move(r));
    }
    cv_.notify_all();
}

void RequestHandler::submit_batch(std::vector<Request> &rs) {
    for (const Request &r : rs) validate(r, owner_->size());
    {
        std::lock_guard<std::mutex> g(mu_);
        DDL_REQUIRE(!stop_, DDL_STATUS_NOT_INITIALIZED, "handler is shutting down");
        std::vector<ReqId> ids;
        ids.reserve(rs.size());
        for (const Request &r : rs) ids.push_back(req_id(r));
        std::vector<size_t> order(rs.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = i;
        auto by_id = [&](size_t a, size_t b) { return ids[a] < ids[b]; };
        if (!std::is_sorted(order.begin(), order.end(), by_id)) std::sort(order.begin(), order.end(), by_id);
        // duplicates inside the batch, then against the pending map by one forward walk
        auto pit = pending_.empty() ? pending_.end() : pending_.lower_bound(ids[order[0]]);
        for (size_t i = 0; i < order.size(); ++i) {
            const ReqId &id = ids[order[i]];
            while (pit != pending_.end() && pit->first < id) ++pit;
            DDL_REQUIRE((pit == pending_.end() || id < pit->first) && (i == 0 || ids[order[i - 1]] < id),
                        DDL_STATUS_DUPLICATE_KEY, "a request with key '" << id.key << "' is already pending");
        }
        // sorted insertion with hints: amortised O(1) per request
        auto hint = pending_.end();
        for (size_t i = order.size(); i-- > 0;) {
            const size_t j = order[i];
            mark_cached_(ids[j], rs[j]);
            hint = pending_.emplace_hint(hint, std::move(ids[j]), std::move(rs[j]));
        }
    }
    cv_.notify_all();
}

void RequestHandler::wait_all() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [this] { return (pending_.empty() && inflight_ == 0) || stop_; });
}

std::atomic<int> g_control_fault{0};
void set_testing_control_fault(int on) { g_control_fault = on ? 1 : 0; }
std::atomic<long long> g_host_coll_fault{-1};
void set_testing_host_coll_fault(long long chunk) { g_host_coll_fault = chunk; }

void RequestHandler::fail_all_(int status) {
    std::vector<Request> left;
    {
        std::lock_guard<std::mutex> g(mu_);
        left.reserve(pending_.size());
        for (auto &kv : pending_) left.push_back(std::move(kv.second));
        pending_.clear();  // the nodes go back to the pool under mu_
        std::fill(pend_flag_.begin(), pend_flag_.end(), 0);
    }
    for (Request &r : left) {
        if (r.done) r.done(status, r.user);
    }
    idle_cv_.notify_all();
}

void RequestHandler::main_() {
    t_handler_thread = true;  // engine.h: no communicator is destroyed on this thread
    try {
        DDL_HIP(hipSetDevice(owner_->device()));
        // the engine thread takes a share of every host pack / unpack: it and the copy threads
        // run on the GPU's NUMA node (config host_numa_bind, read when the handler starts)
        if (config().host_numa_bind.load()) {
            local_cpus_ = gpu_local_cpus(owner_->device());
            bind_this_thread(local_cpus_);
        }
        ControlChannel *ch = ch_;  // null at size 1
        const int P = owner_->size(), rank = owner_->rank();
        for (;;) {
            if (P == 1 || rank == 0) {
                std::vector<ReqId> keys;
                {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [this] { return stop_ || failed_.load() || !pending_.empty(); });
                    if (failed_.load()) fail(failed_.load(), "a keyed round failed on the device");
                    if (stop_) break;
                    // optional fusion window: let more registrations join this round
                    const long long cycle_us = config().cycle_time_us.load();
                    if (cycle_us > 0)
                        cv_.wait_for(lk, std::chrono::microseconds(cycle_us), [this] { return stop_; });
                    if (stop_) break;
                    if (P == 1) {  // (rank 0 of a ring builds its proposal in root_round_)
                        keys.reserve(pending_.size());
                        const int order = pending_.begin()->first.order;
                        for (auto &kv : pending_)
                            if (kv.first.order == order) keys.push_back(kv.first);
                    }
                }
                if (P == 1) execute_(keys);
                else root_round_();  // negotiation lap times: DDL_LOG level 3 in root_round_
            } else {
                if (failed_.load()) fail(failed_.load(), "a keyed round failed on the device");
                Token t;
                bool got = ch->recv(t, 50);
                if (!got) {
                    std::lock_guard<std::mutex> g(mu_);
                    if (stop_ && pending_.empty()) {
                        // rank 0 shuts the channel down; keep listening a little for it
                        Token s;
                        if (ch->recv(s, 5000) && s.type == TOKEN_SHUT_DOWN) ch->send(s);
                        break;
                    }
                    continue;
                }
                if (t.type == TOKEN_SHUT_DOWN) {
                    ch->send(t);  // the acknowledgement
                    break;
                }
                member_round_(t);
            }
        }
        if (P > 1 && rank == 0) {  // SHUT_DOWN to every member, then their acknowledgements
            Token s;                // (the reference's SHUT_DOWN lap, RingTokenCommunicateHandler.cc:34-48)
            s.type = TOKEN_SHUT_DOWN;
            s.request = TOKEN_REQUEST_SHUTDOWN;
            s.msg = "shut down";
            ch->send(s);
            for (int r = 1; r < P; ++r) {
                Token back;
                try {
                    while (ch->recv_from(r, back, 5000) && back.type != TOKEN_SHUT_DOWN) {
                    }
                } catch (const Error &) {  // a member that already left closed its link
                }
            }
        }
    } catch (const Error &e) {
        DDL_LOG(0, "request handler stopped: " << e.msg);
        // a freeze taken by this round's snapshot is cleared here, and the user collectives waiting
        // behind it (or issued later) fail instead of blocking: with the round's place unknown their
        // order against the keyed data plane is no longer defined
        owner_->round_abort(e.status, e.msg);
        // the other ends see the link close (EOF) and stop as well, instead of waiting for a token
        if (ch_) ch_->close_all();
        fail_all_(e.status);
    } catch (const std::exception &e) {
        DDL_LOG(0, "request handler stopped: " << e.what());
        owner_->round_abort(DDL_STATUS_COMM_ERROR, e.what());
        if (ch_) ch_->close_all();
        fail_all_(DDL_STATUS_COMM_ERROR);
    }
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    idle_cv_.notify_all();
}

namespace {
// Rank 0's view of one round: the agreed set is the proposal's entries that every member kept.
// String rounds: each answer is a subsequence of the proposal (members walk it in order).
// Cached rounds: index sets.
Agreed decide(bool cached, const std::vector<uint32_t> &idx, const std::vector<std::string> &strs,
              const std::vector<Token> &answers, ControlChannel &ch) {
    Agreed a;
    a.cached = cached;
    if (cached) {
        std::vector<uint32_t> agreed(idx);
        std::sort(agreed.begin(), agreed.end());
        for (const Token &t : answers) {
            std::vector<uint32_t> theirs = ch.cache.decode(t.msg);
            std::sort(theirs.begin(), theirs.end());
            std::vector<uint32_t> both;
            std::set_intersection(agreed.begin(), agreed.end(), theirs.begin(), theirs.end(), std::back_inserter(both));
            agreed.swap(both);
        }
        a.idx = std::move(agreed);
        return a;
    }
    std::vector<int> kept(strs.size(), 0);
    for (const Token &t : answers) {
        size_t j = 0;
        for (const std::string &k : decode_keys(t.msg)) {
            while (j < strs.size() && strs[j] != k) ++j;
            DDL_REQUIRE(j < strs.size(), DDL_STATUS_COMM_ERROR, "token protocol: answer '" << k << "' not proposed");
            ++kept[j++];
        }
    }
    for (size_t j = 0; j < strs.size(); ++j)
        if (kept[j] == (int)answers.size()) a.wire.push_back(strs[j]);
    return a;
}
}  // namespace

Agreed negotiate_root(ControlChannel &ch, bool cached, const std::vector<uint32_t> &idx,
                      const std::vector<std::string> &strs, int request_type,
                      const std::function<long long()> &snapshot) {
    const uint64_t cfg = config().shared_hash();
    Token t;
    t.type = cached ? TOKEN_SYNC_CACHED : TOKEN_SYNC;
    t.request = (uint8_t)request_type;
    t.cfg = cfg;
    t.msg = cached ? ch.cache.encode(idx) : encode_keys(strs);
    ch.send(t);  // the proposal to every member
    std::vector<Token> answers(ch.size() - 1);
    bool cfg_ok = true;
    long long release = -1;
    std::vector<uint64_t> hashes(ch.size(), cfg);
    for (int r = 1; r < ch.size(); ++r) {
        ch.recv_from(r, answers[r - 1], -1);
        DDL_REQUIRE(answers[r - 1].type == t.type, DDL_STATUS_COMM_ERROR,
                    "token protocol: expected SYNC from rank " << r << ", got " << (int)answers[r - 1].type);
        hashes[r] = answers[r - 1].cfg;
        cfg_ok = cfg_ok && answers[r - 1].cfg == cfg;
        release = std::max<long long>(release, answers[r - 1].seq);
    }
    if (snapshot) release = std::max(release, snapshot());
    Agreed a = decide(cached, idx, strs, answers, ch);
    a.cfg_ok = cfg_ok;
    a.release = release;
    if (!cfg_ok) {
        try {
            check_config_agreement(0, hashes);
        } catch (const Error &e) {
            DDL_LOG(0, "keyed round refused: " << e.msg);
        }
    }
    Token c;
    c.type = cached ? TOKEN_COMMUNICATE_CACHED : TOKEN_COMMUNICATE;
    c.request = (uint8_t)request_type;
    c.cfg = cfg_ok ? cfg : kCfgMismatch;
    c.seq = release;
    c.msg = cached ? ch.cache.encode(a.idx) : encode_keys(a.wire);
    ch.send(c);  // the agreed set to every member
    if (cached) {
        ++ch.cached_rounds;
    } else {
        std::sort(a.wire.begin(), a.wire.end());
        ++ch.string_rounds;
    }
    return a;
}

// Nothing to drain in the star (the ring's COMMUNICATE lap came back to rank 0 here).
void negotiate_root_finish(ControlChannel &) {}

Agreed negotiate_member(ControlChannel &ch, const Token &sync,
                        const std::function<std::vector<std::string>(const std::vector<std::string> &)> &by_string,
                        const std::function<std::vector<uint32_t>(const std::vector<uint32_t> &)> &by_index,
                        const std::function<long long()> &snapshot) {
    DDL_REQUIRE(sync.type == TOKEN_SYNC || sync.type == TOKEN_SYNC_CACHED, DDL_STATUS_COMM_ERROR,
                "token protocol: expected SYNC, got " << (int)sync.type);
    const bool cached = sync.type == TOKEN_SYNC_CACHED;
    Token s;
    s.type = sync.type;
    s.request = sync.request;
    s.msg = cached ? ch.cache.encode(by_index(ch.cache.decode(sync.msg))) : encode_keys(by_string(decode_keys(sync.msg)));
    // the config this rank runs the round under: read once its first proposed request is registered
    // (by_string / by_index wait for it), not when the proposal arrives
    s.cfg = config().shared_hash();
    s.seq = snapshot ? snapshot() : -1;
    ch.send(s);  // this rank's intersection with the proposal
    Token c;
    ch.recv(c, -1);
    DDL_REQUIRE(c.type == (cached ? TOKEN_COMMUNICATE_CACHED : TOKEN_COMMUNICATE), DDL_STATUS_COMM_ERROR,
                "token protocol: expected COMMUNICATE, got " << (int)c.type);
    Agreed a;
    a.cached = cached;
    a.cfg_ok = c.cfg != kCfgMismatch;
    a.release = c.seq;
    if (!a.cfg_ok)
        DDL_LOG(0, "keyed round refused: the ranks' shared tunables differ (this rank's config hash " << std::hex
                                                                                                   << s.cfg << std::dec << ")");
    if (cached) {
        a.idx = ch.cache.decode(c.msg);
        ++ch.cached_rounds;
    } else {
        a.wire = decode_keys(c.msg);
        std::sort(a.wire.begin(), a.wire.end());
        ++ch.string_rounds;
    }
    return a;
}

void RequestHandler::forget_ids_() {
    cache_req_.clear();
    for (auto &m : cache_by_key_) m.clear();
    pend_flag_.clear();
    for (auto &kv : pending_) kv.second.cidx = -1;
}

// The agreed ids in execution order. A string round teaches the id table the new ids (every
// rank learns the same list in the same order); the pending requests among them get their
// index, so the next round with the same key set goes by index.
std::vector<ReqId> RequestHandler::agreed_ids_(const Agreed &a) {
    std::vector<ReqId> ids;
    std::lock_guard<std::mutex> g(mu_);
    if (a.cached) {
        ids.reserve(a.idx.size());
        for (uint32_t i : a.idx) {
            DDL_REQUIRE(i < cache_req_.size(), DDL_STATUS_COMM_ERROR, "token: id index out of range");
            ids.push_back(cache_req_[i]);
        }
        std::sort(ids.begin(), ids.end());
        return ids;
    }
    ControlChannel &ch = *ch_;
    if (ch.cache.learn(a.wire)) forget_ids_();
    for (size_t j = cache_req_.size(); j < ch.cache.size(); ++j) {  // mirror every new table entry
        ReqId rid = parse_wire_id(ch.cache.at((uint32_t)j));
        cache_by_key_[rid.order][rid.key] = (uint32_t)j;
        pend_flag_.push_back(0);
        auto it = pending_.find(rid);
        if (it != pending_.end()) {
            it->second.cidx = (int64_t)j;
            pend_flag_[j] = 1;
        }
        cache_req_.push_back(std::move(rid));
    }
    ids.reserve(a.wire.size());
    for (const auto &w : a.wire) ids.push_back(parse_wire_id(w));
    return ids;
}

// Rank 0: propose every registered id of one type (SYNC to every member — each intersects and
// answers), then announce the agreed set (COMMUNICATE) and run it.
void RequestHandler::root_round_() {
    ControlChannel &ch = *ch_;
    // one request type per round (the token carries one RequestType): the type of the first
    // registered id, as the reference proposes registeredRequest_.begin() (:184-190)
    std::vector<std::string> strs;
    std::vector<uint32_t> idx;
    bool cached = true;
    int type = kReqAllreduce;
    {
        std::lock_guard<std::mutex> g(mu_);
        if (!pending_.empty()) type = pending_.begin()->second.type;
        for (auto &kv : pending_) {
            if (kv.second.type != type) continue;
            if (kv.second.cidx < 0) cached = false;
            if (cached) idx.push_back((uint32_t)kv.second.cidx);
        }
        if (!cached)
            for (auto &kv : pending_)
                if (kv.second.type == type) strs.push_back(wire_id(kv.first));
        cached = cached && !idx.empty();
    }
    const Agreed a = negotiate_root(ch, cached, idx, strs, type, [this] { return owner_->round_freeze(); });
    negotiate_root_finish(ch);
    run_agreed_(a);
}

void RequestHandler::run_agreed_(const Agreed &a) {
    struct Unfreeze {  // user collectives go on whatever happens to the round
        Communicator *c;
        ~Unfreeze() { c->round_unfreeze(); }
    } unfreeze{owner_};
    owner_->round_release(a.release);
    std::vector<ReqId> ids = agreed_ids_(a);
    owner_->round_enter(a.release);
    execute_(ids, a.cfg_ok ? DDL_STATUS_OK : DDL_STATUS_CONFIG_MISMATCH);
}

// Other ranks: answer the SYNC once the first proposed id is registered here (the reference
// parks the READY token the same way, RingTokenCommunicateHandler.cc:225-250) with the
// intersection, then take COMMUNICATE and run the agreed set (:302-310).
void RequestHandler::member_round_(Token &t) {
    const Agreed a = negotiate_member(
        *ch_, t,
        [this](const std::vector<std::string> &keys) {
            std::vector<ReqId> proposed;
            for (const auto &w : keys) proposed.push_back(parse_wire_id(w));
            std::vector<std::string> mine;
            std::unique_lock<std::mutex> lk(mu_);
            if (!proposed.empty()) cv_.wait(lk, [&] { return stop_ || pending_.count(proposed.front()) > 0; });
            for (size_t i = 0; i < proposed.size(); ++i)
                if (pending_.count(proposed[i])) mine.push_back(keys[i]);
            return mine;
        },
        [this](const std::vector<uint32_t> &proposed) {
            std::vector<uint32_t> mine;
            std::unique_lock<std::mutex> lk(mu_);
            auto held = [&](uint32_t i) { return i < pend_flag_.size() && pend_flag_[i]; };
            if (!proposed.empty()) cv_.wait(lk, [&] { return stop_ || held(proposed.front()); });
            for (uint32_t i : proposed)
                if (held(i)) mine.push_back(i);
            return mine;
        },
        [this] {
            const long long at = owner_->round_freeze();
            // test hook (ddl_testing_control_fault): the control link is lost right after this
            // rank froze its user collectives for the round — the answer below cannot be sent
            if (g_control_fault.exchange(0)) ch_->close_all();
            return at;
        });
    run_agreed_(a);
}

void *RequestHandler::ensure_(void *&buf, size_t &cap, size_t need) {
    if (need > cap) {
        if (buf) {  // may still be read on the device; no hipFree on a data path (engine.h retire_device)
            retire_device(buf);
            buf = nullptr;
            cap = 0;
        }
        const size_t sz = need + need / 2;  // x1.5 growth (MPIRingTokenCommunication.cc:13, 480)
        DDL_HIP(hipMalloc(&buf, sz));
        cap = sz;
    }
    return buf;
}

size_t RequestHandler::record_plan_(size_t &nplans) {
    hipEvent_t e = nullptr;
    {
        std::lock_guard<std::mutex> g(done_mu_);
        if (!event_pool_.empty()) {
            e = event_pool_.back();
            event_pool_.pop_back();
        }
    }
    if (!e) DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    round_events_.push_back(e);
    DDL_HIP(hipEventRecord(e, stream_));
    return nplans++;
}

void RequestHandler::wait_inputs_(const Request &r, std::vector<hipEvent_t> &waited) {
    if (!r.ready || std::find(waited.begin(), waited.end(), r.ready->e) != waited.end()) return;
    DDL_HIP(hipStreamWaitEvent(stream_, r.ready->e, 0));
    waited.push_back(r.ready->e);
}

namespace {
// Element slice [b, e) of request q inside plan p.
void plan_slice(const Plan &p, size_t q, size_t n, size_t *b, size_t *e) {
    *b = q == p.req_begin ? p.elem_begin : 0;
    *e = q == p.req_end ? p.elem_end : n;
}
}  // namespace

void RequestHandler::host_pieces_(const std::vector<HostSeg> &segs, const std::vector<size_t> &starts, size_t off,
                                  size_t len, char *pinned, bool pack, std::vector<CopyPool::Piece> &out) {
    // segment i holds [starts[i], starts[i] + bytes) of the staged stream (padding between
    // segments is neither packed nor unpacked)
    const size_t end = off + len;
    for (size_t i = (size_t)(std::upper_bound(starts.begin(), starts.end(), off) - starts.begin()) - 1;
         i < segs.size() && starts[i] < end; ++i) {
        const size_t lo = std::max(off, starts[i]), hi = std::min(end, starts[i] + segs[i].bytes);
        if (hi <= lo) continue;  // empty segment, or `off` past its data
        if (pack) out.push_back(CopyPool::Piece{pinned + (lo - off), segs[i].src + (lo - starts[i]), hi - lo});
        else out.push_back(CopyPool::Piece{segs[i].dst + (lo - starts[i]), pinned + (lo - off), hi - lo});
    }
}

namespace {
constexpr size_t round256(size_t b) { return (b + 255) & ~size_t(255); }

// Offsets of the segments in the staged stream: back to back, or 256-byte-rounded (padded).
template <class Seg>
size_t seg_starts(const std::vector<Seg> &segs, bool padded, std::vector<size_t> &starts) {
    starts.resize(segs.size());
    size_t total = 0;
    for (size_t i = 0; i < segs.size(); ++i) {
        starts[i] = total;
        total += padded ? round256(segs[i].bytes) : segs[i].bytes;
    }
    return total;
}

// Host range [p, p + bytes) is pinned (page-locked) host memory inside one allocation. With
// `alias` the range must also be mapped into the device's address space, 16-byte aligned (the
// unpack kernel's vector path; byte stores over PCIe would crawl): *alias = the device address of
// p — p itself for torch pin_memory / hipHostMalloc, the mapping's address for a hipHostRegister'ed
// range. A failed query (pageable memory) leaves no sticky error behind.
bool mapped_host_range(const void *p, size_t bytes, char **alias = nullptr) {
    if (bytes == 0) {
        if (alias) *alias = static_cast<char *>(const_cast<void *>(p));
        return true;
    }
    if (!p || (alias && (reinterpret_cast<uintptr_t>(p) & 15u) != 0)) return false;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
    void *start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, const_cast<void *>(p)) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, const_cast<void *>(p)) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(start), q = reinterpret_cast<uintptr_t>(p);
    if (!start || q < s0 || q + bytes > s0 + size) return false;
    if (alias) {
        if (!a.devicePointer || (reinterpret_cast<uintptr_t>(a.devicePointer) & 15u) != 0) return false;
        *alias = static_cast<char *>(a.devicePointer);
    }
    return true;
}
}  // namespace

bool RequestHandler::mapped_host_dsts_(std::vector<HostSeg> &segs) {
    if (segs.empty()) return true;
    // the first query alone: a pageable output (the common staged case) answers in one call
    if (!mapped_host_range(segs[0].dst, segs[0].bytes, &segs[0].ddst)) return false;
    std::atomic<bool> all{true};
    pool_for_config_().parallel(segs.size() - 1, [&](size_t lo, size_t hi) {
        for (size_t i = lo + 1; i < hi + 1 && all.load(std::memory_order_relaxed); ++i)
            if (!mapped_host_range(segs[i].dst, segs[i].bytes, &segs[i].ddst)) all = false;
    });
    return all.load();
}

size_t RequestHandler::host_slots_(size_t total) {
    size_t chunk = (size_t)config().host_chunk_bytes.load() & ~size_t(255);  // a multiple of es
    if (chunk < 4096) chunk = 4096;
    if (chunk > total) chunk = round256(total);
    if (host_slot_bytes_ < chunk) {
        for (hipStream_t st : {h2d_, d2h_, stream_})
            if (st) DDL_HIP(hipStreamSynchronize(st));
        for (int k = 0; k < kHostSlots; ++k) {  // outgrown slots kept until ddl_finalize (engine.h retire_*)
            retire_host(pin_[k]);
            retire_host(pout_[k]);
            retire_device(dslot_[k]);
            pin_[k] = pout_[k] = dslot_[k] = nullptr;
            slot_used_[k] = false;
        }
        host_slot_bytes_ = 0;
        for (int k = 0; k < kHostSlots; ++k) {
            DDL_HIP(hipHostMalloc(&pin_[k], chunk, hipHostMallocDefault));
            DDL_HIP(hipHostMalloc(&pout_[k], chunk, hipHostMallocDefault));
            DDL_HIP(hipMalloc(&dslot_[k], chunk));
        }
        host_slot_bytes_ = chunk;
    }
    if (!h2d_) {
        h2d_ = create_engine_stream(owner_->keyed_queue_class());
        d2h_ = create_engine_stream(owner_->keyed_queue_class());
        for (hipEvent_t &e : hev_) DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    return chunk;
}

CopyPool &RequestHandler::pool_for_config_() {
    // rebuilt when the setting changed (only the engine thread runs host plans, so no plan is
    // using the old pool here); r02's thread-count sweep ran every setting on the first pool
    const int want = (int)std::max(0ll, config().host_copy_threads.load());
    if (!pool_ || pool_->threads() != want) {
        if (lane_) lane_->drain();  // no unpack job may still use out_pool_
        pool_.reset();
        pool_.reset(new CopyPool(want, local_cpus_));
        out_pool_.reset();
        out_pool_.reset(new CopyPool(want, local_cpus_));
    }
    if (!lane_) lane_.reset(new AsyncLane(local_cpus_));
    return *pool_;
}

namespace {
// Waits for a plan's event without holding a core for a whole long round: queries with yields
// for the first 200 us (a plan about to land — small rounds keep their latency), then sleeps
// between queries (each sleep ~20-70 us with the kernel's timer slack), so the completion thread
// does not spin beside the engine thread, the host copies and the framework's own threads. Also
// the unpack lane's wait for a D2H: hipEventSynchronize from a helper thread held up the engine
// thread's own HIP calls on the same streams (r04 s2: ~27 ms per pageable C5 batch outside every
// timed section of the staging loop; 3.9 ms once polled).
hipError_t wait_plan(hipEvent_t e) {
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q != hipErrorNotReady) return q;
        if (clk::now() - t0 < std::chrono::microseconds(200)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}
}  // namespace

void RequestHandler::host_staged_(const std::vector<HostSeg> &segs, size_t es, bool upload,
                                  const std::function<void(void *, size_t)> &coll, bool padded, bool device_unpack) {
    std::vector<size_t> starts;
    const size_t total = seg_starts(segs, padded || device_unpack, starts);
    if (total == 0) return;
    const size_t chunk = host_slots_(total);
    pool_for_config_();
    if (device_unpack) config().host_zero_copy_plans.fetch_add(1);
    // chunk boundaries (the same on every rank)
    const std::vector<size_t> cut = host_chunk_cuts(total, chunk);
    const size_t nchunks = cut.size() - 1;
    std::vector<CopyPool::Piece> pieces;
    // timeline statistics (config "host_pack_us" / "host_wait_us" / "host_unpack_us"): where the
    // engine thread spends a host plan — packing chunks, waiting for a slot's DMA / device work,
    // unpacking chunks
    using clk = std::chrono::steady_clock;
    auto ns_since = [](clk::time_point t0) {  // summed in ns: a 4 KiB chunk's unpack is < 1 us
        return (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
    };
    // staged outputs: chunk j's D2H lands in the download slot pout_[j % kHostSlots] and its host
    // unpack runs on the unpack lane (out_pool_'s copy threads) — concurrently with the engine
    // thread's packs of the next chunks into the upload slots. Before the D2H of chunk j + kHostSlots
    // reuses the download slot, the engine thread waits for chunk j's unpack (host_unpack_us).
    std::vector<uint64_t> unpacked(nchunks, 0);  // lane job of chunk j
    const int dev = owner_->device();
    auto unpack_async = [&](size_t j) {
        const int k = (int)(j % kHostSlots);
        std::vector<CopyPool::Piece> pc;
        host_pieces_(segs, starts, cut[j], cut[j + 1] - cut[j], static_cast<char *>(pout_[k]), false, pc);
        const hipEvent_t landed = hev_[3 * k + 2];  // re-recorded only after this job (wait_unpack)
        CopyPool *op = out_pool_.get();
        unpacked[j] = lane_->submit([dev, landed, op, ns_since, pc = std::move(pc)] {
            DeviceGuard g(dev);
            // D2H of chunk j landed (polled: see wait_plan). The lane's two phases are timed apart
            // (config "host_lane_d2h_wait_us" / "host_lane_copy_us" / "host_lane_copy_bytes",
            // VERDICT r5 next #4): the wait says how long the DMA kept the lane, the copy what
            // rate the pinned download slot -> pageable output memcpy reaches
            clk::time_point t0 = clk::now();
            const hipError_t q = wait_plan(landed);
            config().host_lane_d2h_wait_ns.fetch_add(ns_since(t0));
            DDL_REQUIRE(q == hipSuccess, DDL_STATUS_HIP_ERROR, "D2H of a staged chunk: " << hipGetErrorString(q));
            t0 = clk::now();
            op->run(pc);
            config().host_lane_copy_ns.fetch_add(ns_since(t0));
            long long bytes = 0;
            for (const CopyPool::Piece &p : pc) bytes += (long long)p.bytes;
            config().host_lane_copy_bytes.fetch_add(bytes);
            config().host_lane_jobs.fetch_add(1);
        });
    };
    auto wait_unpack = [&](size_t j) {
        const clk::time_point t0 = clk::now();
        lane_->wait(unpacked[j]);
        config().host_unpack_ns.fetch_add(ns_since(t0));
    };
    std::vector<void *> dst;
    std::vector<size_t> len;
    // no unpack job may outlive the plan: if posting throws midway (a collective, a
    // HIP call, a failed unpack), the lane finishes the jobs already submitted — they write into
    // the requests' outputs — before the error reaches complete_() and done(), after which the
    // caller may free those outputs; drain() also clears the lane's error, so it cannot surface in
    // a later plan's wait
    try {
        for (size_t i = 0; i < nchunks; ++i) {
            const int k = (int)(i % kHostSlots);
            const size_t off = cut[i], n = cut[i + 1] - off;
            // the device slot's last user may still be in flight (a device unpack)
            if (slot_used_[k]) DDL_HIP(hipStreamWaitEvent(h2d_, hev_[3 * k + 2], 0));
            if (upload) {
                // the pinned slot's last upload must have left it (device-unpack plans do not wait
                // for their D2H on the host)
                clk::time_point t0 = clk::now();
                if (slot_used_[k]) DDL_HIP(hipEventSynchronize(hev_[3 * k]));
                config().host_wait_ns.fetch_add(ns_since(t0));
                t0 = clk::now();
                pieces.clear();
                host_pieces_(segs, starts, off, n, static_cast<char *>(pin_[k]), true, pieces);
                pool_->run(pieces);  // packs chunk i while the device works on chunks i-1, i-2, ...
                DDL_HIP(hipMemcpyAsync(dslot_[k], pin_[k], n, hipMemcpyHostToDevice, h2d_));
                config().host_pack_ns.fetch_add(ns_since(t0));
            }
            DDL_HIP(hipEventRecord(hev_[3 * k], h2d_));
            DDL_HIP(hipStreamWaitEvent(stream_, hev_[3 * k], 0));
            const clk::time_point t_coll = clk::now();
            const long long fault = g_host_coll_fault.load();
            if (fault >= 0 && (long long)i >= fault) {  // test hook (ddl_testing_host_coll_fault)
                g_host_coll_fault = -1;
                fail(DDL_STATUS_COMM_ERROR, "test fault: host plan collective of chunk " + std::to_string(i));
            }
            coll(dslot_[k], n / es);
            config().host_coll_ns.fetch_add(ns_since(t_coll));
            DDL_HIP(hipEventRecord(hev_[3 * k + 1], stream_));
            DDL_HIP(hipStreamWaitEvent(d2h_, hev_[3 * k + 1], 0));
            if (device_unpack) {
                // the unpack kernel writes the chunk's pieces straight into the pinned outputs over
                // PCIe; it lays piece j at the rounded sum of the pieces before it, which is its
                // offset in the padded stream (chunks start at multiples of 256, so a cut never
                // falls inside a segment's padding)
                dst.clear();
                len.clear();
                size_t flat = 0;
                for (size_t j = (size_t)(std::upper_bound(starts.begin(), starts.end(), off) - starts.begin()) - 1;
                     j < segs.size() && starts[j] < off + n; ++j) {
                    const size_t lo = std::max(off, starts[j]), hi = std::min(off + n, starts[j] + segs[j].bytes);
                    if (hi <= lo) continue;
                    DDL_REQUIRE(flat == lo - off, DDL_STATUS_ERROR_UNKNOWN, "device-unpack chunk layout");
                    dst.push_back(segs[j].ddst + (lo - starts[j]));  // the device's address of the output
                    len.push_back(hi - lo);
                    flat += round256(hi - lo);
                }
                fp_.copier.run(1, dslot_[k], dst.data(), len.data(), (int)dst.size(), d2h_);
            } else {
                if (i >= (size_t)kHostSlots) wait_unpack(i - kHostSlots);  // download slot k free again
                const clk::time_point t_post = clk::now();
                DDL_HIP(hipMemcpyAsync(pout_[k], dslot_[k], n, hipMemcpyDeviceToHost, d2h_));
                config().host_d2h_post_ns.fetch_add(ns_since(t_post));
            }
            DDL_HIP(hipEventRecord(hev_[3 * k + 2], d2h_));
            slot_used_[k] = true;
            if (!device_unpack) {
                const clk::time_point t_sub = clk::now();
                unpack_async(i);
                config().host_unpack_submit_ns.fetch_add(ns_since(t_sub));
            }
        }
        if (device_unpack) {
            // the plan's event (recorded on stream_ next) covers the last unpack, hence every unpack
            DDL_HIP(hipStreamWaitEvent(stream_, hev_[3 * ((nchunks - 1) % kHostSlots) + 2], 0));
            return;
        }
        for (size_t j = nchunks > (size_t)kHostSlots ? nchunks - kHostSlots : 0; j < nchunks; ++j) wait_unpack(j);
    } catch (...) {
        lane_->drain();
        // device-unpack plans: copier kernels of the chunks already posted on d2h_ write into the
        // caller's pinned outputs; they must finish before done(error) lets the caller free those
        // (ADVICE r5). The H2D / compute work of posted chunks reads the caller's inputs and the
        // slots: drained too, so the next plan starts from idle streams.
        (void)hipStreamSynchronize(h2d_);
        (void)hipStreamSynchronize(stream_);
        (void)hipStreamSynchronize(d2h_);
        throw;
    }
}

void RequestHandler::release_registrations() {
    std::lock_guard<std::mutex> g(reg_mu_);
    DeviceGuard dg(owner_->device());
    {
        std::lock_guard<std::mutex> q(unreg_mu_);
        unreg_q_.clear();  // everything goes anyway
    }
    if (!reg_.empty()) unregister_all_();
}

void RequestHandler::unregister_range(const void *ptr, size_t bytes) {
    if (!ptr || !bytes) return;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr), hi = lo + bytes;
    std::unique_lock<std::mutex> g(reg_mu_, std::try_to_lock);
    if (!g.owns_lock()) {  // a host plan is being posted: the engine drains the queue before its next lookup
        std::lock_guard<std::mutex> q(unreg_mu_);
        unreg_q_.emplace_back(lo, hi);
        return;
    }
    DeviceGuard dg(owner_->device());
    drain_unregisters_();
    drop_overlapping_(lo, hi);
}

void RequestHandler::drain_unregisters_() {
    std::vector<std::pair<uintptr_t, uintptr_t>> q;
    {
        std::lock_guard<std::mutex> g(unreg_mu_);
        q.swap(unreg_q_);
    }
    for (const auto &r : q) drop_overlapping_(r.first, r.second);
}

void RequestHandler::drop_overlapping_(uintptr_t lo, uintptr_t hi) {
    std::vector<uintptr_t> drop;
    for (auto &e : reg_)
        if (e.first < hi && lo < e.first + e.second.first) drop.push_back(e.first);
    if (drop.empty()) return;
    for (hipStream_t st : {h2d_, d2h_, stream_})  // plans in flight may still DMA from / to them
        if (st) DDL_HIP(hipStreamSynchronize(st));
    for (uintptr_t a : drop) {
        (void)hipHostUnregister(reinterpret_cast<void *>(a));
        reg_bytes_ -= reg_[a].first;
        config().host_registered_bytes.fetch_sub((long long)reg_[a].first);
        config().host_unregistered_ranges.fetch_add(1);
        reg_.erase(a);
    }
    (void)hipGetLastError();
}

void RequestHandler::unregister_all_() {
    for (hipStream_t st : {h2d_, d2h_, stream_})  // rounds in flight may still DMA from / to them
        if (st) DDL_HIP(hipStreamSynchronize(st));
    for (auto &e : reg_) {
        (void)hipHostUnregister(reinterpret_cast<void *>(e.first));
        config().host_registered_bytes.fetch_sub((long long)e.second.first);
    }
    (void)hipGetLastError();
    reg_.clear();
    reg_bytes_ = 0;
}

void RequestHandler::register_hosts_(const std::vector<std::pair<const void *, size_t>> &ranges) {
    constexpr uintptr_t kPage = 4096;
    drain_unregisters_();  // ranges freed since the last lookup are not hits
    const size_t cap = (size_t)config().host_register_cache_bytes.load();
    // 1) the page ranges of the tensors not pinned already, merged where they share pages (small
    //    tensors of one heap page; hipHostRegister refuses a page registered twice)
    std::vector<std::pair<uintptr_t, uintptr_t>> want;
    for (const auto &r : ranges) {
        if (!r.first || r.second == 0) continue;
        const uintptr_t lo = reinterpret_cast<uintptr_t>(r.first) & ~(kPage - 1);
        const uintptr_t hi = (reinterpret_cast<uintptr_t>(r.first) + r.second + kPage - 1) & ~(kPage - 1);
        auto it = reg_.upper_bound(lo);  // inside an entry already: touch it
        if (it != reg_.begin() && std::prev(it)->first <= lo && hi <= std::prev(it)->first + std::prev(it)->second.first) {
            std::prev(it)->second.second = ++reg_tick_;
            config().host_register_hits.fetch_add(1);
            continue;
        }
        if (mapped_host_range(r.first, r.second)) continue;  // pinned already (the framework's own)
        want.emplace_back(lo, hi);
    }
    std::sort(want.begin(), want.end());
    std::vector<std::pair<uintptr_t, uintptr_t>> merged;
    for (const auto &w : want) {
        if (!merged.empty() && w.first < merged.back().second) merged.back().second = std::max(merged.back().second, w.second);
        else merged.push_back(w);
    }
    if (merged.empty()) return;
    bool synced = false;
    auto release = [&](uintptr_t a) {
        if (!synced) {  // rounds in flight may still DMA from / to it
            for (hipStream_t st : {h2d_, d2h_, stream_})
                if (st) DDL_HIP(hipStreamSynchronize(st));
            synced = true;
        }
        (void)hipHostUnregister(reinterpret_cast<void *>(a));
        (void)hipGetLastError();
        reg_bytes_ -= reg_[a].first;
        config().host_registered_bytes.fetch_sub((long long)reg_[a].first);
        reg_.erase(a);
    };
    for (auto m : merged) {
        // 2) entries overlapping it (a tensor that grew, moved or shares a page) join the union
        std::vector<uintptr_t> drop;
        for (auto &e : reg_)
            if (e.first < m.second && m.first < e.first + e.second.first) {
                drop.push_back(e.first);
                m.first = std::min(m.first, e.first);
                m.second = std::max(m.second, (uintptr_t)(e.first + e.second.first));
            }
        const size_t bytes = m.second - m.first;
        if (bytes > cap) continue;
        for (uintptr_t a : drop) release(a);
        while (reg_bytes_ + bytes > cap && !reg_.empty()) {  // least recently used out
            auto lru = reg_.begin();
            for (auto e = reg_.begin(); e != reg_.end(); ++e)
                if (e->second.second < lru->second.second) lru = e;
            release(lru->first);
        }
        if (hipHostRegister(reinterpret_cast<void *>(m.first), bytes, hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();  // e.g. registered by someone else: staged as before
            config().host_register_failures.fetch_add(1);
            continue;
        }
        reg_[m.first] = std::make_pair(bytes, ++reg_tick_);
        reg_bytes_ += bytes;
        config().host_registered_bytes.fetch_add((long long)bytes);
    }
}

// allreduceRequests (MPIRingTokenCommunication.cc:105-157): dtype groups in ascending enum order,
// ids lexicographic inside, plans capped at the fusion threshold.
void RequestHandler::allreduce_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans) {
    // (dtype, host): dtype groups in ascending enum order; host-resident requests — all of them
    // in the reference, which only has CPU tensors — form their own groups after the device ones
    std::map<std::pair<int, int>, std::vector<size_t>> groups;
    for (size_t i = 0; i < reqs.size(); ++i) {
        if (reqs[i].n == 0) dones.push_back(Done{kNoPlan, i, DDL_STATUS_OK});  // nothing to reduce
        else groups[std::make_pair(reqs[i].dtype, reqs[i].host ? 1 : 0)].push_back(i);
    }
    std::vector<hipEvent_t> waited;
    for (auto &g : groups) {
        const int dt = g.first.first;
        const bool host = g.first.second != 0;
        const size_t es = dtype_size(dt);
        std::vector<size_t> elems, esz;
        for (size_t i : g.second) {
            elems.push_back(reqs[i].n);
            esz.push_back(es);
        }
        // a host group holds the registration lock while its plans are posted: release_registrations
        // (ddl_set_config on the user's thread) then waits, and its stream sync covers every plan
        // already posted with a device alias of a registered range
        std::unique_lock<std::mutex> rg(reg_mu_, std::defer_lock);
        if (host) rg.lock();
        if (host && config().host_register_cache_bytes.load() > 0) {
            std::vector<std::pair<const void *, size_t>> ranges;  // pageable tensors used again and again
            for (size_t i : g.second) {
                ranges.emplace_back(reqs[i].in, reqs[i].n * es);
                if (reqs[i].out != reqs[i].in) ranges.emplace_back(reqs[i].out, reqs[i].n * es);
            }
            register_hosts_(ranges);  // registered once, kept
        }
        for (const Plan &p : make_plans(elems, esz, (size_t)config().fusion_threshold_bytes.load())) {
            for (size_t q = p.req_begin; q <= p.req_end; ++q) wait_inputs_(reqs[g.second[q]], waited);
            if (host) {
                // memcpy in -> MPI_Allreduce -> memcpy out (MPIRingTokenCommunication.cc:548-733),
                // the allreduce on the device through pinned chunks
                std::vector<HostSeg> segs;
                size_t message = 0;
                for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                    const Request &r = reqs[g.second[q]];
                    size_t b, e;
                    plan_slice(p, q, r.n, &b, &e);
                    segs.push_back(HostSeg{static_cast<const char *>(r.in) + b * es, static_cast<char *>(r.out) + b * es,
                                           (e - b) * es});
                    message += (e - b) * es;
                }
                if (data_->size() == 1 && config().one_rank_shortcut.load()) {
                    std::vector<CopyPool::Piece> pieces;
                    for (const HostSeg &sg : segs)
                        if (sg.src != sg.dst) pieces.push_back(CopyPool::Piece{sg.dst, sg.src, sg.bytes});
                    pool_for_config_().run(pieces);
                } else {
                    // chunks of the padded stream either way, so ranks that differ in which
                    // outputs are pinned still issue the same collectives
                    auto coll = [&](void *d, size_t elems) {
                        data_->allreduce(d, d, elems, dt, DDL_ALLREDUCE_OP_SUM, stream_, message);
                    };
                    const auto t_check = std::chrono::steady_clock::now();
                    const bool mapped = config().host_zero_copy.load() && mapped_host_dsts_(segs);
                    const auto t_plan = std::chrono::steady_clock::now();
                    config().host_check_ns.fetch_add(
                        std::chrono::duration_cast<std::chrono::nanoseconds>(t_plan - t_check).count());
                    host_staged_(segs, es, true, coll, true, mapped);
                    config().host_plan_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                        std::chrono::steady_clock::now() - t_plan)
                                                        .count());
                }
            } else if (data_->size() == 1 && config().one_rank_shortcut.load()) {
                // a one-rank world: the sum is the input; move bytes only where out != in
                for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                    const Request &r = reqs[g.second[q]];
                    size_t b, e;
                    plan_slice(p, q, r.n, &b, &e);
                    if (r.in != r.out && e > b)
                        DDL_HIP(hipMemcpyAsync(static_cast<char *>(r.out) + b * es,
                                               static_cast<const char *>(r.in) + b * es, (e - b) * es,
                                               hipMemcpyDeviceToDevice, stream_));
                }
            } else if (p.req_begin == p.req_end) {
                const Request &r = reqs[g.second[p.req_begin]];
                const size_t cnt = p.elem_end - p.elem_begin;
                data_->allreduce(static_cast<const char *>(r.in) + p.elem_begin * es,
                                 static_cast<char *>(r.out) + p.elem_begin * es, cnt, dt, r.op, stream_);
            } else {
                std::vector<const void *> srcs;
                std::vector<void *> dsts;
                std::vector<size_t> bytes;
                for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                    const Request &r = reqs[g.second[q]];
                    size_t b, e;
                    plan_slice(p, q, r.n, &b, &e);
                    srcs.push_back(static_cast<const char *>(r.in) + b * es);
                    dsts.push_back(static_cast<char *>(r.out) + b * es);
                    bytes.push_back((e - b) * es);
                }
                fp_.run(srcs, dsts, bytes, dt, (size_t)config().fusion_pipeline_bytes.load(), stream_,
                        [&](void *buf, size_t elems, size_t message) {
                            data_->allreduce(buf, buf, elems, dt, DDL_ALLREDUCE_OP_SUM, stream_, message);
                        });
            }
            const size_t plan = record_plan_(nplans);
            for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                const Request &r = reqs[g.second[q]];
                const size_t e = q == p.req_end ? p.elem_end : r.n;
                if (e == r.n) dones.push_back(Done{plan, g.second[q], DDL_STATUS_OK});
            }
        }
    }
}

// broadcastRequests (MPIRingTokenCommunication.cc:367-419): dtype groups, plans, broadcast of
// the packed plan from the root. The reference broadcasts every group from the first request's
// root; requests are grouped by (dtype, root) here so mixed roots stay correct.
void RequestHandler::broadcast_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans) {
    std::map<std::tuple<int, int, int>, std::vector<size_t>> groups;  // (dtype, root, host)
    for (size_t i = 0; i < reqs.size(); ++i) {
        if (reqs[i].n == 0) dones.push_back(Done{kNoPlan, i, DDL_STATUS_OK});
        else groups[std::make_tuple(reqs[i].dtype, reqs[i].root, reqs[i].host ? 1 : 0)].push_back(i);
    }
    const int me = data_->rank();
    std::vector<hipEvent_t> waited;
    for (auto &g : groups) {
        const int dt = std::get<0>(g.first), root = std::get<1>(g.first);
        const bool host = std::get<2>(g.first) != 0;
        const size_t es = dtype_size(dt);
        std::vector<size_t> elems, esz;
        for (size_t i : g.second) {
            elems.push_back(reqs[i].n);
            esz.push_back(es);
        }
        // a host group holds the registration lock while its plans are posted: release_registrations
        // (ddl_set_config on the user's thread) then waits, and its stream sync covers every plan
        // already posted with a device alias of a registered range
        std::unique_lock<std::mutex> rg(reg_mu_, std::defer_lock);
        if (host) rg.lock();
        if (host && config().host_register_cache_bytes.load() > 0) {
            std::vector<std::pair<const void *, size_t>> ranges;  // pageable tensors used again and again
            for (size_t i : g.second) {
                ranges.emplace_back(reqs[i].in, reqs[i].n * es);
                if (reqs[i].out != reqs[i].in) ranges.emplace_back(reqs[i].out, reqs[i].n * es);
            }
            register_hosts_(ranges);  // registered once, kept
        }
        for (const Plan &p : make_plans(elems, esz, (size_t)config().fusion_threshold_bytes.load())) {
            for (size_t q = p.req_begin; q <= p.req_end; ++q) wait_inputs_(reqs[g.second[q]], waited);
            if (host) {
                // root: pack in -> H2D -> broadcast -> D2H -> unpack to out; others only receive
                std::vector<HostSeg> segs;
                for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                    const Request &r = reqs[g.second[q]];
                    size_t b, e;
                    plan_slice(p, q, r.n, &b, &e);
                    segs.push_back(HostSeg{static_cast<const char *>(r.in) + b * es, static_cast<char *>(r.out) + b * es,
                                           (e - b) * es});
                }
                host_staged_(segs, es, me == root,
                             [&](void *d, size_t elems) { data_->broadcast(d, elems, dt, root, stream_); });
            } else if (p.req_begin == p.req_end) {
                const Request &r = reqs[g.second[p.req_begin]];
                const size_t cnt = p.elem_end - p.elem_begin;
                char *out = static_cast<char *>(r.out) + p.elem_begin * es;
                if (me == root && r.in != r.out)
                    DDL_HIP(hipMemcpyAsync(out, static_cast<const char *>(r.in) + p.elem_begin * es, cnt * es,
                                           hipMemcpyDeviceToDevice, stream_));
                data_->broadcast(out, cnt, dt, root, stream_);
            } else {
                std::vector<const void *> srcs;
                std::vector<void *> dsts;
                std::vector<size_t> bytes;
                for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                    const Request &r = reqs[g.second[q]];
                    size_t b, e;
                    plan_slice(p, q, r.n, &b, &e);
                    srcs.push_back(static_cast<const char *>(r.in) + b * es);
                    dsts.push_back(static_cast<char *>(r.out) + b * es);
                    bytes.push_back((e - b) * es);
                }
                const size_t total = SegmentCopier::flat_bytes(bytes.data(), (int)bytes.size());
                void *fb = fp_.ensure(0, total, stream_);
                if (me == root)
                    fp_.copier.run(0, fb, const_cast<void *const *>(srcs.data()), bytes.data(), (int)srcs.size(),
                                   stream_);
                data_->broadcast(fb, total / es, dt, root, stream_);
                fp_.copier.run(1, fb, dsts.data(), bytes.data(), (int)dsts.size(), stream_);
            }
            const size_t plan = record_plan_(nplans);
            for (size_t q = p.req_begin; q <= p.req_end; ++q) {
                const Request &r = reqs[g.second[q]];
                const size_t e = q == p.req_end ? p.elem_end : r.n;
                if (e == r.n) dones.push_back(Done{plan, g.second[q], DDL_STATUS_OK});
            }
        }
    }
}

// allgatherRequests (MPIRingTokenCommunication.cc:160-364), per dtype group: allgather every
// rank's first dims (u64), allocate each output (first dim = sum over ranks), then one
// allgatherv of the packed requests and an unpack into the outputs in rank order. A single
// request gathers straight into its output (rank-major blocks are the concatenation).
void RequestHandler::allgather_reqs_(std::vector<Request> &reqs, std::vector<Done> &dones, size_t &nplans) {
    std::map<std::pair<int, int>, std::vector<size_t>> groups;  // (dtype, host)
    for (size_t i = 0; i < reqs.size(); ++i) groups[std::make_pair(reqs[i].dtype, reqs[i].host ? 1 : 0)].push_back(i);
    const int P = data_->size(), me = data_->rank();
    std::vector<hipEvent_t> waited;
    for (auto &g : groups) {
        const int dt = g.first.first;
        const bool host = g.first.second != 0;
        const size_t es = dtype_size(dt), m = g.second.size();
        // 1) first dims of every rank: fd[q * m + j]
        std::vector<uint64_t> fd(P * m);
        for (size_t j = 0; j < m; ++j) fd[me * m + j] = reqs[g.second[j]].first_dim;
        if (P > 1) {
            ensure_(dims_, dims_bytes_, fd.size() * 8);
            std::vector<size_t> cnt(P, m), dsp(P);
            for (int q = 0; q < P; ++q) dsp[q] = q * m;
            DDL_HIP(hipMemcpyAsync(static_cast<char *>(dims_) + me * m * 8, fd.data() + me * m, m * 8,
                                   hipMemcpyHostToDevice, stream_));
            data_->allgatherv(static_cast<char *>(dims_) + me * m * 8, dims_, cnt.data(), dsp.data(), DDL_UINT64,
                              stream_);
            DDL_HIP(hipMemcpyAsync(fd.data(), dims_, fd.size() * 8, hipMemcpyDeviceToHost, stream_));
            DDL_HIP(hipStreamSynchronize(stream_));
        }
        // 2) outputs
        std::vector<size_t> total_rows(m, 0);
        for (size_t j = 0; j < m; ++j) {
            Request &r = reqs[g.second[j]];
            for (int q = 0; q < P; ++q) total_rows[j] += fd[q * m + j];
            const size_t bytes = total_rows[j] * r.row_elems * es;
            r.out = r.alloc(total_rows[j], bytes, r.user);
            DDL_REQUIRE(bytes == 0 || r.out, DDL_STATUS_ERROR_UNKNOWN, "allgather output allocation failed for '" << r.key << "'");
        }
        for (size_t j = 0; j < m; ++j) wait_inputs_(reqs[g.second[j]], waited);
        // 3) data
        if (host) {
            // host tensors: this rank's rows packed back to back through a pinned buffer, one
            // allgatherv on the device, then every rank's rows unpacked into the host outputs
            std::vector<size_t> blk(P, 0);
            for (int q = 0; q < P; ++q)
                for (size_t j = 0; j < m; ++j) blk[q] += fd[q * m + j] * reqs[g.second[j]].row_elems * es;
            size_t all = 0;
            std::vector<size_t> cnt(P), dsp(P);
            for (int q = 0; q < P; ++q) {
                cnt[q] = blk[q] / es;
                dsp[q] = all / es;
                all += blk[q];
            }
            if (all) {
                void *fb = fp_.ensure(0, std::max<size_t>(blk[me], 256), stream_);
                ensure_(gather_, gather_bytes_, all);
                if (pin_gather_bytes_ < all) {
                    retire_host(pin_gather_);  // no hipHostFree on a data path (engine.h retire_host)
                    pin_gather_ = nullptr;
                    pin_gather_bytes_ = 0;
                    DDL_HIP(hipHostMalloc(&pin_gather_, all + all / 2, hipHostMallocDefault));
                    pin_gather_bytes_ = all + all / 2;
                }
                char *pin = static_cast<char *>(pin_gather_);
                size_t off = 0;
                for (size_t j = 0; j < m; ++j) {
                    const Request &r = reqs[g.second[j]];
                    const size_t b = fd[me * m + j] * r.row_elems * es;
                    std::memcpy(pin + off, r.in, b);
                    off += b;
                }
                DDL_HIP(hipMemcpyAsync(fb, pin, blk[me], hipMemcpyHostToDevice, stream_));
                data_->allgatherv(fb, gather_, cnt.data(), dsp.data(), dt, stream_);
                DDL_HIP(hipMemcpyAsync(pin, gather_, all, hipMemcpyDeviceToHost, stream_));
                DDL_HIP(hipStreamSynchronize(stream_));
                std::vector<size_t> row_off(m, 0);
                off = 0;
                for (int q = 0; q < P; ++q)
                    for (size_t j = 0; j < m; ++j) {
                        const Request &r = reqs[g.second[j]];
                        const size_t b = fd[q * m + j] * r.row_elems * es;
                        std::memcpy(static_cast<char *>(r.out) + row_off[j] * r.row_elems * es, pin + off, b);
                        row_off[j] += fd[q * m + j];
                        off += b;
                    }
            }
        } else if (m == 1) {
            const Request &r = reqs[g.second[0]];
            std::vector<size_t> cnt(P), dsp(P);
            size_t acc = 0;
            for (int q = 0; q < P; ++q) {
                cnt[q] = fd[q] * r.row_elems;
                dsp[q] = acc;
                acc += cnt[q];
            }
            if (acc) data_->allgatherv(r.in, r.out, cnt.data(), dsp.data(), dt, stream_);
        } else {
            // rank q's block: its m requests, each 256-byte aligned (the copier's flat layout)
            std::vector<size_t> blk(P, 0);
            std::vector<size_t> seg_bytes(P * m);
            for (int q = 0; q < P; ++q)
                for (size_t j = 0; j < m; ++j) {
                    seg_bytes[q * m + j] = fd[q * m + j] * reqs[g.second[j]].row_elems * es;
                    blk[q] += (seg_bytes[q * m + j] + 255) & ~size_t(255);
                }
            size_t all = 0;
            std::vector<size_t> cnt(P), dsp(P);
            for (int q = 0; q < P; ++q) {
                cnt[q] = blk[q] / es;
                dsp[q] = all / es;
                all += blk[q];
            }
            if (all) {
                void *fb = fp_.ensure(0, std::max<size_t>(blk[me], 256), stream_);
                ensure_(gather_, gather_bytes_, all);
                std::vector<const void *> srcs(m);
                for (size_t j = 0; j < m; ++j) srcs[j] = reqs[g.second[j]].in;
                fp_.copier.run(0, fb, const_cast<void *const *>(srcs.data()), seg_bytes.data() + me * m, (int)m,
                               stream_);
                data_->allgatherv(fb, gather_, cnt.data(), dsp.data(), dt, stream_);
                std::vector<void *> dsts(P * m);
                std::vector<size_t> row_off(m, 0);  // rows of request j written so far
                for (int q = 0; q < P; ++q)
                    for (size_t j = 0; j < m; ++j) {
                        const Request &r = reqs[g.second[j]];
                        dsts[q * m + j] = static_cast<char *>(r.out) + row_off[j] * r.row_elems * es;
                        row_off[j] += fd[q * m + j];
                    }
                fp_.copier.run(1, gather_, dsts.data(), seg_bytes.data(), (int)(P * m), stream_);
            }
        }
        const size_t plan = record_plan_(nplans);
        for (size_t j = 0; j < m; ++j) dones.push_back(Done{plan, g.second[j], DDL_STATUS_OK});
    }
}

void RequestHandler::execute_(const std::vector<ReqId> &ids, int forced) {
    if (ids.empty()) return;
    // phase times of the round at log level 2 (take / enqueue / wait + done, microseconds)
    using clk = std::chrono::steady_clock;
    const bool timed = log_level() >= 2;
    const clk::time_point t0 = timed ? clk::now() : clk::time_point();
    std::vector<Request> reqs;
    reqs.reserve(ids.size());
    {
        std::lock_guard<std::mutex> g(mu_);
        // the agreed ids come in (type, key) order, the pending map's order: one forward walk
        // (a compare or two per id) instead of a lookup per id
        const bool sorted = std::is_sorted(ids.begin(), ids.end());
        auto it = sorted ? pending_.lower_bound(ids.front()) : pending_.end();
        for (const auto &k : ids) {
            if (sorted) {
                while (it != pending_.end() && it->first < k) ++it;
            } else {
                it = pending_.find(k);
            }
            DDL_REQUIRE(it != pending_.end() && !(k < it->first), DDL_STATUS_COMM_ERROR,
                        "agreed request '" << k.key << "' is not registered");
            if (it->second.cidx >= 0) pend_flag_[it->second.cidx] = 0;
            reqs.push_back(std::move(it->second));
            it = pending_.erase(it);
        }
        inflight_ += reqs.size();
    }
    std::vector<Done> dones;
    size_t nplans = 0;
    int status = forced;
    const clk::time_point t1 = timed ? clk::now() : clk::time_point();
    round_events_.clear();
    if (forced == DDL_STATUS_OK) try {
        for (const Request &r : reqs)
            DDL_REQUIRE(r.type == reqs[0].type, DDL_STATUS_COMM_ERROR, "agreed requests of mixed types");
        switch (reqs[0].type) {
            case kReqAllreduce: allreduce_reqs_(reqs, dones, nplans); break;
            case kReqBroadcast: broadcast_reqs_(reqs, dones, nplans); break;
            case kReqAllgather: allgather_reqs_(reqs, dones, nplans); break;
            default: fail(DDL_STATUS_ERROR_UNKNOWN, "unknown request type");
        }
    } catch (const Error &e) {
        DDL_LOG(0, "collective of agreed requests failed: " << e.msg);
        status = e.status;
    }
    Round rd;
    rd.reqs = std::move(reqs);
    rd.dones = std::move(dones);
    rd.events.swap(round_events_);
    rd.status = status;
    rd.nplans = nplans;
    rd.t0 = t0;
    rd.t1 = t1;
    if (timed) rd.t2 = clk::now();
    const bool pipelined = config().pipeline_rounds.load() != 0;
    size_t bytes = 0;
    for (const Request &r : rd.reqs) bytes += r.n * dtype_size(r.dtype);
    bool idle;
    {
        std::lock_guard<std::mutex> g(done_mu_);
        idle = rounds_queued_ == rounds_done_;  // no earlier round waiting or completing
    }
    // nothing earlier in flight and the round is to be waited for anyway (unpipelined, failed)
    // or small (its data plane takes microseconds): complete it here — done() order holds and
    // the hand-off to the completion thread (a thread wake-up each way) is saved
    if (idle && (!pipelined || status != DDL_STATUS_OK || bytes <= kInlineRoundBytes)) {
        complete_(rd);
        if (status != DDL_STATUS_OK && status != forced) fail(status, "keyed collective failed");
        return;
    }
    unsigned long long seq;
    {
        std::lock_guard<std::mutex> g(done_mu_);
        rounds_.push_back(std::move(rd));
        seq = ++rounds_queued_;
    }
    done_cv_.notify_all();
    // pipelined: back to negotiating while the device runs this round; otherwise (and after a
    // failed enqueue, whose done() calls must have fired before the handler stops) wait for it
    if (status != DDL_STATUS_OK || !pipelined) {
        std::unique_lock<std::mutex> lk(done_mu_);
        done_cv_.wait(lk, [&] { return rounds_done_ >= seq; });
    }
    if (status != DDL_STATUS_OK && status != forced) fail(status, "keyed collective failed");
}


// done() in plan order as each request's last element lands (MPIRTC.cc:593-597, 690-725).
void RequestHandler::complete_(Round &rd) {
    using clk = std::chrono::steady_clock;
    int status = rd.status;
    std::vector<char> fired(rd.reqs.size(), 0);
    size_t synced = kNoPlan;  // dones are in plan order: wait for each plan's event once
    for (const Done &d : rd.dones) {
        if (status == DDL_STATUS_OK && d.plan != kNoPlan && d.plan != synced) {
            hipError_t he = wait_plan(rd.events[d.plan]);
            if (he != hipSuccess) status = DDL_STATUS_HIP_ERROR;
            synced = d.plan;
        }
        const Request &r = rd.reqs[d.req];
        fired[d.req] = 1;
        if (r.done) r.done(status == DDL_STATUS_OK ? d.status : status, r.user);
    }
    for (size_t i = 0; i < rd.reqs.size(); ++i)
        if (!fired[i] && rd.reqs[i].done)
            rd.reqs[i].done(status == DDL_STATUS_OK ? DDL_STATUS_ERROR_UNKNOWN : status, rd.reqs[i].user);
    if (status == DDL_STATUS_OK) {  // waited for: safe to record again
        std::lock_guard<std::mutex> g(done_mu_);
        event_pool_.insert(event_pool_.end(), rd.events.begin(), rd.events.end());
    } else {
        for (hipEvent_t e : rd.events) (void)hipEventDestroy(e);
        if (rd.status == DDL_STATUS_OK) {  // a device failure the engine thread has not seen
            {
                std::lock_guard<std::mutex> g(mu_);
                int expected = 0;
                failed_.compare_exchange_strong(expected, status);
            }
            cv_.notify_all();
        }
    }
    rd.events.clear();
    const size_t n = rd.reqs.size();
    rd.reqs.clear();  // the requests' input-ready events go with them
    {
        std::lock_guard<std::mutex> g(mu_);
        inflight_ -= n;
    }
    idle_cv_.notify_all();
    if (log_level() >= 2 && rd.t0 != clk::time_point()) {
        auto us = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
        };
        DDL_LOG(2, "round: " << n << " requests, " << rd.nplans << " plans; take " << us(rd.t0, rd.t1) << " us, enqueue "
                             << us(rd.t1, rd.t2) << " us, wait + done " << us(rd.t2, clk::now()) << " us");
    }
}

void RequestHandler::completer_() {
    t_handler_thread = true;  // done() callbacks run here (engine.h)
    (void)hipSetDevice(owner_->device());
    for (;;) {
        Round rd;
        {
            std::unique_lock<std::mutex> lk(done_mu_);
            done_cv_.wait(lk, [this] { return done_stop_ || !rounds_.empty(); });
            if (rounds_.empty()) break;  // stopping, and every handed-over round has completed
            rd = std::move(rounds_.front());
            rounds_.pop_front();
        }
        complete_(rd);
        {
            std::lock_guard<std::mutex> g(done_mu_);
            ++rounds_done_;
        }
        done_cv_.notify_all();
    }
}

}  // namespace ddl
