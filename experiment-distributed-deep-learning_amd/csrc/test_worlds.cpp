// test_worlds.cpp — see test_worlds.h (testing library only).
#include "test_worlds.h"

#include <algorithm>
#include <sstream>
#include <thread>

namespace ddl {

void CallbackTransport::allgather(const GatherOp &g, hipStream_t stream) {
    char *recv = static_cast<char *>(g.recv);
    if (recv + (size_t)rank_ * g.bytes != g.send)  // in place: the own block is already there
        DDL_HIP(hipMemcpyAsync(recv + (size_t)rank_ * g.bytes, g.send, g.bytes, hipMemcpyDeviceToDevice, stream));
    std::vector<P2POp> ops;
    for (int d = 1; d < size_; ++d) {
        const int to = (rank_ + d) % size_, from = (rank_ + size_ - d) % size_;
        ops.push_back(P2POp{true, to, 0, const_cast<void *>(g.send), g.bytes});
        ops.push_back(P2POp{false, from, 0, recv + (size_t)from * g.bytes, g.bytes});
    }
    group(ops, stream);
}

CallbackTransport::~CallbackTransport() {
    if (pinned_) (void)hipHostFree(pinned_);
}

void CallbackTransport::group(const std::vector<P2POp> &ops, hipStream_t stream) {
    if (ops.empty()) return;
    // copies through pinned memory, ordered on `stream` only: a synchronous or pageable copy
    // would also wait for what the caller's framework queued on the default stream (the rest
    // of a backward pass, say)
    size_t need = 0;
    for (const P2POp &op : ops) need += (op.bytes + 255) & ~size_t(255);
    if (need > pinned_bytes_) {
        DDL_HIP(hipStreamSynchronize(stream));
        if (pinned_) DDL_HIP(hipHostFree(pinned_));
        pinned_ = nullptr;
        pinned_bytes_ = 0;
        DDL_HIP(hipHostMalloc(&pinned_, need, hipHostMallocDefault));
        pinned_bytes_ = need;
    }
    std::vector<ddl_p2p_op> v(ops.size());
    std::vector<char *> host(ops.size());
    for (size_t i = 0, off = 0; i < ops.size(); ++i) {
        host[i] = pinned_ + off;
        off += (ops[i].bytes + 255) & ~size_t(255);
        if (ops[i].send && ops[i].bytes)
            DDL_HIP(hipMemcpyAsync(host[i], ops[i].ptr, ops[i].bytes, hipMemcpyDeviceToHost, stream));
        v[i] = ddl_p2p_op{ops[i].send ? 1 : 0, ops[i].peer, ops[i].tag, host[i], ops[i].bytes};
    }
    DDL_HIP(hipStreamSynchronize(stream));  // the sends' data is on the host, the receive buffers free
    host_group(v);
    for (size_t i = 0; i < ops.size(); ++i)
        if (!ops[i].send && ops[i].bytes)
            DDL_HIP(hipMemcpyAsync(ops[i].ptr, host[i], ops[i].bytes, hipMemcpyHostToDevice, stream));
    DDL_HIP(hipStreamSynchronize(stream));  // the pinned buffer is reused by the next group
}

void CallbackTransport::host_group(std::vector<ddl_p2p_op> &ops) {
    if (ops.empty()) return;
    for (ddl_p2p_op &o : ops) {
        if (world_ranks_.empty()) continue;
        DDL_REQUIRE(o.peer >= 0 && o.peer < (int)world_ranks_.size(), DDL_STATUS_ERROR_UNKNOWN, "bad peer " << o.peer);
        o.peer = world_ranks_[o.peer];
    }
    const int rc = hooks_->group(tag_, ops.data(), (int)ops.size(), hooks_->user);
    DDL_REQUIRE(rc == 0, DDL_STATUS_COMM_ERROR, "test transport: group callback failed (" << rc << ")");
}

std::unique_ptr<Transport> make_callback_transport(const std::shared_ptr<TestHooks> &hooks, long long tag,
                                                   std::vector<int> world_ranks, int rank, int size) {
    return std::unique_ptr<Transport>(new CallbackTransport(hooks, tag, std::move(world_ranks), rank, size));
}

ThreadFabric::ThreadFabric(int P, ncclComm_t loopback) : P_(P), q_((size_t)P * P) {
    if (loopback) loop_.reset(new RcclTransport(loopback));
}

ThreadFabric::~ThreadFabric() {
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
}

hipEvent_t ThreadFabric::event_() {
    {
        std::lock_guard<std::mutex> g(mu_);
        if (next_event_ < events_.size()) return events_[next_event_++];
    }
    hipEvent_t e;
    DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::lock_guard<std::mutex> g(mu_);
    events_.push_back(e);
    next_event_ = events_.size();
    return e;
}

void ThreadFabric::recycle() {
    std::lock_guard<std::mutex> g(mu_);
    next_event_ = 0;
}

void ThreadFabric::abort() {
    {
        std::lock_guard<std::mutex> g(mu_);
        aborted_ = true;
    }
    cv_.notify_all();
}

void ThreadFabric::group(int rank, const std::vector<P2POp> &ops, hipStream_t stream) {
    if (ops.empty()) return;
    DDL_TRACE("fabric rank " << rank << " group of " << ops.size() << " ops on " << (void *)stream);
    // 1) post every send: the send buffers are ready at this point of `stream`
    hipEvent_t ready = event_();
    DDL_HIP(hipEventRecord(ready, stream));
    dep::record(ready, stream);
    std::vector<std::shared_ptr<Send>> mine;
    {
        std::lock_guard<std::mutex> g(mu_);
        for (const P2POp &op : ops) {
            if (!op.send) continue;
            DDL_REQUIRE(op.peer >= 0 && op.peer < P_ && op.peer != rank, DDL_STATUS_ERROR_UNKNOWN, "bad peer " << op.peer);
            auto sd = std::make_shared<Send>(Send{op.ptr, op.bytes, op.tag, ready});
            q_[(size_t)rank * P_ + op.peer].push_back(sd);
            mine.push_back(sd);
        }
    }
    cv_.notify_all();
    // 2) receives in posting order: the peer's matching send once it is POSTED (enqueue only)
    for (const P2POp &op : ops) {
        if (op.send) continue;
        std::shared_ptr<Send> sd;
        {
            std::unique_lock<std::mutex> g(mu_);
            auto &qq = q_[(size_t)op.peer * P_ + rank];
            cv_.wait(g, [&] { return aborted_ || !qq.empty(); });
            DDL_REQUIRE(!aborted_, DDL_STATUS_COMM_ERROR, "thread fabric aborted");
            sd = qq.front();
            qq.pop_front();
        }
        DDL_REQUIRE(sd->bytes == op.bytes && sd->tag == op.tag, DDL_STATUS_ERROR_UNKNOWN,
                    "thread fabric: rank " << rank << " receives " << op.bytes << " B (tag " << op.tag << ") from "
                                           << op.peer << ", whose matching send is " << sd->bytes << " B (tag "
                                           << sd->tag << ")");
        DDL_TRACE("fabric rank " << rank << " recv " << op.bytes << " B from " << op.peer << " tag " << op.tag << " "
                                  << sd->ptr << " -> " << op.ptr);
        DDL_HIP(hipStreamWaitEvent(stream, sd->ready, 0));
        dep::wait(stream, sd->ready);
        if (op.bytes && loop_) {  // the bytes through RCCL: a self pair in one group on this stream
            std::lock_guard<std::mutex> lg(loop_mu_);
            loop_->group({P2POp{true, 0, op.tag, const_cast<void *>(sd->ptr), op.bytes},
                          P2POp{false, 0, op.tag, op.ptr, op.bytes}},
                         stream);
            ++loopback_pairs;
        } else if (op.bytes) {
            DDL_HIP(hipMemcpyAsync(op.ptr, sd->ptr, op.bytes, hipMemcpyDeviceToDevice, stream));
        }
        if (dep::on()) {
            std::ostringstream os;
            os << "recv rank " << rank << " <- " << op.peer << " tag " << op.tag;
            dep::op(stream, os.str(), {dep::rd(sd->ptr, op.bytes), dep::wr(op.ptr, op.bytes)});
        }
        hipEvent_t copied = event_();
        DDL_HIP(hipEventRecord(copied, stream));
        dep::record(copied, stream);
        {
            std::lock_guard<std::mutex> g(mu_);
            sd->copied = copied;
        }
        cv_.notify_all();
    }
    // 3) the group completes for a sender once every receiver's copy has run (device order):
    //    the host waits only for the receivers to have ENQUEUED their copies
    for (const auto &sd : mine) {
        hipEvent_t copied;
        {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return aborted_ || sd->copied != nullptr; });
            DDL_REQUIRE(!aborted_, DDL_STATUS_COMM_ERROR, "thread fabric aborted");
            copied = sd->copied;
        }
        DDL_HIP(hipStreamWaitEvent(stream, copied, 0));
        dep::wait(stream, copied);
    }
}

void ThreadTransport::allgather(const GatherOp &g, hipStream_t stream) {
    const int P = fab_->size();
    char *recv = static_cast<char *>(g.recv);
    if (recv + (size_t)rank_ * g.bytes != g.send) {
        DDL_HIP(hipMemcpyAsync(recv + (size_t)rank_ * g.bytes, g.send, g.bytes, hipMemcpyDeviceToDevice, stream));
        if (dep::on())
            dep::op(stream, dep_label("gather own block", rank_, 0),
                    {dep::rd(g.send, g.bytes), dep::wr(recv + (size_t)rank_ * g.bytes, g.bytes)});
    }
    std::vector<P2POp> ops;
    for (int d = 1; d < P; ++d) {
        const int to = (rank_ + d) % P, from = (rank_ + P - d) % P;
        ops.push_back(P2POp{true, to, 0, const_cast<void *>(g.send), g.bytes});
        ops.push_back(P2POp{false, from, 0, recv + (size_t)from * g.bytes, g.bytes});
    }
    group(ops, stream);
}

ThreadWorld::ThreadWorld(int nranks, int device, ncclComm_t loopback) : P_(nranks), device_(device) {
    fab_ = std::make_shared<ThreadFabric>(nranks, loopback);
    for (int r = 0; r < nranks; ++r) {
        ex_.emplace_back(new RingExecutor(r, nranks, device, std::unique_ptr<Transport>(new ThreadTransport(fab_, r))));
        hipStream_t s;
        DDL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        streams_.push_back(s);
        hipEvent_t e;
        DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        done_.push_back(e);
    }
    DDL_HIP(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
}

ThreadWorld::~ThreadWorld() {
    (void)hipDeviceSynchronize();
    ex_.clear();
    for (hipStream_t s : streams_) (void)hipStreamDestroy(s);
    for (hipEvent_t e : done_) (void)hipEventDestroy(e);
    if (fork_) (void)hipEventDestroy(fork_);
}

void ThreadWorld::run_(hipStream_t user, const std::function<void(int, hipStream_t)> &body) {
    DDL_HIP(hipEventRecord(fork_, user));
    dep::record(fork_, user);
    for (int r = 0; r < P_; ++r) {
        DDL_HIP(hipStreamWaitEvent(streams_[r], fork_, 0));
        dep::wait(streams_[r], fork_);
    }
    std::vector<std::thread> th;
    std::vector<Error> errs;
    std::mutex emu;
    for (int r = 0; r < P_; ++r)
        th.emplace_back([&, r] {
            try {
                DDL_HIP(hipSetDevice(device_));
                body(r, streams_[r]);
                DDL_HIP(hipEventRecord(done_[r], streams_[r]));
                dep::record(done_[r], streams_[r]);
            } catch (const Error &e) {
                std::lock_guard<std::mutex> g(emu);
                errs.push_back(e);
                fab_->abort();
            }
        });
    for (auto &t : th) t.join();
    if (!errs.empty()) {
        (void)hipDeviceSynchronize();
        fab_ = std::make_shared<ThreadFabric>(P_);  // a fresh fabric: the aborted one has stale posts
        for (int r = 0; r < P_; ++r)
            ex_[r].reset(new RingExecutor(r, P_, device_, std::unique_ptr<Transport>(new ThreadTransport(fab_, r))));
        throw errs.front();
    }
    for (int r = 0; r < P_; ++r) {
        DDL_HIP(hipStreamWaitEvent(user, done_[r], 0));
        dep::wait(user, done_[r]);
    }
    fab_->recycle();
}

void ThreadWorld::allreduce(const void *const *in, void *const *out, size_t n, int dtype, hipStream_t user,
                            const RingConfig &cfg) {
    run_(user, [&](int r, hipStream_t s) { ex_[r]->allreduce(in[r], out[r], n, dtype, s, cfg); });
}

void ThreadWorld::broadcast(void *const *bufs, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg) {
    run_(user, [&](int r, hipStream_t s) { ex_[r]->broadcast(bufs[r], n, dtype, root, s, cfg); });
}

void ThreadWorld::allgatherv(const void *const *sends, void *const *recvs, const size_t *counts, const size_t *displs,
                             int dtype, hipStream_t user) {
    run_(user, [&](int r, hipStream_t s) { ex_[r]->allgatherv(sends[r], recvs[r], counts, displs, dtype, s); });
}

void ThreadWorld::allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                                  hipStream_t user, const RingConfig &cfg) {
    run_(user, [&](int r, hipStream_t s) {
        ex_[r]->allreduce_batch(in + (size_t)r * count, out + (size_t)r * count, n, count, dtype, s, cfg);
    });
}

size_t ThreadWorld::fused_allreduce(const void *const *srcs, void *const *dsts, const size_t *bytes, int count,
                                    int dtype, hipStream_t user, const RingConfig &cfg, size_t cap) {
    while (pipes_.size() < (size_t)P_) pipes_.emplace_back(new FusionPipe);
    const std::vector<size_t> b(bytes, bytes + count);
    run_(user, [&](int r, hipStream_t s) {
        const std::vector<const void *> src(srcs + (size_t)r * count, srcs + (size_t)(r + 1) * count);
        const std::vector<void *> dst(dsts + (size_t)r * count, dsts + (size_t)(r + 1) * count);
        pipes_[r]->run(src, dst, b, dtype, cap, s, [&](void *buf, size_t elems, size_t message) {
            RingConfig c = cfg;
            c.order_bytes = message;
            ex_[r]->allreduce(buf, buf, elems, dtype, s, c);
        });
    });
    return pipes_[0]->subplans();
}

LocalWorld::LocalWorld(int nranks, int device, ncclComm_t loopback) : P_(nranks) {
    for (int r = 0; r < nranks; ++r) res_.emplace_back(new RankResources(device, config_compute_cu_mask()));
    progs_.resize(nranks);
    if (loopback) {
        loop_.reset(new RcclTransport(loopback));
        DDL_HIP(hipStreamCreateWithFlags(&loop_stream_, hipStreamNonBlocking));
        DDL_HIP(hipEventCreateWithFlags(&loop_join_, hipEventDisableTiming));
    }
}

LocalWorld::~LocalWorld() {
    for (hipEvent_t e : loop_ev_) (void)hipEventDestroy(e);
    if (loop_join_) (void)hipEventDestroy(loop_join_);
    if (loop_stream_) (void)hipStreamDestroy(loop_stream_);
}

const P2POp &LocalWorld::match_(int r, size_t t, const P2POp &op, std::map<std::pair<int, int>, int> &seen) const {
    int skip = seen[std::make_pair(op.peer, op.tag)]++;
    for (const P2POp &o : progs_[op.peer].ticks[t].ops)
        if (o.send && o.peer == r && o.tag == op.tag && skip-- == 0) {
            DDL_REQUIRE(o.bytes == op.bytes, DDL_STATUS_ERROR_UNKNOWN,
                        "local world: recv of " << op.bytes << " B matches a send of " << o.bytes << " B");
            return o;
        }
    fail(DDL_STATUS_ERROR_UNKNOWN, "local world: unmatched recv rank " + std::to_string(r) + " tick " +
                                       std::to_string(t) + " tag " + std::to_string(op.tag));
}

void LocalWorld::allreduce(const void *const *in, void *const *out, size_t n, int dtype,
                           hipStream_t user, const RingConfig &cfg) {
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    if (n == 0) return;
    if (P_ == 1) {
        if (in[0] != out[0]) DDL_HIP(hipMemcpyAsync(out[0], in[0], n * es, hipMemcpyDeviceToDevice, user));
        return;
    }
    const bool capture = stream_capturing(user);
    for (int r = 0; r < P_; ++r) {
        void *st = res_[r]->ensure_staging(program_staging_elems(n, es, P_, cfg) * es, capture);
        build_program(progs_[r], r, P_, in[r], out[r], st, n, dtype, cfg);
    }
    run_(dtype, user);
}

void LocalWorld::allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                                 hipStream_t user, const RingConfig &cfg) {
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    if (P_ == 1) {
        for (int b = 0; b < count; ++b)
            if (n[b] && in[b] != out[b]) DDL_HIP(hipMemcpyAsync(out[b], in[b], n[b] * es, hipMemcpyDeviceToDevice, user));
        return;
    }
    const bool capture = stream_capturing(user);
    const size_t elems = std::max<size_t>(1, batch_staging_elems(n, count, es, P_, cfg));
    for (int r = 0; r < P_; ++r) {
        void *st = res_[r]->ensure_staging(elems * es, capture);
        build_batch_program(progs_[r], r, P_, in + (size_t)r * count, out + (size_t)r * count, n, count, st, dtype, cfg);
    }
    run_(dtype, user);
}

void LocalWorld::broadcast(void *const *bufs, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg) {
    DDL_REQUIRE(dtype_size(dtype) != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    if (n == 0 || P_ == 1) return;
    for (int r = 0; r < P_; ++r) build_broadcast(progs_[r], r, P_, root, bufs[r], n, dtype, cfg);
    run_(dtype, user);
}

void LocalWorld::allgatherv(const void *const *sends, void *const *recvs, const size_t *counts, const size_t *displs,
                            int dtype, hipStream_t user) {
    DDL_REQUIRE(dtype_size(dtype) != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    for (int r = 0; r < P_; ++r) build_allgatherv(progs_[r], r, P_, sends[r], recvs[r], counts, displs, dtype);
    run_(dtype, user);
}

void LocalWorld::run_(int dtype, hipStream_t user) {
    const size_t T = progs_[0].ticks.size();
    if (T == 0) return;
    for (int r = 0; r < P_; ++r) {
        DDL_REQUIRE(progs_[r].ticks.size() == T, DDL_STATUS_ERROR_UNKNOWN, "local world: tick counts differ");
        res_[r]->ensure_events(T);
    }
    while (loop_ && loop_ev_.size() < T) {
        hipEvent_t e;
        DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        loop_ev_.push_back(e);
    }
    // posted through a Poster as RingExecutor::run_ is: real streams eagerly; inside a capture a
    // serial order (default) or a single-stream DAG (config capture_mode)
    Poster p(Poster::mode_for(user), user);
    auto comm = [&](int r) { return res_[r]->comm; };
    auto compute = [&](int r) { return res_[r]->compute; };
    auto record = [&](hipEvent_t e, hipStream_t st) { p.record(e, st); };
    auto wait = [&](hipStream_t st, hipEvent_t e) { p.wait(st, e); };
    auto copy = [&](void *dst, const void *src, size_t bytes, hipStream_t st) {
        DDL_TRACE("copy " << bytes << " B on " << (void *)st);
        const hipStream_t s = p.on(st);
        DDL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
        p.posted(st);
        if (dep::on()) dep::op(s, "local copy", {dep::rd(src, bytes), dep::wr(dst, bytes)});
    };
    DDL_TRACE("local world run: P " << P_ << " ticks " << T << " mode " << (int)p.mode() << " user " << (void *)user);
    hipEvent_t fork = res_[0]->fork_ev;
    record(fork, user);
    for (int r = 0; r < P_; ++r) {
        wait(comm(r), fork);
        wait(compute(r), fork);
    }
    if (loop_) wait(loop_stream_, fork);
    for (size_t t = 0; t < T; ++t) {
        // 1) each rank's comm stream reaches the tick (after its reduce dependency)
        for (int r = 0; r < P_; ++r) {
            const Tick &tk = progs_[r].ticks[t];
            RankResources &rr = *res_[r];
            if (tk.wait_reduce >= 0) {
                int w = last_reduce_at_or_before(progs_[r], tk.wait_reduce);
                if (w >= 0) wait(comm(r), rr.red_ev[w]);
            }
            for (const CopyOp &c : tk.copies) copy(c.dst, c.src, c.bytes, comm(r));
            record(rr.pre_ev[t], comm(r));
        }
        // 1b) allgather ticks: rank q's block into every rank's recv at q * bytes, once q has
        //     reached the tick (copies, or self pairs through RCCL on the loopback)
        if (progs_[0].ticks[t].gather.bytes) {
            std::vector<P2POp> pairs;
            for (int r = 0; r < P_; ++r) {
                const GatherOp &g = progs_[r].ticks[t].gather;
                for (int q = 0; q < P_; ++q) {
                    const GatherOp &src = progs_[q].ticks[t].gather;
                    DDL_REQUIRE(src.bytes == g.bytes, DDL_STATUS_ERROR_UNKNOWN, "local world: allgather sizes differ");
                    char *dst = static_cast<char *>(g.recv) + (size_t)q * g.bytes;
                    if (dst == src.send) continue;  // in place: rank q's own block
                    if (loop_) {
                        pairs.push_back(P2POp{true, 0, 0, const_cast<void *>(src.send), g.bytes});
                        pairs.push_back(P2POp{false, 0, 0, dst, g.bytes});
                    } else {
                        wait(comm(r), res_[q]->pre_ev[t]);
                        copy(dst, src.send, g.bytes, comm(r));
                    }
                }
            }
            if (loop_) {
                for (int r = 0; r < P_; ++r) wait(loop_stream_, res_[r]->pre_ev[t]);
                loop_->group(pairs, p.on(loop_stream_));
                p.posted(loop_stream_);
                record(loop_ev_[t], loop_stream_);
                for (int r = 0; r < P_; ++r) wait(comm(r), loop_ev_[t]);
                loop_pairs_ += (long long)pairs.size() / 2;
            } else {
                // every rank's block is read by the others: none may run ahead and overwrite
                for (int r = 0; r < P_; ++r) record(res_[r]->pre_ev[t], comm(r));
                for (int r = 0; r < P_; ++r)
                    for (int q = 0; q < P_; ++q) wait(comm(r), res_[q]->pre_ev[t]);
            }
        }
        if (loop_) {
            // 2') every matched pair of the tick through RCCL as a self send / self recv, posted
            //     in matching order in one group on the transport stream, which waits for every
            //     rank to reach the tick; every rank's comm stream then waits for the group
            std::vector<P2POp> pairs;
            for (int r = 0; r < P_; ++r) {
                std::map<std::pair<int, int>, int> seen;
                for (const P2POp &op : progs_[r].ticks[t].ops) {
                    if (op.send) continue;
                    const P2POp &s = match_(r, t, op, seen);
                    pairs.push_back(P2POp{true, 0, op.tag, s.ptr, s.bytes});
                    pairs.push_back(P2POp{false, 0, op.tag, op.ptr, op.bytes});
                }
            }
            if (!pairs.empty()) {
                for (int r = 0; r < P_; ++r) wait(loop_stream_, res_[r]->pre_ev[t]);
                loop_->group(pairs, p.on(loop_stream_));
                p.posted(loop_stream_);
                record(loop_ev_[t], loop_stream_);
                for (int r = 0; r < P_; ++r) wait(comm(r), loop_ev_[t]);
                loop_pairs_ += (long long)pairs.size() / 2;
            }
        } else {
            // 2) receives: copy from the matching send of the peer, once the peer reached the tick
            //    (the k-th recv from a peer with a tag matches the k-th send to us with that tag,
            //    as RCCL matches p2p operations between a pair in posting order)
            for (int r = 0; r < P_; ++r) {
                RankResources &rr = *res_[r];
                std::map<std::pair<int, int>, int> seen;
                for (const P2POp &op : progs_[r].ticks[t].ops) {
                    if (op.send) continue;
                    const P2POp &match = match_(r, t, op, seen);
                    wait(comm(r), res_[op.peer]->pre_ev[t]);
                    DDL_TRACE("recv copy " << op.bytes << " B on " << (void *)comm(r));
                    const hipStream_t s = p.on(comm(r));
                    DDL_HIP(hipMemcpyAsync(op.ptr, match.ptr, op.bytes, hipMemcpyDeviceToDevice, s));
                    p.posted(comm(r));
                    if (dep::on())
                        dep::op(s, dep_label("local recv", r, t), {dep::rd(match.ptr, op.bytes), dep::wr(op.ptr, op.bytes)});
                }
                record(rr.post_ev[t], comm(r));
            }
            // 3) a group completes for the sender only once its receivers have the data
            for (int r = 0; r < P_; ++r) {
                for (const P2POp &op : progs_[r].ticks[t].ops)
                    if (op.send) wait(comm(r), res_[op.peer]->post_ev[t]);
            }
        }
        // 4) reduce of the received slices
        for (int r = 0; r < P_; ++r) {
            const Tick &tk = progs_[r].ticks[t];
            RankResources &rr = *res_[r];
            if (!tk.has_reduce) continue;
            record(rr.comm_ev[t], comm(r));
            wait(compute(r), rr.comm_ev[t]);
            DDL_TRACE("reduce launch on " << (void *)compute(r));
            const hipStream_t cs = p.on(compute(r));
            launch_tick_reduce(tk, dtype, cs);
            p.posted(compute(r));
            if (dep::on()) dep::op(cs, dep_label(tk.multi ? "fold" : "reduce", r, t), tick_reduce_access(tk, dtype));
            record(rr.red_ev[t], compute(r));
        }
    }
    for (int r = 0; r < P_; ++r) {
        record(res_[r]->join_ev, comm(r));
        record(res_[r]->join_cp_ev, compute(r));
        wait(user, res_[r]->join_ev);
        wait(user, res_[r]->join_cp_ev);
    }
    if (loop_) {  // the transport stream too (its groups are joined through the comm streams already)
        record(loop_join_, loop_stream_);
        wait(user, loop_join_);
    }
    p.finish();
}

RcclLoopback &rccl_loopback() {
    static RcclLoopback *l = new RcclLoopback();  // leaked: no static-destruction order issues
    return *l;
}

LocalWorld &RcclLoopback::world(int nranks) {
    DDL_REQUIRE(comm != nullptr, DDL_STATUS_NOT_INITIALIZED, "ddl_rccl_loopback_init has not been called");
    int dev = 0;
    DDL_HIP(hipGetDevice(&dev));
    auto key = std::make_pair(nranks, comm);
    auto it = worlds.find(key);
    if (it == worlds.end()) it = worlds.emplace(key, std::unique_ptr<LocalWorld>(new LocalWorld(nranks, dev, comm))).first;
    return *it->second;
}

LocalWorld &local_world(int nranks) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::unique_ptr<LocalWorld>> worlds;
    int dev = 0;
    DDL_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(mu);
    auto key = std::make_pair(nranks, dev);
    auto it = worlds.find(key);
    if (it == worlds.end()) it = worlds.emplace(key, std::unique_ptr<LocalWorld>(new LocalWorld(nranks, dev))).first;
    return *it->second;
}

}  // namespace ddl
