// executor.cpp — see executor.h.
#include "executor.h"

#include "engine.h"

#include "deptrace.h"

#include <algorithm>
#include <map>
#include <thread>

namespace ddl {

namespace {
std::atomic<int> g_drop_wait_tick{-1};
}
void set_testing_drop_wait(int tick) { g_drop_wait_tick = tick; }

bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

namespace dep {
std::atomic<Sink *> g_sink{nullptr};
}

void Transport::host_group(std::vector<ddl_p2p_op> &) {
    fail(DDL_STATUS_ERROR_UNKNOWN, "host groups need the test transport");
}

void RcclTransport::group(const std::vector<P2POp> &ops, hipStream_t stream) {
    if (ops.empty()) return;
    const RcclApi &api = rccl();
    rccl_check(api.GroupStart(), "ncclGroupStart");
    ncclResult_t first_err = ncclSuccess;
    for (const P2POp &op : ops) {
        ncclResult_t r = op.send ? api.Send(op.ptr, op.bytes, ncclInt8, op.peer, comm_, stream)
                                 : api.Recv(op.ptr, op.bytes, ncclInt8, op.peer, comm_, stream);
        if (r != ncclSuccess && first_err == ncclSuccess) first_err = r;
    }
    ncclResult_t e = api.GroupEnd();
    rccl_check(first_err, "ncclSend/ncclRecv");
    rccl_check(e, "ncclGroupEnd");
    if (dep::on()) {
        std::vector<dep::Access> acc;
        for (const P2POp &op : ops) acc.push_back(op.send ? dep::rd(op.ptr, op.bytes) : dep::wr(op.ptr, op.bytes));
        dep::op(stream, "rccl group", std::move(acc));
    }
}

void RcclTransport::allgather(const GatherOp &g, hipStream_t stream) {
    rccl_check(rccl().AllGather(g.send, g.recv, g.bytes, ncclInt8, comm_, stream), "ncclAllGather");
    // (the other ranks' blocks are written too; their extent is the communicator's size)
    if (dep::on()) dep::op(stream, "rccl allgather", {dep::rd(g.send, g.bytes), dep::wr(g.recv, g.bytes)});
}

hipStream_t create_engine_stream(QueueClass qc, int cu_mask_every) {
    if (cu_mask_every >= 2 || qc == QueueClass::kPooled) {
        // a CU-masked stream already has a hardware queue of its own
        return create_compute_stream(cu_mask_every);
    }
    int least = 0, greatest = 0;
    DDL_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s = nullptr;
    DDL_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, qc == QueueClass::kHigh ? greatest : least));
    return s;
}

hipStream_t create_compute_stream(int every) {
    hipStream_t s = nullptr;
    int ncu = device_cu_count();
    if (every >= 2 && ncu > 0) {
        // CU c off when c % every == every - 1: the reduce / fold kernels keep their full HBM rate
        // on such masks (tools/cu_mask_probe.py: every 8th, 4th or 2nd CU off, 6.56-6.59 TB/s vs
        // 6.59 on all 256) and leave the masked-off CUs free for RCCL's send / recv kernels
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu; ++c)
            if (c % every != every - 1) mask[(size_t)c / 32] |= 1u << (c % 32);
        // (hipExtStreamCreateWithCUMask takes no flags: the masked stream is a blocking one, ordered
        // with the legacy NULL stream, where the unmasked one below is non-blocking)
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return s;
        (void)hipGetLastError();  // a runtime without CU masks: an ordinary stream
        DDL_LOG(1, "compute_cu_mask " << every << ": hipExtStreamCreateWithCUMask failed, using an unmasked stream");
    }
    DDL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

RankResources::RankResources(int dev, int cu_mask_every, QueueClass qc) : device(dev) {
    comm = create_engine_stream(qc);
    compute = create_engine_stream(qc, cu_mask_every);
    DDL_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    DDL_HIP(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
    DDL_HIP(hipEventCreateWithFlags(&join_cp_ev, hipEventDisableTiming));
}

RankResources::~RankResources() {
    // best effort: called at teardown, errors are ignored
    for (auto *v : {&comm_ev, &red_ev, &pre_ev, &post_ev})
        for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (join_ev) (void)hipEventDestroy(join_ev);
    if (join_cp_ev) (void)hipEventDestroy(join_cp_ev);
    if (comm) (void)hipStreamDestroy(comm);
    if (compute) (void)hipStreamDestroy(compute);
    if (staging_) (void)hipFree(staging_);
    for (void *p : retired_) (void)hipFree(p);
}

void RankResources::ensure_events(size_t ticks) {
    for (auto *v : {&comm_ev, &red_ev, &pre_ev, &post_ev}) {
        while (v->size() < ticks) {
            hipEvent_t e;
            DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            v->push_back(e);
        }
    }
}

void *RankResources::ensure_staging(size_t bytes, bool capturing) {
    if (bytes > staging_bytes_) {
        DDL_REQUIRE(!capturing, DDL_STATUS_INVALID_ARGUMENT,
                    "the staging buffer would grow (to " << bytes << " B) inside a stream capture: run this "
                    "collective once before capturing it");
        if (staging_ && staging_captured_) {
            // a captured graph may replay with this address at any time: keep it allocated
            retired_.push_back(staging_);
            staging_ = nullptr;
            staging_captured_ = false;
        } else if (staging_) {
            // a previous call may still read it on the device; and hipFree would synchronise the
            // whole device, which can deadlock against other communicators' RCCL kernels: kept
            // until ddl_finalize (retire_device)
            retire_device(staging_);
            staging_ = nullptr;
        }
        size_t sz = bytes + bytes / 4;  // grow with headroom (the reference grows x1.5, MPIRTC.cc:13)
        DDL_HIP(hipMalloc(&staging_, sz));
        staging_bytes_ = sz;
    }
    if (capturing) staging_captured_ = true;
    return staging_;
}

double launch_tick_reduce(const Tick &tk, int dtype, hipStream_t stream) {
    const double es = (double)dtype_size(dtype);
    if (tk.multi) {
        // fold steps in order on the compute stream; consecutive independent steps of one shape
        // (a grouped allreduce's buckets) share a launch, kMaxFoldBatch at a time
        double bytes = 0;
        std::vector<SegTableN> batch;
        auto flush = [&] {
            if (!batch.empty()) launch_sumN_batch(batch.data(), (int)batch.size(), dtype, stream);
            batch.clear();
        };
        auto meets = [es](const void *p, uint64_t pn, const void *q, uint64_t qn) {
            const uintptr_t a = (uintptr_t)p, b = (uintptr_t)q;
            return a < b + qn * es && b < a + pn * es;
        };
        for (const SegTableN &f : tk.folds) {
            bool joins = !batch.empty() && (int)batch.size() < kMaxFoldBatch && f.nb == batch[0].nb &&
                         f.order == batch[0].order;
            for (size_t i = 0; joins && i < batch.size(); ++i) {  // no step reads or writes another's output
                const SegTableN &g = batch[i];
                joins = !meets(f.out, f.n, g.out, g.n) && !meets(f.a, f.n, g.out, g.n) && !meets(g.a, g.n, f.out, f.n);
                for (int k = 0; joins && k < f.nb; ++k) joins = !meets(f.b[k], f.n, g.out, g.n);
                for (int k = 0; joins && k < g.nb; ++k) joins = !meets(g.b[k], g.n, f.out, f.n);
            }
            if (!joins) flush();
            batch.push_back(f);
            bytes += (f.nb + 2.0) * (double)f.n * es;
        }
        flush();
        return bytes;
    }
    launch_sum2(tk.reduce, dtype, stream, ring_variant());
    double elems = 0;
    for (int s = 0; s < tk.reduce.count; ++s) elems += (double)tk.reduce.n[s];
    return 3.0 * elems * es;
}

std::vector<dep::Access> tick_reduce_access(const Tick &tk, int dtype) {
    const size_t es = dtype_size(dtype);
    std::vector<dep::Access> acc;
    if (tk.multi) {
        for (const SegTableN &f : tk.folds) {
            acc.push_back(dep::rd(f.a, f.n * es));
            for (int i = 0; i < f.nb; ++i) acc.push_back(dep::rd(f.b[i], f.n * es));
            acc.push_back(dep::wr(f.out, f.n * es));
        }
    } else {
        for (int s = 0; s < tk.reduce.count; ++s) {
            acc.push_back(dep::rd(tk.reduce.a[s], tk.reduce.n[s] * es));
            acc.push_back(dep::rd(tk.reduce.b[s], tk.reduce.n[s] * es));
            acc.push_back(dep::wr(tk.reduce.out[s], tk.reduce.n[s] * es));
        }
    }
    return acc;
}

std::string dep_label(const char *what, int rank, size_t tick) {
    std::ostringstream os;
    os << what << " rank " << rank << " tick " << tick;
    return os.str();
}

int last_reduce_at_or_before(const RingProgram &p, int w) {
    for (int t = w; t >= 0; --t)
        if (p.ticks[t].has_reduce) return t;
    return -1;
}

RingExecutor::RingExecutor(int rank, int size, int device, std::unique_ptr<Transport> transport, QueueClass qc)
    : rank_(rank), size_(size), transport_(std::move(transport)),
      res_(device, size > 1 ? config_compute_cu_mask() : 0, qc) {}

RingExecutor::~RingExecutor() {
    for (auto *v : {&timed_, &free_pairs_})
        for (auto &p : *v) {
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
}

void RingExecutor::set_timing(bool on) { timing_ = on; }

KernelStats RingExecutor::collect_stats() {
    KernelStats s;
    for (size_t i = 0; i < timed_.size(); ++i) {
        DDL_HIP(hipEventSynchronize(timed_[i].second));
        float ms = 0;
        DDL_HIP(hipEventElapsedTime(&ms, timed_[i].first, timed_[i].second));
        s.ms += ms;
        s.bytes += timed_bytes_[i];
        s.launches += 1;
        free_pairs_.push_back(timed_[i]);
    }
    timed_.clear();
    timed_bytes_.clear();
    return s;
}

void RingExecutor::allreduce(const void *in, void *out, size_t n, int dtype, hipStream_t user,
                             const RingConfig &cfg) {
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    if (n == 0) return;
    if (size_ == 1) {  // P = 1: out = in (the reference never completes here)
        if (in != out) DDL_HIP(hipMemcpyAsync(out, in, n * es, hipMemcpyDeviceToDevice, user));
        return;
    }
    void *staging = res_.ensure_staging(program_staging_elems(n, es, size_, cfg) * es, stream_capturing(user));
    build_program(prog_, rank_, size_, in, out, staging, n, dtype, cfg);
    run_(dtype, user);
}

void RingExecutor::allreduce_batch(const void *const *in, void *const *out, const size_t *n, int count, int dtype,
                                   hipStream_t user, const RingConfig &cfg) {
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    if (size_ == 1) {
        for (int b = 0; b < count; ++b)
            if (n[b] && in[b] != out[b]) DDL_HIP(hipMemcpyAsync(out[b], in[b], n[b] * es, hipMemcpyDeviceToDevice, user));
        return;
    }
    void *staging = res_.ensure_staging(std::max<size_t>(1, batch_staging_elems(n, count, es, size_, cfg)) * es,
                                        stream_capturing(user));
    build_batch_program(prog_, rank_, size_, in, out, n, count, staging, dtype, cfg);
    run_(dtype, user);
}

void RingExecutor::broadcast(void *buf, size_t n, int dtype, int root, hipStream_t user, const RingConfig &cfg) {
    DDL_REQUIRE(dtype_size(dtype) != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    DDL_REQUIRE(root >= 0 && root < size_, DDL_STATUS_INVALID_ARGUMENT, "root " << root << " outside [0, " << size_ << ")");
    if (n == 0 || size_ == 1) return;
    build_broadcast(prog_, rank_, size_, root, buf, n, dtype, cfg);
    run_(dtype, user);
}

void RingExecutor::allgatherv(const void *send, void *recv, const size_t *counts, const size_t *displs, int dtype,
                              hipStream_t user) {
    DDL_REQUIRE(dtype_size(dtype) != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
    build_allgatherv(prog_, rank_, size_, send, recv, counts, displs, dtype);
    run_(dtype, user);
}

Poster::Mode Poster::mode_for(hipStream_t user) {
    if (!stream_capturing(user)) return kStreams;
    const int m = config_capture_mode();
    return m == 0 ? kSerial : kDag;
}

Poster::Poster(Mode m, hipStream_t user) : m_(m), user_(user) {
    if (m_ != kDag) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t *deps = nullptr;
    size_t nd = 0;
    DDL_HIP(hipStreamGetCaptureInfo_v2(user_, &cs, &id, &g, &deps, &nd));
    DDL_REQUIRE(cs == hipStreamCaptureStatusActive, DDL_STATUS_ERROR_UNKNOWN, "DAG posting outside a capture");
    tail_[user_].assign(deps, deps + nd);
}

hipStream_t Poster::on(hipStream_t s) {
    if (m_ == kStreams) return s;
    if (m_ == kSerial) return user_;
    std::vector<hipGraphNode_t> &t = tail_[s];
    DDL_HIP(hipStreamUpdateCaptureDependencies(user_, t.empty() ? nullptr : t.data(), t.size(),
                                               hipStreamSetCaptureDependencies));
    return user_;
}

void Poster::posted(hipStream_t s) {
    if (m_ != kDag) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t *deps = nullptr;
    size_t nd = 0;
    DDL_HIP(hipStreamGetCaptureInfo_v2(user_, &cs, &id, &g, &deps, &nd));
    tail_[s].assign(deps, deps + nd);
}

void Poster::record(hipEvent_t e, hipStream_t s) {
    DDL_TRACE("record ev " << (void *)e << " on " << (void *)s);
    if (m_ == kStreams) {
        DDL_HIP(hipEventRecord(e, s));
        dep::record(e, s);
    } else if (m_ == kDag) {
        ev_[e] = tail_[s];
    }
}

void Poster::wait(hipStream_t s, hipEvent_t e) {
    DDL_TRACE("wait " << (void *)s << " on ev " << (void *)e);
    if (m_ == kStreams) {
        DDL_HIP(hipStreamWaitEvent(s, e, 0));
        dep::wait(s, e);
    } else if (m_ == kDag) {
        std::vector<hipGraphNode_t> &t = tail_[s];
        for (hipGraphNode_t n : ev_[e])
            if (std::find(t.begin(), t.end(), n) == t.end()) t.push_back(n);
    }
}

void Poster::finish() {
    if (m_ != kDag) return;
    std::vector<hipGraphNode_t> &t = tail_[user_];
    DDL_HIP(hipStreamUpdateCaptureDependencies(user_, t.empty() ? nullptr : t.data(), t.size(),
                                               hipStreamSetCaptureDependencies));
}

void RingExecutor::run_(int dtype, hipStream_t user) {
    if (prog_.ticks.empty()) return;
    DDL_TRACE("executor rank " << rank_ << "/" << size_ << " run: " << prog_.ticks.size() << " ticks, user " << (void *)user);
    // Eagerly the program forks from the caller's stream onto the comm / compute streams and joins
    // back. Inside a graph capture the Poster turns the same posting into a serial order on the
    // captured stream (default) or a single-stream DAG (config capture_mode; executor.h,
    // DESIGN §9).
    const bool capturing = stream_capturing(user);
    DDL_REQUIRE(!capturing || !transport_ || transport_->capturable(), DDL_STATUS_INVALID_ARGUMENT,
                "this communicator's transport synchronises the host and cannot be captured into a graph");
    Poster p(Poster::mode_for(user), user);
    const bool timing = timing_ && !capturing;
    const hipStream_t comm = res_.comm, compute = res_.compute;
    res_.ensure_events(prog_.ticks.size());
    p.record(res_.fork_ev, user);
    p.wait(comm, res_.fork_ev);
    p.wait(compute, res_.fork_ev);
    const int drop = g_drop_wait_tick.load();
    for (size_t t = 0; t < prog_.ticks.size(); ++t) {
        const Tick &tk = prog_.ticks[t];
        if (tk.wait_reduce >= 0 && (int)t != drop) {
            int w = last_reduce_at_or_before(prog_, tk.wait_reduce);
            if (w >= 0) p.wait(comm, res_.red_ev[w]);
        }
        for (const CopyOp &c : tk.copies) {
            const hipStream_t s = p.on(comm);
            DDL_HIP(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToDevice, s));
            p.posted(comm);
            if (dep::on()) dep::op(s, dep_label("copy", rank_, t), {dep::rd(c.src, c.bytes), dep::wr(c.dst, c.bytes)});
        }
        if (transport_) {
            if (tk.gather.bytes) {
                transport_->allgather(tk.gather, p.on(comm));
                p.posted(comm);
            }
            if (!tk.ops.empty()) {
                transport_->group(tk.ops, p.on(comm));
                p.posted(comm);
            }
        } else {
            DDL_REQUIRE(tk.ops.empty() && !tk.gather.bytes, DDL_STATUS_ERROR_UNKNOWN, "no transport for a multi-rank program");
        }
        if (tk.has_reduce) {
            p.record(res_.comm_ev[t], comm);
            p.wait(compute, res_.comm_ev[t]);
            std::pair<hipEvent_t, hipEvent_t> tp{nullptr, nullptr};
            if (timing) {
                if (free_pairs_.empty()) {
                    DDL_HIP(hipEventCreate(&tp.first));
                    DDL_HIP(hipEventCreate(&tp.second));
                } else {
                    tp = free_pairs_.back();
                    free_pairs_.pop_back();
                }
                DDL_HIP(hipEventRecord(tp.first, compute));
            }
            const hipStream_t cs = p.on(compute);
            const double bytes = launch_tick_reduce(tk, dtype, cs);
            p.posted(compute);
            if (dep::on()) dep::op(cs, dep_label(tk.multi ? "fold" : "reduce", rank_, t), tick_reduce_access(tk, dtype));
            if (timing) {
                DDL_HIP(hipEventRecord(tp.second, compute));
                timed_.push_back(tp);
                timed_bytes_.push_back(bytes);
            }
            p.record(res_.red_ev[t], compute);
        }
    }
    // join both forked streams back into the caller's: every stream a capture forked must be
    // joined before it ends (the compute stream of a program with no reduce — broadcast,
    // allgatherv — only waited on the fork)
    p.record(res_.join_ev, comm);
    p.record(res_.join_cp_ev, compute);
    p.wait(user, res_.join_ev);
    p.wait(user, res_.join_cp_ev);
    p.finish();
}

}  // namespace ddl
