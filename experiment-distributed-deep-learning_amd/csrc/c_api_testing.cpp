// c_api_testing.cpp — the test / measurement C-ABI (include/ddl_amd_testing.h), linked into
// libddl_amd_testing.so only, beside the same engine objects and the deployment surface
// (c_api.cpp): the host-callback test transport, handle-based control channels, raw kernels,
// the virtual-rank worlds (device copies, RCCL loopback, threads), mutation knobs, the
// happens-before recorder and schedule introspection.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "abi.h"
#include "handler.h"
#include "test_worlds.h"

using namespace ddl;
using namespace ddl::abi;

namespace {

// ddl_pack / ddl_unpack share one copier (its table slots are not thread-safe).
std::mutex &abi_copier_mu() {
    static std::mutex mu;
    return mu;
}
SegmentCopier &abi_copier() {
    static SegmentCopier *c = new SegmentCopier();  // leaked: no destruction-order issues at exit
    return *c;
}

std::mutex &channels_mu() {
    static std::mutex mu;
    return mu;
}
std::map<long long, std::shared_ptr<ControlChannel>> &channels() {
    static auto *m = new std::map<long long, std::shared_ptr<ControlChannel>>();
    return *m;
}
std::shared_ptr<ControlChannel> channel(long long h) {
    std::lock_guard<std::mutex> g(channels_mu());
    auto it = channels().find(h);
    DDL_REQUIRE(it != channels().end(), DDL_STATUS_INVALID_ARGUMENT, "unknown control channel " << h);
    return it->second;
}

// One negotiation round with a fixed key set ('\n'-separated) over `ch`: the agreed keys,
// '\n'-separated and lexicographic, into out (the handler's protocol without the data plane).
void negotiate_keys(ControlChannel &ch, const char *keys, char *out, size_t len) {
    DDL_REQUIRE(keys && out && len > 0, DDL_STATUS_INVALID_ARGUMENT, "bad negotiate args");
    DDL_REQUIRE(ch.connected(), DDL_STATUS_NOT_INITIALIZED, "control channel not connected");
    std::vector<std::string> mine;
    std::string s(keys);
    size_t pos = 0;
    while (pos < s.size()) {
        size_t nl = s.find('\n', pos);
        if (nl == std::string::npos) nl = s.size();
        if (nl > pos) mine.push_back(std::string(request_type_name(kReqAllreduce)) + "::" + s.substr(pos, nl - pos));
        pos = nl + 1;
    }
    std::sort(mine.begin(), mine.end());
    mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
    // this rank's ids by table index, as the handler keeps them
    std::vector<uint8_t> held(ch.cache.size(), 0);
    std::vector<uint32_t> idx;
    bool cached = !mine.empty();
    for (const auto &k : mine) {
        uint32_t i;
        if (ch.cache.lookup(k, &i)) {
            held[i] = 1;
            idx.push_back(i);
        } else {
            cached = false;
        }
    }
    Agreed a;
    if (ch.rank() == 0) {
        a = negotiate_root(ch, cached, idx, mine);
        negotiate_root_finish(ch);
    } else {
        Token t;
        ch.recv(t, -1);
        a = negotiate_member(
            ch, t,
            [&](const std::vector<std::string> &proposed) {
                std::vector<std::string> both;
                for (const auto &k : proposed)
                    if (std::binary_search(mine.begin(), mine.end(), k)) both.push_back(k);
                return both;
            },
            [&](const std::vector<uint32_t> &proposed) {
                std::vector<uint32_t> both;
                for (uint32_t i : proposed)
                    if (i < held.size() && held[i]) both.push_back(i);
                return both;
            });
    }
    std::vector<std::string> agreed;
    if (a.cached) {
        for (uint32_t i : a.idx) agreed.push_back(ch.cache.at(i));
        std::sort(agreed.begin(), agreed.end());
    } else {
        agreed = a.wire;
        ch.cache.learn(agreed);
    }
    DDL_REQUIRE(a.cfg_ok, DDL_STATUS_CONFIG_MISMATCH,
                "negotiation refused: the ranks' shared tunables differ (config hash here " << std::hex
                                                                                           << config().shared_hash() << ")");
    std::string res;
    for (const auto &k : agreed) res.append(k.substr(k.find("::") + 2)).append("\n");
    DDL_REQUIRE(res.size() < len, DDL_STATUS_INVALID_ARGUMENT, "output buffer too small");
    std::memcpy(out, res.c_str(), res.size() + 1);
}

// One thread world per (ranks, device, compute_cu_mask): its executors' compute streams are
// created with the mask in force when the world is.
// ddl_testing_thread_transport: 0 = device copies, 1 = RCCL loopback (the thread worlds made while
// it is 1 move their bytes through the RCCL loopback communicator)
std::atomic<int> g_thread_rccl{0};
std::mutex g_thread_mu;
std::map<std::tuple<int, int, int, ncclComm_t>, std::unique_ptr<ThreadWorld>> *g_thread_worlds =
    new std::map<std::tuple<int, int, int, ncclComm_t>, std::unique_ptr<ThreadWorld>>();

// Lock order: the loopback's mutex, then g_thread_mu — as ddl_rccl_loopback_finalize takes them — so
// the loopback communicator cannot be destroyed between reading it and building the world on it
// (ADVICE r4). A world returned here is used after the locks are released: finalize must not run
// concurrently with thread-transport calls (the tests call it between them).
ThreadWorld &thread_world(int nranks) {
    int dev = current_device();
    ncclComm_t loop = nullptr;
    std::unique_lock<std::mutex> lg;
    if (g_thread_rccl.load()) {
        RcclLoopback &l = rccl_loopback();
        lg = std::unique_lock<std::mutex>(l.mu);
        DDL_REQUIRE(l.comm, DDL_STATUS_NOT_INITIALIZED, "thread transport 1 needs ddl_rccl_loopback_init first");
        loop = l.comm;
    }
    std::lock_guard<std::mutex> g(g_thread_mu);
    auto key = std::make_tuple(nranks, dev, config_compute_cu_mask(), loop);
    auto it = g_thread_worlds->find(key);
    if (it == g_thread_worlds->end())
        it = g_thread_worlds->emplace(key, std::unique_ptr<ThreadWorld>(new ThreadWorld(nranks, dev, loop))).first;
    return *it->second;
}

void testing_finalize() {
    std::lock_guard<std::mutex> g(channels_mu());
    channels().clear();
}

struct RegisterFinalize {
    RegisterFinalize() { add_finalize_hook(&testing_finalize); }
} g_register_finalize;

}  // namespace

extern "C" {

int ddl_init_test_transport(int rank, int size, int device, ddl_test_group_fn group, ddl_test_max_fn max,
                            void *user) {
    return guarded([&] {
        DDL_REQUIRE(size >= 1 && rank >= 0 && rank < size && group, DDL_STATUS_INVALID_ARGUMENT,
                    "bad test transport arguments");
        const char *allow = std::getenv("DDL_ALLOW_TEST_TRANSPORT");
        DDL_REQUIRE(allow && std::string(allow) == "1", DDL_STATUS_INVALID_ARGUMENT,
                    "ddl_init_test_transport is a test harness (host-synchronised groups, no RCCL): set "
                    "DDL_ALLOW_TEST_TRANSPORT=1 to use it; deployments call ddl_init");
        DDL_REQUIRE(!Registry::get().initialized(), DDL_STATUS_INVALID_ARGUMENT, "already initialized");
        DDL_HIP(hipSetDevice(device));
        auto hooks = std::make_shared<TestHooks>();
        hooks->group = group;
        hooks->max = max;
        hooks->user = user;
        hooks->make_transport = &make_callback_transport;
        Registry::get().set_world(new_communicator(rank, size, device, nullptr, hooks, 0));
        DDL_LOG(1, "initialized rank " << rank << "/" << size << " on device " << device << " (test transport)");
    });
}

int ddl_control_connect_ranked(int rank, int size, const char *endpoints) {
    return guarded([&] {
        DDL_REQUIRE(endpoints, DDL_STATUS_INVALID_ARGUMENT, "null endpoints");
        standalone_control()->connect(rank, size, split_endpoints(endpoints), 120000);
    });
}

int ddl_control_negotiate(const char *keys, char *out, size_t len) {
    return guarded([&] { negotiate_keys(*standalone_control(), keys, out, len); });
}

// ---- handle-based control channels (several token rings in one process: tools, CPU tests) ----
long long ddl_control_channel_open(char *endpoint_out, size_t len) {
    long long h = 0;
    int st = guarded([&] {
        auto ch = std::make_shared<ControlChannel>();
        std::string ep = ch->listen();
        DDL_REQUIRE(endpoint_out && len > ep.size(), DDL_STATUS_INVALID_ARGUMENT, "endpoint buffer too small");
        std::memcpy(endpoint_out, ep.c_str(), ep.size() + 1);
        std::lock_guard<std::mutex> g(channels_mu());
        h = reinterpret_cast<long long>(ch.get());
        channels()[h] = ch;
    });
    return st == DDL_STATUS_OK ? h : 0;
}

int ddl_control_channel_connect(long long h, int rank, int size, const char *endpoints) {
    return guarded([&] {
        DDL_REQUIRE(endpoints, DDL_STATUS_INVALID_ARGUMENT, "null endpoints");
        channel(h)->connect(rank, size, split_endpoints(endpoints), 120000);
    });
}

int ddl_control_channel_negotiate(long long h, const char *keys, char *out, size_t len) {
    return guarded([&] { negotiate_keys(*channel(h), keys, out, len); });
}

int ddl_control_channel_close(long long h) {
    return guarded([&] {
        std::lock_guard<std::mutex> g(channels_mu());
        DDL_REQUIRE(channels().erase(h) == 1, DDL_STATUS_INVALID_ARGUMENT, "unknown control channel " << h);
    });
}

int ddl_allreduce_variant(ddl_communicator_id id, const void *send, void *recv, size_t elements, int dtype,
                          int op, void *hip_stream, int variant) {
    return guarded([&] {
        auto c = Registry::get().find(id);
        if (variant == 0) {
            c->allreduce(send, recv, elements, dtype, op, as_stream(hip_stream));
            return;
        }
        DDL_REQUIRE(variant == 1, DDL_STATUS_INVALID_ARGUMENT, "variant " << variant);
        DDL_REQUIRE(op == DDL_ALLREDUCE_OP_SUM, DDL_STATUS_INVALID_ARGUMENT, "only SUM");
        c->rccl_allreduce(send, recv, elements, dtype, as_stream(hip_stream));
    });
}

int ddl_testing_round_log(ddl_communicator_id id, long long *user_collectives, long long *releases, int max_releases,
                          int *count) {
    return guarded([&] {
        DDL_REQUIRE(user_collectives && count, DDL_STATUS_INVALID_ARGUMENT, "null output");
        auto c = Registry::get().find(id);
        *user_collectives = c->user_collectives();
        std::vector<long long> log = c->round_log();
        *count = (int)log.size();
        for (int i = 0; i < (int)log.size() && i < max_releases && releases; ++i) releases[i] = log[i];
    });
}

int ddl_testing_agree_config(int rank, int size, ddl_test_group_fn group, void *user) {
    return guarded([&] {
        DDL_REQUIRE(size >= 1 && rank >= 0 && rank < size && group, DDL_STATUS_INVALID_ARGUMENT,
                    "bad agreement arguments");
        std::vector<uint64_t> all(size, 0);
        all[rank] = config().shared_hash();
        std::vector<ddl_p2p_op> ops;
        for (int d = 1; d < size; ++d) {
            const int to = (rank + d) % size, from = (rank + size - d) % size;
            ops.push_back(ddl_p2p_op{1, to, 4002, &all[rank], sizeof(uint64_t)});
            ops.push_back(ddl_p2p_op{0, from, 4002, &all[from], sizeof(uint64_t)});
        }
        if (!ops.empty())
            DDL_REQUIRE(group(0, ops.data(), (int)ops.size(), user) == 0, DDL_STATUS_COMM_ERROR,
                        "agreement exchange failed");
        check_config_agreement(rank, all);
    });
}

int ddl_local_tune(int nranks, size_t elements, int dtype, void *hip_stream, int *chosen, int *count,
                   long long *configs, float *ms, int max_candidates) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 2 && nranks <= 16, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        const size_t es = dtype_size(dtype), bytes = elements * es;
        DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
        DDL_REQUIRE(elements > 0, DDL_STATUS_INVALID_ARGUMENT, "empty bucket");
        (void)current_device();
        hipStream_t stream = as_stream(hip_stream);
        std::vector<void *> bufs(2 * nranks, nullptr);
        auto release = [&] {
            (void)hipStreamSynchronize(stream);
            for (void *p : bufs)
                if (p) (void)hipFree(p);
        };
        TuneResult r;
        try {
            for (void *&p : bufs) {
                DDL_HIP(hipMalloc(&p, bytes));
                DDL_HIP(hipMemsetAsync(p, 0, bytes, stream));
            }
            LocalWorld &w = local_world(nranks);
            r = run_tuning(
                nranks, bytes, stream, config().ring(),
                [&](const RingConfig &c) { w.allreduce(bufs.data(), bufs.data() + nranks, elements, dtype, stream, c); },
                [](float *, int) {});
        } catch (...) {
            release();
            throw;
        }
        release();
        export_tune(r, chosen, count, configs, ms, max_candidates);
    });
}

// ---- kernels ------------------------------------------------------------------------------
int ddl_reduce_sum2_variant(int variant, void *out, const void *a, const void *b, size_t elements,
                            int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(variant >= -1 && variant <= (kVariantMask | kRunForm | kRun4), DDL_STATUS_INVALID_ARGUMENT, "variant " << variant);
        SegTable t;
        t.count = 1;
        t.a[0] = a;
        t.b[0] = b;
        t.out[0] = out;
        t.n[0] = elements;
        launch_sum2(t, dtype, as_stream(hip_stream), variant);
    });
}

int ddl_reduce_fold_ordered(void *out, const void *a, const void *const *ins, int nb, size_t elements, int dtype,
                            int order, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nb >= 1 && nb <= kMaxInputs && ins, DDL_STATUS_INVALID_ARGUMENT, "fold inputs " << nb);
        SegTableN t;
        t.a = a;
        t.out = out;
        t.n = elements;
        t.nb = nb;
        t.order = order;
        for (int i = 0; i < nb; ++i) t.b[i] = ins[i];
        launch_sumN(t, dtype, as_stream(hip_stream));
    });
}

int ddl_reduce_fold_batch(int count, void *const *outs, const void *const *as, const void *const *ins, int nb,
                          const size_t *elements, int dtype, int order, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(count >= 1 && count <= kMaxFoldBatch && outs && as && ins && elements, DDL_STATUS_INVALID_ARGUMENT,
                    "fold batch of " << count << " (1.." << kMaxFoldBatch << ")");
        DDL_REQUIRE(nb >= 1 && nb <= kMaxInputs, DDL_STATUS_INVALID_ARGUMENT, "fold inputs " << nb);
        std::vector<SegTableN> t(count);
        for (int p = 0; p < count; ++p) {
            t[p].a = as[p];
            t[p].out = outs[p];
            t[p].n = elements[p];
            t[p].nb = nb;
            t[p].order = order;
            for (int i = 0; i < nb; ++i) t[p].b[i] = ins[(size_t)p * nb + i];
        }
        launch_sumN_batch(t.data(), count, dtype, as_stream(hip_stream));
    });
}

int ddl_reduce_fold(void *out, const void *a, const void *const *ins, int nb, size_t elements, int dtype,
                    void *hip_stream) {
    return ddl_reduce_fold_ordered(out, a, ins, nb, elements, dtype, kFoldLeft, hip_stream);
}

int ddl_reduce_sum2(void *out, const void *a, const void *b, size_t elements, int dtype, void *hip_stream) {
    return ddl_reduce_sum2_variant(-1, out, a, b, elements, dtype, hip_stream);
}

int ddl_reduce_local(void *acc, const void *in, size_t elements, int dtype, void *hip_stream) {
    return ddl_reduce_sum2_variant(-1, acc, acc, in, elements, dtype, hip_stream);
}

int ddl_pack(void *dst, const void *const *srcs, const size_t *bytes, int count, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(count >= 0 && (count == 0 || (dst && srcs && bytes)), DDL_STATUS_INVALID_ARGUMENT, "bad pack args");
        std::lock_guard<std::mutex> g(abi_copier_mu());
        abi_copier().run(0, dst, const_cast<void *const *>(srcs), bytes, count, as_stream(hip_stream));
    });
}

int ddl_unpack(void *const *dsts, const void *src, const size_t *bytes, int count, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(count >= 0 && (count == 0 || (src && dsts && bytes)), DDL_STATUS_INVALID_ARGUMENT, "bad unpack args");
        std::lock_guard<std::mutex> g(abi_copier_mu());
        abi_copier().run(1, const_cast<void *>(src), dsts, bytes, count, as_stream(hip_stream));
    });
}

int ddl_local_ring_allreduce(int nranks, const void *const *sends, void *const *recvs, size_t elements,
                             int dtype, int op, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        DDL_REQUIRE(op == DDL_ALLREDUCE_OP_SUM, DDL_STATUS_INVALID_ARGUMENT, "only SUM");
        DDL_REQUIRE(sends && recvs, DDL_STATUS_INVALID_ARGUMENT, "null buffer arrays");
        (void)current_device();
        local_world(nranks).allreduce(sends, recvs, elements, dtype, as_stream(hip_stream), config().ring());
    });
}

int ddl_local_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                              const size_t *elements, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && count >= 0 && (count == 0 || (sends && recvs && elements)),
                    DDL_STATUS_INVALID_ARGUMENT, "bad local allreduce batch");
        (void)current_device();
        local_world(nranks).allreduce_batch(sends, recvs, elements, count, dtype, as_stream(hip_stream), config().ring());
    });
}

int ddl_local_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        DDL_REQUIRE(root >= 0 && root < nranks, DDL_STATUS_INVALID_ARGUMENT, "root " << root);
        DDL_REQUIRE(bufs, DDL_STATUS_INVALID_ARGUMENT, "null buffer array");
        (void)current_device();
        local_world(nranks).broadcast(bufs, elements, dtype, root, as_stream(hip_stream), config().ring());
    });
}

int ddl_local_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                         const size_t *displs, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        DDL_REQUIRE(sends && recvs && counts && displs, DDL_STATUS_INVALID_ARGUMENT, "null argument");
        (void)current_device();
        local_world(nranks).allgatherv(sends, recvs, counts, displs, dtype, as_stream(hip_stream));
    });
}

// ---- thread world: the production RingExecutor per rank, asynchronous transport --------------------
int ddl_testing_thread_allreduce(int nranks, const void *const *sends, void *const *recvs, size_t elements, int dtype,
                                 void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && sends && recvs, DDL_STATUS_INVALID_ARGUMENT, "bad thread allreduce");
        thread_world(nranks).allreduce(sends, recvs, elements, dtype, as_stream(hip_stream), config().ring());
    });
}

int ddl_testing_thread_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                                       const size_t *elements, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && count >= 0 && (count == 0 || (sends && recvs && elements)),
                    DDL_STATUS_INVALID_ARGUMENT, "bad thread allreduce batch");
        thread_world(nranks).allreduce_batch(sends, recvs, elements, count, dtype, as_stream(hip_stream),
                                             config().ring());
    });
}

int ddl_testing_thread_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype,
                                 void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && root >= 0 && root < nranks && bufs, DDL_STATUS_INVALID_ARGUMENT,
                    "bad thread broadcast");
        thread_world(nranks).broadcast(bufs, elements, dtype, root, as_stream(hip_stream), config().ring());
    });
}

int ddl_testing_thread_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                                  const size_t *displs, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && sends && recvs && counts && displs, DDL_STATUS_INVALID_ARGUMENT,
                    "bad thread allgatherv");
        thread_world(nranks).allgatherv(sends, recvs, counts, displs, dtype, as_stream(hip_stream));
    });
}

int ddl_testing_thread_fused_allreduce(int nranks, int count, const void *const *srcs, void *const *dsts,
                                       const size_t *bytes, int dtype, void *hip_stream, size_t *subplans) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && count >= 1 && srcs && dsts && bytes, DDL_STATUS_INVALID_ARGUMENT,
                    "bad thread fused allreduce");
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
        for (int i = 0; i < count; ++i)
            DDL_REQUIRE(bytes[i] % es == 0, DDL_STATUS_INVALID_ARGUMENT, "segment " << i << " is not whole elements");
        const size_t j = thread_world(nranks).fused_allreduce(srcs, dsts, bytes, count, dtype, as_stream(hip_stream),
                                                              config().ring(),
                                                              (size_t)config().fusion_pipeline_bytes.load());
        if (subplans) *subplans = j;
    });
}

int ddl_testing_thread_transport(int rccl, long long *loopback_pairs) {
    return guarded([&] {
        DDL_REQUIRE(rccl == 0 || rccl == 1, DDL_STATUS_INVALID_ARGUMENT, "thread transport " << rccl);
        if (loopback_pairs) {
            long long n = 0;
            std::lock_guard<std::mutex> g(g_thread_mu);
            for (auto &kv : *g_thread_worlds)
                if (std::get<3>(kv.first)) n += kv.second->loopback_pairs();
            *loopback_pairs = n;
        }
        g_thread_rccl = rccl;
    });
}

int ddl_testing_control_fault(int on) {
    return guarded([&] { set_testing_control_fault(on); });
}

int ddl_testing_host_coll_fault(long long chunk) {
    return guarded([&] { set_testing_host_coll_fault(chunk); });
}

int ddl_testing_fold_variant(int variant) {
    return guarded([&] {
        DDL_REQUIRE(variant == -1 || variant == 4 || variant == 5, DDL_STATUS_INVALID_ARGUMENT,
                    "fold variant " << variant << " (4, 5 or -1)");
        set_testing_fold_variant(variant);
    });
}

int ddl_testing_drop_wait(int tick) {
    return guarded([&] { set_testing_drop_wait(tick); });
}

int ddl_testing_dep_trace(int on) {
    return guarded([&] {
        if (on) dep::start();
        else dep::stop();
    });
}

int ddl_testing_dep_check(long long *counts, char *report, size_t len) {
    return guarded([&] {
        DDL_REQUIRE(counts, DDL_STATUS_INVALID_ARGUMENT, "null counts");
        const dep::Report r = dep::check();
        counts[0] = r.ops;
        counts[1] = r.conflicts;
        counts[2] = r.ordered;
        counts[3] = r.ordered_reduce;
        counts[4] = r.races;
        if (report && len) {
            const size_t k = std::min(len - 1, r.first.size());
            std::memcpy(report, r.first.data(), k);
            report[k] = 0;
        }
    });
}

int ddl_testing_compute_stream_cus(int every, int *enabled, int *total) {
    return guarded([&] {
        DDL_REQUIRE(enabled && total, DDL_STATUS_INVALID_ARGUMENT, "null output");
        RankResources rr(current_device(), every);
        const int ncu = device_cu_count();
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        DDL_HIP(hipExtStreamGetCUMask(rr.compute, (uint32_t)mask.size(), mask.data()));
        int on = 0;
        for (int c = 0; c < ncu; ++c) on += (mask[(size_t)c / 32] >> (c % 32)) & 1u;
        *enabled = on;
        *total = ncu;
    });
}

int ddl_testing_stream_priorities(ddl_communicator_id id, int *prio) {
    return guarded([&] {
        DDL_REQUIRE(prio, DDL_STATUS_INVALID_ARGUMENT, "null output");
        auto c = Registry::get().find(id);
        const RankResources &rr = c->executor().resources();
        DDL_HIP(hipStreamGetPriority(rr.comm, &prio[0]));
        DDL_HIP(hipStreamGetPriority(rr.compute, &prio[1]));
        prio[2] = prio[3] = DDL_TESTING_NO_STREAM;
        if (RequestHandler *h = c->handler_if_created()) DDL_HIP(hipStreamGetPriority(h->stream(), &prio[2]));
        if (auto kd = c->keyed_data()) DDL_HIP(hipStreamGetPriority(kd->executor().resources().comm, &prio[3]));
    });
}

int ddl_testing_host_chunk_cuts(size_t total_bytes, size_t chunk_bytes, size_t *cuts, size_t cap, size_t *count) {
    return guarded([&] {
        DDL_REQUIRE(count && (cuts || cap == 0), DDL_STATUS_INVALID_ARGUMENT, "null output");
        DDL_REQUIRE(chunk_bytes >= 256 && chunk_bytes % 256 == 0, DDL_STATUS_INVALID_ARGUMENT,
                    "chunk_bytes " << chunk_bytes << " is not a positive multiple of 256");
        const std::vector<size_t> cut = host_chunk_cuts(total_bytes, chunk_bytes);
        for (size_t i = 0; i < cut.size() && i < cap; ++i) cuts[i] = cut[i];
        *count = cut.size();
    });
}

// ---- RCCL loopback (one GPU, real RCCL transport) --------------------------------------------
int ddl_rccl_loopback_init(int device) {
    return guarded([&] {
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        DDL_REQUIRE(l.comm == nullptr, DDL_STATUS_INVALID_ARGUMENT, "RCCL loopback already initialized");
        DDL_HIP(hipSetDevice(device));
        char uid[sizeof(ncclUniqueId)];
        DDL_REQUIRE(ddl_get_unique_id(uid, sizeof uid) == DDL_STATUS_OK, DDL_STATUS_COMM_ERROR, last_error());
        l.comm = rccl_init_rank(0, 1, uid, sizeof uid);
        l.owned.push_back(l.comm);
    });
}

int ddl_rccl_loopback_split(int color, int key, int *rank, int *size) {
    return guarded([&] {
        DDL_REQUIRE(rank && size, DDL_STATUS_INVALID_ARGUMENT, "null output");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        DDL_REQUIRE(l.comm != nullptr, DDL_STATUS_NOT_INITIALIZED, "ddl_rccl_loopback_init has not been called");
        *rank = -1;
        *size = 0;
        ncclComm_t nc = rccl_split(l.comm, color, key, rank, size);
        if (!nc) return;  // color < 0: in no communicator; the current one stays
        l.owned.push_back(nc);
        l.comm = nc;
    });
}

int ddl_rccl_loopback_allreduce(int nranks, const void *const *sends, void *const *recvs, size_t elements, int dtype,
                                void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        DDL_REQUIRE(sends && recvs, DDL_STATUS_INVALID_ARGUMENT, "null buffer arrays");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        l.world(nranks).allreduce(sends, recvs, elements, dtype, as_stream(hip_stream), config().ring());
    });
}

int ddl_rccl_loopback_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                                      const size_t *elements, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && count >= 0 && (count == 0 || (sends && recvs && elements)),
                    DDL_STATUS_INVALID_ARGUMENT, "bad loopback allreduce batch");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        l.world(nranks).allreduce_batch(sends, recvs, elements, count, dtype, as_stream(hip_stream), config().ring());
    });
}

int ddl_rccl_loopback_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype,
                                void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && root >= 0 && root < nranks && bufs, DDL_STATUS_INVALID_ARGUMENT,
                    "bad loopback broadcast");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        l.world(nranks).broadcast(bufs, elements, dtype, root, as_stream(hip_stream), config().ring());
    });
}

int ddl_rccl_loopback_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                                 const size_t *displs, int dtype, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 1 && nranks <= 64 && sends && recvs && counts && displs, DDL_STATUS_INVALID_ARGUMENT,
                    "bad loopback allgatherv");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        l.world(nranks).allgatherv(sends, recvs, counts, displs, dtype, as_stream(hip_stream));
    });
}

int ddl_rccl_loopback_allgather(const void *send, void *recv, size_t bytes, void *hip_stream) {
    return guarded([&] {
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        DDL_REQUIRE(l.comm != nullptr, DDL_STATUS_NOT_INITIALIZED, "ddl_rccl_loopback_init has not been called");
        RcclTransport(l.comm).allgather(GatherOp{send, recv, bytes}, as_stream(hip_stream));
    });
}

int ddl_rccl_loopback_max(float *values, int count, void *hip_stream) {
    return guarded([&] {
        DDL_REQUIRE(values, DDL_STATUS_INVALID_ARGUMENT, "null values");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        DDL_REQUIRE(l.comm != nullptr, DDL_STATUS_NOT_INITIALIZED, "ddl_rccl_loopback_init has not been called");
        rccl_max_floats(l.comm, values, count, as_stream(hip_stream));
    });
}

int ddl_rccl_loopback_tune(int nranks, size_t elements, int dtype, void *hip_stream, int *chosen, int *count,
                           long long *configs, float *ms, int max_candidates) {
    return guarded([&] {
        DDL_REQUIRE(nranks >= 2 && nranks <= 16, DDL_STATUS_INVALID_ARGUMENT, "nranks " << nranks);
        const size_t es = dtype_size(dtype), bytes = elements * es;
        DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dtype);
        DDL_REQUIRE(elements > 0, DDL_STATUS_INVALID_ARGUMENT, "empty bucket");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        hipStream_t stream = as_stream(hip_stream);
        std::vector<void *> bufs(2 * nranks, nullptr);
        auto release = [&] {
            (void)hipStreamSynchronize(stream);
            for (void *p : bufs)
                if (p) (void)hipFree(p);
        };
        TuneResult r;
        try {
            for (void *&p : bufs) {
                DDL_HIP(hipMalloc(&p, bytes));
                DDL_HIP(hipMemsetAsync(p, 0, bytes, stream));
            }
            LocalWorld &w = l.world(nranks);
            // the candidates run through RCCL; the agreement is the product's ncclAllReduce(MAX)
            r = run_tuning(
                nranks, bytes, stream, config().ring(),
                [&](const RingConfig &c) { w.allreduce(bufs.data(), bufs.data() + nranks, elements, dtype, stream, c); },
                [&](float *v, int nc) { rccl_max_floats(l.comm, v, nc, stream); });
        } catch (...) {
            release();
            throw;
        }
        release();
        export_tune(r, chosen, count, configs, ms, max_candidates);
    });
}

int ddl_rccl_loopback_stats(int nranks, long long *pairs) {
    return guarded([&] {
        DDL_REQUIRE(pairs, DDL_STATUS_INVALID_ARGUMENT, "null output");
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        *pairs = l.world(nranks).loopback_pairs();
    });
}

int ddl_rccl_loopback_finalize(void) {
    return guarded([&] {
        RcclLoopback &l = rccl_loopback();
        std::lock_guard<std::mutex> g(l.mu);
        (void)hipDeviceSynchronize();
        l.worlds.clear();
        {  // thread worlds moving their bytes through these communicators go first
            std::lock_guard<std::mutex> tg(g_thread_mu);
            for (auto it = g_thread_worlds->begin(); it != g_thread_worlds->end();)
                it = std::get<3>(it->first) ? g_thread_worlds->erase(it) : std::next(it);
        }
        for (auto it = l.owned.rbegin(); it != l.owned.rend(); ++it) (void)rccl().CommDestroy(*it);
        l.owned.clear();
        l.comm = nullptr;
    });
}

// ---- schedule introspection -----------------------------------------------------------------
int ddl_ring_count(int nranks, int max_rings) {
    if (nranks < 1) return 0;
    return (int)rings_for(nranks, max_rings).size();
}

int ddl_ring_perm(int nranks, int max_rings, int ring, int *perm_out) {
    return guarded([&] {
        const auto &rings = rings_for(nranks, max_rings);
        DDL_REQUIRE(ring >= 0 && ring < (int)rings.size() && perm_out, DDL_STATUS_INVALID_ARGUMENT, "bad ring " << ring);
        for (int p = 0; p < nranks; ++p) perm_out[p] = rings[ring][p];
    });
}

int ddl_chunk_range(size_t elements, int dtype, int nranks, int rings, int ring, int chunk, size_t *begin,
                    size_t *end) {
    return guarded([&] {
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es && nranks >= 1 && rings >= 1 && ring >= 0 && ring < rings && chunk >= 0 && chunk < nranks &&
                        begin && end,
                    DDL_STATUS_INVALID_ARGUMENT, "bad chunk query");
        Range r = chunk_range(elements, es, nranks, rings, ring, chunk);
        *begin = r.begin;
        *end = r.end;
    });
}

int ddl_ring_shape(size_t elements, int dtype, int nranks, int *rings, int *slices) {
    return guarded([&] {
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es && nranks >= 1 && rings && slices, DDL_STATUS_INVALID_ARGUMENT, "bad shape query");
        size_t stride;
        ring_shape(elements, es, nranks, config().ring(), rings, slices, &stride);
    });
}

namespace {

// Symbolic base addresses: every pointer of a program decodes to (buffer, element offset).
char *sym_base(int i) { return (char *)(uintptr_t(i + 1) << 44); }

void dump_program(const RingProgram &prog, size_t es, long long *ops_out, size_t max_ops, size_t *nops) {
    auto decode = [&](const void *p, long long *buf, long long *off) {
        uintptr_t v = reinterpret_cast<uintptr_t>(p);
        *buf = (long long)(v >> 44) - 1;
        *off = (long long)((v & ((uintptr_t(1) << 44) - 1)) / es);
    };
    std::vector<long long> rows;
    for (size_t t = 0; t < prog.ticks.size(); ++t) {
        const Tick &tk = prog.ticks[t];
        for (const CopyOp &c : tk.copies) {
            long long dbuf, doff, sbuf, soff;
            decode(c.dst, &dbuf, &doff);
            decode(c.src, &sbuf, &soff);
            DDL_REQUIRE(sbuf == 0, DDL_STATUS_ERROR_UNKNOWN, "copy source outside the input");
            long long row[8] = {(long long)t, 4, -1, -1, dbuf, doff, (long long)(c.bytes / es), soff};
            rows.insert(rows.end(), row, row + 8);
        }
        if (tk.gather.bytes) {
            // {tick, 11, send buffer, send offset, recv buffer, recv offset, elements per rank,
            //  the tick's reduce wait (-1: none)}
            long long sbuf, soff, rbuf, roff;
            decode(tk.gather.send, &sbuf, &soff);
            decode(tk.gather.recv, &rbuf, &roff);
            long long row[8] = {(long long)t, 11, sbuf, soff, rbuf, roff, (long long)(tk.gather.bytes / es),
                                tk.wait_reduce};
            rows.insert(rows.end(), row, row + 8);
        }
        for (const P2POp &op : tk.ops) {
            long long buf, off;
            decode(op.ptr, &buf, &off);
            long long row[8] = {(long long)t, op.send ? 0 : 1, op.peer, op.tag, buf, off, (long long)(op.bytes / es), tk.wait_reduce};
            rows.insert(rows.end(), row, row + 8);
        }
        for (int sgi = 0; sgi < tk.reduce.count; ++sgi) {
            long long obuf, ooff, abuf, aoff, bbuf, boff;
            decode(tk.reduce.out[sgi], &obuf, &ooff);
            decode(tk.reduce.a[sgi], &abuf, &aoff);
            decode(tk.reduce.b[sgi], &bbuf, &boff);
            DDL_REQUIRE(abuf == 0 && aoff == ooff && bbuf == 2 && obuf == 1, DDL_STATUS_ERROR_UNKNOWN,
                        "unexpected reduce operands");
            long long row[8] = {(long long)t, 2, -1, sgi, obuf, ooff, (long long)tk.reduce.n[sgi], boff};
            rows.insert(rows.end(), row, row + 8);
        }
        if (tk.has_reduce && tk.multi) {
            // the classic direct fold (one left-order step, a = in at the output offset, every
            // other input a staging slot): one row per received input, in fold order
            //   {tick, 3, inputs - 1, i, 1, output offset, count, staging offset}
            if (tk.folds.size() == 1 && tk.folds[0].order == kFoldLeft) {
                const SegTableN &f = tk.folds[0];
                long long obuf, ooff, abuf, aoff;
                decode(f.out, &obuf, &ooff);
                decode(f.a, &abuf, &aoff);
                bool staged = obuf == 1 && abuf == 0 && aoff == ooff;
                for (int i = 0; i < f.nb; ++i) {
                    long long bbuf, boff;
                    decode(f.b[i], &bbuf, &boff);
                    staged = staged && bbuf == 2;
                }
                if (staged) {
                    for (int i = 0; i < f.nb; ++i) {
                        long long bbuf, boff;
                        decode(f.b[i], &bbuf, &boff);
                        long long row[8] = {(long long)t, 3, f.nb, i, obuf, ooff, (long long)f.n, boff};
                        rows.insert(rows.end(), row, row + 8);
                    }
                    continue;
                }
            }
            // general fold steps, in execution order: one row per input, input 0 = a:
            //   {tick, kind, inputs, i, source buffer, source offset, count, output offset}
            // kind 5 + order into the output buffer, 8 + order into staging (a partial sum);
            // order 0 left, 1 MPICH's pre-fold + pairwise tree, 2 binomial
            for (const SegTableN &f : tk.folds) {
                long long obuf, ooff;
                decode(f.out, &obuf, &ooff);
                DDL_REQUIRE(obuf == 1 || obuf == 2, DDL_STATUS_ERROR_UNKNOWN, "fold output outside out / staging");
                const int ni = f.nb + 1;
                const long long kind = (obuf == 1 ? 5 : 8) + f.order;
                for (int i = 0; i < ni; ++i) {
                    long long sbuf, soff;
                    decode(i == 0 ? f.a : f.b[i - 1], &sbuf, &soff);
                    long long row[8] = {(long long)t, kind, ni, i, sbuf, soff, (long long)f.n, ooff};
                    rows.insert(rows.end(), row, row + 8);
                }
            }
        }
    }
    *nops = rows.size() / 8;
    DDL_REQUIRE(*nops <= max_ops && (rows.empty() || ops_out), DDL_STATUS_INVALID_ARGUMENT,
                "op buffer too small: need " << *nops);
    std::copy(rows.begin(), rows.end(), ops_out);
}

}  // namespace

int ddl_ring_program(int rank, int nranks, size_t elements, int dtype, long long *ops_out, size_t max_ops,
                     size_t *nops) {
    return guarded([&] {
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es && nranks >= 1 && rank >= 0 && rank < nranks && nops, DDL_STATUS_INVALID_ARGUMENT,
                    "bad program query");
        RingProgram prog;
        build_program(prog, rank, nranks, sym_base(0), sym_base(1), sym_base(2), elements, dtype, config().ring());
        dump_program(prog, es, ops_out, max_ops, nops);
    });
}

int ddl_broadcast_program(int rank, int nranks, int root, size_t elements, int dtype, long long *ops_out,
                          size_t max_ops, size_t *nops) {
    return guarded([&] {
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es && nranks >= 1 && rank >= 0 && rank < nranks && nops, DDL_STATUS_INVALID_ARGUMENT,
                    "bad program query");
        RingProgram prog;
        build_broadcast(prog, rank, nranks, root, sym_base(1), elements, dtype, config().ring());
        dump_program(prog, es, ops_out, max_ops, nops);
    });
}

int ddl_allgather_program(int rank, int nranks, const size_t *counts, const size_t *displs, int dtype,
                          long long *ops_out, size_t max_ops, size_t *nops) {
    return guarded([&] {
        const size_t es = dtype_size(dtype);
        DDL_REQUIRE(es && nranks >= 1 && rank >= 0 && rank < nranks && nops && counts && displs,
                    DDL_STATUS_INVALID_ARGUMENT, "bad program query");
        RingProgram prog;
        build_allgatherv(prog, rank, nranks, sym_base(0), sym_base(1), counts, displs, dtype);
        dump_program(prog, es, ops_out, max_ops, nops);
    });
}

int ddl_make_plans(const size_t *elements, const size_t *esizes, size_t count, size_t limit, size_t *plans_out,
                   size_t max_plans, size_t *nplans) {
    return guarded([&] {
        DDL_REQUIRE(nplans && (count == 0 || (elements && esizes)), DDL_STATUS_INVALID_ARGUMENT, "bad plan args");
        std::vector<size_t> e(elements, elements + count), s(esizes, esizes + count);
        auto plans = make_plans(e, s, limit);
        *nplans = plans.size();
        DDL_REQUIRE(plans.size() <= max_plans && (plans.empty() || plans_out), DDL_STATUS_INVALID_ARGUMENT,
                    "plan buffer too small: need " << plans.size());
        for (size_t i = 0; i < plans.size(); ++i) {
            plans_out[4 * i] = plans[i].req_begin;
            plans_out[4 * i + 1] = plans[i].elem_begin;
            plans_out[4 * i + 2] = plans[i].req_end;
            plans_out[4 * i + 3] = plans[i].elem_end;
        }
    });
}

}  // extern "C"
