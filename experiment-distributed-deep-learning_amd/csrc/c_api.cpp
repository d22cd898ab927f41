// c_api.cpp — the deployment C-ABI (include/ddl_amd.h): exactly these symbols are exported by
// libddl_amd.so (ddl_amd.map). Every entry point converts internal errors into a status code; no
// C++ exception crosses the ABI. The test / measurement entry points (include/ddl_amd_testing.h)
// are in c_api_testing.cpp, linked into libddl_amd_testing.so only.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "engine.h"
#include "abi.h"
#include "handler.h"

using namespace ddl;
using namespace ddl::abi;

namespace {

// The submitter's input-ready event: device requests are ordered after hip_stream's current
// position; host requests are ready at submission (CPU tensors, as the reference's op inputs).
std::shared_ptr<ReadyEvent> ready_event(int memory, void *hip_stream) {
    DDL_REQUIRE(memory == DDL_MEMORY_DEVICE || memory == DDL_MEMORY_HOST, DDL_STATUS_INVALID_ARGUMENT,
                "memory must be DDL_MEMORY_DEVICE (0) or DDL_MEMORY_HOST (1), not " << memory);
    return memory == DDL_MEMORY_HOST ? nullptr : std::make_shared<ReadyEvent>(as_stream(hip_stream));
}

}  // namespace

extern "C" {

int ddl_version(void) { return 2; }

#ifndef DDL_SRC_HASH
#define DDL_SRC_HASH "unknown"
#endif
const char *ddl_build_info(void) { return "src=" DDL_SRC_HASH " arch=gfx950"; }
const char *ddl_last_error(void) { return last_error(); }
const char *ddl_dtype_name(int dtype) { return dtype_name(dtype); }
size_t ddl_dtype_size(int dtype) { return dtype_size(dtype); }

int ddl_get_unique_id(void *out, size_t len) {
    return guarded([&] {
        DDL_REQUIRE(out && len >= sizeof(ncclUniqueId), DDL_STATUS_INVALID_ARGUMENT,
                    "unique id buffer needs " << sizeof(ncclUniqueId) << " bytes");
        ncclUniqueId id;
        rccl_check(rccl().GetUniqueId(&id), "ncclGetUniqueId");
        std::memcpy(out, &id, sizeof id);
    });
}

int ddl_init(int rank, int size, int device, const void *unique_id, size_t len) {
    return guarded([&] {
        DDL_REQUIRE(size >= 1 && rank >= 0 && rank < size, DDL_STATUS_INVALID_ARGUMENT,
                    "bad rank/size " << rank << "/" << size);
        DDL_REQUIRE(!Registry::get().initialized(), DDL_STATUS_INVALID_ARGUMENT, "already initialized");
        DDL_HIP(hipSetDevice(device));
        ncclComm_t nc = size > 1 ? rccl_init_rank(rank, size, unique_id, len) : nullptr;
        Registry::get().set_world(new_communicator(rank, size, device, nc));
        DDL_LOG(1, "initialized rank " << rank << "/" << size << " on device " << device
                                       << (size > 1 ? std::string(" rccl=") + rccl().path : ""));
    });
}

int ddl_init_single(int device) { return ddl_init(0, 1, device, nullptr, 0); }

int ddl_control_listen(char *endpoint_out, size_t len) {
    return guarded([&] {
        std::string ep = standalone_control()->listen();
        DDL_REQUIRE(endpoint_out && len > ep.size(), DDL_STATUS_INVALID_ARGUMENT, "endpoint buffer too small");
        std::memcpy(endpoint_out, ep.c_str(), ep.size() + 1);
    });
}

int ddl_control_connect(const char *endpoints) {
    return guarded([&] {
        DDL_REQUIRE(endpoints, DDL_STATUS_INVALID_ARGUMENT, "null endpoints");
        auto world = Registry::get().world();
        auto ch = standalone_control();
        ch->connect(world->rank(), world->size(), split_endpoints(endpoints), 120000);
        standalone_control() = std::make_shared<ControlChannel>();
        // collective: the world's token ring and its keyed data-plane communicator
        world->enable_keyed(ch);
    });
}

int ddl_control_stats(long long *string_rounds, long long *cached_rounds) {
    return guarded([&] {
        DDL_REQUIRE(string_rounds && cached_rounds, DDL_STATUS_INVALID_ARGUMENT, "null output");
        ControlChannel *ch = standalone_control().get();
        if (Registry::get().initialized() && Registry::get().world()->control())
            ch = Registry::get().world()->control();
        *string_rounds = ch->string_rounds;
        *cached_rounds = ch->cached_rounds;
    });
}

int ddl_finalize(void) {
    return guarded([&] {
        Registry::get().clear();
        DDL_REQUIRE(wait_deferred_deletions(60000), DDL_STATUS_ERROR_UNKNOWN,
                    "a communicator released by its own handler thread is still being destroyed after 60 s");
        free_retired();
        standalone_control() = std::make_shared<ControlChannel>();
        run_finalize_hooks();
    });
}

int ddl_is_initialized(void) { return Registry::get().initialized() ? 1 : 0; }

int ddl_set_config(const char *key, long long value) {
    return guarded([&] {
        DDL_REQUIRE(key, DDL_STATUS_INVALID_ARGUMENT, "null key");
        std::string k(key);
        Config &c = config();
        if (k == "slice_bytes") c.slice_bytes = value;
        else if (k == "algo") {
            DDL_REQUIRE(value >= kAlgoRing && value <= kAlgoDirectGather, DDL_STATUS_INVALID_ARGUMENT,
                        "algo must be 0 (ring), 1 (direct), 2 (one-shot), 3 (gather-fold) or 4 (direct-gather)");
            c.algo = value;
        } else if (k == "rings") c.rings = value;
        else if (k == "max_slices") c.max_slices = value;
        else if (k == "fusion_threshold_bytes") {
            DDL_REQUIRE(value > 0, DDL_STATUS_INVALID_ARGUMENT, "fusion threshold must be > 0");
            c.fusion_threshold_bytes = value;
        } else if (k == "log_level") c.log_level = value;
        else if (k == "cycle_time_us") c.cycle_time_us = value;
        else if (k == "host_chunk_bytes") {
            DDL_REQUIRE(value >= 4096, DDL_STATUS_INVALID_ARGUMENT, "host_chunk_bytes must be >= 4096");
            c.host_chunk_bytes = value;
        } else if (k == "host_copy_threads") {
            DDL_REQUIRE(value >= 0 && value <= 64, DDL_STATUS_INVALID_ARGUMENT, "host_copy_threads must be in [0, 64]");
            c.host_copy_threads = value;
        } else if (k == "host_zero_copy") c.host_zero_copy = value ? 1 : 0;
        else if (k == "host_numa_bind") c.host_numa_bind = value ? 1 : 0;
        else if (k == "host_register_cache_bytes") {
            DDL_REQUIRE(value >= 0, DDL_STATUS_INVALID_ARGUMENT, "host_register_cache_bytes must be >= 0");
            c.host_register_cache_bytes = value;
            if (value == 0)  // off: every cached registration goes now (before the caller frees memory)
                for (auto &comm : Registry::get().all())
                    if (RequestHandler *h = comm->handler_if_created()) h->release_registrations();
        }
        else if (k == "tune") c.tune = value ? 1 : 0;
        else if (k == "fusion_pipeline_bytes") {
            DDL_REQUIRE(value >= 0, DDL_STATUS_INVALID_ARGUMENT, "fusion_pipeline_bytes must be >= 0");
            c.fusion_pipeline_bytes = value;
        } else if (k == "one_rank_shortcut") c.one_rank_shortcut = value ? 1 : 0;
        else if (k == "pipeline_rounds") c.pipeline_rounds = value ? 1 : 0;
        else if (k == "reference_order") c.reference_order = value ? 1 : 0;
        else if (k == "capture_mode") {
            DDL_REQUIRE(value != 1, DDL_STATUS_INVALID_ARGUMENT,
                        "capture_mode 1 (forked streams) was removed in r04: HIP 7.0's hipStreamEndCapture crashes "
                        "on three or more cross-waiting forked streams (DESIGN §9); 2 keeps the overlap");
            DDL_REQUIRE(value == 0 || value == 2, DDL_STATUS_INVALID_ARGUMENT,
                        "capture_mode must be 0 (serial) or 2 (single-stream DAG)");
            c.capture_mode = value;
        } else if (k == "compute_cu_mask") {
            DDL_REQUIRE(value == 0 || value == 2 || value == 4 || value == 8, DDL_STATUS_INVALID_ARGUMENT,
                        "compute_cu_mask must be 0 (all CUs), 2, 4 or 8 (every n-th CU left to RCCL)");
            c.compute_cu_mask = value;
        } else if (k == "queue_isolation") c.queue_isolation = value ? 1 : 0;
        else if (k == "rccl_min_ctas" || k == "rccl_max_ctas") {
            DDL_REQUIRE(value >= 0 && value <= 256, DDL_STATUS_INVALID_ARGUMENT,
                        k << " must be 0 (RCCL's default) or a channel count in [1, 256]");
            (k == "rccl_min_ctas" ? c.rccl_min_ctas : c.rccl_max_ctas) = value;
        } else if (k == "fold_form") {
            DDL_REQUIRE(value >= 0 && value <= 2, DDL_STATUS_INVALID_ARGUMENT,
                        "fold_form must be 0 (auto), 1 (tile form) or 2 (run form)");
            set_fold_form((int)value);
        }
        else fail(DDL_STATUS_INVALID_ARGUMENT, "unknown config key '" + k + "'");
        c.epoch.fetch_add(1);
    });
}

long long ddl_get_config(const char *key) {
    if (!key) return -1;
    std::string k(key);
    Config &c = config();
    if (k == "slice_bytes") return c.slice_bytes;
    if (k == "algo") return c.algo;
    if (k == "rings") return c.rings;
    if (k == "max_slices") return c.max_slices;
    if (k == "fusion_threshold_bytes") return c.fusion_threshold_bytes;
    if (k == "log_level") return c.log_level;
    if (k == "cycle_time_us") return c.cycle_time_us;
    if (k == "host_chunk_bytes") return c.host_chunk_bytes;
    if (k == "tune") return c.tune;
    if (k == "host_copy_threads") return c.host_copy_threads;
    if (k == "host_zero_copy") return c.host_zero_copy;
    if (k == "host_register_cache_bytes") return c.host_register_cache_bytes;
    if (k == "host_numa_bind") return c.host_numa_bind;
    if (k == "host_registered_bytes") return c.host_registered_bytes;    // statistic, not settable
    if (k == "host_register_failures") return c.host_register_failures;  // statistic, not settable
    if (k == "host_register_hits") return c.host_register_hits;          // statistic, not settable
    if (k == "host_unregistered_ranges") return c.host_unregistered_ranges;  // statistic, not settable
    if (k == "host_zero_copy_plans") return c.host_zero_copy_plans;  // statistic, not settable
    if (k == "host_pack_us") return c.host_pack_ns / 1000;      // statistic, not settable
    if (k == "host_wait_us") return c.host_wait_ns / 1000;      // statistic, not settable
    if (k == "host_unpack_us") return c.host_unpack_ns / 1000;  // statistic, not settable
    if (k == "host_check_us") return c.host_check_ns / 1000;    // statistic, not settable
    if (k == "host_plan_us") return c.host_plan_ns / 1000;      // statistic, not settable
    if (k == "host_coll_us") return c.host_coll_ns / 1000;      // statistic, not settable
    if (k == "host_d2h_post_us") return c.host_d2h_post_ns / 1000;  // statistic, not settable
    if (k == "host_unpack_submit_us") return c.host_unpack_submit_ns / 1000;  // statistic, not settable
    if (k == "host_lane_d2h_wait_us") return c.host_lane_d2h_wait_ns / 1000;  // statistic, not settable
    if (k == "host_lane_copy_us") return c.host_lane_copy_ns / 1000;          // statistic, not settable
    if (k == "host_lane_copy_bytes") return c.host_lane_copy_bytes;           // statistic, not settable
    if (k == "host_lane_jobs") return c.host_lane_jobs;                       // statistic, not settable
    if (k == "fusion_pipeline_bytes") return c.fusion_pipeline_bytes;
    if (k == "one_rank_shortcut") return c.one_rank_shortcut;
    if (k == "pipeline_rounds") return c.pipeline_rounds;
    if (k == "reference_order") return c.reference_order;
    if (k == "capture_mode") return c.capture_mode;
    if (k == "fold_form") return get_fold_form();
    if (k == "compute_cu_mask") return c.compute_cu_mask;
    if (k == "queue_isolation") return c.queue_isolation;
    if (k == "rccl_min_ctas") return c.rccl_min_ctas;
    if (k == "rccl_max_ctas") return c.rccl_max_ctas;
    return -1;
}

// ---- reference c_api.h surface (src/cpp/c_api.cc:11-65) ------------------------------------
int communicator_rank(ddl_communicator_id id) {
    int r = -1;
    if (guarded([&] { r = Registry::get().find(id)->rank(); }) != DDL_STATUS_OK) return -1;
    return r;
}

int communicator_size(ddl_communicator_id id) {
    int s = -1;
    if (guarded([&] { s = Registry::get().find(id)->size(); }) != DDL_STATUS_OK) return -1;
    return s;
}

ddl_communicator_id world_communicator(void) {
    ddl_communicator_id id = 0;
    if (guarded([&] { id = Registry::get().world()->id(); }) != DDL_STATUS_OK) return 0;
    return id;
}

ddl_communicator_id split_communicator(ddl_communicator_id id, int color, int key) {
    ddl_communicator_id out = 0;
    int st = guarded([&] {
        auto c = Registry::get().find(id)->split(color, key);
        Registry::get().add(c);
        out = c->id();
    });
    return st == DDL_STATUS_OK ? out : 0;
}

void detach_communicator(ddl_communicator_id id) {
    (void)guarded([&] { Registry::get().detach(id); });
}

void py_info(const char *s) { DDL_LOG(1, "[py]: " << (s ? s : "")); }
void py_debug(const char *s) { DDL_LOG(2, "[py]: " << (s ? s : "")); }
void py_error(const char *s) { DDL_LOG(0, "[py]: " << (s ? s : "")); }

// ---- data plane ---------------------------------------------------------------------------
int ddl_allreduce(ddl_communicator_id id, const void *send, void *recv, size_t elements, int dtype,
                  int op, void *hip_stream) {
    return guarded([&] { Registry::get().find(id)->allreduce(send, recv, elements, dtype, op, as_stream(hip_stream)); });
}

int ddl_allreduce_batch(ddl_communicator_id id, int count, const void *const *sends, void *const *recvs,
                        const size_t *elements, int dtype, int op, void *hip_stream) {
    return guarded([&] {
        Registry::get().find(id)->allreduce_batch(sends, recvs, elements, count, dtype, op, as_stream(hip_stream));
    });
}

int ddl_broadcast(ddl_communicator_id id, void *buf, size_t elements, int dtype, int root, void *hip_stream) {
    return guarded([&] { Registry::get().find(id)->broadcast(buf, elements, dtype, root, as_stream(hip_stream)); });
}

int ddl_allgatherv(ddl_communicator_id id, const void *send, size_t send_elements, void *recv,
                   const size_t *recv_counts, const size_t *displs, int dtype, void *hip_stream) {
    return guarded([&] {
        auto c = Registry::get().find(id);
        DDL_REQUIRE(recv_counts && displs, DDL_STATUS_INVALID_ARGUMENT, "null counts/displs");
        DDL_REQUIRE(recv_counts[c->rank()] == send_elements, DDL_STATUS_INVALID_ARGUMENT,
                    "send_elements " << send_elements << " != recv_counts[rank] " << recv_counts[c->rank()]);
        c->allgatherv(send, recv, recv_counts, displs, dtype, as_stream(hip_stream));
    });
}

int ddl_allgather(ddl_communicator_id id, const void *send, size_t send_elements, void *recv, size_t recv_elements,
                  int dtype, void *hip_stream) {
    return guarded([&] {
        auto c = Registry::get().find(id);
        DDL_REQUIRE(send_elements == recv_elements, DDL_STATUS_INVALID_ARGUMENT,
                    "send_elements " << send_elements << " != recv_elements " << recv_elements);
        std::vector<size_t> counts(c->size(), recv_elements), displs(c->size());
        for (int q = 0; q < c->size(); ++q) displs[q] = (size_t)q * recv_elements;
        c->allgatherv(send, recv, counts.data(), displs.data(), dtype, as_stream(hip_stream));
    });
}

int ddl_allreduce_host(ddl_communicator_id id, const void *send, void *recv, size_t elements, int dtype, int op) {
    return guarded([&] { Registry::get().find(id)->allreduce_host(send, recv, elements, dtype, op); });
}

int ddl_comm_transport(ddl_communicator_id id, int *kind, int *ranks) {
    return guarded([&] {
        DDL_REQUIRE(kind && ranks, DDL_STATUS_INVALID_ARGUMENT, "null output");
        Registry::get().find(id)->transport(kind, ranks);
    });
}

int ddl_tune_result(ddl_communicator_id id, size_t bucket_bytes, int *chosen, int *count, long long *configs,
                    float *ms, int max_candidates) {
    return guarded([&] {
        export_tune(Registry::get().find(id)->tune_result(bucket_bytes), chosen, count, configs, ms, max_candidates);
    });
}

int ddl_allreduce_submit_mem(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                             int dtype, int op, int memory, void *hip_stream, ddl_done_fn done, void *user) {
    return guarded([&] {
        DDL_REQUIRE(key, DDL_STATUS_INVALID_ARGUMENT, "null key");
        auto c = Registry::get().find(id);
        DeviceGuard g(c->device());
        Request r;
        r.key = key;
        r.in = in;
        r.out = out;
        r.n = elements;
        r.dtype = dtype;
        r.op = op;
        r.done = done;
        r.user = user;
        r.host = memory == DDL_MEMORY_HOST;
        r.ready = ready_event(memory, hip_stream);
        c->handler().submit(r);
    });
}

int ddl_allreduce_submit(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                         int dtype, int op, void *hip_stream, ddl_done_fn done, void *user) {
    return ddl_allreduce_submit_mem(id, key, in, out, elements, dtype, op, DDL_MEMORY_DEVICE, hip_stream, done, user);
}

int ddl_broadcast_submit_mem(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                             int dtype, int root, int memory, void *hip_stream, ddl_done_fn done, void *user) {
    return guarded([&] {
        DDL_REQUIRE(key, DDL_STATUS_INVALID_ARGUMENT, "null key");
        auto c = Registry::get().find(id);
        DeviceGuard g(c->device());
        Request r;
        r.type = kReqBroadcast;
        r.key = key;
        r.in = in;
        r.out = out;
        r.n = elements;
        r.dtype = dtype;
        r.root = root;
        r.done = done;
        r.user = user;
        r.host = memory == DDL_MEMORY_HOST;
        r.ready = ready_event(memory, hip_stream);
        c->handler().submit(r);
    });
}

int ddl_broadcast_submit(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                         int dtype, int root, void *hip_stream, ddl_done_fn done, void *user) {
    return ddl_broadcast_submit_mem(id, key, in, out, elements, dtype, root, DDL_MEMORY_DEVICE, hip_stream, done,
                                    user);
}

int ddl_allgather_submit_mem(ddl_communicator_id id, const char *key, const void *in, size_t first_dim,
                             size_t row_elements, int dtype, int memory, void *hip_stream, ddl_alloc_fn alloc,
                             ddl_done_fn done, void *user) {
    return guarded([&] {
        DDL_REQUIRE(key, DDL_STATUS_INVALID_ARGUMENT, "null key");
        auto c = Registry::get().find(id);
        DeviceGuard g(c->device());
        Request r;
        r.type = kReqAllgather;
        r.key = key;
        r.in = in;
        r.first_dim = first_dim;
        r.row_elems = row_elements;
        r.n = first_dim * row_elements;
        r.dtype = dtype;
        r.alloc = alloc;
        r.done = done;
        r.user = user;
        r.host = memory == DDL_MEMORY_HOST;
        r.ready = ready_event(memory, hip_stream);
        c->handler().submit(r);
    });
}

int ddl_allgather_submit(ddl_communicator_id id, const char *key, const void *in, size_t first_dim, size_t row_elements,
                         int dtype, void *hip_stream, ddl_alloc_fn alloc, ddl_done_fn done, void *user) {
    return ddl_allgather_submit_mem(id, key, in, first_dim, row_elements, dtype, DDL_MEMORY_DEVICE, hip_stream, alloc,
                                    done, user);
}

int ddl_allreduce_submit_batch_mem(ddl_communicator_id id, int count, const char *const *keys, const void *const *ins,
                                   void *const *outs, const size_t *elements, const int *dtypes, int op, int memory,
                                   void *hip_stream, ddl_done_fn done, void *const *users) {
    return guarded([&] {
        DDL_REQUIRE(count >= 0 && (count == 0 || (keys && ins && outs && elements && dtypes)),
                    DDL_STATUS_INVALID_ARGUMENT, "bad batch arguments");
        if (count == 0) return;
        auto c = Registry::get().find(id);
        DeviceGuard g(c->device());
        auto ready = ready_event(memory, hip_stream);
        std::vector<Request> rs(count);
        for (int i = 0; i < count; ++i) {
            DDL_REQUIRE(keys[i], DDL_STATUS_INVALID_ARGUMENT, "null key " << i);
            rs[i].key = keys[i];
            rs[i].in = ins[i];
            rs[i].out = outs[i];
            rs[i].n = elements[i];
            rs[i].dtype = dtypes[i];
            rs[i].op = op;
            rs[i].done = done;
            rs[i].user = users ? users[i] : nullptr;
            rs[i].host = memory == DDL_MEMORY_HOST;
            rs[i].ready = ready;
        }
        c->handler().submit_batch(rs);
    });
}

int ddl_allreduce_submit_batch(ddl_communicator_id id, int count, const char *const *keys, const void *const *ins,
                               void *const *outs, const size_t *elements, const int *dtypes, int op,
                               void *hip_stream, ddl_done_fn done, void *const *users) {
    return ddl_allreduce_submit_batch_mem(id, count, keys, ins, outs, elements, dtypes, op, DDL_MEMORY_DEVICE,
                                          hip_stream, done, users);
}

int ddl_kernel_timing(ddl_communicator_id id, int on) {
    return guarded([&] {
        auto c = Registry::get().find(id);
        std::lock_guard<std::mutex> g(c->mutex());
        c->executor().set_timing(on != 0);
    });
}

int ddl_kernel_stats(ddl_communicator_id id, long long *launches, double *bytes, double *ms) {
    return guarded([&] {
        DDL_REQUIRE(launches && bytes && ms, DDL_STATUS_INVALID_ARGUMENT, "null output");
        auto c = Registry::get().find(id);
        std::lock_guard<std::mutex> g(c->mutex());
        DeviceGuard dg(c->device());
        KernelStats s = c->executor().collect_stats();
        *launches = s.launches;
        *bytes = s.bytes;
        *ms = s.ms;
    });
}

int ddl_host_unregister(const void *ptr, size_t bytes) {
    return guarded([&] {
        for (auto &comm : Registry::get().all())
            if (RequestHandler *h = comm->handler_if_created()) h->unregister_range(ptr, bytes);
    });
}

int ddl_wait_all(ddl_communicator_id id) {
    return guarded([&] { Registry::get().find(id)->handler().wait_all(); });
}

}  // extern "C"
