/*
 * ddl_amd.h — C-ABI of the MI355X gradient-bucket allreduce engine.
 *
 * This is the drop-in boundary for the reference's allreduce hot path
 * (LYL232/Experiment-Distributed-Deep-Learning, paths relative to its src/):
 *
 *   reference                                             replaced by
 *   ---------------------------------------------------   -----------------------------
 *   cpp/c_api.h:15-17   communicator_rank/size            communicator_rank/size
 *   cpp/c_api.h:19      world_communicator                world_communicator
 *   cpp/c_api.h:33-35   split/detach_communicator         split_communicator/detach_communicator
 *   cpp/c_api.h:37-41   py_info/py_debug/py_error         py_info/py_debug/py_error
 *   cpp/global/initialize.cc:57-65 + MPIBackend.cc:77-97  ddl_get_unique_id + ddl_init
 *     (MPI_Init_thread at dlopen)                          (explicit RCCL bootstrap)
 *   cpp/communicate/backend/Communicator.h:45-48 /        ddl_allreduce (device buffers; at
 *     mpi/MPICommunicator.cc:14-28  (MPI_Allreduce SUM)     P > 2 by default the direct schedule:
 *                                                          reduce-scatter of slices to every peer
 *                                                          over RCCL send/recv, a HIP fold of the P
 *                                                          inputs in MPICH's order, allgather; a
 *                                                          ring at P = 2; autotuned per size class)
 *   cpp/op/tensorflow/AllreduceOp.cc:32-66 →              ddl_allreduce_submit
 *     TensorsCollectiveCommunicateController::handleRequest (keyed async request, done callback)
 *     (.../controller/TensorsCollectiveCommunicateController.h:14-34)
 *
 * Conventions (mirroring the reference):
 *   - communicator ids are 64-bit integers (Communicator::ID = long long, Communicator.h:20);
 *   - dtypes use tensorflow::DataType numbers, as the reference does (def.h:10 uses
 *     tensorflow::DataType; ascending enum order is the fusion group order,
 *     MPIRingTokenCommunication.cc:735-749);
 *   - every call returns an int status (StatusCode, def.h:70-74, extended); no C++
 *     exception crosses this boundary; ddl_last_error() describes the last failure
 *     on the calling thread;
 *   - buffers are device (HBM) pointers; hip_stream is a hipStream_t (NULL = legacy
 *     default stream); calls are stream-ordered and never synchronise the host unless
 *     documented.
 */
#ifndef DDL_AMD_H
#define DDL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* tensorflow::DataType numeric values (reference def.h:10-53 comment block). */
enum ddl_dtype {
    DDL_FLOAT = 1,
    DDL_DOUBLE = 2,
    DDL_INT32 = 3,
    DDL_INT64 = 9,
    DDL_BFLOAT16 = 14, /* extension: the reference rejects it (AllreduceOp.cc:18) */
    DDL_HALF = 19,     /* extension: the reference rejects it (MPIBackend.cc:48-66) */
    DDL_UINT64 = 23
};

/* StatusCode (reference def.h:70-74) + extensions. */
enum ddl_status {
    DDL_STATUS_OK = 0,
    DDL_STATUS_COMM_ERROR = 1, /* was STATUS_MPI_ERROR: RCCL / control-channel failure */
    DDL_STATUS_ERROR_UNKNOWN = 2,
    DDL_STATUS_INVALID_ARGUMENT = 3,
    DDL_STATUS_UNSUPPORTED_DTYPE = 4,
    DDL_STATUS_HIP_ERROR = 5,
    DDL_STATUS_NOT_INITIALIZED = 6,
    DDL_STATUS_DUPLICATE_KEY = 7, /* TensorCommunicateRequest.h:21: one pending request per key */
    DDL_STATUS_CONFIG_MISMATCH = 8 /* the ranks' shared tunables differ (see ddl_set_config): the
                                      collective or keyed round fails on every rank, nothing runs */
};

/* Where a keyed request's buffers live: SURVEY §8(b)'s device_ptr_flag. The reference's op is
 * CPU-only (AllreduceOp.cc:68): its tensors are host memory, copied into the MPI buffer
 * (MPIRingTokenCommunication.cc:548-733). Host requests are staged through pinned chunks to the
 * device and back; device requests stay in HBM. */
enum ddl_memory { DDL_MEMORY_DEVICE = 0, DDL_MEMORY_HOST = 1 };

/* Communicator::AllreduceOperation (reference Communicator.h:22-24): SUM only. */
enum ddl_allreduce_op { DDL_ALLREDUCE_OP_SUM = 0 };

typedef long long ddl_communicator_id;

/* Completion callback of a keyed request: TensorCommunicateRequest::done(StatusCode)
 * (reference TensorCommunicateRequest.h:41). Runs on the communicator's engine thread. */
typedef void (*ddl_done_fn)(int status, void *user);

/* Output allocation of a keyed allgather, called on the engine thread once the gathered first
 * dimension is known (the reference allocates through OpContext::allocateOutput,
 * MPIRingTokenCommunication.cc:299-306): returns a device buffer of `bytes` for an output of
 * `first_dim` rows, or NULL on failure (the request then completes with an error). */
typedef void *(*ddl_alloc_fn)(size_t first_dim, size_t bytes, void *user);

/* ---- library / lifecycle ------------------------------------------------------- */
int ddl_version(void);
/* "src=<sha1 of the engine sources, 16 hex> arch=gfx950": which sources this library was built
 * from (tests rebuild a stale library rather than test it). */
const char *ddl_build_info(void);
const char *ddl_last_error(void);
const char *ddl_dtype_name(int dtype);
size_t ddl_dtype_size(int dtype); /* 0 for unsupported */

/* RCCL bootstrap id (128 bytes). Rank 0 creates it and the launcher distributes it. */
int ddl_get_unique_id(void *out, size_t len);
/* Creates the world communicator for this process (one process per GPU). */
int ddl_init(int rank, int size, int device, const void *unique_id, size_t len);

/* Same, for a single-process world (size 1); no RCCL involved. */
int ddl_init_single(int device);
/* Optional control channel for keyed requests at size > 1: TCP links in a star around rank 0
 * (3 hops per negotiation round at any size), replacing the MPI p2p token ring
 * (MPIRingTokenCommunication.cc:29-102) with the same token header. ddl_control_listen opens a
 * listener and returns "ip:port"; ddl_control_connect takes every rank's endpoint, separated by
 * ';', in rank order. */
int ddl_control_listen(char *endpoint_out, size_t len);
int ddl_control_connect(const char *endpoints);
/* Negotiation rounds so far by token form: ids as strings, or as indices into the table of ids
 * agreed in earlier rounds (a repeated key set, e.g. every training step's gradients). */
int ddl_control_stats(long long *string_rounds, long long *cached_rounds);
int ddl_finalize(void);
int ddl_is_initialized(void);

/* Tunables: "algo" (0 multi-ring, 1 direct all-to-all, 2 one-shot, 3 gather-fold: one
 * ncclAllGather then the rank-order fold, 4 direct-gather: the direct reduce-scatter then one
 * in-place ncclAllGather of the reduced chunks when they are equal), "slice_bytes", "rings", "max_slices",
 * "fusion_threshold_bytes", "log_level", "cycle_time_us", "host_chunk_bytes" (host-staged
 * transfers move in chunks of this size, default 32 MiB), "tune",
 * "host_copy_threads" (memcpy workers of the keyed host staging), "host_zero_copy" (1, default:
 * a keyed host allreduce plan whose outputs are all pinned and mapped on the device — torch
 * pin_memory, hipHostMalloc, hipHostRegister — is unpacked by the fusion kernel straight into
 * them over PCIe, no D2H copy or host memcpy; 0: always stage through the pinned slots; the
 * read-only "host_zero_copy_plans" counts the plans that took that path),
 * "host_numa_bind" (1, default: the handler's engine thread and copy threads bind to the CPUs of
 * the GPU's NUMA node, where pinned host memory lives; 0: placement left to the OS),
 * "host_register_cache_bytes" (0, default = off; > 0: pageable host tensors of keyed requests
 * are hipHostRegister'ed once and the registrations kept, least recently used out past this many
 * bytes, so repeated allreduce(cpu_tensor) calls take the pinned paths — a cached range must be
 * released with ddl_host_unregister before its memory is freed (the torch mirror does this for
 * the tensors it submits); setting it to 0 unregisters every cached range at once, after
 * ddl_wait_all; read-only statistics "host_registered_bytes", "host_register_hits",
 * "host_register_failures", "host_unregistered_ranges"), the read-only timeline of keyed host plans "host_pack_us" / "host_wait_us" /
 * "host_unpack_us" (microseconds the engine thread spent packing chunks, waiting for a pinned
 * slot's DMA / device work, waiting for the unpack lane — staged results are unpacked by their own
 * copy threads while the next chunks are packed), "capture_mode" (0, default: inside a
 * hipGraph capture the program is posted serially on the captured stream — one chain; 2: as a
 * single-stream DAG, every op on the captured stream with its dependencies set explicitly, which
 * keeps the recv / reduce / send overlap in the graph; r03's 1, the forked comm / compute
 * streams, crashed HIP 7.0's hipStreamEndCapture and is refused since r04 — DESIGN §9; so is its
 * older key "capture_forked"), "compute_cu_mask" (0,
 * default: all CUs; 8 / 4 / 2: the compute streams of multi-rank executors and handlers — the
 * reduce / fold / pack kernels that overlap RCCL's send / recv kernels — avoid every 8th / 4th /
 * 2nd CU, which stay free for RCCL; each masked stream takes a hardware queue of its own; read
 * when a communicator's executor / handler is created), "fold_form" (0, default:
 * the N-input fold in its run form from 4 MiB chunks of 7+ inputs, its tile form otherwise; 1 /
 * 2: always the tile / run form), "rccl_min_ctas" / "rccl_max_ctas" (0, default: RCCL's own
 * choice, NCCL_CONFIG_UNDEF_INT; 1..256: ncclConfig_t.minCTAs / maxCTAs of every RCCL
 * communicator created afterwards — ddl_init's ncclCommInitRankConfig, ddl_comm_split's and the
 * keyed data plane's ncclCommSplit — bounding its channel count and with it the p2p channels the
 * direct schedule's concurrent sends and receives spread over; shared tunables),
 * "queue_isolation" (0, default: every engine stream at the default priority; 1: the streams of
 * multi-rank RCCL communicators are created in three stream-priority classes, each of which HIP
 * maps to a pool of in-order hardware queues of its own — the world's direct collectives at the
 * default priority, the world's keyed data plane at the greatest, split communicators at the
 * least — so one communicator's queued RCCL kernels cannot hold another's behind them; env
 * DDL_QUEUE_ISOLATION seeds it; read when a communicator is created; local),
 * "fusion_pipeline_bytes" (keyed fusion plans above this run as a pack / allreduce / unpack
 * pipeline of sub-plans of at most this size; 0 = unpipelined), "one_rank_shortcut" (1: a
 * one-rank world skips the keyed data plane; 0: runs it, for tests), "pipeline_rounds" (1,
 * default: a completion thread fires a keyed round's done() calls as its plans land while the
 * engine thread negotiates the next round; 0: each round is waited for first), "reference_order" (1,
 * default: every allreduce sum equals the reference's MPI_Allreduce — MPICH 3.3.2 — bit for
 * bit: the direct and one-shot folds add the P inputs in rank order in MPICH's tree, picked by
 * the message size, and "algo" 0 runs as the direct schedule at P > 2; 0: ring order and left
 * folds, within (P-1)·u·Σ|x| of the reference).
 * With "tune" = 1 (default) a communicator of P > 1 ranks picks the schedule (algo, rings,
 * slice size) per bucket-size class (floor(log2 bytes)) the first time it sees that class: a
 * collective timing of a fixed candidate list on scratch buffers, max over ranks, argmin.
 * The shared tunables (algo, slice_bytes, rings, max_slices, fusion_threshold_bytes, tune,
 * fusion_pipeline_bytes, reference_order, host_chunk_bytes, rccl_min_ctas, rccl_max_ctas) must
 * be equal on every rank of a
 * communicator. Direct collectives: the ranks exchange a hash of them at a communicator's first
 * collective and at the next collective after this rank's values changed; a mismatch found there
 * fails that collective on every rank with DDL_STATUS_CONFIG_MISMATCH instead of building
 * different programs. That exchange is itself collective, so it is only matched when EVERY rank
 * changes its shared values between the same two collectives (to equal or different values);
 * changing them on some ranks only, after the first collective, is unsupported — those ranks post
 * an exchange the others never match, and the communicator hangs (there is no per-collective
 * check: it would cost a host-synchronising exchange on every call). Keyed rounds carry each
 * rank's hash in their tokens, so they detect any difference, one-sided included.
 * A change of the shared tunables drops the tuned choices; the other keys are per process. */
int ddl_set_config(const char *key, long long value);
long long ddl_get_config(const char *key);

/* How the ranks of communicator `id` are connected: *kind 0 = one rank (no transport), 1 = RCCL
 * (*ranks = ncclCommCount of its RCCL communicator), 2 = the test transport (*ranks = size). */
int ddl_comm_transport(ddl_communicator_id id, int *kind, int *ranks);

/* ---- reference c_api.h surface ----------------------------------------------------- */
int communicator_rank(ddl_communicator_id id);
int communicator_size(ddl_communicator_id id);
ddl_communicator_id world_communicator(void);
ddl_communicator_id split_communicator(ddl_communicator_id id, int color, int key);
void detach_communicator(ddl_communicator_id id);
void py_info(const char *log_str);
void py_debug(const char *log_str);
void py_error(const char *log_str);

/* ---- data plane ---------------------------------------------------------------------- */
/* recv = SUM over ranks of send (elementwise), bit for bit the reference's MPI_Allreduce (MPICH
 * 3.3.2's order) with reference_order 1. The schedule is the tuned one for the bucket's size
 * class: by default at P > 2 the direct reduce-scatter (slices of every chunk to every peer over
 * RCCL send/recv, one HIP fold per slice in MPICH's tree) + allgather; one-shot / gather-fold for
 * small buckets; at P = 2 the ring. recv may equal send (in place). Stream-ordered: no host
 * synchronisation (except the first bucket of a size class, which the autotuner times). */
int ddl_allreduce(ddl_communicator_id id, const void *send, void *recv, size_t elements,
                  int dtype, int op, void *hip_stream);

/* Grouped form of ddl_allreduce for `count` buckets of one dtype (MI355X extension: a DDP-style
 * bucket list in one call): recvs[b] = SUM over ranks of sends[b] (elements[b] each; in place when
 * recvs[b] == sends[b]); with reference_order 1 (the default) bit for bit what ddl_allreduce
 * gives each bucket on its own (both are MPICH's order for the bucket's own size); with
 * reference_order 0 each bucket is summed in the batch schedule's order (direct: rank-order fold;
 * one-shot: left fold), which may differ in the last bits from the ring or other schedule a solo
 * ddl_allreduce of that bucket's size class was tuned to. One program
 * for all buckets — tick by tick one RCCL group carries every bucket's slices and the folds of up
 * to 8 buckets share a kernel launch — instead of a program, two or more groups and a fold launch
 * per bucket. The schedule is the one tuned for the largest bucket (direct, or one-shot for small
 * buckets). Stream-ordered; collective: every rank passes the same count and element counts. */
int ddl_allreduce_batch(ddl_communicator_id id, int count, const void *const *sends, void *const *recvs,
                        const size_t *elements, int dtype, int op, void *hip_stream);

/* Communicator::broadcast (reference Communicator.h:81-92, MPI_Bcast at MPICommunicator.cc:77-90):
 * root's `elements` of `buf` into every rank's `buf`. Scatter + direct allgather over RCCL
 * send/recv (each xGMI link out of the root carries 2S/P, not S). Stream-ordered. */
int ddl_broadcast(ddl_communicator_id id, void *buf, size_t elements, int dtype, int root, void *hip_stream);
/* Communicator::allgather, per-rank counts (Communicator.h:50-66, MPI_Allgatherv at
 * MPICommunicator.cc:31-60): rank q's recv_counts[q] elements land at recv + displs[q] (in
 * elements) on every rank; send_elements must equal recv_counts[rank]. Stream-ordered. */
int ddl_allgatherv(ddl_communicator_id id, const void *send, size_t send_elements, void *recv,
                   const size_t *recv_counts, const size_t *displs, int dtype, void *hip_stream);
/* Communicator::allgather, equal counts (Communicator.h:68-79): rank q's block at q*recv_elements. */
int ddl_allgather(ddl_communicator_id id, const void *send, size_t send_elements, void *recv,
                  size_t recv_elements, int dtype, void *hip_stream);

/* Host-resident buckets (the reference's deployment case: CPU tensors behind the MPI buffers,
 * MPIRingTokenCommunication.cc:548-733): chunked H2D -> ddl_allreduce -> D2H pipeline on three
 * streams ("host_chunk_bytes", default 32 MiB; 4 chunk slots in HBM in flight). Pageable memory is
 * registered for the call; pinned memory avoids that cost. Synchronous: returns when `recv`
 * holds the result. Collective: every rank calls it with the same element count. */
int ddl_allreduce_host(ddl_communicator_id id, const void *send, void *recv, size_t elements,
                       int dtype, int op);

/* Autotuner record for the size class of `bucket_bytes` on communicator `id`: *chosen = index
 * of the schedule in use (-1 = class not tuned yet), *count = candidates; for the first
 * max_candidates of them configs[4i..4i+3] = {algo, rings, slice_bytes, max_slices} and
 * ms[i] = mean time per allreduce (max over ranks). configs/ms may be NULL. */
int ddl_tune_result(ddl_communicator_id id, size_t bucket_bytes, int *chosen, int *count,
                    long long *configs, float *ms, int max_candidates);
/* Keyed asynchronous request (TF op Allreduce semantics): registered under `key`,
 * negotiated across ranks, fused by dtype in lexicographic key order, then `done` fires.
 * `in`/`out` must stay valid until `done`. Work is ordered after `hip_stream`'s current
 * position; `done` fires once `out` is final.
 * Keyed rounds and direct collectives on one communicator (the reference's MPI_THREAD_MULTIPLE,
 * MPIBackend.cc:77-86): a communicator with a token ring reduces its keyed rounds on a private
 * RCCL communicator, and every round is placed after the same number of the communicator's
 * direct collectives (ddl_allreduce[_batch], ddl_broadcast, ddl_allgather[v], ddl_allreduce_host,
 * split_communicator) on every rank, so both RCCL communicators see their work in one order
 * everywhere. A direct collective issued while a round is being placed waits for the placement
 * (one negotiation). If the communicator's handler stops on an error (a control link lost, a
 * token-protocol fault), its pending requests complete with that status, and from then on every
 * direct collective on the communicator returns it too instead of waiting for a placement that
 * can no longer happen: the communicator is unusable, finalize and re-initialise. */
int ddl_allreduce_submit(ddl_communicator_id id, const char *key, const void *in, void *out,
                         size_t elements, int dtype, int op, void *hip_stream,
                         ddl_done_fn done, void *user);
/* Keyed broadcast (TF op Broadcast, op/tensorflow/BroadcastOp.cc; TensorBroadcastRequest.h:13-40):
 * `out` on every rank receives root's `in`. Negotiated and fused like allreduce requests
 * (dtype groups, plans, MPIRingTokenCommunication.cc:367-419); requests of different roots
 * run as separate groups. */
int ddl_broadcast_submit(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                         int dtype, int root, void *hip_stream, ddl_done_fn done, void *user);
/* Keyed allgather (TF op Allgather, op/tensorflow/AllgatherOp.cc; TensorAllgatherRequest.h):
 * `in` holds first_dim rows of row_elements; the output holds every rank's rows in rank order
 * (first dims may differ per rank, row_elements may not). Once the gathered first dim is known
 * `alloc(total_rows, bytes, user)` supplies the output buffer, then `done` fires
 * (MPIRingTokenCommunication.cc:160-364). */
int ddl_allgather_submit(ddl_communicator_id id, const char *key, const void *in, size_t first_dim,
                         size_t row_elements, int dtype, void *hip_stream, ddl_alloc_fn alloc,
                         ddl_done_fn done, void *user);
/* Batch form of ddl_allreduce_submit: registers `count` keyed requests at once (one input-ready
 * event on hip_stream, one wake-up of the engine thread); users[i] (or NULL) is passed to done for
 * request i. All-or-nothing: a duplicate key rejects the whole batch. */
int ddl_allreduce_submit_batch(ddl_communicator_id id, int count, const char *const *keys,
                               const void *const *ins, void *const *outs, const size_t *elements,
                               const int *dtypes, int op, void *hip_stream, ddl_done_fn done,
                               void *const *users);
/* The same four submissions with the memory kind of in / out (ddl_memory). Host buffers are
 * ready at submission (no stream wait) and must stay valid until done; a keyed allgather's alloc
 * then returns host memory. Host and device requests of one dtype fuse into separate plans
 * (device groups first); with only host requests the plans are the reference's. */
int ddl_allreduce_submit_mem(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                             int dtype, int op, int memory, void *hip_stream, ddl_done_fn done, void *user);
int ddl_allreduce_submit_batch_mem(ddl_communicator_id id, int count, const char *const *keys,
                                   const void *const *ins, void *const *outs, const size_t *elements,
                                   const int *dtypes, int op, int memory, void *hip_stream, ddl_done_fn done,
                                   void *const *users);
int ddl_broadcast_submit_mem(ddl_communicator_id id, const char *key, const void *in, void *out, size_t elements,
                             int dtype, int root, int memory, void *hip_stream, ddl_done_fn done, void *user);
int ddl_allgather_submit_mem(ddl_communicator_id id, const char *key, const void *in, size_t first_dim,
                             size_t row_elements, int dtype, int memory, void *hip_stream, ddl_alloc_fn alloc,
                             ddl_done_fn done, void *user);
/* Blocks until every request submitted on `id` so far has completed. */
int ddl_wait_all(ddl_communicator_id id);

/* Completion groups (MI355X extension, csrc/completion.cpp): a native done callback for bindings
 * whose own callbacks are costly — a Python done() per request costs ~10 us of interpreter time,
 * 40-60 ms per 4096-tensor batch. Create a group of `count` slots, pass ddl_completion_done as the
 * ddl_done_fn and slot i's pointer (ddl_completion_slots: `count` of them from `first` into out)
 * as request i's `user`; done() stores the status in slot i and wakes its waiters.
 * ddl_completion_wait blocks (no callback into the binding) until slot `index` completed or
 * `timeout_s` (< 0: no limit; 0: a test) passed: DDL_STATUS_OK with *status = the request's
 * status, or DDL_STATUS_ERROR_UNKNOWN while it is still pending. ddl_completion_poll copies the
 * first `count` slots' statuses (-1: pending; statuses may be NULL when count is 0) and returns
 * how many slots are pending. ddl_completion_destroy is the owner's release: the group is freed
 * once every slot has completed too, so done() calls after it stay safe. */
void *ddl_completion_create(int count);
int ddl_completion_slots(void *group, int first, int count, void **out);
void ddl_completion_done(int status, void *user);
int ddl_completion_wait(void *group, int index, double timeout_s, int *status);
int ddl_completion_poll(void *group, int *statuses, int count);
void ddl_completion_destroy(void *group);

/* With "host_register_cache_bytes" > 0: the host range [ptr, ptr + bytes) is about to be freed —
 * call this BEFORE freeing (munmap / free / the framework's deallocator) any host tensor that was
 * part of a keyed request. Every cached registration overlapping the range is dropped (at once,
 * or — while the engine is posting a host plan — before its next cache lookup), so a later
 * tensor placed at the same address is registered afresh instead of being taken for the old,
 * now unmapped pages (a device access through the stale registration faults). The torch mirror
 * (ddl.torch.tensor_communicate) calls it from a finalizer of every host tensor it submits while
 * the cache is on. A no-op for ranges that are not cached. */
int ddl_host_unregister(const void *ptr, size_t bytes);

/* Measurement: bracket every reduce-kernel launch of ddl_allreduce on `id` with timing
 * events on the engine's compute stream (the stream the kernel runs on). ddl_kernel_stats
 * waits for the recorded events and returns launches, algorithmic HBM bytes (per launch: a
 * two-input ring step 3 * elements * sizeof(T); a fold of nb received inputs
 * (nb + 2) * elements * sizeof(T) — the own input, the nb inputs, one write) and summed kernel
 * milliseconds, then resets. */
int ddl_kernel_timing(ddl_communicator_id id, int on);
int ddl_kernel_stats(ddl_communicator_id id, long long *launches, double *bytes, double *ms);

#ifdef __cplusplus
}
#endif

/* The test / diagnostic entry points (ddl_init_test_transport, ddl_p2p_op, ddl_control_negotiate*,
 * ddl_allreduce_variant, ddl_reduce_*, ddl_pack / ddl_unpack, ddl_local_*, ddl_testing_*,
 * ddl_rccl_loopback_*, the schedule introspection) are declared in ddl_amd_testing.h and exported
 * only by lib/libddl_amd_testing.so (the same engine objects plus the harness); lib/libddl_amd.so
 * exports exactly this header. Define DDL_AMD_WITH_TESTING_API before including this header to
 * get both (and link the testing library). ddl_init_test_transport also needs
 * DDL_ALLOW_TEST_TRANSPORT=1 in the environment. */
#ifdef DDL_AMD_WITH_TESTING_API
#include "ddl_amd_testing.h"
#endif

#endif /* DDL_AMD_H */
