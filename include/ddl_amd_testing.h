/*
 * ddl_amd_testing.h — test, measurement and diagnostic entry points of libddl_amd.so.
 *
 * NOT the deployment surface: a framework binding uses include/ddl_amd.h only. These entry
 * points exist so that the engine's parts can be checked and measured on their own (and on a
 * one-GPU box): the host-callback test transport, P virtual ranks on one GPU (copies or a
 * one-rank RCCL communicator standing in for the mesh), the reduce / fold / pack kernels as
 * launched by the schedules, program and plan introspection, and standalone token channels.
 * tests/, tools/ and bench.py use them; nothing on the product path calls them.
 */
#ifndef DDL_AMD_TESTING_H
#define DDL_AMD_TESTING_H

#include "ddl_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- test transport ------------------------------------------------------------------
 * A world communicator whose point-to-point groups and
 * the autotuner's max-reduce go through host callbacks instead of RCCL, so the multi-process
 * engine — control channel, keyed handler, fusion, schedules, streams, kernels — can run as
 * several processes sharing one GPU (RCCL refuses two ranks on one device). `comm_tag` names
 * the communicator (0 = world; splits agree on theirs), so the callbacks can keep concurrent
 * communicators apart. The engine synchronises the group's stream, stages every
 * send into host memory, calls the group callback — which must complete the whole exchange on
 * the host buffers before it returns, 0 = success — and copies the received host buffers to
 * the device. `peer` is a world rank (splits map their ranks); `comm_tag` differs between any two
 * communicators that share a pair of ranks. `max` is no longer called (the autotuner agrees
 * through `group`); it may be NULL.
 * Refused (DDL_STATUS_INVALID_ARGUMENT) unless the environment sets DDL_ALLOW_TEST_TRANSPORT=1:
 * its host-synchronised groups must never stand in for RCCL by accident. */
typedef struct ddl_p2p_op {
    int send;     /* 1 send, 0 receive */
    int peer;     /* world rank of the peer */
    int tag;      /* matches a send with its receive inside one group (posting order per tag) */
    void *ptr;    /* host staging buffer of `bytes` */
    size_t bytes;
} ddl_p2p_op;
typedef int (*ddl_test_group_fn)(long long comm_tag, const ddl_p2p_op *ops, int count, void *user);
typedef int (*ddl_test_max_fn)(long long comm_tag, float *values, int count, void *user);
int ddl_init_test_transport(int rank, int size, int device, ddl_test_group_fn group, ddl_test_max_fn max,
                            void *user);

/* The order between keyed rounds and direct collectives on communicator `id`: the direct
 * collectives issued so far and the release point of each keyed round (the round ran after that
 * many direct collectives; the first min(count, max_releases) of the last 2048-4096 rounds). */
int ddl_testing_round_log(ddl_communicator_id id, long long *user_collectives, long long *releases, int max_releases,
                          int *count);
/* The direct path's shared-config agreement on the host alone (no device, no communicator): this
 * rank's Config hash to every other rank through `group` (one group of sends and receives,
 * ddl_p2p_op over host buffers), then the comparison the engine makes at a communicator's first
 * collective — DDL_STATUS_CONFIG_MISMATCH on every rank when any two differ. */
int ddl_testing_agree_config(int rank, int size, ddl_test_group_fn group, void *user);

/* Control channel without a world communicator (tools / CPU tests of the token protocol). */
int ddl_control_connect_ranked(int rank, int size, const char *endpoints);
/* One negotiation round over the control channel with a fixed key set ('\n'-separated):
 * writes the agreed keys ('\n'-separated, lexicographic) to out. Same protocol as the
 * keyed-request handler, without the data plane. */
int ddl_control_negotiate(const char *keys, char *out, size_t len);

/* Several independent token rings in one process (tools, CPU tests of per-communicator rings):
 * _open listens and returns a handle (0 on failure) and "ip:port"; _connect joins the ring of
 * `size` ranks; _negotiate is ddl_control_negotiate on that ring. Every communicator of size > 1
 * made by split_communicator owns such a ring (RingTokenCommunicateController.cc:53-79). */
long long ddl_control_channel_open(char *endpoint_out, size_t len);
int ddl_control_channel_connect(long long channel, int rank, int size, const char *endpoints);
int ddl_control_channel_negotiate(long long channel, const char *keys, char *out, size_t len);
int ddl_control_channel_close(long long channel);

/* Comparator entry for measurement: variant 0 = the engine's ring (= ddl_allreduce),
 * variant 1 = RCCL's built-in ncclAllReduce on the same communicator. */
int ddl_allreduce_variant(ddl_communicator_id id, const void *send, void *recv, size_t elements,
                          int dtype, int op, void *hip_stream, int variant);


/* The same tuning procedure on ddl_local_ring_allreduce's P virtual ranks (one GPU, copies
 * for the transport; no cross-rank agreement needed): a test/diagnostic entry. */
int ddl_local_tune(int nranks, size_t elements, int dtype, void *hip_stream, int *chosen, int *count,
                   long long *configs, float *ms, int max_candidates);


/* ---- HIP kernels exposed for measurement and tests ----------------------------------- */
/* acc[i] = acc[i] + in[i]  (the per-hop reduce of the ring). */
int ddl_reduce_local(void *acc, const void *in, size_t elements, int dtype, void *hip_stream);
/* out[i] = a[i] + b[i]; out may alias a or b. */
int ddl_reduce_sum2(void *out, const void *a, const void *b, size_t elements, int dtype,
                    void *hip_stream);
/* Kernel variant selection for measurement (bit set; -1 = the engine's default):
 * 1 = non-temporal loads of a, 2 = non-temporal loads of b, 4 = non-temporal stores,
 * 8 = operand b staged through LDS by global_load_lds_dwordx4, 16 = write-through (sc0 sc1)
 * stores of out (ignored with 8). */
int ddl_reduce_sum2_variant(int variant, void *out, const void *a, const void *b,
                            size_t elements, int dtype, void *hip_stream);
/* The direct schedule's fold: out[i] = a[i] + ins[0][i] + ... + ins[nb-1][i], 1 <= nb <= 15,
 * left to right; fp16/bf16 accumulate in fp32 and round once. out may alias a. */
int ddl_reduce_fold(void *out, const void *a, const void *const *ins, int nb, size_t elements, int dtype,
                    void *hip_stream);
/* The same fold in a given order of the inputs x_0 = a, x_1 = ins[0], ...: order 0 left to right,
 * 1 MPICH 3.3.2's MPI_Allreduce order above 2048 bytes (the first 2*rem inputs folded in pairs,
 * then a pairwise tree over the pof2 leaves), 2 its order up to 2048 bytes (binomial tree).
 * fp16/bf16 fold left in fp32 whatever the order. The reference-order schedules launch this. */
int ddl_reduce_fold_ordered(void *out, const void *a, const void *const *ins, int nb, size_t elements, int dtype,
                            int order, void *hip_stream);

/* Up to 8 such folds in ONE launch (the grouped allreduce's batched fold; blockIdx.y = problem):
 * problem p computes outs[p] = as[p] + ins[p * nb + 0] + ... + ins[p * nb + nb - 1] over elements[p]
 * in `order`. No problem may read another's output. */
int ddl_reduce_fold_batch(int count, void *const *outs, const void *const *as, const void *const *ins, int nb,
                          const size_t *elements, int dtype, int order, void *hip_stream);

/* Fusion pack/unpack (device): gathers `count` segments into one contiguous buffer and
 * scatters it back (executeCommunicatePlan_'s memcpy in/out, MPIRingTokenCommunication.cc:548-733). */
int ddl_pack(void *dst, const void *const *srcs, const size_t *bytes, int count, void *hip_stream);
int ddl_unpack(void *const *dsts, const void *src, const size_t *bytes, int count,
               void *hip_stream);

/* ---- single-GPU rehearsal of the ring schedule --------------------------------------- */
/* Runs the exact per-rank ring schedule for `nranks` virtual ranks inside this process on
 * the current device, with device-to-device copies standing in for RCCL send/recv.
 * sends[r]/recvs[r] are rank r's buffers. Stream-ordered on hip_stream. */
int ddl_local_ring_allreduce(int nranks, const void *const *sends, void *const *recvs,
                             size_t elements, int dtype, int op, void *hip_stream);

/* ddl_allreduce_batch over P virtual ranks: sends[r * count + b] / recvs[r * count + b] are rank r's
 * bucket b of elements[b]. _local: device copies for the moves (LocalWorld); _thread: the
 * production executor per rank over the asynchronous thread fabric; _rccl_loopback: every matched
 * pair through RCCL (declared with the loopback below). */
int ddl_local_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                              const size_t *elements, int dtype, void *hip_stream);
int ddl_testing_thread_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                                       const size_t *elements, int dtype, void *hip_stream);

/* Broadcast / allgatherv of P virtual ranks on one GPU (as ddl_local_ring_allreduce). */
int ddl_local_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype, void *hip_stream);
int ddl_local_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                         const size_t *displs, int dtype, void *hip_stream);

/* ---- thread world: the production executor, asynchronously --------------------------------
 * P threads, each driving its own RingExecutor (the class ddl_allreduce runs at N > 1) over an
 * in-process transport with RCCL's asynchronous contract: a group rendezvous with its peers only
 * on the host ENQUEUE; a receive is a stream wait on the sender's event plus a D2D copy; the
 * sender's stream waits for the receiver's copy event; nothing synchronises the host. Every
 * rank works on its own stream forked from / joined to hip_stream. sends[r] / recvs[r] / bufs[r]
 * are rank r's buffers; the schedule is the configured one (ddl_set_config "algo", ...). */
int ddl_testing_thread_allreduce(int nranks, const void *const *sends, void *const *recvs, size_t elements, int dtype,
                                 void *hip_stream);
int ddl_testing_thread_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype,
                                 void *hip_stream);
int ddl_testing_thread_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                                  const size_t *displs, int dtype, void *hip_stream);
/* The keyed path's multi-request plan on every virtual rank (the handler's FusionPipe: pack ->
 * allreduce -> unpack, cut into sub-plans above config "fusion_pipeline_bytes", two fusion buffers,
 * pack / unpack on a side stream), each sub-plan's allreduce through the rank's RingExecutor in the
 * whole plan's MPICH order. srcs[r * count + i] / dsts[r * count + i] are rank r's segment i of
 * bytes[i] bytes (whole elements of dtype); *subplans (may be NULL) = the sub-plans per rank. */
int ddl_testing_thread_fused_allreduce(int nranks, int count, const void *const *srcs, void *const *dsts,
                                       const size_t *bytes, int dtype, void *hip_stream, size_t *subplans);
/* Data movement of the thread worlds made from now on: rccl = 0 device copies (default); 1 every
 * matched send / receive pair goes through RcclTransport::group as a self send + self receive on
 * the RCCL loopback communicator (ddl_rccl_loopback_init first), posted on the receiver's stream
 * after its wait on the sender's event — the production executor, asynchronous, handing its bytes
 * to RCCL. *loopback_pairs (may be NULL) = pairs moved through RCCL so far by such worlds. */
int ddl_testing_thread_transport(int rccl, long long *loopback_pairs);
/* Fault injection for the keyed handler's error path: with on = 1, the next keyed round a member
 * rank joins closes that rank's control link right after it froze its user collectives for the
 * round (a link lost mid-round). Every rank's handler then stops, its pending requests complete
 * with an error, and later user collectives on the communicator return that error instead of
 * blocking behind the round that can no longer be placed. */
int ddl_testing_control_fault(int on);
/* Fault for the host staging loop: the next keyed host plan fails at chunk `chunk`
 * (its collective is not posted; -1 turns it off). The staged unpacks of the chunks before it
 * have all landed when the requests' done() reports the error. */
int ddl_testing_host_coll_fault(long long chunk);
/* A/B knob of the N-input fold's cache policy (reduce_kernels.hip fold_variant): 4 = plain loads +
 * write-through store, 5 = non-temporal loads + write-through store, -1 = the size rule. */
int ddl_testing_fold_variant(int variant);
/* Mutation for the ordering tests: RingExecutor skips the reduce wait (wait_reduce) of program
 * tick `tick` (-1 restores the product behaviour). A test that cannot see this is blind. */
int ddl_testing_drop_wait(int tick);
/* Happens-before tracing of the work the executors post (deptrace.h): _trace(1) clears the log
 * and starts it, _trace(0) stops it. _check replays the log with vector clocks (stream order plus
 * event record -> stream wait edges) and compares every pair of ops on different streams whose
 * byte ranges overlap, one of them writing: counts[0..4] = {ops, such conflicting pairs, pairs
 * ordered by the posted dependencies, ordered pairs with a reduce / fold on one side, unordered
 * pairs = races}; `report` gets the first races, one per line. Independent of timing and of how
 * streams share hardware queues. */
int ddl_testing_dep_trace(int on);
int ddl_testing_dep_check(long long *counts, char *report, size_t len);
/* The CUs enabled on an executor compute stream created with every `every`-th CU masked off
 * (config "compute_cu_mask"; 0 = unmasked), read back with hipExtStreamGetCUMask. */
int ddl_testing_compute_stream_cus(int every, int *enabled, int *total);
/* The stream priorities of a communicator's engine streams (config "queue_isolation", executor.h
 * QueueClass): prio[0] / prio[1] its executor's comm / compute stream, prio[2] its keyed
 * handler's stream, prio[3] its private keyed data-plane communicator's comm stream
 * (DDL_TESTING_NO_STREAM where that object does not exist yet). hipDeviceGetStreamPriorityRange
 * gives the meaning: lower is more urgent, 0 is the default. */
#define DDL_TESTING_NO_STREAM (-1000)
int ddl_testing_stream_priorities(ddl_communicator_id id, int *prio);
/* The chunk boundaries of a host-staged transfer (ddl_allreduce_host, the keyed handler's host
 * plans): whole chunks of chunk_bytes, the last one short. Writes min(count, cap) boundaries
 * cut[0] = 0 < ... < cut[count - 1] = total_bytes into cuts and sets *count. Pure host arithmetic
 * (no device). */
int ddl_testing_host_chunk_cuts(size_t total_bytes, size_t chunk_bytes, size_t *cuts, size_t cap, size_t *count);

/* ---- RCCL loopback: the production RCCL transport on one GPU (TEST / DIAGNOSTIC) ---------
 * A one-rank RCCL communicator (ncclGetUniqueId + ncclCommInitRank, the calls ddl_init makes at
 * size > 1) carries the matched send/recv pairs of P virtual ranks' programs as self-send /
 * self-recv pairs, posted through the engine's RcclTransport::group in matching order — the
 * data path that replaces MPI_Allreduce (MPICommunicator.cc:14-28) with RCCL doing the moves.
 * _split runs ncclCommSplit (MPICommunicator.cc:92-101) on the current loopback communicator;
 * the split becomes current (color < 0: *rank = -1, *size = 0, nothing changes). _max is the
 * autotuner's cross-rank agreement (ncclAllReduce(MAX)); _tune runs the autotuner with the
 * candidates over RCCL and that agreement. _stats: self pairs posted so far for P ranks. */
int ddl_rccl_loopback_init(int device);
int ddl_rccl_loopback_split(int color, int key, int *rank, int *size);
int ddl_rccl_loopback_allreduce(int nranks, const void *const *sends, void *const *recvs, size_t elements,
                                int dtype, void *hip_stream);
int ddl_rccl_loopback_allreduce_batch(int nranks, int count, const void *const *sends, void *const *recvs,
                                      const size_t *elements, int dtype, void *hip_stream);
int ddl_rccl_loopback_broadcast(int nranks, int root, void *const *bufs, size_t elements, int dtype,
                                void *hip_stream);
int ddl_rccl_loopback_allgatherv(int nranks, const void *const *sends, void *const *recvs, const size_t *counts,
                                 const size_t *displs, int dtype, void *hip_stream);
/* RcclTransport::allgather (ncclAllGather, the gather-fold schedule's transport) on the one-rank
 * loopback communicator: recv[0..bytes) = send. */
int ddl_rccl_loopback_allgather(const void *send, void *recv, size_t bytes, void *hip_stream);
int ddl_rccl_loopback_max(float *values, int count, void *hip_stream);
int ddl_rccl_loopback_tune(int nranks, size_t elements, int dtype, void *hip_stream, int *chosen, int *count,
                           long long *configs, float *ms, int max_candidates);
int ddl_rccl_loopback_stats(int nranks, long long *pairs);
int ddl_rccl_loopback_finalize(void);

/* ---- schedule introspection (host only, no GPU needed) -------------------------------- */
int ddl_ring_count(int nranks, int max_rings);
/* perm_out[p] = rank at ring position p (length nranks). */
int ddl_ring_perm(int nranks, int max_rings, int ring, int *perm_out);
/* Element range [begin, end) of (ring, chunk) in a bucket of `elements` of `dtype`. */
int ddl_chunk_range(size_t elements, int dtype, int nranks, int rings, int ring, int chunk,
                    size_t *begin, size_t *end);
/* Rings and reduce-scatter slices the schedule uses for a bucket under the current config. */
int ddl_ring_shape(size_t elements, int dtype, int nranks, int *rings, int *slices);
/* Rank `rank`'s ring program as rows of 8 int64:
 *   send/recv: {tick, 0=send|1=recv, peer, ring, buffer(0 in, 1 out, 2 staging), offset, count, wait_tick}
 *   reduce:    {tick, 2, -1, segment, 1 (out), offset, count, staging offset}  (out = in + staging)
 *   fold:      {tick, 3, nb, input i, 1 (out), offset, count, staging offset of input i}
 *              (direct schedule: out = in + input 0 + ... + input nb-1, fp16/bf16 in fp32)
 * Offsets and counts in elements. Host only. */
int ddl_ring_program(int rank, int nranks, size_t elements, int dtype, long long *ops_out,
                     size_t max_ops, size_t *nops);
/* Broadcast program of `rank` (buffer 1 = the broadcast buffer) and allgatherv program
 * (buffer 0 = send, 1 = recv), same row format; copy rows: {tick, 4, -1, -1, 1, dst offset,
 * count, src offset in buffer 0}. */
int ddl_broadcast_program(int rank, int nranks, int root, size_t elements, int dtype, long long *ops_out,
                          size_t max_ops, size_t *nops);
int ddl_allgather_program(int rank, int nranks, const size_t *counts, const size_t *displs, int dtype,
                          long long *ops_out, size_t max_ops, size_t *nops);
/* Fusion plans (requestBegin, elementBegin, requestEnd, elementEnd) over `count` requests of
 * one dtype group, capped at `limit` bytes (makeCollectiveCommunicatePlan,
 * MPIRingTokenCommunication.cc:495-546). plans_out holds 4*max_plans entries. */
int ddl_make_plans(const size_t *elements, const size_t *esizes, size_t count, size_t limit,
                   size_t *plans_out, size_t max_plans, size_t *nplans);

#ifdef __cplusplus
}
#endif

#endif /* DDL_AMD_TESTING_H */
