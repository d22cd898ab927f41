/* The reference's CPU op, driven from plain C through the deployment library alone
 * (include/ddl_amd.h, lib/libddl_amd.so): what a native binding of the reference — its TF
 * AllreduceOp (op/tensorflow/AllreduceOp.cc:17-68, a DEVICE_CPU kernel) or a cgo / JNI caller —
 * does, with host buffers as the reference's tensors are.
 *
 *   1. the synchronous host-resident allreduce (replaces Communicator::allreduce ->
 *      MPI_Allreduce, MPICommunicator.cc:14-28): C1's fp32[1024] bucket, x = rank + i;
 *   2. keyed requests on host memory (the op's ComputeAsync -> handleRequest, AllreduceOp.cc:32-66):
 *      a batch of mixed-dtype buckets under TF-style op names, completed through a completion
 *      group (the library's own done function: no callback into the binding), waited per slot;
 *   3. the reference's c_api.h names (world_communicator, communicator_rank / _size,
 *      split_communicator, detach_communicator).
 *
 * One process, one GPU (a size-1 world): the sum over one rank is the input itself, which the
 * program checks bit for bit; `one_rank_shortcut` = 0 makes the engine run the whole data plane
 * anyway (pinned staging, H2D, the fused allreduce, D2H). Build (tests/test_examples_cpu.py does):
 *
 *   gcc -std=c99 -Wall -Wextra -Werror -Iinclude examples/c_host_allreduce.c \
 *       -Lexperiment-distributed-deep-learning_amd/lib -lddl_amd \
 *       -Wl,-rpath,<abs>/experiment-distributed-deep-learning_amd/lib -o c_host_allreduce
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ddl_amd.h"

#define CHECK(call)                                                                    \
    do {                                                                               \
        int st_ = (call);                                                              \
        if (st_ != DDL_STATUS_OK) {                                                    \
            fprintf(stderr, "%s failed: status %d: %s\n", #call, st_, ddl_last_error()); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

enum { kBuckets = 6 };

int main(int argc, char **argv) {
    const int device = argc > 1 ? atoi(argv[1]) : 0;
    CHECK(ddl_init_single(device));
    CHECK(ddl_set_config("one_rank_shortcut", 0));
    const ddl_communicator_id world = world_communicator();
    const int rank = communicator_rank(world), size = communicator_size(world);
    if (world == 0 || rank != 0 || size != 1) {
        fprintf(stderr, "world %lld: rank %d of %d\n", (long long)world, rank, size);
        return 1;
    }

    /* 1. C1: fp32[1024], synchronous, host buffers */
    float send[1024], recv[1024];
    for (int i = 0; i < 1024; ++i) send[i] = (float)(rank + i);
    memset(recv, 0, sizeof recv);
    CHECK(ddl_allreduce_host(world, send, recv, 1024, DDL_FLOAT, DDL_ALLREDUCE_OP_SUM));
    if (memcmp(send, recv, sizeof send) != 0) {
        fprintf(stderr, "ddl_allreduce_host: the one-rank sum differs from the input\n");
        return 1;
    }

    /* 2. keyed host requests, one batch, a completion group */
    static const size_t elements[kBuckets] = {1, 1000, 4099, 65536, 300000, 7};
    static const int dtypes[kBuckets] = {DDL_FLOAT, DDL_DOUBLE, DDL_INT32, DDL_FLOAT, DDL_INT64, DDL_HALF};
    const char *keys[kBuckets] = {"dense/kernel:0", "dense/bias:0", "embedding:0", "conv1/kernel:0",
                                  "step_counts:0", "scale:0"};
    void *ins[kBuckets], *outs[kBuckets], *users[kBuckets];
    for (int b = 0; b < kBuckets; ++b) {
        const size_t bytes = elements[b] * ddl_dtype_size(dtypes[b]);
        ins[b] = malloc(bytes);
        outs[b] = malloc(bytes);
        if (!ins[b] || !outs[b]) return 1;
        for (size_t j = 0; j < bytes; ++j) ((unsigned char *)ins[b])[j] = (unsigned char)(j * 31 + b);
        if (dtypes[b] == DDL_HALF)  /* finite fp16 values only: 0x3c00 | low bits */
            for (size_t j = 0; j < elements[b]; ++j) ((uint16_t *)ins[b])[j] = (uint16_t)(0x3c00 | (j & 0x3ff));
        memset(outs[b], 0xff, bytes);
    }
    void *group = ddl_completion_create(kBuckets);
    if (!group) return 1;
    CHECK(ddl_completion_slots(group, 0, kBuckets, users));
    CHECK(ddl_allreduce_submit_batch_mem(world, kBuckets, keys, (const void *const *)ins, outs, elements, dtypes,
                                         DDL_ALLREDUCE_OP_SUM, DDL_MEMORY_HOST, NULL, ddl_completion_done,
                                         users));
    for (int b = 0; b < kBuckets; ++b) {
        int status = -1;
        CHECK(ddl_completion_wait(group, b, 60.0, &status));
        CHECK(status);
        if (memcmp(ins[b], outs[b], elements[b] * ddl_dtype_size(dtypes[b])) != 0) {
            fprintf(stderr, "keyed request %s: the one-rank sum differs from the input\n", keys[b]);
            return 1;
        }
    }
    if (ddl_completion_poll(group, NULL, 0) != 0) return 1;
    ddl_completion_destroy(group);

    /* 3. a split of the world, used and detached */
    const ddl_communicator_id sub = split_communicator(world, 0, rank);
    if (sub == 0 || communicator_size(sub) != 1) {
        fprintf(stderr, "split_communicator: %s\n", ddl_last_error());
        return 1;
    }
    memset(recv, 0, sizeof recv);
    CHECK(ddl_allreduce_host(sub, send, recv, 1024, DDL_FLOAT, DDL_ALLREDUCE_OP_SUM));
    if (memcmp(send, recv, sizeof send) != 0) return 1;
    detach_communicator(sub);

    for (int b = 0; b < kBuckets; ++b) {
        free(ins[b]);
        free(outs[b]);
    }
    CHECK(ddl_finalize());
    printf("c_host_allreduce: ok (%s; C1 fp32[1024] host allreduce, %d keyed host buckets, split)\n",
           ddl_build_info(), kBuckets);
    return 0;
}
