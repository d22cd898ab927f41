// fusion.h — the data plane of one multi-request fusion plan: pack -> allreduce -> unpack.
//
// The reference copies every request of a plan into one MPI buffer, reduces it and copies it back
// (executeCommunicatePlan_, MPIRingTokenCommunication.cc:548-733). Here the copies are the pack /
// unpack kernels (SegmentCopier, pack.hip), and a plan above `cap` bytes (config
// fusion_pipeline_bytes) is cut into sub-plans J of at most that size (segments split at 256-byte
// multiples) over two fusion buffers:
//   side:    pack 0, pack 1, unpack 0, pack 2, unpack 1, ...   (unpack j waits allreduce j)
//   stream:          ar 0,   ar 1,     ar 2, ...               (ar j waits pack j)
// so the pack of j+1 and the unpack of j-1 run under the allreduce of j. Buffer j%2 is reused by
// pack j+2, issued on `side` after unpack j. Each sub-plan is an allreduce of its own; it is told
// the whole plan's message size, so with reference_order every sub-plan folds in the order MPICH
// uses for the whole plan and the cut changes no bit.
//
// One FusionPipe per engine thread: the keyed handler owns one (handler.cpp) and the thread world
// one per virtual rank (executor.cpp, ddl_testing_thread_fused_allreduce), so the same code runs
// under the production executor on one GPU.
#pragma once

#include <functional>
#include <vector>

#include "common.h"

namespace ddl {

class FusionPipe {
public:
    FusionPipe() = default;
    ~FusionPipe();
    FusionPipe(const FusionPipe &) = delete;
    FusionPipe &operator=(const FusionPipe &) = delete;

    // Fusion buffer i (0 or 1) of at least `need` bytes; an outgrown buffer is retired, not freed
    // (common.h retire_device): earlier uses of it may still be in flight.
    void *ensure(int i, size_t need, hipStream_t stream);
    // elems of the plan's dtype in `buf`, reduced in place on the pipe's stream; `message_bytes`
    // = the whole plan's unpadded bytes (the reference's MPI_Allreduce message)
    using Allreduce = std::function<void(void *buf, size_t elems, size_t message_bytes)>;
    // pack -> allreduce -> unpack of srcs[i] -> dsts[i] (bytes[i] each) on `stream`, pipelined in
    // sub-plans above `cap` bytes (0: never)
    void run(const std::vector<const void *> &srcs, const std::vector<void *> &dsts,
             const std::vector<size_t> &bytes, int dtype, size_t cap, hipStream_t stream, const Allreduce &ar);
    size_t subplans() const { return last_subplans_; }  // of the last run

    SegmentCopier copier;
    // hardware-queue class of the side stream (executor.h QueueClass; set by the owning handler)
    QueueClass qc = QueueClass::kPooled;

private:
    hipEvent_t event_(size_t i);
    void *buf_[2] = {nullptr, nullptr};
    size_t cap_[2] = {0, 0};
    hipStream_t side_ = nullptr;
    std::vector<hipEvent_t> events_;
    size_t last_subplans_ = 0;
};

}  // namespace ddl
