// rccl_api.h — RCCL entry points resolved at run time.
//
// The engine uses exactly one RCCL per process: the copy PyTorch already loaded (its
// libtorch_hip.so depends on librccl.so) when present, else the system librccl.so.1 — so a
// torch-based training script never ends up with two RCCL runtimes. Only types come from
// <rccl/rccl.h>; nothing links against RCCL.
#pragma once

#include <rccl/rccl.h>

namespace ddl {

struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    // optional (null when the loaded RCCL lacks it): needed only for a non-default ncclConfig_t
    ncclResult_t (*CommInitRankConfig)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t *, ncclConfig_t *) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GetVersion)(int *) = nullptr;
    ncclResult_t (*CommCount)(const ncclComm_t, int *) = nullptr;
    ncclResult_t (*CommUserRank)(const ncclComm_t, int *) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    const char *path = "";
};

// Loads (once) and returns the RCCL API; throws ddl::Error if RCCL cannot be loaded.
const RcclApi &rccl();

// Throws a DDL_STATUS_COMM_ERROR with the RCCL message when r != ncclSuccess.
void rccl_check(ncclResult_t r, const char *what);

}  // namespace ddl
