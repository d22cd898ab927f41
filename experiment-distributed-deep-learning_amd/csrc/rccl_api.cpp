// rccl_api.cpp — dlopen-based RCCL binding (see rccl_api.h).
#include "rccl_api.h"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>
#include <string>

#include "common.h"

namespace ddl {

namespace {

void *open_rccl(std::string &path) {
    // 1) an RCCL already in the process (PyTorch's), matched by the names it was loaded under
    const char *loaded[] = {"librccl.so", "librccl.so.1"};
    for (const char *name : loaded) {
        if (void *h = dlopen(name, RTLD_NOW | RTLD_NOLOAD)) {
            path = std::string(name) + " (already loaded)";
            return h;
        }
    }
    // 2) explicit override, then the system copy
    std::string cands[3];
    int nc = 0;
    if (const char *env = std::getenv("DDL_RCCL_LIB")) cands[nc++] = env;
    cands[nc++] = "librccl.so.1";
    cands[nc++] = "/opt/rocm/lib/librccl.so.1";
    for (int i = 0; i < nc; ++i) {
        if (void *h = dlopen(cands[i].c_str(), RTLD_NOW | RTLD_LOCAL)) {
            path = cands[i];
            return h;
        }
    }
    return nullptr;
}

template <typename F>
void bind(void *h, F &fn, const char *name) {
    fn = reinterpret_cast<F>(dlsym(h, name));
    DDL_REQUIRE(fn != nullptr, DDL_STATUS_COMM_ERROR, "RCCL symbol " << name << " not found");
}

}  // namespace

const RcclApi &rccl() {
    static std::once_flag once;
    static RcclApi api;
    static std::string err;
    static std::string path;
    std::call_once(once, [] {
        void *h = open_rccl(path);
        if (!h) {
            const char *e = dlerror();
            err = std::string("cannot load RCCL: ") + (e ? e : "not found");
            return;
        }
        try {
            bind(h, api.GetUniqueId, "ncclGetUniqueId");
            bind(h, api.CommInitRank, "ncclCommInitRank");
            bind(h, api.CommDestroy, "ncclCommDestroy");
            bind(h, api.CommAbort, "ncclCommAbort");
            bind(h, api.CommSplit, "ncclCommSplit");
            bind(h, api.CommGetAsyncError, "ncclCommGetAsyncError");
            bind(h, api.Send, "ncclSend");
            bind(h, api.Recv, "ncclRecv");
            bind(h, api.GroupStart, "ncclGroupStart");
            bind(h, api.GroupEnd, "ncclGroupEnd");
            bind(h, api.AllReduce, "ncclAllReduce");
            bind(h, api.AllGather, "ncclAllGather");
            bind(h, api.GetVersion, "ncclGetVersion");
            bind(h, api.CommCount, "ncclCommCount");
            bind(h, api.CommUserRank, "ncclCommUserRank");
            bind(h, api.GetErrorString, "ncclGetErrorString");
            api.CommInitRankConfig =
                reinterpret_cast<decltype(api.CommInitRankConfig)>(dlsym(h, "ncclCommInitRankConfig"));
            api.path = path.c_str();
        } catch (const Error &e) {
            err = e.msg;
            api = RcclApi();
        }
    });
    DDL_REQUIRE(err.empty(), DDL_STATUS_COMM_ERROR, err);
    return api;
}

void rccl_check(ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return;
    const RcclApi &api = rccl();
    fail(DDL_STATUS_COMM_ERROR, std::string(what) + " failed: " +
                                    (api.GetErrorString ? api.GetErrorString(r) : "rccl error"));
}

}  // namespace ddl
