// The engine's own programs captured into hipGraphs from C++ (one HIP runtime: the system's, which
// libddl_amd.so links): VERDICT r2 next #3 — is the hipStreamEndCapture crash of r02 the engine's
// (an unjoined forked stream, an event reused across the capture boundary) or the runtime's?
//   ./capture_engine <mode> <capture_mode 0|2>
//   modes: direct3   P = 3 virtual ranks, direct schedule, 300 and 70001 fp32 (D2D moves)
//          ring2     P = 2 ring (reference_order 0)
//          bcast3    P = 3 broadcast (no reduce: the compute streams only wait on the fork)
//          gatherv3  P = 3 allgatherv
//          loop5     P = 5 direct over the one-rank RCCL loopback (RCCL groups in the graph)
// Every HIP call's status is printed; the replay is compared with the eager result on the same
// inputs (bit for bit).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ddl_amd_testing.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        std::printf("  %-60s -> %s\n", #x, hipGetErrorString(e_));                            \
        std::fflush(stdout);                                                                   \
        if (e_ != hipSuccess) return 1;                                                        \
    } while (0)
#define DK(x)                                                                                  \
    do {                                                                                       \
        int s_ = (x);                                                                          \
        if (s_ != 0) {                                                                         \
            std::printf("  %s -> status %d: %s\n", #x, s_, ddl_last_error());                 \
            std::fflush(stdout);                                                               \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

static int run(const std::string &mode, size_t n, hipStream_t s) {
    const int P = mode == "ring2" ? 2 : mode == "loop5" ? 5 : 3;
    std::vector<float *> in(P), out(P);
    std::vector<float> host(n);
    for (int r = 0; r < P; ++r) {
        CK(hipMalloc(&in[r], n * 4 * P));
        CK(hipMalloc(&out[r], n * 4 * P));
        for (size_t i = 0; i < n; ++i) host[i] = (float)((i * 2654435761u + 977u * r) % 1000) / 997.0f - 0.4f;
        CK(hipMemcpy(in[r], host.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemset(out[r], 0, n * 4 * P));
    }
    std::vector<size_t> counts(P), displs(P);
    for (int r = 0; r < P; ++r) {
        counts[r] = n / P + (size_t)r;
        displs[r] = r ? displs[r - 1] + counts[r - 1] : 0;
    }
    auto call = [&]() -> int {
        if (mode == "bcast3") return ddl_local_broadcast(P, 1, (void *const *)in.data(), n, DDL_FLOAT, s);
        if (mode == "gatherv3")
            return ddl_local_allgatherv(P, (const void *const *)in.data(), (void *const *)out.data(), counts.data(),
                                        displs.data(), DDL_FLOAT, s);
        if (mode == "loop5")
            return ddl_rccl_loopback_allreduce(P, (const void *const *)in.data(), (void *const *)out.data(), n,
                                               DDL_FLOAT, s);
        return ddl_local_ring_allreduce(P, (const void *const *)in.data(), (void *const *)out.data(), n, DDL_FLOAT,
                                        DDL_ALLREDUCE_OP_SUM, s);
    };
    std::printf("[%s n=%zu] eager\n", mode.c_str(), n);
    DK(call());
    CK(hipStreamSynchronize(s));
    // eager results (broadcast: in place on `in`, so keep its outputs and restore its inputs)
    std::vector<std::vector<float>> want(P, std::vector<float>(n * P));
    float *const *res = mode == "bcast3" ? in.data() : out.data();
    for (int r = 0; r < P; ++r) CK(hipMemcpy(want[r].data(), res[r], n * 4 * P, hipMemcpyDeviceToHost));
    std::printf("[%s n=%zu] begin capture\n", mode.c_str(), n);
    std::fflush(stdout);
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    const int st = call();
    std::printf("  captured call -> status %d %s\n", st, st ? ddl_last_error() : "");
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(s, &g));
    if (st) return 1;
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    std::printf("  graph nodes: %zu\n", nodes);
    hipGraphExec_t x = nullptr;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    for (int r = 0; r < P; ++r) CK(hipMemset(out[r], 0, n * 4 * P));
    CK(hipStreamSynchronize(s));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipGraphLaunch(x, s));
        CK(hipStreamSynchronize(s));
    }
    bool same = true;
    std::vector<float> got(n * P);
    for (int r = 0; r < P; ++r) {
        CK(hipMemcpy(got.data(), res[r], n * 4 * P, hipMemcpyDeviceToHost));
        same = same && std::memcmp(got.data(), want[r].data(), n * 4 * P) == 0;
    }
    std::printf("[%s n=%zu] replay x3 equals eager: %s\n", mode.c_str(), n, same ? "yes" : "NO");
    CK(hipGraphExecDestroy(x));
    CK(hipGraphDestroy(g));
    for (int r = 0; r < P; ++r) {
        CK(hipFree(in[r]));
        CK(hipFree(out[r]));
    }
    return same ? 0 : 2;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::printf("usage: %s <direct3|ring2|bcast3|gatherv3|loop5> <capture_mode 0|2>\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    CK(hipSetDevice(0));
    DK(ddl_set_config("tune", 0));
    DK(ddl_set_config("slice_bytes", 64 << 10));
    DK(ddl_set_config("capture_mode", std::atoi(argv[2])));  // 0 serial, 2 single-stream DAG
    if (mode == "ring2") {
        DK(ddl_set_config("reference_order", 0));
        DK(ddl_set_config("algo", 0));
    } else {
        DK(ddl_set_config("algo", 1));
    }
    if (mode == "loop5") DK(ddl_rccl_loopback_init(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int rc = 0;
    for (size_t n : {(size_t)300, (size_t)70001})
        if ((rc = run(mode, n, s)) != 0) break;
    if (mode == "loop5") DK(ddl_rccl_loopback_finalize());
    std::printf("%s capture_mode=%s: %s\n", mode.c_str(), argv[2], rc == 0 ? "ok" : "FAILED");
    return rc;
}
