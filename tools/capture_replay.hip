// Replays a posting trace of the engine (DDL_LOG_LEVEL=4 "[ddl trace]" lines of LocalWorld::run_:
// event records, stream waits, D2D copies, reduce launches) inside hipStreamBeginCapture with fresh
// streams and events, to find which part of the engine's forked-stream program makes
// hipStreamEndCapture fail. Diagnostic only.
//   ./capture_replay <trace file> <flags>
//     flags: E = replay the same program eagerly first (events / streams used before the capture,
//            as the engine's are), C = include the copies, K = include the kernels,
//            1 = events only on a single extra stream per original stream (no change), empty = "-",
//            D = single-stream DAG posting: every op goes on the origin stream, its dependencies set
//                explicitly (hipStreamUpdateCaptureDependencies) from the logical stream's node set;
//                records / waits become node-set bookkeeping (no forked stream at all)
// The trace's first "local world run" block is the eager call, the second the captured one; the
// second is replayed (its stream and event handles are mapped to fresh objects).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("  %s -> %s\n", #x, hipGetErrorString(e_));                           \
            std::fflush(stdout);                                                               \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void noop() {}

__global__ void inc(float *p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1.0f;
}

struct Op {
    char kind;  // 'r' record, 'w' wait, 'c' copy, 'k' kernel
    std::string a, b;  // r: event, stream; w: stream, event; c/k: stream
    size_t bytes = 0;
};

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const std::string flags = argv[2];
    const bool eager = flags.find('E') != std::string::npos, copies = flags.find('C') != std::string::npos,
               kernels = flags.find('K') != std::string::npos, anchors = flags.find('A') != std::string::npos;
    std::ifstream f(argv[1]);
    std::string line;
    int block = 0;
    std::vector<Op> ops;
    std::string user;
    while (std::getline(f, line)) {
        if (line.rfind("[ddl trace]", 0) != 0) continue;
        std::istringstream is(line.substr(12));
        std::string w0;
        is >> w0;
        if (w0 == "local") {
            ++block;
            size_t u = line.find("user ");
            if (block == 2) user = line.substr(u + 5);
            continue;
        }
        if (block != 2) continue;
        Op op;
        std::string x, y, z;
        if (w0 == "record") {  // record ev E on S
            is >> x >> op.a >> y >> op.b;
            op.kind = 'r';
        } else if (w0 == "wait") {  // wait S on ev E
            is >> op.a >> x >> y >> op.b;
            op.kind = 'w';
        } else if (w0 == "recv" || w0 == "copy") {  // recv copy N B on S | copy N B on S
            if (w0 == "recv") is >> x;
            is >> op.bytes >> y >> z >> op.a;
            op.kind = 'c';
        } else if (w0 == "reduce") {  // reduce launch on S
            is >> x >> y >> op.a;
            op.kind = 'k';
        } else {
            continue;
        }
        ops.push_back(op);
    }
    std::printf("replay: %zu ops, user stream %s, flags '%s'\n", ops.size(), user.c_str(), flags.c_str());
    std::map<std::string, hipStream_t> st;
    std::map<std::string, hipEvent_t> ev;
    hipStream_t o;
    CK(hipStreamCreateWithFlags(&o, hipStreamNonBlocking));
    st[user] = o;
    for (const Op &op : ops) {
        for (const std::string *sname : {&op.a, &op.b}) {
            if (sname->empty()) continue;
        }
        const std::string &sn = op.kind == 'r' ? op.b : op.a;
        if (!st.count(sn)) CK(hipStreamCreateWithFlags(&st[sn], hipStreamNonBlocking));
        if (op.kind == 'r' || op.kind == 'w') {
            const std::string &en = op.kind == 'r' ? op.a : op.b;
            if (!ev.count(en)) CK(hipEventCreateWithFlags(&ev[en], hipEventDisableTiming));
        }
    }
    std::printf("  %zu streams, %zu events\n", st.size(), ev.size());
    float *buf;
    const int n = 1 << 16;
    CK(hipMalloc(&buf, n * 4 * 2));
    CK(hipMemset(buf, 0, n * 4 * 2));
    // flag digits after '@' (e.g. "CK@40"): replay only the first k ops, then join every stream
    // touched so far back into the origin (a fresh event per stream) — bisects the crash
    size_t limit = ops.size();
    if (flags.find('@') != std::string::npos) limit = std::strtoul(flags.c_str() + flags.find('@') + 1, nullptr, 10);
    if (limit > ops.size()) limit = ops.size();
    // ":i,j,k" (1-based op numbers): replay only those ops (then join every touched stream)
    std::vector<char> keep(ops.size(), 1);
    if (flags.find(':') != std::string::npos) {
        std::fill(keep.begin(), keep.end(), 0);
        const char *p = flags.c_str() + flags.find(':') + 1;
        while (*p) {
            char *end;
            const unsigned long i = std::strtoul(p, &end, 10);
            if (i >= 1 && i <= ops.size()) keep[i - 1] = 1;
            p = *end ? end + 1 : end;
        }
        limit = 0;  // forces the join of touched streams
        for (size_t i = 0; i < ops.size(); ++i)
            if (keep[i]) limit = i + 1;
        if (limit == ops.size()) limit = ops.size() - 1;
    }
    const bool dag = flags.find('D') != std::string::npos;
    auto post_dag = [&]() -> int {
        std::map<std::string, std::vector<hipGraphNode_t>> tail, evn;
        auto add = [](std::vector<hipGraphNode_t> &a, const std::vector<hipGraphNode_t> &b) {
            for (hipGraphNode_t x : b)
                if (std::find(a.begin(), a.end(), x) == a.end()) a.push_back(x);
        };
        auto node_op = [&](const std::string &s, const std::function<void()> &fn) -> int {
            std::vector<hipGraphNode_t> &t = tail[s];
            CK(hipStreamUpdateCaptureDependencies(o, t.empty() ? nullptr : t.data(), t.size(),
                                                  hipStreamSetCaptureDependencies));
            fn();
            hipStreamCaptureStatus cs;
            unsigned long long id = 0;
            hipGraph_t cg = nullptr;
            const hipGraphNode_t *deps = nullptr;
            size_t nd = 0;
            CK(hipStreamGetCaptureInfo_v2(o, &cs, &id, &cg, &deps, &nd));
            t.assign(deps, deps + nd);
            return 0;
        };
        for (size_t i = 0; i < limit; ++i) {
            if (!keep[i]) continue;
            const Op &op = ops[i];
            switch (op.kind) {
                case 'r': evn[op.a] = tail[op.b]; break;
                case 'w': add(tail[op.a], evn[op.b]); break;
                case 'c':
                    if (copies && node_op(op.a, [&] { (void)hipMemcpyAsync(buf + n, buf, op.bytes, hipMemcpyDeviceToDevice, o); }))
                        return 1;
                    break;
                case 'k':
                    if (kernels && node_op(op.a, [&] { hipLaunchKernelGGL(inc, dim3(2), dim3(256), 0, o, buf, 300); }))
                        return 1;
                    break;
            }
        }
        std::vector<hipGraphNode_t> all = tail[user];  // join every logical stream into the origin
        for (auto &kv : tail) add(all, kv.second);
        CK(hipStreamUpdateCaptureDependencies(o, all.empty() ? nullptr : all.data(), all.size(),
                                              hipStreamSetCaptureDependencies));
        std::printf("  dag: %zu logical streams, %zu terminal nodes\n", tail.size(), all.size());
        return 0;
    };
    auto post = [&]() -> int {
        if (dag) return post_dag();
        std::map<std::string, int> touched, anchored;
        for (size_t i = 0; i < limit; ++i) {
            if (!keep[i]) continue;
            const Op &op = ops[i];
            touched[op.kind == 'r' ? op.b : op.a] = 1;
            // 'A': the engine's fix — an empty node on every stream before its first event record
            if (anchors && op.kind == 'r' && op.b != user && !anchored[op.b]) {
                hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, st[op.b]);
                anchored[op.b] = 1;
            }
            switch (op.kind) {
                case 'r': CK(hipEventRecord(ev[op.a], st[op.b])); break;
                case 'w': CK(hipStreamWaitEvent(st[op.a], ev[op.b], 0)); break;
                case 'c':
                    if (copies) CK(hipMemcpyAsync(buf + n, buf, op.bytes, hipMemcpyDeviceToDevice, st[op.a]));
                    break;
                case 'k':
                    if (kernels) hipLaunchKernelGGL(inc, dim3(2), dim3(256), 0, st[op.a], buf, 300);
                    break;
            }
        }
        if (limit < ops.size())
            for (auto &kv : touched) {
                if (kv.first == user) continue;
                hipEvent_t j;
                CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
                CK(hipEventRecord(j, st[kv.first]));
                CK(hipStreamWaitEvent(o, j, 0));
            }
        return 0;
    };
    if (flags == "Z" || flags == "F") {  // controls: an empty capture / fork + join with no nodes
        CK(hipStreamBeginCapture(o, hipStreamCaptureModeGlobal));
        if (flags == "F") {
            hipEvent_t fk, jn[8];
            hipStream_t side[8];
            CK(hipEventCreateWithFlags(&fk, hipEventDisableTiming));
            CK(hipEventRecord(fk, o));
            for (int i = 0; i < 6; ++i) {
                CK(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
                CK(hipEventCreateWithFlags(&jn[i], hipEventDisableTiming));
                CK(hipStreamWaitEvent(side[i], fk, 0));
                CK(hipEventRecord(jn[i], side[i]));
                CK(hipStreamWaitEvent(o, jn[i], 0));
            }
        }
        std::printf("  control '%s' posted; ending\n", flags.c_str());
        std::fflush(stdout);
        hipGraph_t g = nullptr;
        CK(hipStreamEndCapture(o, &g));
        size_t nodes = 0;
        CK(hipGraphGetNodes(g, nullptr, &nodes));
        std::printf("replay '%s': ok (%zu nodes)\n", flags.c_str(), nodes);
        return 0;
    }
    if (eager && !dag) {
        if (post()) return 1;
        CK(hipDeviceSynchronize());
        std::printf("  eager replay ok\n");
        std::fflush(stdout);
    }
    CK(hipStreamBeginCapture(o, hipStreamCaptureModeGlobal));
    if (post()) return 1;
    std::printf("  posted in capture; ending\n");
    std::fflush(stdout);
    if (flags.find('I') != std::string::npos) {  // the capture's state right before it ends
        hipGraph_t cg = nullptr;
        for (auto &kv : st) {
            hipStreamCaptureStatus cs;
            unsigned long long id = 0;
            const hipGraphNode_t *deps = nullptr;
            size_t nd = 0;
            CK(hipStreamGetCaptureInfo_v2(kv.second, &cs, &id, &cg, &deps, &nd));
            std::printf("  stream %s%s: status %d id %llu deps %zu:", kv.first.c_str(), kv.first == user ? " (origin)" : "",
                        (int)cs, id, nd);
            for (size_t i = 0; i < nd; ++i) std::printf(" %p", (void *)deps[i]);
            std::printf("\n");
        }
        size_t nn = 0, ne = 0;
        CK(hipGraphGetNodes(cg, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        CK(hipGraphGetNodes(cg, nodes.data(), &nn));
        CK(hipGraphGetEdges(cg, nullptr, nullptr, &ne));
        std::vector<hipGraphNode_t> from(ne), to(ne);
        CK(hipGraphGetEdges(cg, from.data(), to.data(), &ne));
        std::printf("  capture graph: %zu nodes, %zu edges\n", nn, ne);
        for (size_t i = 0; i < nn; ++i) {
            hipGraphNodeType t;
            CK(hipGraphNodeGetType(nodes[i], &t));
            std::printf("   node %p type %d\n", (void *)nodes[i], (int)t);
        }
        for (size_t i = 0; i < ne; ++i) std::printf("   edge %p -> %p\n", (void *)from[i], (void *)to[i]);
        std::fflush(stdout);
    }
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(o, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    hipGraphExec_t x;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, o));
    CK(hipStreamSynchronize(o));
    std::printf("replay '%s': ok (%zu nodes)\n", flags.c_str(), nodes);
    return 0;
}
