// deptrace.h — happens-before tracing of the work the engine posts on HIP streams (test /
// diagnostic). The engine itself only carries the hooks: op() / record() / wait() forward to a
// Sink when one is installed and cost one relaxed atomic load otherwise. The recorder and its
// checker (start / stop / check, deptrace.cpp) are linked into the testing library only
// (libddl_amd_testing.so, ddl_testing_dep_trace); the deployment library never installs a sink.
//
// Every op the executors post — copies, transport receives / RCCL groups, reduce and fold
// launches — is logged with the byte ranges it reads and writes, and every event record and
// stream wait with its stream and event, in the order the host issues them. check() replays the
// log with vector clocks: stream order, plus record -> wait edges (a wait orders the waiting
// stream after the event's most recent record at the time of the wait, as hipStreamWaitEvent
// does). It reports every pair of ops on different streams whose byte ranges overlap, at least
// one of them writing, that neither happens before the other.
//
// The verdict depends only on what was posted — not on how the runtime maps streams onto its
// hardware queues (GPU_MAX_HW_QUEUES = 4 shares them between many streams, and a shared queue
// runs its work in submission order, which can mask a missing wait) nor on how long a kernel
// runs. So a dropped hipStreamWaitEvent is seen on every box (tests/test_thread_world_gpu.py).
// Work posted before tracing started is taken as complete.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace ddl {
namespace dep {

struct Access {
    uintptr_t lo, hi;  // [lo, hi) bytes
    bool write;
};
inline Access rd(const void *p, size_t bytes) { return Access{(uintptr_t)p, (uintptr_t)p + bytes, false}; }
inline Access wr(const void *p, size_t bytes) { return Access{(uintptr_t)p, (uintptr_t)p + bytes, true}; }

// Receiver of the posting log (the testing library's recorder).
class Sink {
public:
    virtual ~Sink() = default;
    virtual void op(hipStream_t s, const std::string &what, std::vector<Access> acc) = 0;
    virtual void record(hipEvent_t e, hipStream_t s) = 0;
    virtual void wait(hipStream_t s, hipEvent_t e) = 0;
};
extern std::atomic<Sink *> g_sink;  // null unless tracing (defined by the engine, executor.cpp)
inline bool on() { return g_sink.load(std::memory_order_relaxed) != nullptr; }

// Call right after the HIP call that posted the op / record / wait on `s`.
inline void op(hipStream_t s, const std::string &what, std::vector<Access> acc) {
    if (Sink *k = g_sink.load(std::memory_order_relaxed)) k->op(s, what, std::move(acc));
}
inline void record(hipEvent_t e, hipStream_t s) {
    if (Sink *k = g_sink.load(std::memory_order_relaxed)) k->record(e, s);
}
inline void wait(hipStream_t s, hipEvent_t e) {
    if (Sink *k = g_sink.load(std::memory_order_relaxed)) k->wait(s, e);
}

// ---- the recorder (deptrace.cpp: testing library only) ----
void start();  // clears the log and installs the recorder
void stop();   // uninstalls it (the log stays for check())

struct Report {
    long long ops = 0;
    long long conflicts = 0;       // pairs on different streams: overlapping ranges, one writing
    long long ordered = 0;         // ... of which one happens before the other
    long long ordered_reduce = 0;  // ... ordered pairs with a reduce / fold on one side
    long long races = 0;           // conflicts - ordered
    std::string first;             // the first races, one per line ("<op a> || <op b>")
};
Report check(size_t max_lines = 16);

}  // namespace dep
}  // namespace ddl
