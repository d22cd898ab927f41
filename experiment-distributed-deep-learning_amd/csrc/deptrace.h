// deptrace.h — happens-before tracing of the work the engine posts on HIP streams (test /
// diagnostic: off unless ddl_testing_dep_trace(1); one relaxed atomic load per posted op when off).
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

extern std::atomic<bool> g_on;
inline bool on() { return g_on.load(std::memory_order_relaxed); }
void start();  // clears the log and starts tracing
void stop();

// Call right after the HIP call that posted the op / record / wait on `s`.
void op(hipStream_t s, const std::string &what, std::vector<Access> acc);
void record(hipEvent_t e, hipStream_t s);
void wait(hipStream_t s, hipEvent_t e);

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
