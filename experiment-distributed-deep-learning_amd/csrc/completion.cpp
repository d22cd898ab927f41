// completion.cpp — completion groups: a native ddl_done_fn for bindings whose own callbacks are
// costly (include/ddl_amd.h, ddl_completion_*).
//
// The reference's op hands every request a done callback (AllreduceOp.cc:32-66, the TF kernel's
// DoneCallback). A Python binding that passes a Python function pays the interpreter for every
// request: ctypes re-enters the interpreter from the engine's completion thread (GIL acquisition,
// argument boxing, the Python body) — about 10 us per call, 40-60 ms for a 4096-tensor batch,
// measured against a native-callback submission of the same batch. Here done() is
// native: it stores the request's status in its slot of a group and wakes whoever waits on that
// slot; the binding waits with ddl_completion_wait, which blocks in C++ (ctypes releases the GIL).
//
// Lifetime: the group is freed when its owner has called ddl_completion_destroy AND every slot has
// completed, so the engine's late done() calls never touch freed memory (a binding may drop its
// handles without waiting).
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "common.h"

namespace ddl {
namespace {

struct Group;

struct Slot {
    Group *group;
    int index;
};

struct Group {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> status;  // -1 pending, else the request's status
    std::vector<Slot> slots;
    int pending;
    int waiters = 0;  // threads blocked in ddl_completion_wait: done() wakes only when someone waits
    bool owner_gone = false;
};

constexpr int kPending = -1;

}  // namespace
}  // namespace ddl

using namespace ddl;

extern "C" {

void *ddl_completion_create(int count) {
    if (count < 0) return nullptr;
    Group *g = new (std::nothrow) Group;
    if (!g) return nullptr;
    g->status.assign((size_t)count, kPending);
    g->slots.resize((size_t)count);
    for (int i = 0; i < count; ++i) g->slots[(size_t)i] = Slot{g, i};
    g->pending = count;
    return g;
}

int ddl_completion_slots(void *group, int first, int count, void **out) {
    Group *g = static_cast<Group *>(group);
    if (!g || first < 0 || count < 0 || first + count > (int)g->slots.size() || (count && !out))
        return DDL_STATUS_INVALID_ARGUMENT;
    for (int i = 0; i < count; ++i) out[i] = &g->slots[(size_t)(first + i)];
    return DDL_STATUS_OK;
}

void ddl_completion_done(int status, void *user) {
    Slot *s = static_cast<Slot *>(user);
    if (!s) return;
    Group *g = s->group;
    bool free_it = false;
    {
        std::lock_guard<std::mutex> l(g->mu);
        if (g->status[(size_t)s->index] != kPending) return;  // a slot completes once
        g->status[(size_t)s->index] = status < 0 ? DDL_STATUS_ERROR_UNKNOWN : status;
        free_it = --g->pending == 0 && g->owner_gone;
        if (!free_it && g->waiters) g->cv.notify_all();
    }
    if (free_it) delete g;
}

int ddl_completion_wait(void *group, int index, double timeout_s, int *status) {
    Group *g = static_cast<Group *>(group);
    if (!g || index < 0 || index >= (int)g->status.size()) return DDL_STATUS_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> l(g->mu);
    auto done = [&] { return g->status[(size_t)index] != kPending; };
    if (!done()) {
        ++g->waiters;
        bool ok = true;
        if (timeout_s < 0) g->cv.wait(l, done);
        else ok = g->cv.wait_for(l, std::chrono::duration<double>(timeout_s), done);
        --g->waiters;
        if (!ok) return DDL_STATUS_ERROR_UNKNOWN;  // still pending
    }
    if (status) *status = g->status[(size_t)index];
    return DDL_STATUS_OK;
}

int ddl_completion_poll(void *group, int *statuses, int count) {
    Group *g = static_cast<Group *>(group);
    if (!g || count < 0 || count > (int)g->status.size() || (count && !statuses)) return -1;
    std::lock_guard<std::mutex> l(g->mu);
    for (int i = 0; i < count; ++i) statuses[i] = g->status[(size_t)i];
    return g->pending;
}

void ddl_completion_destroy(void *group) {
    Group *g = static_cast<Group *>(group);
    if (!g) return;
    bool free_it;
    {
        std::lock_guard<std::mutex> l(g->mu);
        g->owner_gone = true;
        free_it = g->pending == 0;
    }
    if (free_it) delete g;
}

}  // extern "C"
