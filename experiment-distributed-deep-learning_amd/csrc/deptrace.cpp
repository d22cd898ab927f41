// deptrace.cpp — the happens-before recorder and checker (see deptrace.h). Testing library only.
#include "deptrace.h"

#include <algorithm>
#include <mutex>
#include <sstream>
#include <unordered_map>

namespace ddl {
namespace dep {

namespace {

struct OpRec {
    int stream;
    uint32_t seq;              // this op's position on its stream (1-based)
    std::vector<uint32_t> vc;  // the stream's vector clock once the op is posted
    std::string what;
    std::vector<Access> acc;
};

struct State : Sink {
    void op(hipStream_t s, const std::string &what, std::vector<Access> acc) override;
    void record(hipEvent_t e, hipStream_t s) override;
    void wait(hipStream_t s, hipEvent_t e) override;
    std::mutex mu;
    std::unordered_map<hipStream_t, int> sid;
    std::vector<std::vector<uint32_t>> vc;                       // per stream
    std::unordered_map<hipEvent_t, std::vector<uint32_t>> ev;   // clock of the event's latest record
    std::vector<OpRec> ops;
};

State &st() {
    static State *s = new State;  // never destroyed: hooks may run during static teardown
    return *s;
}

int stream_id_(State &s, hipStream_t h) {
    auto it = s.sid.find(h);
    if (it != s.sid.end()) return it->second;
    const int id = (int)s.vc.size();
    s.sid.emplace(h, id);
    s.vc.emplace_back();
    return id;
}

uint32_t at(const std::vector<uint32_t> &v, int i) { return (size_t)i < v.size() ? v[(size_t)i] : 0u; }

void join_into(std::vector<uint32_t> &dst, const std::vector<uint32_t> &src) {
    if (dst.size() < src.size()) dst.resize(src.size(), 0u);
    for (size_t i = 0; i < src.size(); ++i) dst[i] = std::max(dst[i], src[i]);
}

bool conflict(const OpRec &a, const OpRec &b) {
    for (const Access &x : a.acc)
        for (const Access &y : b.acc)
            if ((x.write || y.write) && x.lo < y.hi && y.lo < x.hi && x.lo < x.hi && y.lo < y.hi) return true;
    return false;
}

bool is_reduce(const OpRec &o) { return o.what.compare(0, 4, "fold") == 0 || o.what.compare(0, 6, "reduce") == 0; }

}  // namespace

void start() {
    State &s = st();
    std::lock_guard<std::mutex> g(s.mu);
    s.sid.clear();
    s.vc.clear();
    s.ev.clear();
    s.ops.clear();
    g_sink = &s;
}

void stop() { g_sink = nullptr; }

void State::op(hipStream_t h, const std::string &what, std::vector<Access> acc) {
    State &s = *this;
    std::lock_guard<std::mutex> g(s.mu);
    const int i = stream_id_(s, h);
    std::vector<uint32_t> &v = s.vc[(size_t)i];
    if (v.size() <= (size_t)i) v.resize((size_t)i + 1, 0u);
    v[(size_t)i] += 1;
    s.ops.push_back(OpRec{i, v[(size_t)i], v, what, std::move(acc)});
}

void State::record(hipEvent_t e, hipStream_t h) {
    State &s = *this;
    std::lock_guard<std::mutex> g(s.mu);
    s.ev[e] = s.vc[(size_t)stream_id_(s, h)];
}

void State::wait(hipStream_t h, hipEvent_t e) {
    State &s = *this;
    std::lock_guard<std::mutex> g(s.mu);
    const int i = stream_id_(s, h);
    auto it = s.ev.find(e);
    if (it != s.ev.end()) join_into(s.vc[(size_t)i], it->second);  // never recorded while tracing: complete
}

Report check(size_t max_lines) {
    State &s = st();
    std::lock_guard<std::mutex> g(s.mu);
    Report r;
    r.ops = (long long)s.ops.size();
    std::ostringstream os;
    size_t lines = 0;
    // every pair once, in posting order; the ops' bounding ranges are compared before their accesses
    std::vector<size_t> idx(s.ops.size());
    std::vector<uintptr_t> lo(s.ops.size(), UINTPTR_MAX), hi(s.ops.size(), 0);
    for (size_t k = 0; k < s.ops.size(); ++k) {
        idx[k] = k;
        for (const Access &a : s.ops[k].acc)
            if (a.lo < a.hi) {
                lo[k] = std::min(lo[k], a.lo);
                hi[k] = std::max(hi[k], a.hi);
            }
    }
    for (size_t x = 0; x < idx.size(); ++x) {
        for (size_t y = x + 1; y < idx.size(); ++y) {
            const size_t i = idx[x], j = idx[y];
            const OpRec &a = s.ops[i], &b = s.ops[j];
            if (a.stream == b.stream || lo[i] >= hi[j] || lo[j] >= hi[i] || !conflict(a, b)) continue;
            ++r.conflicts;
            const bool hb = a.seq <= at(b.vc, a.stream) || b.seq <= at(a.vc, b.stream);
            if (hb) {
                ++r.ordered;
                if (is_reduce(a) || is_reduce(b)) ++r.ordered_reduce;
            } else {
                ++r.races;
                if (lines < max_lines) {
                    os << a.what << " || " << b.what << "\n";
                    ++lines;
                }
            }
        }
    }
    r.first = os.str();
    return r;
}

}  // namespace dep
}  // namespace ddl
