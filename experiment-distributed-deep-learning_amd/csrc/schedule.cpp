// schedule.cpp — ring construction, bucket partition and per-rank tick lists.
#include "schedule.h"

#include <algorithm>
#include <map>
#include <mutex>

namespace ddl {

namespace {

struct RingSearch {
    int P;
    std::vector<std::vector<char>> used;  // used[u][v]: directed edge u->v taken
    std::vector<std::vector<int>> cycles;
    int want;

    bool next_cycle(std::vector<int> &path, std::vector<char> &visited, std::vector<int> &out) {
        // first Hamiltonian cycle (DFS, ascending vertex order) avoiding used edges
        if ((int)path.size() == P) {
            if (!used[path.back()][path[0]]) { out = path; return true; }
            return false;
        }
        for (int v = 0; v < P; ++v) {
            if (visited[v] || used[path.back()][v]) continue;
            visited[v] = 1;
            path.push_back(v);
            if (next_cycle(path, visited, out)) return true;
            path.pop_back();
            visited[v] = 0;
        }
        return false;
    }

    // Enumerate candidate cycles in DFS order and backtrack over them.
    void all_cycles(std::vector<int> &path, std::vector<char> &visited,
                    std::vector<std::vector<int>> &res) {
        if ((int)path.size() == P) {
            if (!used[path.back()][path[0]]) res.push_back(path);
            return;
        }
        for (int v = 0; v < P; ++v) {
            if (visited[v] || used[path.back()][v]) continue;
            visited[v] = 1;
            path.push_back(v);
            all_cycles(path, visited, res);
            path.pop_back();
            visited[v] = 0;
        }
    }

    void mark(const std::vector<int> &c, char val) {
        for (int i = 0; i < P; ++i) used[c[i]][c[(i + 1) % P]] = val;
    }

    bool rec(std::vector<std::vector<int>> &best) {
        if ((int)cycles.size() == want) return true;
        if (cycles.size() > best.size()) best = cycles;
        std::vector<int> path{0};
        std::vector<char> visited(P, 0);
        visited[0] = 1;
        std::vector<std::vector<int>> cands;
        all_cycles(path, visited, cands);
        for (const auto &c : cands) {
            mark(c, 1);
            cycles.push_back(c);
            if (rec(best)) return true;
            cycles.pop_back();
            mark(c, 0);
        }
        return false;
    }
};

std::vector<std::vector<int>> search_rings(int P, int max_rings) {
    std::vector<std::vector<int>> res;
    std::vector<int> nat(P);
    for (int i = 0; i < P; ++i) nat[i] = i;
    res.push_back(nat);
    if (P <= 2 || max_rings <= 1) return res;
    if (P > 8) {
        // beyond one node the exhaustive search is out of reach (it enumerates (P-1)! cycles):
        // stride rings r -> r + s for s coprime to P are Hamiltonian and pairwise edge-disjoint
        for (int st = 2; st < P && (int)res.size() < std::min(P - 1, max_rings); ++st) {
            int a = P, b = st;
            while (b) { int t = a % b; a = b; b = t; }
            if (a != 1) continue;
            std::vector<int> ring(P);
            for (int i = 0; i < P; ++i) ring[i] = (int)((long long)i * st % P);
            res.push_back(ring);
        }
        return res;
    }
    RingSearch s;
    s.P = P;
    s.used.assign(P, std::vector<char>(P, 0));
    s.want = std::min(P - 1, max_rings);
    s.mark(nat, 1);
    s.cycles.push_back(nat);
    std::vector<std::vector<int>> best = s.cycles;
    if (s.rec(best)) return s.cycles;
    return best;
}

}  // namespace

const std::vector<std::vector<int>> &rings_for(int P, int max_rings) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::vector<std::vector<int>>> cache;
    if (P < 1) P = 1;
    if (max_rings < 1) max_rings = 1;
    if (max_rings > kMaxRings) max_rings = kMaxRings;
    std::lock_guard<std::mutex> g(mu);
    auto key = std::make_pair(P, max_rings);
    auto it = cache.find(key);
    if (it == cache.end()) it = cache.emplace(key, search_rings(P, max_rings)).first;
    return it->second;
}

Range chunk_range(size_t n, size_t esize, int P, int R, int ring, int chunk) {
    const size_t G = kGranuleBytes / esize;
    const size_t ng = (n + G - 1) / G;
    const size_t parts = (size_t)R * (size_t)P;
    const size_t q = (size_t)ring * (size_t)P + (size_t)chunk;
    const size_t gb = (size_t)(((unsigned __int128)ng * q) / parts);
    const size_t ge = (size_t)(((unsigned __int128)ng * (q + 1)) / parts);
    Range r;
    r.begin = gb * G < n ? gb * G : n;
    r.end = ge * G < n ? ge * G : n;
    return r;
}

Range slice_range(const Range &chunk, size_t esize, int K, int k) {
    const size_t G = kGranuleBytes / esize;
    const size_t len = chunk.size();
    const size_t ng = (len + G - 1) / G;
    const size_t gb = ng * (size_t)k / (size_t)K, ge = ng * (size_t)(k + 1) / (size_t)K;
    Range r;
    r.begin = chunk.begin + (gb * G < len ? gb * G : len);
    r.end = chunk.begin + (ge * G < len ? ge * G : len);
    return r;
}

void ring_shape(size_t n, size_t esize, int P, const RingConfig &cfg_in, int *R, int *K,
                size_t *staging_stride) {
    const RingConfig cfg = effective_config(cfg_in, P);
    if (cfg.algo == kAlgoOneShot) {  // one tick, whole bucket per peer
        *R = 1;
        *K = 1;
        *staging_stride = (n + 63) & ~size_t(63);
        return;
    }
    if (cfg.algo == kAlgoGatherFold) {  // the allgather's blocks are contiguous: stride = block
        *R = 1;
        *K = 1;
        *staging_stride = gather_stride(n, esize);
        return;
    }
    int r = is_direct(cfg.algo) ? 1 : (int)rings_for(P, cfg.rings).size();
    // Small buckets: fewer rings so every message stays >= 64 KiB (latency-bound regime).
    const size_t bytes = n * esize;
    while (r > 1 && bytes / ((size_t)r * (size_t)P) < (64u << 10)) --r;
    size_t max_chunk = 0;
    for (int j = 0; j < r; ++j)
        for (int c = 0; c < P; ++c) {
            size_t s = chunk_range(n, esize, P, r, j, c).size();
            max_chunk = s > max_chunk ? s : max_chunk;
        }
    int k = 1;
    if (cfg.slice_bytes > 0) {
        size_t want = (max_chunk * esize + cfg.slice_bytes - 1) / cfg.slice_bytes;
        k = (int)(want < 1 ? 1 : want);
    }
    if (k > cfg.max_slices) k = cfg.max_slices;
    if (k < 1) k = 1;
    *R = r;
    *K = k;
    *staging_stride = (max_chunk + 63) & ~size_t(63);
}

size_t program_staging_elems(size_t n, size_t esize, int P, const RingConfig &cfg_in) {
    const RingConfig cfg = effective_config(cfg_in, P);
    int R, K;
    size_t stride;
    ring_shape(n, esize, P, cfg, &R, &K, &stride);
    return program_staging_slots(P, cfg.algo, R) * stride;
}

size_t program_staging_slots(int P, int algo, int R) {
    if (P <= 1) return 0;
    if (algo == kAlgoRing) return 2 * (size_t)R;
    if (algo == kAlgoGatherFold) return (size_t)P + 1 + fold_temp_slots(P);
    return (size_t)(P - 1 + fold_temp_slots(P));
}

int fold_temp_count(int K, int order) {
    const int W = kMaxInputs + 1;
    if (K <= W) return 0;
    if (order == kFoldLeft) return 1;  // one running partial
    int used = 0, level = K;
    if (order == kFoldMpichTree) {  // pre-folded pairs
        int pof2 = 1;
        while (pof2 * 2 <= K) pof2 *= 2;
        used += K - pof2;
        level = pof2;
    }
    while (level > W) {  // block sums of aligned blocks of W (single leftovers pass through)
        int next = 0;
        for (int b = 0; b < level; b += W) {
            if (std::min(level, b + W) - b > 1) ++used;
            ++next;
        }
        level = next;
    }
    return used;
}

void plan_fold(std::vector<SegTableN> &steps, const std::vector<const void *> &xs, void *out, size_t n, int order,
               const std::function<void *(int)> &temp) {
    const size_t W = kMaxInputs + 1;
    int used = 0;
    auto step = [&](const std::vector<const void *> &in, int ord, void *dst) {
        SegTableN t;
        t.a = in[0];
        t.nb = (int)in.size() - 1;
        for (int i = 0; i < t.nb; ++i) t.b[i] = in[i + 1];
        t.out = dst;
        t.n = n;
        t.order = ord;
        steps.push_back(t);
    };
    DDL_REQUIRE(xs.size() >= 2, DDL_STATUS_ERROR_UNKNOWN, "fold of " << xs.size() << " inputs");
    if (xs.size() <= W) {
        step(xs, order, out);
        return;
    }
    if (order == kFoldLeft) {  // ((x_0 + ... + x_15) + x_16 + ... + x_30) + ...: one partial
        void *acc = temp(used++);
        step(std::vector<const void *>(xs.begin(), xs.begin() + W), kFoldLeft, acc);
        for (size_t i = W; i < xs.size();) {
            const size_t take = std::min(W - 1, xs.size() - i);
            std::vector<const void *> in{acc};
            in.insert(in.end(), xs.begin() + i, xs.begin() + i + take);
            i += take;
            step(in, kFoldLeft, i == xs.size() ? out : acc);
        }
        return;
    }
    std::vector<const void *> level = xs;
    if (order == kFoldMpichTree) {  // leaves: pre-folded pairs, then the rest; pof2 of them
        size_t pof2 = 1;
        while (pof2 * 2 <= xs.size()) pof2 *= 2;
        const size_t rem = xs.size() - pof2;
        level.clear();
        for (size_t t = 0; t < rem; ++t) {
            void *d = temp(used++);
            step({xs[2 * t], xs[2 * t + 1]}, kFoldLeft, d);
            level.push_back(d);
        }
        for (size_t t = rem; t < pof2; ++t) level.push_back(xs[t + rem]);
    }
    // a binomial tree (the pairwise tree over pof2 leaves is one) restricted to aligned blocks
    // of W is the block's own binomial tree; the block sums then continue the same tree
    while (level.size() > W) {
        std::vector<const void *> next;
        for (size_t b = 0; b < level.size(); b += W) {
            const size_t e = std::min(level.size(), b + W);
            if (e - b == 1) {
                next.push_back(level[b]);
                continue;
            }
            void *d = temp(used++);
            step(std::vector<const void *>(level.begin() + b, level.begin() + e), kFoldBinomial, d);
            next.push_back(d);
        }
        level.swap(next);
    }
    step(level, kFoldBinomial, out);
    DDL_REQUIRE(used == fold_temp_count((int)xs.size(), order), DDL_STATUS_ERROR_UNKNOWN, "fold temp slots miscounted");
}

namespace {

// Direct reduce-scatter / allgather on a fully connected mesh. Chunk c (of P) is reduced by rank
// c. RS tick k: send slice k of chunk q to every peer q, receive slice k of my chunk from every
// peer into its staging slot; then one N-input fold: kFoldLeft out = in + x_{me+1} + x_{me+2}
// + ... (the ring's left-fold order for ring 0); the reference orders fold x_0, ..., x_{P-1} in
// rank order (x_me = in) in MPICH's tree. AG tick k (waits the fold of slice k): send my
// reduced slice to every peer, receive theirs straight into out.
void build_direct(RingProgram &prog, int rank, int P, const char *inb, char *outb, char *stb, size_t n,
                  size_t es, int order, bool rank_order, bool collective_ag) {
    const int K = prog.K;
    const Range mine = chunk_range(n, es, P, 1, 0, rank);
    for (int k = 0; k < K; ++k) {
        Tick t;
        t.reduce.count = 0;
        const Range ms = slice_range(mine, es, K, k);
        for (int d = 1; d < P; ++d) {
            const int q = (rank + d) % P;  // peer
            const Range qs = slice_range(chunk_range(n, es, P, 1, 0, q), es, K, k);
            if (qs.size()) t.ops.push_back(P2POp{true, q, d, const_cast<char *>(inb + qs.begin * es), qs.size() * es});
            if (ms.size()) {
                // receive from the rank d positions before me: fold order me, me+1, ..., so the
                // peer at offset d' = P - d ... keep slot = offset of the sender after me
                const int from = (rank + P - d) % P;
                const int slot = (from - rank + P) % P - 1;  // sender me+1 -> slot 0
                char *st = stb + ((size_t)slot * prog.staging_stride + (ms.begin - mine.begin)) * es;
                t.ops.push_back(P2POp{false, from, d, st, ms.size() * es});
            }
        }
        if (ms.size()) {
            t.has_reduce = true;
            t.multi = true;
            const size_t off = ms.begin - mine.begin;
            auto slot = [&](int s) -> const void * { return stb + ((size_t)s * prog.staging_stride + off) * es; };
            const void *own = inb + ms.begin * es;
            // ring order: in, x_{me+1}, x_{me+2}, ... (slot s holds sender me+1+s); reference
            // order: x_0, ..., x_{P-1} in rank order (x_me = in) — in MPICH's tree, or left to
            // right in fp32 for fp16 / bf16, which the reference rejects (the oracle's rank-order fold)
            std::vector<const void *> xs;
            for (int q = 0; q < P; ++q) {
                const int who = rank_order ? q : (rank + q) % P;
                xs.push_back(who == rank ? own : slot((who - rank + P) % P - 1));
            }
            plan_fold(t.folds, xs, outb + ms.begin * es, ms.size(), order, [&](int j) {
                return static_cast<void *>(stb + ((size_t)(P - 1 + j) * prog.staging_stride + off) * es);
            });
        }
        prog.ticks.push_back(std::move(t));
    }
    if (collective_ag) {
        // every chunk is n / P elements at q * n / P (direct_gather_eligible): one in-place
        // allgather of the reduced chunks once the last fold has run (the compute stream is in
        // order, so waiting for the last fold waits for all of them)
        Tick t;
        t.reduce.count = 0;
        t.wait_reduce = K - 1;
        t.gather = GatherOp{outb + mine.begin * es, outb, mine.size() * es};
        prog.ticks.push_back(std::move(t));
        return;
    }
    for (int k = 0; k < K; ++k) {
        Tick t;
        t.reduce.count = 0;
        t.wait_reduce = k;
        const Range ms = slice_range(mine, es, K, k);
        for (int d = 1; d < P; ++d) {
            const int q = (rank + d) % P;
            const int from = (rank + P - d) % P;
            const Range fs = slice_range(chunk_range(n, es, P, 1, 0, from), es, K, k);
            if (ms.size()) t.ops.push_back(P2POp{true, q, d, outb + ms.begin * es, ms.size() * es});
            if (fs.size()) t.ops.push_back(P2POp{false, from, d, outb + fs.begin * es, fs.size() * es});
        }
        prog.ticks.push_back(std::move(t));
    }
}

// One-shot allreduce for latency-bound buckets: tick 0 sends the whole input to every peer and
// receives every peer's whole input into staging slot (peer - me - 1) mod P, then folds the P
// inputs in rank order 0, 1, ..., P-1 (in for me, a slot otherwise) — left to right, or in
// MPICH's tree with `order` — so every rank computes the same sum bit for bit (fp16/bf16
// accumulated in fp32, rounded once per fold step: once up to 16 ranks). Tick 1 only waits for the
// fold, so the comm stream's tail covers it (the executor joins the caller on the comm stream).
// In place is safe: the fold runs after the group, i.e. after every send has read `in`.
void build_oneshot(RingProgram &prog, int rank, int P, const char *inb, char *outb, char *stb, size_t n,
                   size_t es, int order) {
    auto slot = [&](int q) { return stb + (size_t)((q - rank + P) % P - 1) * prog.staging_stride * es; };
    Tick t;
    t.reduce.count = 0;
    for (int d = 1; d < P; ++d) {
        const int to = (rank + d) % P, from = (rank + P - d) % P;
        t.ops.push_back(P2POp{true, to, d, const_cast<char *>(inb), n * es});
        t.ops.push_back(P2POp{false, from, d, slot(from), n * es});
    }
    t.has_reduce = true;
    t.multi = true;
    std::vector<const void *> xs;
    for (int q = 0; q < P; ++q) xs.push_back(q == rank ? static_cast<const void *>(inb) : slot(q));
    plan_fold(t.folds, xs, outb, n, order,
              [&](int j) { return static_cast<void *>(stb + (size_t)(P - 1 + j) * prog.staging_stride * es); });
    prog.ticks.push_back(std::move(t));
    Tick join;
    join.reduce.count = 0;
    join.wait_reduce = 0;
    prog.ticks.push_back(std::move(join));
}

// Gather-fold for latency-bound buckets: tick 0 gathers every rank's bucket into staging slots
// 0..P-1 (slot q = rank q's input; RCCL's ncclAllGather, one collective call instead of 2(P-1)
// p2p ops in a group), then folds the P inputs in rank order (`in` for me) exactly as the
// one-shot schedule does — same sum, bit for bit, on every rank. The blocks of an allgather are
// contiguous, so the slot stride is the bucket itself when that keeps the slots 16-byte aligned
// (the fold's vector loads); otherwise the input is first copied into the padded slot P and the
// gather moves padded blocks. Tick 1 only waits for the fold (the caller's join covers it).
void build_gatherfold(RingProgram &prog, int rank, int P, const char *inb, char *outb, char *stb, size_t n,
                      size_t es, int order) {
    const size_t stride = prog.staging_stride;
    auto slot = [&](int q) { return stb + (size_t)q * stride * es; };
    Tick t;
    t.reduce.count = 0;
    const void *src = inb;
    if (stride != n) {  // padded blocks: gather from a padded copy of the input
        t.copies.push_back(CopyOp{inb, slot(P), n * es});
        src = slot(P);
    }
    t.gather = GatherOp{src, stb, stride * es};
    t.has_reduce = true;
    t.multi = true;
    std::vector<const void *> xs;
    for (int q = 0; q < P; ++q) xs.push_back(q == rank ? static_cast<const void *>(inb) : slot(q));
    plan_fold(t.folds, xs, outb, n, order, [&](int j) { return static_cast<void *>(slot(P + 1 + j)); });
    prog.ticks.push_back(std::move(t));
    Tick join;
    join.reduce.count = 0;
    join.wait_reduce = 0;
    prog.ticks.push_back(std::move(join));
}

}  // namespace

void build_program(RingProgram &prog, int rank, int P, const void *in, void *out, void *staging,
                   size_t n, int dtype, const RingConfig &cfg_in) {
    const RingConfig cfg = effective_config(cfg_in, P);
    const size_t es = dtype_size(dtype);
    prog.P = P;
    prog.rank = rank;
    prog.n = n;
    prog.esize = es;
    prog.algo = cfg.algo;
    prog.ticks.clear();
    ring_shape(n, es, P, cfg, &prog.R, &prog.K, &prog.staging_stride);
    prog.staging_slots = program_staging_slots(P, cfg.algo, prog.R);
    if (P <= 1 || n == 0) return;
    // fold order of the direct / one-shot N-input reduce (kFoldLeft: ring 0's order)
    // (fp16 / bf16, which the reference rejects, always fold left in fp32)
    const bool half = dtype == DDL_HALF || dtype == DDL_BFLOAT16;
    const int order =
        cfg.ref_order && !half ? mpich_fold_order(cfg.order_bytes ? cfg.order_bytes : n * es, es, P) : kFoldLeft;
    if (cfg.algo == kAlgoOneShot) {
        build_oneshot(prog, rank, P, static_cast<const char *>(in), static_cast<char *>(out),
                      static_cast<char *>(staging), n, es, order);
        return;
    }
    if (cfg.algo == kAlgoGatherFold) {
        build_gatherfold(prog, rank, P, static_cast<const char *>(in), static_cast<char *>(out),
                         static_cast<char *>(staging), n, es, order);
        return;
    }
    if (is_direct(cfg.algo)) {
        build_direct(prog, rank, P, static_cast<const char *>(in), static_cast<char *>(out),
                     static_cast<char *>(staging), n, es, order, cfg.ref_order != 0,
                     cfg.algo == kAlgoDirectGather && direct_gather_eligible(n, es, P));
        return;
    }
    const int R = prog.R, K = prog.K;
    const auto &rings = rings_for(P, cfg.rings);
    std::vector<int> pos(R), succ(R), pred(R);
    for (int j = 0; j < R; ++j) {
        const auto &ring = rings[j];
        int p = 0;
        while (ring[p] != rank) ++p;
        pos[j] = p;
        succ[j] = ring[(p + 1) % P];
        pred[j] = ring[(p + P - 1) % P];
    }
    const char *inb = static_cast<const char *>(in);
    char *outb = static_cast<char *>(out);
    char *stb = static_cast<char *>(staging);
    auto mod = [P](int x) { return ((x % P) + P) % P; };

    // reduce-scatter: tick index = s*K + k
    for (int s = 0; s < P - 1; ++s) {
        for (int k = 0; k < K; ++k) {
            Tick t;
            t.reduce.count = 0;
            if (s > 0) t.wait_reduce = (s - 1) * K + k;
            for (int j = 0; j < R; ++j) {
                const Range sc = chunk_range(n, es, P, R, j, mod(pos[j] - s));
                const Range rc = chunk_range(n, es, P, R, j, mod(pos[j] - s - 1));
                const Range ss = slice_range(sc, es, K, k);
                const Range rs = slice_range(rc, es, K, k);
                if (ss.size()) {
                    const char *src = (s == 0 ? inb : outb) + ss.begin * es;
                    t.ops.push_back(P2POp{true, succ[j], j, const_cast<char *>(src), ss.size() * es});
                }
                if (rs.size()) {
                    // staging is double-buffered by step parity: the recv of step s never lands
                    // in the region the reduce of step s-1 may still be reading (chunks differ
                    // by up to one granule, so their slice boundaries differ)
                    char *st = stb + ((size_t)(2 * j + (s & 1)) * prog.staging_stride + (rs.begin - rc.begin)) * es;
                    t.ops.push_back(P2POp{false, pred[j], j, st, rs.size() * es});
                    const int c = t.reduce.count++;
                    t.reduce.a[c] = inb + rs.begin * es;
                    t.reduce.b[c] = st;
                    t.reduce.out[c] = outb + rs.begin * es;
                    t.reduce.n[c] = rs.size();
                }
            }
            t.has_reduce = t.reduce.count > 0;
            prog.ticks.push_back(std::move(t));
        }
    }
    // allgather: the first step waits for the last reduce-scatter reduce (compute stream is
    // in order, so that covers every slice)
    const int last_rs = (P - 1) * K - 1;
    for (int s = 0; s < P - 1; ++s) {
        Tick t;
        t.reduce.count = 0;
        if (s == 0) t.wait_reduce = last_rs;
        for (int j = 0; j < R; ++j) {
            const Range sc = chunk_range(n, es, P, R, j, mod(pos[j] + 1 - s));
            const Range rc = chunk_range(n, es, P, R, j, mod(pos[j] - s));
            if (sc.size()) t.ops.push_back(P2POp{true, succ[j], j, outb + sc.begin * es, sc.size() * es});
            if (rc.size()) t.ops.push_back(P2POp{false, pred[j], j, outb + rc.begin * es, rc.size() * es});
        }
        prog.ticks.push_back(std::move(t));
    }
}

RingConfig batch_bucket_config(RingConfig cfg, int P) {
    cfg = effective_config(cfg, P);
    // a merged tick posts one group and one allgather at most: every bucket runs a p2p schedule
    // whose reduce is a fold (direct; one-shot where picked) — the ring's two-input steps and the
    // collective allgathers of gather-fold / direct-gather are not merged
    if (cfg.algo != kAlgoOneShot) {
        cfg.algo = kAlgoDirect;
        cfg.rings = 1;
    }
    return cfg;
}

namespace {
size_t batch_block_elems(size_t n, size_t es, int P, const RingConfig &cfg) {
    const size_t e = program_staging_elems(n, es, P, cfg);
    const size_t g = kGranuleBytes / es;  // every bucket's block starts 256-byte aligned
    return (e + g - 1) / g * g;
}
}  // namespace

size_t batch_staging_elems(const size_t *ns, int count, size_t es, int P, const RingConfig &cfg_in) {
    const RingConfig cfg = batch_bucket_config(cfg_in, P);
    size_t total = 0;
    for (int b = 0; b < count; ++b)
        if (ns[b]) total += batch_block_elems(ns[b], es, P, cfg);
    return total;
}

void build_batch_program(RingProgram &prog, int rank, int P, const void *const *ins, void *const *outs,
                         const size_t *ns, int count, void *staging, int dtype, const RingConfig &cfg_in) {
    const RingConfig cfg = batch_bucket_config(cfg_in, P);
    const size_t es = dtype_size(dtype);
    prog.P = P;
    prog.rank = rank;
    prog.esize = es;
    prog.algo = cfg.algo;
    prog.R = 1;
    prog.K = 0;
    prog.n = 0;
    prog.staging_stride = 0;
    prog.staging_slots = 0;
    prog.ticks.clear();
    if (P <= 1) return;
    RingProgram part;
    char *st = static_cast<char *>(staging);
    for (int b = 0; b < count; ++b) {
        if (ns[b] == 0) continue;
        build_program(part, rank, P, ins[b], outs[b], st, ns[b], dtype, cfg);
        st += batch_block_elems(ns[b], es, P, cfg) * es;
        prog.n += ns[b];
        prog.K = std::max(prog.K, part.K);
        if (prog.ticks.size() < part.ticks.size()) prog.ticks.resize(part.ticks.size());
        for (size_t t = 0; t < part.ticks.size(); ++t) {
            Tick &dst = prog.ticks[t];
            Tick &src = part.ticks[t];
            DDL_REQUIRE(!src.gather.bytes && (!src.has_reduce || src.multi), DDL_STATUS_ERROR_UNKNOWN,
                        "grouped allreduce: tick " << t << " of bucket " << b << " cannot be merged");
            dst.reduce.count = 0;
            dst.copies.insert(dst.copies.end(), src.copies.begin(), src.copies.end());
            dst.ops.insert(dst.ops.end(), src.ops.begin(), src.ops.end());
            if (src.has_reduce) {
                dst.has_reduce = true;
                dst.multi = true;
                dst.folds.insert(dst.folds.end(), src.folds.begin(), src.folds.end());
            }
            dst.wait_reduce = std::max(dst.wait_reduce, src.wait_reduce);
        }
    }
}

void build_broadcast(RingProgram &prog, int rank, int P, int root, void *buf, size_t n, int dtype,
                     const RingConfig &cfg) {
    const size_t es = dtype_size(dtype);
    DDL_REQUIRE(root >= 0 && root < P, DDL_STATUS_INVALID_ARGUMENT, "root " << root << " outside [0, " << P << ")");
    prog.P = P;
    prog.rank = rank;
    prog.n = n;
    prog.esize = es;
    prog.algo = kAlgoDirect;
    prog.R = 1;
    prog.staging_stride = 0;
    prog.staging_slots = 0;
    prog.ticks.clear();
    size_t max_chunk = 0;
    for (int c = 0; c < P; ++c) max_chunk = std::max(max_chunk, chunk_range(n, es, P, 1, 0, c).size());
    int K = 1;
    if (cfg.slice_bytes > 0) K = (int)std::max<size_t>(1, (max_chunk * es + cfg.slice_bytes - 1) / cfg.slice_bytes);
    K = std::max(1, std::min(K, cfg.max_slices));
    prog.K = K;
    if (P <= 1 || n == 0) return;
    char *b = static_cast<char *>(buf);
    auto slice = [&](int c, int k) { return slice_range(chunk_range(n, es, P, 1, 0, c), es, K, k); };
    for (int t = 0; t <= K; ++t) {
        Tick tk;
        tk.reduce.count = 0;
        if (t < K) {  // scatter slice t
            if (rank == root) {
                for (int d = 1; d < P; ++d) {
                    const int c = (root + d) % P;
                    const Range r = slice(c, t);
                    if (r.size()) tk.ops.push_back(P2POp{true, c, 0, b + r.begin * es, r.size() * es});
                }
            } else {
                const Range r = slice(rank, t);
                if (r.size()) tk.ops.push_back(P2POp{false, root, 0, b + r.begin * es, r.size() * es});
            }
        }
        if (t >= 1) {  // allgather slice t-1: every chunk owner sends to every non-root peer
            const int k = t - 1;
            const Range mine = slice(rank, k);
            for (int d = 1; d < P; ++d) {
                const int q = (rank + d) % P;
                if (q != root && mine.size()) tk.ops.push_back(P2POp{true, q, 1, b + mine.begin * es, mine.size() * es});
            }
            if (rank != root) {
                for (int d = 1; d < P; ++d) {
                    const int q = (rank + P - d) % P;
                    const Range r = slice(q, k);
                    if (r.size()) tk.ops.push_back(P2POp{false, q, 1, b + r.begin * es, r.size() * es});
                }
            }
        }
        prog.ticks.push_back(std::move(tk));
    }
}

void build_allgatherv(RingProgram &prog, int rank, int P, const void *send, void *recv,
                      const size_t *counts, const size_t *displs, int dtype) {
    const size_t es = dtype_size(dtype);
    prog.P = P;
    prog.rank = rank;
    prog.esize = es;
    prog.algo = kAlgoDirect;
    prog.R = 1;
    prog.K = 1;
    prog.staging_stride = 0;
    prog.staging_slots = 0;
    prog.ticks.clear();
    prog.n = 0;
    for (int q = 0; q < P; ++q) prog.n += counts[q];
    if (prog.n == 0) return;
    char *r = static_cast<char *>(recv);
    Tick tk;
    tk.reduce.count = 0;
    const size_t mine = counts[rank] * es;
    char *dst = r + displs[rank] * es;
    if (mine && dst != send) tk.copies.push_back(CopyOp{send, dst, mine});
    for (int d = 1; d < P; ++d) {
        const int to = (rank + d) % P, from = (rank + P - d) % P;
        if (mine) tk.ops.push_back(P2POp{true, to, 0, const_cast<void *>(send), mine});
        if (counts[from]) tk.ops.push_back(P2POp{false, from, 0, r + displs[from] * es, counts[from] * es});
    }
    prog.ticks.push_back(std::move(tk));
}

}  // namespace ddl
