// schedule.h — the ring reduce-scatter / allgather schedule (host side, no GPU calls).
//
// Replaces what MPICH does inside MPI_Allreduce at the reference's data-plane call
// (src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28) with an explicit multi-ring
// schedule for a fully connected xGMI node:
//   * R rings = edge-disjoint directed Hamiltonian cycles of the P ranks (ring 0 is the
//     natural ring r -> r+1, the direction of the reference's token ring,
//     RingTokenCommunicateHandler.cc:52-54); P = 8 gives 7 rings, one per xGMI link;
//   * the bucket splits into R*P chunks of 256-byte granules (ring j owns chunks j*P..j*P+P-1);
//   * reduce-scatter: P-1 steps, each chunk split into K slices so the recv of slice k+1
//     overlaps the reduce of slice k; allgather: P-1 steps, received straight into `out`.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

#include "common.h"

namespace ddl {

struct Range {
    size_t begin = 0, end = 0;
    size_t size() const { return end > begin ? end - begin : 0; }
};

constexpr size_t kGranuleBytes = 256;
constexpr int kMaxRings = kMaxSegments;  // one reduce segment per ring per launch

// Edge-disjoint directed Hamiltonian cycles of K_P (deterministic DFS; ring 0 = identity).
// Returns at most max_rings rings; each ring is the list of ranks in ring order.
const std::vector<std::vector<int>> &rings_for(int P, int max_rings);

// Element range of (ring, chunk) — granules split evenly over R*P parts.
Range chunk_range(size_t n, size_t esize, int P, int R, int ring, int chunk);
// Element range of slice k of K inside `chunk` (granule-aligned, relative to the bucket).
Range slice_range(const Range &chunk, size_t esize, int K, int k);

struct P2POp {
    bool send;
    int peer;
    int tag;  // ring index: matches a send with its recv inside one tick
    void *ptr;
    size_t bytes;
};

struct CopyOp {  // device-to-device copy posted on the comm stream before the tick's group
    const void *src;
    void *dst;
    size_t bytes;
};

// A collective allgather posted on the comm stream after the tick's copies: every rank's
// `bytes` at `send` land at recv + q * bytes on every rank q (ncclAllGather over RCCL).
struct GatherOp {
    const void *send = nullptr;
    void *recv = nullptr;
    size_t bytes = 0;
};

struct Tick {
    std::vector<CopyOp> copies;
    std::vector<P2POp> ops;
    GatherOp gather;       // valid when gather.bytes > 0
    SegTable reduce;       // valid when has_reduce && !multi
    // valid when has_reduce && multi (direct / one-shot): N-input fold steps run in order; one
    // step up to 16 ranks, a chain or tree of steps through temp slots beyond (plan_fold)
    std::vector<SegTableN> folds;
    bool has_reduce = false;
    bool multi = false;
    int wait_reduce = -1;  // the comm stream waits for this tick's reduce before posting ops
};

enum Algo : int {
    kAlgoRing = 0,    // multi-ring reduce-scatter + allgather (edge-disjoint Hamiltonian cycles)
    kAlgoDirect = 1,  // every rank exchanges with every peer at once (fully connected mesh)
    kAlgoOneShot = 2, // small buckets: every rank sends its whole bucket to every peer in one
                      // group and folds all P inputs in rank order (one group instead of 2)
    kAlgoGatherFold = 3, // small buckets: one ncclAllGather of the bucket (RCCL's low-latency
                         // collective path instead of 2(P-1) grouped p2p ops), then the same
                         // rank-order fold as one-shot
    kAlgoDirectGather = 4, // the direct reduce-scatter (p2p ticks + rank-order folds), then ONE
                           // in-place ncclAllGather of the reduced chunks instead of K p2p
                           // allgather ticks; needs equal chunks (direct_gather_eligible), else
                           // it runs as kAlgoDirect
};

// Direct-gather's allgather is one collective over equal, contiguous chunks: every chunk of
// chunk_range(n, es, P, 1, 0, q) has n / P elements exactly when the bucket is a whole number of
// P-granule groups.
inline bool direct_gather_eligible(size_t n, size_t esize, int P) {
    return P > 1 && n > 0 && (n * esize) % (kGranuleBytes * (size_t)P) == 0;
}
inline bool is_direct(int algo) { return algo == kAlgoDirect || algo == kAlgoDirectGather; }

// Largest bucket the autotuner tries the one-shot schedule on.
constexpr size_t kOneShotMaxBytes = 1u << 20;

struct RingConfig {
    int algo = kAlgoRing;
    int rings = kMaxRings;            // upper bound; clipped to what the topology allows
    size_t slice_bytes = 2u << 20;    // target bytes per reduce-scatter message
    int max_slices = 8;
    // Reference order: the sum of every element equals the reference's MPI_Allreduce (MPICH
    // 3.3.2) bit for bit. Direct and one-shot fold the P inputs in rank order in MPICH's tree
    // (FoldOrder kFoldMpichTree / kFoldBinomial, picked by the message size); the ring, whose
    // order cannot follow it at P > 2, runs as the direct schedule there (effective_config).
    // 0: direct folds left in ring 0's order, the ring runs as configured.
    int ref_order = 0;
    size_t order_bytes = 0;  // message size that picks MPICH's algorithm (0 = this bucket's)
};

// The schedule that actually runs for P ranks: with ref_order, a ring at P > 2 becomes the
// direct schedule with the same slicing. Every builder and shape query goes through it.
inline RingConfig effective_config(RingConfig c, int P) {
    if (c.ref_order && c.algo == kAlgoRing && P > 2) {
        c.algo = kAlgoDirect;
        c.rings = 1;
    }
    return c;
}

// Fold steps that compute out = x_0 + ... + x_{K-1} (xs in the order the sum takes them) in
// FoldOrder `order`, each step at most kMaxInputs + 1 inputs over n elements. Up to 16 inputs
// it is one step. Beyond: kFoldLeft chains 16-input steps through one partial; the MPICH orders
// fold aligned blocks of 16 (pre-folded pairs first for kFoldMpichTree), then the block sums,
// which is the same tree. Partial sums go to temp(0), temp(1), ... (n elements each, at most
// fold_temp_slots(K) of them).
void plan_fold(std::vector<SegTableN> &steps, const std::vector<const void *> &xs, void *out, size_t n, int order,
               const std::function<void *(int)> &temp);
// Partial sums plan_fold(K inputs) needs in `order` (a dry run of its steps), and the most any
// order needs (what staging reserves: the order also depends on dtype and message size).
int fold_temp_count(int K, int order);
inline int fold_temp_slots(int K) {
    int m = 0;
    for (int o : {kFoldLeft, kFoldMpichTree, kFoldBinomial}) m = fold_temp_count(K, o) > m ? fold_temp_count(K, o) : m;
    return m;
}

// Per-rank tick list of one allreduce. `staging` must hold staging_elems(R, stride) elements:
// two slots per ring (reduce-scatter step parity), ring j / parity q at (2j + q) * stride.
inline size_t staging_elems(int R, size_t stride) { return 2 * (size_t)R * stride; }
struct RingProgram {
    int P = 1, R = 1, K = 1, rank = 0, algo = kAlgoRing;
    size_t n = 0, esize = 0;
    size_t staging_stride = 0;  // elements per staging slot
    size_t staging_slots = 0;   // ring: 2 per ring (step parity); direct / one-shot: P-1 (one per peer);
                                // gather-fold: P (one per rank) + 1 (padded copy of the input)
    std::vector<Tick> ticks;
};

// Number of rings and slices the schedule uses for this problem (direct: R = 1, K slices).
void ring_shape(size_t n, size_t esize, int P, const RingConfig &cfg, int *R, int *K,
                size_t *staging_stride);
// Staging elements the program needs, and its staging slots.
size_t program_staging_elems(size_t n, size_t esize, int P, const RingConfig &cfg);
size_t program_staging_slots(int P, int algo, int R);
// Gather-fold slot stride (elements): the bucket itself when its byte size keeps every slot
// 16-byte aligned, else the bucket rounded up to 64 elements (the input is copied in first).
inline size_t gather_stride(size_t n, size_t esize) { return (n * esize) % 16 == 0 ? n : (n + 63) & ~size_t(63); }

// Builds rank `rank`'s program. in/out are that rank's buffers, staging its scratch.
void build_program(RingProgram &prog, int rank, int P, const void *in, void *out, void *staging,
                   size_t n, int dtype, const RingConfig &cfg);

// Grouped allreduce of `count` buckets of one dtype (ins[b] -> outs[b], ns[b] elements) as ONE
// program: every bucket's own program (batch_bucket_config: the direct schedule, or one-shot where
// the config picks it), merged tick by tick — tick t posts every bucket's tick-t copies and p2p ops
// as one group and folds every bucket's tick-t slices in as few launches as kMaxFoldBatch allows
// (launch_tick_reduce); the merged tick waits for the latest reduce any bucket's tick waits for
// (the compute stream is in order, so that covers the others). Per element the sums are exactly the
// buckets' own (same fold, same order; `cfg.order_bytes` 0: each bucket's own message size). Bucket
// b's staging is its own block of batch_staging_elems' layout.
RingConfig batch_bucket_config(RingConfig cfg, int P);
size_t batch_staging_elems(const size_t *ns, int count, size_t esize, int P, const RingConfig &cfg);
void build_batch_program(RingProgram &prog, int rank, int P, const void *const *ins, void *const *outs,
                         const size_t *ns, int count, void *staging, int dtype, const RingConfig &cfg);

// Broadcast of `root`'s n elements into every rank's `buf` (MPICommunicator.cc:77-90 is
// MPI_Bcast): scatter (root sends chunk c to rank c) + direct allgather of the chunks, K
// slices pipelined so the allgather of slice k shares a tick with the scatter of slice k+1.
// Every xGMI link out of the root carries 2S/P instead of S. Ticks 0..K; tag 0 scatter,
// tag 1 allgather (within a tick, ops to one peer are posted tag 0 first on both sides).
void build_broadcast(RingProgram &prog, int rank, int P, int root, void *buf, size_t n, int dtype,
                     const RingConfig &cfg);

// Allgatherv (MPICommunicator.cc:31-60 is MPI_Allgatherv): rank q's counts[q] elements land at
// recv + displs[q] on every rank. One tick: a copy of the own block (unless already in
// place) and, for every peer, one send of the own block and one recv of the peer's block.
void build_allgatherv(RingProgram &prog, int rank, int P, const void *send, void *recv,
                      const size_t *counts, const size_t *displs, int dtype);

}  // namespace ddl
