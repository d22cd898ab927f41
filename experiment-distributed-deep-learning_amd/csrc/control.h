// control.h — host control channel: TCP links carrying negotiation tokens.
//
// Replaces the reference's token transport over MPI point-to-point
// (communicate/tensor/collective/controller/rtc/mpi/MPIRingTokenCommunication.cc:29-102). The
// reference passes the token around a ring (rank -> rank+1), so a round's two laps cost 2P
// hops. Here the links form a star around rank 0: rank 0 sends the proposal to every member,
// each member answers with its intersection, rank 0 intersects the answers and sends the
// agreed set to every member — 3 hops at any P, the members' hops in parallel (a single-key
// round at P = 8 on 8 cores: 0.35 ms as a ring). A token on the wire is the same packed header
// the reference sends with MPI_Pack — {u8 type, u8 request type, u64 length} (10 bytes,
// :25,44-53) — then a 16-byte engine extension {u64 config hash, i64 user-collective count}
// (the round's config agreement and its place among the communicator's user collectives, see
// handler.h), then `length` bytes of key list.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace ddl {

// Token types / request types: reference rtc/Token.h:20-33, plus the two cached-id forms of
// SYNC / COMMUNICATE (the key set as indices into IdCache instead of strings).
enum TokenType : uint8_t { TOKEN_READY = 0, TOKEN_SYNC = 1, TOKEN_COMMUNICATE = 2, TOKEN_SHUT_DOWN = 3,
                           TOKEN_SYNC_CACHED = 4, TOKEN_COMMUNICATE_CACHED = 5 };
enum TokenRequest : uint8_t { TOKEN_REQUEST_SHUTDOWN = 0, TOKEN_REQUEST_ALLREDUCE = 1, TOKEN_REQUEST_BROADCAST = 2,
                            TOKEN_REQUEST_ALLGATHER = 3 };

struct Token {
    uint8_t type = TOKEN_READY;
    uint8_t request = TOKEN_REQUEST_ALLREDUCE;
    uint64_t cfg = 0;  // sender's shared-config hash (kCfgMismatch in a COMMUNICATE: ranks disagree)
    int64_t seq = -1;  // user collectives issued (SYNC answers) / the round's release point (COMMUNICATE)
    std::string msg;
};
constexpr uint64_t kCfgMismatch = ~0ull;

// Request ids agreed in earlier rounds, in agreement order. Every rank appends the same agreed
// lists in the same order, so the tables are identical across ranks and a proposal made only
// of known ids can travel as indices (a bitmap or a u32 list, whichever is shorter) instead of
// "Type::key" strings — for a training step's 4096 gradient keys, ~0.5 KB instead of ~100 KB
// per hop.
class IdCache {
public:
    bool lookup(const std::string &id, uint32_t *idx) const;
    const std::string &at(uint32_t i) const;
    size_t size() const { return ids_.size(); }
    // Appends the unseen ids of an agreed list (in list order). Past kMax entries the table is
    // cleared first — the same decision on every rank; returns true then.
    bool learn(const std::vector<std::string> &agreed);
    std::string encode(const std::vector<uint32_t> &idx) const;
    std::vector<uint32_t> decode(const std::string &msg) const;
    void clear();
    static constexpr size_t kMax = 1u << 20;

private:
    std::unordered_map<std::string, uint32_t> index_;
    std::vector<std::string> ids_;
};

class ControlChannel {
public:
    ControlChannel() = default;
    ~ControlChannel();
    ControlChannel(const ControlChannel &) = delete;
    ControlChannel &operator=(const ControlChannel &) = delete;

    // Opens the listening socket; returns "host:port" (host from $DDL_CONTROL_HOST, default
    // 127.0.0.1 — one node).
    std::string listen();
    // Rank 0 accepts one connection from every other rank; the others connect to rank 0's
    // endpoint (their own listeners are closed unused).
    void connect(int rank, int size, const std::vector<std::string> &endpoints, int timeout_ms);
    bool connected() const;

    // Member: to rank 0. Rank 0: to every member, in rank order.
    void send(const Token &t);
    // Member: the next token from rank 0. Blocks until one arrives, or returns false after
    // timeout_ms (< 0: forever).
    bool recv(Token &t, int timeout_ms);
    // Rank 0: the next token from member `from` (1 .. size-1).
    bool recv_from(int from, Token &t, int timeout_ms);
    int rank() const { return rank_; }
    int size() const { return size_; }
    void close_all();

    IdCache cache;                 // see IdCache; reset by connect / close_all
    long long string_rounds = 0;   // negotiation rounds by token form (ddl_control_stats)
    long long cached_rounds = 0;

private:
    int listen_fd_ = -1;
    std::vector<int> fd_;  // rank 0: fd_[r] links member r (fd_[0] unused); member: fd_[0] links rank 0
    int rank_ = 0, size_ = 1;
};

// One request id ("<Type>::<key>", e.g. "Allreduce::grad_0") per line — the reference's token
// message format (RingTokenCommunicateHandler.cc:10-11, 140-147, 412-437).
std::string encode_keys(const std::vector<std::string> &keys);
std::vector<std::string> decode_keys(const std::string &msg);

}  // namespace ddl
