// control.cpp — see control.h.
#include "control.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "common.h"

namespace ddl {

namespace {

void write_all(int fd, const void *p, size_t n) {
    const char *c = static_cast<const char *>(p);
    while (n) {
        ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR) continue;
        DDL_REQUIRE(w > 0, DDL_STATUS_COMM_ERROR, "control channel send failed: " << std::strerror(errno));
        c += w;
        n -= (size_t)w;
    }
}

void read_all(int fd, void *p, size_t n) {
    char *c = static_cast<char *>(p);
    while (n) {
        ssize_t r = ::recv(fd, c, n, 0);
        if (r < 0 && errno == EINTR) continue;
        DDL_REQUIRE(r > 0, DDL_STATUS_COMM_ERROR,
                    "control channel closed by peer" << (r < 0 ? std::string(": ") + std::strerror(errno) : ""));
        c += r;
        n -= (size_t)r;
    }
}

void split_endpoint(const std::string &ep, std::string &host, int &port) {
    size_t c = ep.rfind(':');
    DDL_REQUIRE(c != std::string::npos, DDL_STATUS_INVALID_ARGUMENT, "bad endpoint '" << ep << "'");
    host = ep.substr(0, c);
    port = std::atoi(ep.c_str() + c + 1);
}

void tune(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

}  // namespace

ControlChannel::~ControlChannel() { close_all(); }

void ControlChannel::close_all() {
    cache.clear();
    if (listen_fd_ >= 0) ::close(listen_fd_);
    listen_fd_ = -1;
    for (int fd : fd_)
        if (fd >= 0) ::close(fd);
    fd_.clear();
}

bool ControlChannel::connected() const {
    if (size_ <= 1 || fd_.empty()) return false;
    if (rank_ != 0) return fd_[0] >= 0;
    for (int r = 1; r < size_; ++r)
        if (fd_[r] < 0) return false;
    return true;
}

std::string ControlChannel::listen() {
    DDL_REQUIRE(listen_fd_ < 0, DDL_STATUS_INVALID_ARGUMENT, "control channel already listening");
    // The token channel is a single-node, same-host channel: it binds to loopback. A deployment
    // that spans hosts opts in by naming the interface address in $DDL_CONTROL_HOST.
    const char *env = std::getenv("DDL_CONTROL_HOST");
    const std::string host = env && *env ? env : "127.0.0.1";
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = 0;
    DDL_REQUIRE(inet_pton(AF_INET, host.c_str(), &a.sin_addr) == 1, DDL_STATUS_INVALID_ARGUMENT,
                "DDL_CONTROL_HOST '" << host << "' is not an IPv4 address");
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    DDL_REQUIRE(listen_fd_ >= 0, DDL_STATUS_COMM_ERROR, "socket: " << std::strerror(errno));
    DDL_REQUIRE(::bind(listen_fd_, (sockaddr *)&a, sizeof a) == 0, DDL_STATUS_COMM_ERROR,
                "bind " << host << ": " << std::strerror(errno));
    DDL_REQUIRE(::listen(listen_fd_, 128) == 0, DDL_STATUS_COMM_ERROR, "listen: " << std::strerror(errno));
    socklen_t len = sizeof a;
    getsockname(listen_fd_, (sockaddr *)&a, &len);
    return host + ":" + std::to_string(ntohs(a.sin_port));
}

void ControlChannel::connect(int rank, int size, const std::vector<std::string> &eps, int timeout_ms) {
    DDL_REQUIRE(size >= 1 && rank >= 0 && rank < size && (int)eps.size() == size,
                DDL_STATUS_INVALID_ARGUMENT, "control connect: " << eps.size() << " endpoints for size " << size);
    rank_ = rank;
    size_ = size;
    cache.clear();
    if (size == 1) return;
    DDL_REQUIRE(listen_fd_ >= 0, DDL_STATUS_INVALID_ARGUMENT, "ddl_control_listen must come first");
    for (int fd : fd_)
        if (fd >= 0) ::close(fd);
    fd_.assign(rank == 0 ? size : 1, -1);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    if (rank != 0) {
        // connect to rank 0 (its listener may not be accepting yet: retry)
        std::string host;
        int port = 0;
        split_endpoint(eps[0], host, port);
        for (;;) {
            int fd = ::socket(AF_INET, SOCK_STREAM, 0);
            DDL_REQUIRE(fd >= 0, DDL_STATUS_COMM_ERROR, "socket: " << std::strerror(errno));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_port = htons((uint16_t)port);
            DDL_REQUIRE(inet_pton(AF_INET, host.c_str(), &a.sin_addr) == 1, DDL_STATUS_INVALID_ARGUMENT,
                        "bad control host '" << host << "'");
            if (::connect(fd, (sockaddr *)&a, sizeof a) == 0) {
                tune(fd);
                int32_t me = rank;
                write_all(fd, &me, sizeof me);
                fd_[0] = fd;
                break;
            }
            ::close(fd);
            DDL_REQUIRE(std::chrono::steady_clock::now() < deadline, DDL_STATUS_COMM_ERROR,
                        "control connect to " << eps[0] << " timed out");
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
    } else {
        // accept every member (a connection announcing an unknown or repeated rank is dropped)
        int missing = size - 1;
        while (missing > 0) {
            pollfd p{listen_fd_, POLLIN, 0};
            int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                           deadline - std::chrono::steady_clock::now()).count();
            DDL_REQUIRE(left > 0, DDL_STATUS_COMM_ERROR, "control accept: " << missing << " rank(s) missing");
            if (::poll(&p, 1, left) <= 0) continue;
            int fd = ::accept(listen_fd_, nullptr, nullptr);
            if (fd < 0) continue;
            int32_t who = -1;
            read_all(fd, &who, sizeof who);
            if (who >= 1 && who < size && fd_[who] < 0) {
                tune(fd);
                fd_[who] = fd;
                --missing;
            } else {
                ::close(fd);
            }
        }
    }
    // the star is complete: no further connections are accepted
    ::close(listen_fd_);
    listen_fd_ = -1;
}

namespace {
void send_token(int fd, const Token &t) {
    unsigned char hdr[26];
    uint64_t len = t.msg.size();
    hdr[0] = t.type;
    hdr[1] = t.request;
    std::memcpy(hdr + 2, &len, 8);  // host byte order, as the reference's MPI_Pack of size_t
    std::memcpy(hdr + 10, &t.cfg, 8);  // the engine's extension
    std::memcpy(hdr + 18, &t.seq, 8);
    write_all(fd, hdr, sizeof hdr);
    if (len) write_all(fd, t.msg.data(), len);
}

bool recv_token(int fd, Token &t, int timeout_ms) {
    if (timeout_ms >= 0) {
        pollfd p{fd, POLLIN, 0};
        int r = ::poll(&p, 1, timeout_ms);
        if (r == 0) return false;
        DDL_REQUIRE(r > 0, DDL_STATUS_COMM_ERROR, "control poll: " << std::strerror(errno));
    }
    unsigned char hdr[26];
    read_all(fd, hdr, sizeof hdr);
    uint64_t len;
    std::memcpy(&len, hdr + 2, 8);
    std::memcpy(&t.cfg, hdr + 10, 8);
    std::memcpy(&t.seq, hdr + 18, 8);
    DDL_REQUIRE(len < (1ull << 32), DDL_STATUS_COMM_ERROR, "control token too long: " << len);
    t.type = hdr[0];
    t.request = hdr[1];
    t.msg.assign(len, '\0');
    if (len) read_all(fd, &t.msg[0], len);
    return true;
}
}  // namespace

void ControlChannel::send(const Token &t) {
    DDL_REQUIRE(connected(), DDL_STATUS_NOT_INITIALIZED, "control channel not connected");
    if (rank_ != 0) {
        send_token(fd_[0], t);
        return;
    }
    for (int r = 1; r < size_; ++r) send_token(fd_[r], t);
}

bool ControlChannel::recv(Token &t, int timeout_ms) {
    DDL_REQUIRE(rank_ != 0 && connected(), DDL_STATUS_NOT_INITIALIZED, "control recv: not a connected member");
    return recv_token(fd_[0], t, timeout_ms);
}

bool ControlChannel::recv_from(int from, Token &t, int timeout_ms) {
    DDL_REQUIRE(rank_ == 0 && from >= 1 && from < size_ && connected(), DDL_STATUS_INVALID_ARGUMENT,
                "control recv_from(" << from << ") on rank " << rank_);
    return recv_token(fd_[from], t, timeout_ms);
}

bool IdCache::lookup(const std::string &id, uint32_t *idx) const {
    auto it = index_.find(id);
    if (it == index_.end()) return false;
    *idx = it->second;
    return true;
}

const std::string &IdCache::at(uint32_t i) const {
    DDL_REQUIRE(i < ids_.size(), DDL_STATUS_COMM_ERROR, "token: cached id " << i << " out of range " << ids_.size());
    return ids_[i];
}

bool IdCache::learn(const std::vector<std::string> &agreed) {
    const bool cleared = ids_.size() + agreed.size() > kMax;  // same decision on every rank
    if (cleared) clear();
    for (const auto &id : agreed) {
        if (index_.count(id)) continue;
        index_.emplace(id, (uint32_t)ids_.size());
        ids_.push_back(id);
    }
    return cleared;
}

void IdCache::clear() {
    index_.clear();
    ids_.clear();
}

// msg[0] = 0: bitmap over the table; 1: little-endian u32 indices
std::string IdCache::encode(const std::vector<uint32_t> &idx) const {
    const size_t bitmap = (ids_.size() + 7) / 8, list = 4 * idx.size();
    std::string m;
    if (bitmap <= list) {
        m.assign(1 + bitmap, '\0');
        for (uint32_t i : idx) m[1 + i / 8] = (char)((unsigned char)m[1 + i / 8] | (1u << (i % 8)));
    } else {
        m.assign(1 + list, '\0');
        m[0] = 1;
        for (size_t k = 0; k < idx.size(); ++k) std::memcpy(&m[1 + 4 * k], &idx[k], 4);
    }
    return m;
}

std::vector<uint32_t> IdCache::decode(const std::string &msg) const {
    std::vector<uint32_t> out;
    DDL_REQUIRE(!msg.empty(), DDL_STATUS_COMM_ERROR, "token: empty cached-id message");
    if (msg[0] == 0) {
        DDL_REQUIRE(msg.size() - 1 <= (ids_.size() + 7) / 8, DDL_STATUS_COMM_ERROR, "token: bitmap beyond the id table");
        for (size_t b = 1; b < msg.size(); ++b) {
            const unsigned char v = (unsigned char)msg[b];
            if (!v) continue;
            for (int k = 0; k < 8; ++k)
                if (v & (1u << k)) out.push_back((uint32_t)((b - 1) * 8 + k));
        }
    } else {
        DDL_REQUIRE(msg[0] == 1 && (msg.size() - 1) % 4 == 0, DDL_STATUS_COMM_ERROR, "token: bad cached-id message");
        for (size_t p = 1; p < msg.size(); p += 4) {
            uint32_t i;
            std::memcpy(&i, &msg[p], 4);
            out.push_back(i);
        }
    }
    for (uint32_t i : out) DDL_REQUIRE(i < ids_.size(), DDL_STATUS_COMM_ERROR, "token: cached id out of range");
    return out;
}

std::string encode_keys(const std::vector<std::string> &keys) {
    std::string s;
    for (const auto &k : keys) s.append(k).append("\n");
    return s;
}

std::vector<std::string> decode_keys(const std::string &msg) {
    std::vector<std::string> keys;
    size_t pos = 0;
    while (pos < msg.size()) {
        size_t nl = msg.find('\n', pos);
        if (nl == std::string::npos) nl = msg.size();
        keys.push_back(msg.substr(pos, nl - pos));
        pos = nl + 1;
    }
    return keys;
}

}  // namespace ddl
