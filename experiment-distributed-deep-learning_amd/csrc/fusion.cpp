// fusion.cpp — see fusion.h.
#include "fusion.h"

#include "deptrace.h"
#include "engine.h"

namespace ddl {

FusionPipe::~FusionPipe() {
    // best effort at teardown
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
    if (side_) (void)hipStreamDestroy(side_);
    for (void *b : buf_)
        if (b) (void)hipFree(b);
}

void *FusionPipe::ensure(int i, size_t need, hipStream_t stream) {
    void *&buf = buf_[i];
    size_t &cap = cap_[i];
    if (need > cap) {
        if (buf) {  // may still be read on the device; no hipFree on a data path (engine.h retire_device)
            retire_device(buf);
            buf = nullptr;
            cap = 0;
        }
        const size_t sz = need + need / 2;  // x1.5 growth (MPIRingTokenCommunication.cc:13, 480)
        DDL_HIP(hipMalloc(&buf, sz));
        cap = sz;
    }
    return buf;
}

hipEvent_t FusionPipe::event_(size_t i) {
    while (events_.size() <= i) {
        hipEvent_t e;
        DDL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        events_.push_back(e);
    }
    return events_[i];
}

void FusionPipe::run(const std::vector<const void *> &srcs, const std::vector<void *> &dsts,
                     const std::vector<size_t> &bytes, int dt, size_t cap, hipStream_t stream, const Allreduce &ar) {
    const size_t es = dtype_size(dt);
    DDL_REQUIRE(es != 0, DDL_STATUS_UNSUPPORTED_DTYPE, "unsupported dtype " << dt);
    DDL_REQUIRE(srcs.size() == bytes.size() && dsts.size() == bytes.size(), DDL_STATUS_INVALID_ARGUMENT,
                "fusion plan: " << srcs.size() << " sources, " << dsts.size() << " destinations, " << bytes.size()
                                << " sizes");
    const size_t total = SegmentCopier::flat_bytes(bytes.data(), (int)bytes.size());
    // the reference's MPI buffer holds the requests back to back (no padding): its byte count
    // picks MPICH's summation order (reference_order)
    size_t message = 0;
    for (size_t b : bytes) message += b;
    cap &= ~size_t(255);
    if (cap == 0 || total <= cap) {
        last_subplans_ = 1;
        void *fb = ensure(0, total, stream);
        copier.run(0, fb, const_cast<void *const *>(reinterpret_cast<const void *const *>(srcs.data())), bytes.data(),
                   (int)srcs.size(), stream);
        ar(fb, total / es, message);
        copier.run(1, fb, dsts.data(), bytes.data(), (int)dsts.size(), stream);
        return;
    }
    struct Sub {
        std::vector<const void *> src;
        std::vector<void *> dst;
        std::vector<size_t> bytes;
        size_t flat = 0;
    };
    std::vector<Sub> subs(1);
    for (size_t i = 0; i < bytes.size(); ++i) {
        size_t off = 0;
        do {
            Sub *cur = &subs.back();
            if (cur->flat >= cap) {
                subs.emplace_back();
                cur = &subs.back();
            }
            // a piece fills the sub-plan up to cap; every cut is a multiple of 256 bytes (and so of
            // the element size) from the segment start
            const size_t room = cap - cur->flat, left = bytes[i] - off;
            const size_t len = left <= room ? left : room;
            cur->src.push_back(static_cast<const char *>(srcs[i]) + off);
            cur->dst.push_back(static_cast<char *>(dsts[i]) + off);
            cur->bytes.push_back(len);
            cur->flat += (len + 255) & ~size_t(255);
            off += len;
        } while (off < bytes[i]);
    }
    size_t maxflat = 0;
    for (const Sub &sb : subs) maxflat = sb.flat > maxflat ? sb.flat : maxflat;
    void *buf[2] = {ensure(0, maxflat, stream), ensure(1, maxflat, stream)};
    if (!side_) side_ = create_engine_stream(qc);
    const size_t J = subs.size();
    last_subplans_ = J;
    // events: [0] fork, [1 + 2j] pack j done, [2 + 2j] allreduce j done, [1 + 2J] join
    for (size_t k = 0; k <= 2 * J + 1; ++k) event_(k);
    DDL_HIP(hipEventRecord(events_[0], stream));  // inputs ready (the caller's waits ran on stream)
    dep::record(events_[0], stream);
    DDL_HIP(hipStreamWaitEvent(side_, events_[0], 0));
    dep::wait(side_, events_[0]);
    auto unpack = [&](size_t j) {
        DDL_HIP(hipStreamWaitEvent(side_, events_[2 + 2 * j], 0));
        dep::wait(side_, events_[2 + 2 * j]);
        copier.run(1, buf[j % 2], subs[j].dst.data(), subs[j].bytes.data(), (int)subs[j].dst.size(), side_);
    };
    for (size_t j = 0; j < J; ++j) {
        Sub &sb = subs[j];
        copier.run(0, buf[j % 2], const_cast<void *const *>(reinterpret_cast<const void *const *>(sb.src.data())),
                   sb.bytes.data(), (int)sb.src.size(), side_);
        DDL_HIP(hipEventRecord(events_[1 + 2 * j], side_));
        dep::record(events_[1 + 2 * j], side_);
        DDL_HIP(hipStreamWaitEvent(stream, events_[1 + 2 * j], 0));
        dep::wait(stream, events_[1 + 2 * j]);
        ar(buf[j % 2], sb.flat / es, message);
        DDL_HIP(hipEventRecord(events_[2 + 2 * j], stream));
        dep::record(events_[2 + 2 * j], stream);
        if (j >= 1) unpack(j - 1);
    }
    unpack(J - 1);
    DDL_HIP(hipEventRecord(events_[1 + 2 * J], side_));
    dep::record(events_[1 + 2 * J], side_);
    DDL_HIP(hipStreamWaitEvent(stream, events_[1 + 2 * J], 0));
    dep::wait(stream, events_[1 + 2 * J]);
}

}  // namespace ddl
