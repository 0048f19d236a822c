// nsx/pipe.hpp — in-process loopback connection with the semantics of the
// reference's unbuffered transport/pipe (transport/pipe/pipe.go), used to feed
// checksum batches from a transport and as the config-1
// harness (64×1500 B over loopback).
//
// Semantics mirrored from pipe.go:
//   - Pipe() returns two connected ends (pipe.go:44-63); bytes written on one
//     are read on the other.
//   - Write hands the caller's buffer to the reader (no intermediate copy) and
//     blocks until the reader has consumed it all, possibly over several Reads
//     (pipe.go:92-124); concurrent writers are serialised (writeMu, :102-103).
//   - Read copies min(len, offered) bytes and reports the count back to the
//     writer (pipe.go:73-90).
//   - Close makes pending and later Read/Write on either end return kClosed
//     (pipe.go:66-71, 84-87, 114-117); Close is idempotent.
//   - Read/Write deadlines return kDeadline (pipe.go:88, 118; chanDeadLine).
//   - Write of an empty buffer returns 0 immediately (pipe.go:97-99).
// Header-only C++17.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <utility>

namespace nsx::pipe {

enum class Err { kOk = 0, kClosed, kDeadline };

using Clock = std::chrono::steady_clock;

class End;

// Shared state of one connection: one rendezvous slot per direction.
struct Shared {
    std::mutex m;
    std::condition_variable cv;
    struct Slot {
        const uint8_t* offered = nullptr;  // writer's remaining bytes
        size_t offered_len = 0;
        size_t taken = 0;      // bytes the reader consumed from the current offer
        bool consumed = false;
    } slot[2];                 // slot[i]: bytes flowing into end i
    bool closed[2] = {false, false};
    std::mutex write_mu[2];    // per-writer serialisation (writeMu)
};

class End {
public:
    End(std::shared_ptr<Shared> s, int me, std::string name, std::string peer)
        : s_(std::move(s)), me_(me), name_(std::move(name)), peer_(std::move(peer)) {}

    const std::string& local_addr() const { return name_; }   // pipe.go:65
    const std::string& remote_addr() const { return peer_; }  // pipe.go:66

    void set_read_deadline(Clock::time_point t) { std::lock_guard<std::mutex> g(s_->m); rdl_ = t; has_rdl_ = true; s_->cv.notify_all(); }
    void set_write_deadline(Clock::time_point t) { std::lock_guard<std::mutex> g(s_->m); wdl_ = t; has_wdl_ = true; s_->cv.notify_all(); }
    // SetReadDeadLine(time.Time{}) / SetWriteDeadLine(time.Time{}): no deadline.
    void clear_read_deadline() { std::lock_guard<std::mutex> g(s_->m); has_rdl_ = false; s_->cv.notify_all(); }
    void clear_write_deadline() { std::lock_guard<std::mutex> g(s_->m); has_wdl_ = false; s_->cv.notify_all(); }

    // Read up to len bytes (pipe.go:73-90).
    Err read(uint8_t* buf, size_t len, size_t* n) {
        *n = 0;
        std::unique_lock<std::mutex> lk(s_->m);
        Shared::Slot& in = s_->slot[me_];
        for (;;) {
            if (dead()) return Err::kClosed;                               // checkReadOK order
            if (has_rdl_ && Clock::now() >= rdl_) return Err::kDeadline;
            if (in.offered && !in.consumed) break;
            if (has_rdl_) s_->cv.wait_until(lk, rdl_);
            else s_->cv.wait(lk);
        }
        const size_t k = len < in.offered_len ? len : in.offered_len;
        if (k) std::memcpy(buf, in.offered, k);
        in.taken = k;
        in.consumed = true;
        s_->cv.notify_all();
        *n = k;
        return Err::kOk;
    }

    // Write all of buf (pipe.go:92-124); *n = bytes delivered.
    Err write(const uint8_t* buf, size_t len, size_t* n) {
        *n = 0;
        {   // checkWriteOK precedes the empty-write shortcut (pipe.go:93-99)
            std::lock_guard<std::mutex> g(s_->m);
            if (dead()) return Err::kClosed;
            if (has_wdl_ && Clock::now() >= wdl_) return Err::kDeadline;
            if (len == 0) return Err::kOk;
        }
        std::lock_guard<std::mutex> wg(s_->write_mu[me_]);
        std::unique_lock<std::mutex> lk(s_->m);
        Shared::Slot& out = s_->slot[1 - me_];
        while (len > 0) {
            if (dead()) return Err::kClosed;
            out.offered = buf;
            out.offered_len = len;
            out.consumed = false;
            s_->cv.notify_all();
            while (!out.consumed) {
                if (dead()) { out.offered = nullptr; return Err::kClosed; }
                if (has_wdl_ && Clock::now() >= wdl_) { out.offered = nullptr; return Err::kDeadline; }
                if (has_wdl_) s_->cv.wait_until(lk, wdl_);
                else s_->cv.wait(lk);
            }
            buf += out.taken;
            len -= out.taken;
            *n += out.taken;
            out.offered = nullptr;
        }
        return Err::kOk;
    }

    // Read exactly len bytes (io.ReadFull over Read): frames a byte stream.
    Err read_full(uint8_t* buf, size_t len) {
        size_t got = 0;
        while (got < len) {
            size_t k = 0;
            const Err e = read(buf + got, len - got, &k);
            if (e != Err::kOk) return e;
            got += k;
        }
        return Err::kOk;
    }

    Err close() {  // pipe.go:68-71: idempotent
        std::lock_guard<std::mutex> g(s_->m);
        s_->closed[me_] = true;
        s_->cv.notify_all();
        return Err::kOk;
    }

private:
    bool dead() const { return s_->closed[0] || s_->closed[1]; }
    std::shared_ptr<Shared> s_;
    int me_;
    std::string name_, peer_;
    Clock::time_point rdl_{}, wdl_{};
    bool has_rdl_ = false, has_wdl_ = false;
};

// pipe.Pipe(name1, name2, clock) (pipe.go:44-63).
inline std::pair<End, End> make_pipe(const std::string& name1, const std::string& name2) {
    auto s = std::make_shared<Shared>();
    return {End(s, 0, name1, name2), End(s, 1, name2, name1)};
}

}  // namespace nsx::pipe
