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
#include <stdexcept>
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

// ---------------------------------------------------------------------------
// Buffered pipe (transport/pipe/buffered.go): each end owns a bounded receive
// buffer of buf_size bytes (bytes.Buffer with fixed capacity, buffered.go:35-58).
//   - Write copies as much as fits in the peer's free space, blocking while it
//     is full, until all bytes are in (buffered.go:110-151); writers serialise.
//   - Read returns buffered bytes even after Close (buffered.go:93-96) and only
//     then reports kClosed; deadlines are checked first (:88-91).
//   - The buffer may be caller-provided memory (e.g. nsx_alloc_pinned), and the
//     receiver can view buffered bytes in place (peek/consume) — the f4 path
//     that hands received frames to nsx_csum_fixed_host without a copy.
// Data stay contiguous: the buffer compacts to the front when a write would run
// past its end (bytes.Buffer's slide).
// Difference: an empty Write returns 0 at once (Go's loop would park once on
// the write condition before returning 0).
struct BufShared {
    std::mutex m;
    std::condition_variable cv;
    struct Buf {
        uint8_t* data = nullptr;
        size_t cap = 0, r = 0, w = 0;  // buffered bytes are data[r, w)
        bool viewed = false;           // a peek() view is live: no sliding
        std::unique_ptr<uint8_t[]> own;
        size_t len() const { return w - r; }
    } buf[2];                          // buf[i]: receive buffer of end i
    bool closed[2] = {false, false};
    std::mutex write_mu[2];
};

class BufferedEnd {
public:
    BufferedEnd(std::shared_ptr<BufShared> s, int me, std::string name, std::string peer)
        : s_(std::move(s)), me_(me), name_(std::move(name)), peer_(std::move(peer)) {}

    const std::string& local_addr() const { return name_; }
    const std::string& remote_addr() const { return peer_; }
    size_t read_buf_size() const { return s_->buf[me_].cap; }       // buffered.go:60
    size_t write_buf_size() const { return s_->buf[1 - me_].cap; }  // buffered.go:61

    void set_read_deadline(Clock::time_point t) { std::lock_guard<std::mutex> g(s_->m); rdl_ = t; has_rdl_ = true; s_->cv.notify_all(); }
    void set_write_deadline(Clock::time_point t) { std::lock_guard<std::mutex> g(s_->m); wdl_ = t; has_wdl_ = true; s_->cv.notify_all(); }
    void clear_read_deadline() { std::lock_guard<std::mutex> g(s_->m); has_rdl_ = false; s_->cv.notify_all(); }
    void clear_write_deadline() { std::lock_guard<std::mutex> g(s_->m); has_wdl_ = false; s_->cv.notify_all(); }

    Err read(uint8_t* b, size_t len, size_t* n) {  // buffered.go:79-108
        *n = 0;
        std::unique_lock<std::mutex> lk(s_->m);
        BufShared::Buf& in = s_->buf[me_];
        for (;;) {
            if (has_rdl_ && Clock::now() >= rdl_) return Err::kDeadline;
            if (in.len() > 0) {
                const size_t k = len < in.len() ? len : in.len();
                if (k) std::memcpy(b, in.data + in.r, k);
                in.r += k;
                if (in.r == in.w && !in.viewed) in.r = in.w = 0;
                *n = k;
                s_->cv.notify_all();  // notifyWrite on the peer
                return Err::kOk;
            }
            if (dead()) return Err::kClosed;
            wait(lk, has_rdl_, rdl_);
        }
    }

    Err write(const uint8_t* b, size_t len, size_t* n) {  // buffered.go:110-151
        *n = 0;
        std::lock_guard<std::mutex> wg(s_->write_mu[me_]);
        std::unique_lock<std::mutex> lk(s_->m);
        BufShared::Buf& out = s_->buf[1 - me_];
        for (bool once = true; once || len > 0; once = false) {
            if (has_wdl_ && Clock::now() >= wdl_) return Err::kDeadline;
            if (dead()) return Err::kClosed;
            const size_t room = out.viewed ? out.cap - out.w : out.cap - out.len();
            const size_t k = len < room ? len : room;
            if (k > 0) {
                if (out.w + k > out.cap) {  // slide to the front
                    std::memmove(out.data, out.data + out.r, out.len());
                    out.w -= out.r;
                    out.r = 0;
                }
                std::memcpy(out.data + out.w, b, k);
                out.w += k;
                b += k;
                len -= k;
                *n += k;
                s_->cv.notify_all();  // notifyRead on the peer
                continue;
            }
            if (len == 0) break;
            wait(lk, has_wdl_, wdl_);
        }
        return Err::kOk;
    }

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

    // Zero-copy receive: wait until at least min_len bytes are buffered (or
    // the buffer is full), then expose them in place. The view stays valid
    // until consume(): meanwhile writers only append behind it, never slide.
    // One viewer per end.
    Err peek(size_t min_len, const uint8_t** view, size_t* avail) {
        *view = nullptr;
        *avail = 0;
        std::unique_lock<std::mutex> lk(s_->m);
        BufShared::Buf& in = s_->buf[me_];
        const size_t want = min_len < in.cap ? min_len : in.cap;
        for (;;) {
            if (has_rdl_ && Clock::now() >= rdl_) return Err::kDeadline;
            if (in.len() >= want && in.len() > 0) break;
            if (dead()) {
                if (in.len() == 0) return Err::kClosed;
                break;  // whatever remains after Close is still readable
            }
            wait(lk, has_rdl_, rdl_);
        }
        in.viewed = true;
        *view = in.data + in.r;
        *avail = in.len();
        return Err::kOk;
    }

    void consume(size_t k) {
        std::lock_guard<std::mutex> g(s_->m);
        BufShared::Buf& in = s_->buf[me_];
        in.r += k < in.len() ? k : in.len();
        in.viewed = false;
        if (in.r == in.w) in.r = in.w = 0;
        s_->cv.notify_all();
    }

    Err close() {  // buffered.go:66-77
        std::lock_guard<std::mutex> g(s_->m);
        s_->closed[me_] = true;
        s_->cv.notify_all();
        return Err::kOk;
    }

private:
    bool dead() const { return s_->closed[0] || s_->closed[1]; }
    void wait(std::unique_lock<std::mutex>& lk, bool has, Clock::time_point t) {
        if (has) s_->cv.wait_until(lk, t);
        else s_->cv.wait(lk);
    }
    std::shared_ptr<BufShared> s_;
    int me_;
    std::string name_, peer_;
    Clock::time_point rdl_{}, wdl_{};
    bool has_rdl_ = false, has_wdl_ = false;
};

// pipe.BufferedPipe(name1, name2, clock, bufSize) (buffered.go:35-58).
// storage1/storage2 (optional, bufSize bytes each, caller-owned and outliving
// the pipe) become end 1's / end 2's receive buffers; bufSize 0 is refused.
inline std::pair<BufferedEnd, BufferedEnd> make_buffered_pipe(const std::string& name1, const std::string& name2,
                                                              size_t buf_size, uint8_t* storage1 = nullptr,
                                                              uint8_t* storage2 = nullptr) {
    if (buf_size == 0) throw std::invalid_argument("buffer size cannot be 0");  // buffered.go:38-40
    auto s = std::make_shared<BufShared>();
    uint8_t* st[2] = {storage1, storage2};
    for (int i = 0; i < 2; ++i) {
        BufShared::Buf& b = s->buf[i];
        if (!st[i]) {
            b.own.reset(new uint8_t[buf_size]);
            st[i] = b.own.get();
        }
        b.data = st[i];
        b.cap = buf_size;
    }
    return {BufferedEnd(s, 0, name1, name2), BufferedEnd(s, 1, name2, name1)};
}

}  // namespace nsx::pipe
