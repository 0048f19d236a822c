// C++ mirror of the reference's transport conformance suite
// (transport/test/conn.go: ConnTestSuite, buffered_conn.go: BufferedConnTestSuite)
// run against nsx::pipe, which restates transport/pipe/pipe.go and buffered.go.
// Each test names the Go test it follows. A watchdog fails the run if any test
// blocks for more than a second (conn.go:23-33).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nsx/pipe.hpp"

using nsx::pipe::Clock;
using nsx::pipe::End;
using nsx::pipe::Err;

static int g_fail = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                             \
        }                                                                         \
    } while (0)

static std::vector<uint8_t> bytes_of(const char* s) { return std::vector<uint8_t>(s, s + std::strlen(s)); }

struct Watchdog {  // SetupTest's one-second timer
    std::atomic<bool> done{false};
    std::thread t;
    explicit Watchdog(const char* name) {
        t = std::thread([this, name] {
            const auto until = Clock::now() + std::chrono::seconds(1);
            while (!done && Clock::now() < until) std::this_thread::sleep_for(std::chrono::milliseconds(2));
            if (!done) {
                std::fprintf(stderr, "%s: timeout exceeded\n", name);
                std::_Exit(3);
            }
        });
    }
    ~Watchdog() { done = true; t.join(); }
};

template <class E>
static void TestReadWrite(E& c1, E& c2) {  // conn.go:41-68: partial reads
    const auto data = bytes_of("Hello, World!");
    std::thread w([&] {
        size_t n = 0;
        CHECK(c1.write(data.data(), data.size(), &n) == Err::kOk);
        CHECK(n == data.size());
    });
    uint8_t buf[10];
    size_t n = 0;
    CHECK(c2.read(buf, sizeof buf, &n) == Err::kOk);
    CHECK(n == sizeof buf && std::memcmp(buf, data.data(), n) == 0);
    CHECK(c2.read(buf, sizeof buf, &n) == Err::kOk);
    CHECK(n == data.size() - sizeof buf && std::memcmp(buf, data.data() + 10, n) == 0);
    w.join();
}

template <class E>
static void TestWriteRace(E& c1, E& c2) {  // conn.go:70-107: writes never interleave
    const auto data = bytes_of("ABCD");
    const int N = 10;
    std::vector<std::thread> ws;
    for (int i = 0; i < N; ++i)
        ws.emplace_back([&] {
            size_t n = 0;
            CHECK(c1.write(data.data(), data.size(), &n) == Err::kOk);
            CHECK(n == data.size());
        });
    std::vector<uint8_t> result;
    uint8_t b[4];
    for (int i = 0; i < N; ++i) {
        size_t n = 0;
        CHECK(c2.read(b, sizeof b, &n) == Err::kOk);
        result.insert(result.end(), b, b + n);
    }
    for (auto& t : ws) t.join();
    std::vector<uint8_t> want;
    for (int i = 0; i < N; ++i) want.insert(want.end(), data.begin(), data.end());
    CHECK(result == want);
}

template <class E>
static void TestReadRace(E& c1, E& c2) {  // conn.go:109-149
    const auto data = bytes_of("ABCD");
    const int N = 10;
    std::thread w([&] {
        for (int i = 0; i < N; ++i) {
            size_t n = 0;
            CHECK(c2.write(data.data(), data.size(), &n) == Err::kOk);
            CHECK(n == data.size());
        }
    });
    std::mutex l;
    std::vector<uint8_t> result;
    std::vector<std::thread> rs;
    for (int i = 0; i < N; ++i)
        rs.emplace_back([&] {
            uint8_t b[4];
            size_t n = 0;
            CHECK(c1.read(b, sizeof b, &n) == Err::kOk);
            CHECK(n == data.size());
            std::lock_guard<std::mutex> g(l);
            result.insert(result.end(), b, b + n);
        });
    for (auto& t : rs) t.join();
    w.join();
    std::vector<uint8_t> want;
    for (int i = 0; i < N; ++i) want.insert(want.end(), data.begin(), data.end());
    CHECK(result == want);
}

template <class E>
static void try_read_write(E& c) {
    uint8_t buf[10] = {0};
    size_t n = 7;
    CHECK(c.read(buf, sizeof buf, &n) == Err::kClosed);
    CHECK(n == 0);
    n = 7;
    CHECK(c.write(buf, sizeof buf, &n) == Err::kClosed);
    CHECK(n == 0);
}

template <class E>
static void TestClose(E& c1, E& c2) {  // conn.go:151-184: both ends see ErrConnClosed
    CHECK(c1.close() == Err::kOk);
    CHECK(c1.close() == Err::kOk);  // once.Do: idempotent
    try_read_write(c1);
    try_read_write(c2);
}

template <class E>
static void TestReadBeforeClose(E& c1, E&) {  // conn.go:186-200: Close wakes a blocked Read
    std::thread r([&] {
        size_t n = 0;
        CHECK(c1.read(nullptr, 0, &n) == Err::kClosed);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(c1.close() == Err::kOk);
    r.join();
}

template <class E>
static void TestWriteBeforeClose(E& c1, E&) {  // conn.go:202-220: Close wakes a blocked Write
    const auto in = bytes_of("hey");
    std::thread w([&] {
        size_t n = 0;
        CHECK(c1.write(in.data(), in.size(), &n) == Err::kClosed);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(c1.close() == Err::kOk);
    w.join();
}

template <class E>
static void TestReadDeadLine(E& c1, E& c2) {  // conn.go:222-253
    c1.set_read_deadline(Clock::now() - std::chrono::seconds(1));
    uint8_t b[1];
    size_t n = 9;
    CHECK(c1.read(b, 1, &n) == Err::kDeadline);
    CHECK(n == 0);
    std::thread w([&] {
        const uint8_t a = 'a';
        size_t k = 0;
        CHECK(c2.write(&a, 1, &k) == Err::kOk);
    });
    c1.clear_read_deadline();
    CHECK(c1.read(b, 1, &n) == Err::kOk);
    CHECK(n == 1 && b[0] == 'a');
    w.join();
}

template <class E>
static void TestWriteDeadLine(E& c1, E&) {  // conn.go:255-279
    c1.set_write_deadline(Clock::now() - std::chrono::seconds(1));
    const uint8_t a = 'a';
    size_t n = 9;
    CHECK(c1.write(&a, 1, &n) == Err::kDeadline);
    CHECK(n == 0);
}

template <class E>
static void TestDeadLineWakesBlockedRead(E& c1, E&) {  // chanDeadLine firing mid-Read
    c1.set_read_deadline(Clock::now() + std::chrono::milliseconds(30));
    uint8_t b[1];
    size_t n = 0;
    const auto t0 = Clock::now();
    CHECK(c1.read(b, 1, &n) == Err::kDeadline);
    CHECK(Clock::now() - t0 >= std::chrono::milliseconds(25));
}

template <class E>
static void TestAddr(E& c1, E& c2) {  // conn.go:281-287
    CHECK(c1.local_addr() == c2.remote_addr());
    CHECK(c2.local_addr() == c1.remote_addr());
    CHECK(c1.local_addr() == "c1" && c2.local_addr() == "c2");
}

template <class E>
static void TestEmptyWrite(E& c1, E&) {  // pipe.go:97-99
    size_t n = 5;
    CHECK(c1.write(nullptr, 0, &n) == Err::kOk && n == 0);
}

template <class E>
static void TestFramedStream(E& c1, E& c2) {  // read_full framing over many small reads
    std::vector<uint8_t> big(1 << 16);
    for (size_t i = 0; i < big.size(); ++i) big[i] = (uint8_t)(i * 131 + 7);
    std::thread w([&] {
        size_t n = 0;
        CHECK(c1.write(big.data(), big.size(), &n) == Err::kOk && n == big.size());
    });
    std::vector<uint8_t> got(big.size());
    size_t off = 0;
    for (size_t step = 1; off < got.size(); step = step * 3 % 1501 + 1) {
        const size_t k = std::min(step, got.size() - off);
        CHECK(c2.read_full(got.data() + off, k) == Err::kOk);
        off += k;
    }
    w.join();
    CHECK(got == big);
}

// --- transport/test/buffered_conn.go (BufferedConnTestSuite) ---------------
static void TestBothWrite(nsx::pipe::BufferedEnd& c1, nsx::pipe::BufferedEnd& c2) {  // buffered_conn.go:23-61
    const size_t size1 = c1.read_buf_size(), size2 = c2.read_buf_size();
    CHECK(c1.write_buf_size() == size2);
    std::thread a([&] {
        std::vector<uint8_t> b(size2, 1);
        size_t n = 0;
        CHECK(c1.write(b.data(), b.size(), &n) == Err::kOk && n == size2);
        CHECK(c2.read(b.data(), b.size(), &n) == Err::kOk && n == size2);
    });
    std::thread b([&] {
        std::vector<uint8_t> v(size1, 2);
        size_t n = 0;
        CHECK(c2.write(v.data(), v.size(), &n) == Err::kOk && n == size1);
        CHECK(c1.read(v.data(), v.size(), &n) == Err::kOk && n == size1);
    });
    a.join();
    b.join();
}

static void TestReadAfterClose(nsx::pipe::BufferedEnd& c1, nsx::pipe::BufferedEnd& c2) {  // buffered_conn.go:63-84
    const size_t size1 = c1.read_buf_size();
    std::vector<uint8_t> b(size1, 7);
    size_t n = 0;
    CHECK(c2.write(b.data(), size1, &n) == Err::kOk && n == size1);
    CHECK(c2.close() == Err::kOk);
    CHECK(c1.read(b.data(), size1, &n) == Err::kOk && n == size1);
    n = 9;
    CHECK(c1.read(b.data(), 1, &n) == Err::kClosed && n == 0);
}

static void TestWriteBlocksWhenFull(nsx::pipe::BufferedEnd& c1, nsx::pipe::BufferedEnd& c2) {
    // a write larger than the buffer completes only as the reader drains it
    std::vector<uint8_t> big(5 * c2.read_buf_size() + 3);
    for (size_t i = 0; i < big.size(); ++i) big[i] = (uint8_t)(i * 29 + 1);
    std::thread w([&] {
        size_t n = 0;
        CHECK(c1.write(big.data(), big.size(), &n) == Err::kOk && n == big.size());
    });
    std::vector<uint8_t> got(big.size());
    CHECK(c2.read_full(got.data(), got.size()) == Err::kOk);
    w.join();
    CHECK(got == big);
}

static void TestPeekConsume(nsx::pipe::BufferedEnd& c1, nsx::pipe::BufferedEnd& c2) {
    // zero-copy frames: the view is stable while writers keep appending
    const size_t cap = c2.read_buf_size(), frame = 6;
    std::vector<uint8_t> src(40 * frame);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 7 + 3);
    std::thread w([&] {
        for (size_t off = 0; off < src.size(); off += frame) {
            size_t n = 0;
            CHECK(c1.write(src.data() + off, frame, &n) == Err::kOk && n == frame);
        }
        c1.close();
    });
    std::vector<uint8_t> got;
    for (;;) {
        const uint8_t* v = nullptr;
        size_t avail = 0;
        const Err e = c2.peek(frame, &v, &avail);
        if (e == Err::kClosed) break;
        CHECK(e == Err::kOk && avail >= std::min(frame, cap) && avail <= cap);
        const size_t take = avail / frame * frame;
        std::vector<uint8_t> snap(v, v + take);
        std::this_thread::sleep_for(std::chrono::microseconds(50));  // let the writer append behind the view
        CHECK(std::memcmp(snap.data(), v, take) == 0);
        got.insert(got.end(), v, v + take);
        c2.consume(take);
    }
    w.join();
    CHECK(got == src);
}

static void TestZeroSizeRefused() {  // buffered.go:38-40 panics on bufSize 0
    bool threw = false;
    try {
        nsx::pipe::make_buffered_pipe("a", "b", 0);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
}

template <class E>
struct Case {
    const char* name;
    void (*fn)(E&, E&);
};

template <class E, class Make, size_t K>
static void run_suite(const char* suite, const Case<E> (&tests)[K], Make make) {
    for (int rep = 0; rep < 20; ++rep)  // races: repeat
        for (auto& t : tests) {
            if (rep && std::strstr(t.name, "Before")) continue;  // 50 ms sleeps: once is enough
            Watchdog wd(t.name);
            auto ends = make();
            t.fn(ends.first, ends.second);
        }
    std::printf("%s: %zu tests x 20 OK\n", suite, K);
}

int main() {
    using nsx::pipe::BufferedEnd;
    const Case<End> unbuffered[] = {{"TestReadWrite", TestReadWrite<End>},
                                    {"TestWriteRace", TestWriteRace<End>},
                                    {"TestReadRace", TestReadRace<End>},
                                    {"TestClose", TestClose<End>},
                                    {"TestReadBeforeClose", TestReadBeforeClose<End>},
                                    {"TestWriteBeforeClose", TestWriteBeforeClose<End>},
                                    {"TestReadDeadLine", TestReadDeadLine<End>},
                                    {"TestWriteDeadLine", TestWriteDeadLine<End>},
                                    {"TestDeadLineWakesBlockedRead", TestDeadLineWakesBlockedRead<End>},
                                    {"TestAddr", TestAddr<End>},
                                    {"TestEmptyWrite", TestEmptyWrite<End>},
                                    {"TestFramedStream", TestFramedStream<End>}};
    run_suite("pipe", unbuffered, [] { return nsx::pipe::make_pipe("c1", "c2"); });
    // BufferedPipe("A", "B", clock, 20) as in pipe/buffered_test.go:18-21; the
    // conn suite's TestWriteBeforeClose is skipped for buffered conns (conn.go:203-205).
    const Case<BufferedEnd> buffered[] = {{"TestReadWrite", TestReadWrite<BufferedEnd>},
                                          {"TestWriteRace", TestWriteRace<BufferedEnd>},
                                          {"TestReadRace", TestReadRace<BufferedEnd>},
                                          {"TestClose", TestClose<BufferedEnd>},
                                          {"TestReadBeforeClose", TestReadBeforeClose<BufferedEnd>},
                                          {"TestReadDeadLine", TestReadDeadLine<BufferedEnd>},
                                          {"TestWriteDeadLine", TestWriteDeadLine<BufferedEnd>},
                                          {"TestDeadLineWakesBlockedRead", TestDeadLineWakesBlockedRead<BufferedEnd>},
                                          {"TestEmptyWrite", TestEmptyWrite<BufferedEnd>},
                                          {"TestFramedStream", TestFramedStream<BufferedEnd>},
                                          {"TestBothWrite", TestBothWrite},
                                          {"TestReadAfterClose", TestReadAfterClose},
                                          {"TestWriteBlocksWhenFull", TestWriteBlocksWhenFull},
                                          {"TestPeekConsume", TestPeekConsume}};
    run_suite("buffered", buffered, [] { return nsx::pipe::make_buffered_pipe("c1", "c2", 20); });
    TestZeroSizeRefused();
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("OK\n");
    return 0;
}
