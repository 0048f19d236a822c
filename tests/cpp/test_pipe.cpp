// C++ mirror of the reference's transport conformance suite
// (transport/test/conn.go: ConnTestSuite) run against nsx::pipe, which restates
// transport/pipe/pipe.go. Each test names the Go test it follows. A watchdog
// fails the run if any test blocks for more than a second (conn.go:23-33).
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

static void TestReadWrite(End& c1, End& c2) {  // conn.go:41-68: partial reads
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

static void TestWriteRace(End& c1, End& c2) {  // conn.go:70-107: writes never interleave
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

static void TestReadRace(End& c1, End& c2) {  // conn.go:109-149
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

static void try_read_write(End& c) {
    uint8_t buf[10] = {0};
    size_t n = 7;
    CHECK(c.read(buf, sizeof buf, &n) == Err::kClosed);
    CHECK(n == 0);
    n = 7;
    CHECK(c.write(buf, sizeof buf, &n) == Err::kClosed);
    CHECK(n == 0);
}

static void TestClose(End& c1, End& c2) {  // conn.go:151-184: both ends see ErrConnClosed
    CHECK(c1.close() == Err::kOk);
    CHECK(c1.close() == Err::kOk);  // once.Do: idempotent
    try_read_write(c1);
    try_read_write(c2);
}

static void TestReadBeforeClose(End& c1, End&) {  // conn.go:186-200: Close wakes a blocked Read
    std::thread r([&] {
        size_t n = 0;
        CHECK(c1.read(nullptr, 0, &n) == Err::kClosed);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(c1.close() == Err::kOk);
    r.join();
}

static void TestWriteBeforeClose(End& c1, End&) {  // conn.go:202-220: Close wakes a blocked Write
    const auto in = bytes_of("hey");
    std::thread w([&] {
        size_t n = 0;
        CHECK(c1.write(in.data(), in.size(), &n) == Err::kClosed);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    CHECK(c1.close() == Err::kOk);
    w.join();
}

static void TestReadDeadLine(End& c1, End& c2) {  // conn.go:222-253
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

static void TestWriteDeadLine(End& c1, End&) {  // conn.go:255-279
    c1.set_write_deadline(Clock::now() - std::chrono::seconds(1));
    const uint8_t a = 'a';
    size_t n = 9;
    CHECK(c1.write(&a, 1, &n) == Err::kDeadline);
    CHECK(n == 0);
}

static void TestDeadLineWakesBlockedRead(End& c1, End&) {  // chanDeadLine firing mid-Read
    c1.set_read_deadline(Clock::now() + std::chrono::milliseconds(30));
    uint8_t b[1];
    size_t n = 0;
    const auto t0 = Clock::now();
    CHECK(c1.read(b, 1, &n) == Err::kDeadline);
    CHECK(Clock::now() - t0 >= std::chrono::milliseconds(25));
}

static void TestAddr(End& c1, End& c2) {  // conn.go:281-287
    CHECK(c1.local_addr() == c2.remote_addr());
    CHECK(c2.local_addr() == c1.remote_addr());
    CHECK(c1.local_addr() == "c1" && c2.local_addr() == "c2");
}

static void TestEmptyWrite(End& c1, End&) {  // pipe.go:97-99
    size_t n = 5;
    CHECK(c1.write(nullptr, 0, &n) == Err::kOk && n == 0);
}

static void TestFramedStream(End& c1, End& c2) {  // read_full framing over many small reads
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

int main() {
    struct T {
        const char* name;
        void (*fn)(End&, End&);
    } tests[] = {{"TestReadWrite", TestReadWrite},
                 {"TestWriteRace", TestWriteRace},
                 {"TestReadRace", TestReadRace},
                 {"TestClose", TestClose},
                 {"TestReadBeforeClose", TestReadBeforeClose},
                 {"TestWriteBeforeClose", TestWriteBeforeClose},
                 {"TestReadDeadLine", TestReadDeadLine},
                 {"TestWriteDeadLine", TestWriteDeadLine},
                 {"TestDeadLineWakesBlockedRead", TestDeadLineWakesBlockedRead},
                 {"TestAddr", TestAddr},
                 {"TestEmptyWrite", TestEmptyWrite},
                 {"TestFramedStream", TestFramedStream}};
    for (int rep = 0; rep < 20; ++rep)  // races: repeat
        for (auto& t : tests) {
            if (rep && std::strstr(t.name, "Before")) continue;  // 50 ms sleeps: once is enough
            Watchdog wd(t.name);
            auto ends = nsx::pipe::make_pipe("c1", "c2");
            t.fn(ends.first, ends.second);
        }
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("pipe: %zu tests x 20 OK\n", sizeof tests / sizeof tests[0]);
    return 0;
}
