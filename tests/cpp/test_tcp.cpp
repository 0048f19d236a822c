// C++ mirror of transport/tcp/tcp_test.go against nsx::tcp (include/nsx/tcp.hpp)
// and the C ABI. Prints one line per golden segment case ("name offset hex raw
// raw_with_pseudo") for tests/test_tcp_cpp.py to compare with
// tests/golden/segments.json, then "OK" if every assertion held.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "nsx/tcp.hpp"

using nsx::tcp::Ctl;
using nsx::tcp::Option;
using nsx::tcp::Segment;

static int failures = 0;
#define CHECK(cond)                                                          \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                      \
        }                                                                    \
    } while (0)

// tcp_test.go:11-24
static void TestSegmentComputeOffset() {
    Segment s;
    const int min_offset = nsx::tcp::kMinSegmentLength / nsx::tcp::kOffsetMultiplier;
    CHECK(s.compute_offset() == min_offset);
    s.options.push_back(Option{});
    CHECK(s.compute_offset() == min_offset + 1);
}

// tcp_test.go:26-32
static void TestSegmentComputeChecksum() {
    Segment s;
    s.data = {'h', 'e', 'l', 'l', 'o'};
    s.checksum = nsx_field(s.compute_checksum());
    const uint16_t checksum = s.compute_checksum();
    CHECK(checksum == 0xFFFF);
    CHECK(nsx_verify(checksum));
    CHECK(s.checksum == 0xBC2D);  // ^0x43D2
}

// tcp_test.go:34-55
static void TestSegmentCodec() {
    Segment original;
    original.src_port = 1;
    original.dst_port = 2;
    original.seq_num = 3;
    original.ack_num = 4;
    original.offset = 5;
    original.window = 6;
    original.checksum = 7;
    original.urgent_ptr = 8;
    original.data = {9};
    original.offset = original.compute_offset();
    const std::vector<uint8_t> b = original.bytes();
    Segment got;
    std::string err;
    CHECK(nsx::tcp::parse_segment(b, got, err));
    CHECK(original == got);
}

// tcp_test.go:57-67
static void TestCTLCodec() {
    Ctl c;
    c.urg = true;
    c.rst = true;
    CHECK(Ctl::from_byte(c.byte()) == c);
}

static void TestParseErrors() {
    Segment s;
    std::string err;
    CHECK(!nsx::tcp::parse_segment(std::vector<uint8_t>(19, 0), s, err) && err == "segment too short");
    std::vector<uint8_t> b(20, 0);
    b[12] = 6;  // data at 24 > 20
    CHECK(!nsx::tcp::parse_segment(b, s, err) && err == "advertised data offset too long");
    b.resize(24, 0);
    b[20] = 9;  // unknown kind: the reference would spin forever
    CHECK(!nsx::tcp::parse_segment(b, s, err) && err == "unknown option kind");
}

static std::string hex(const std::vector<uint8_t>& b) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (uint8_t x : b) {
        s.push_back(d[x >> 4]);
        s.push_back(d[x & 15]);
    }
    return s;
}

// The struct-level golden cases of tests/golden/make_golden.py::segments().
static void golden() {
    std::vector<std::pair<std::string, Segment>> cases;
    Segment a;
    a.data = {'h', 'e', 'l', 'l', 'o'};
    cases.push_back({"TestSegmentComputeChecksum", a});
    Segment b;
    b.src_port = 1; b.dst_port = 2; b.seq_num = 3; b.ack_num = 4; b.offset = 5; b.window = 6; b.checksum = 7;
    b.urgent_ptr = 8; b.data = {9};
    cases.push_back({"TestSegmentCodec", b});
    Segment c;
    c.src_port = 80; c.dst_port = 443; c.control.urg = true; c.control.rst = true;
    c.data.assign(11, 'x');
    cases.push_back({"ctl_urg_rst", c});
    Segment d;
    d.src_port = 1; d.options.push_back(Option{1, 0, {}}); d.data = {'a', 'b', 'c'};
    cases.push_back({"option_noop", d});
    Segment e;
    e.src_port = 1234; e.dst_port = 80; e.seq_num = 0xDEADBEEF; e.ack_num = 0x01020304;
    e.control.syn = true; e.control.ack = true; e.window = 65535;
    e.options.push_back(Option{2, 4, {0x05, 0xB4, 0, 0}});
    e.data = {'p', 'a', 'y', 'l', 'o', 'a', 'd', '!'};
    cases.push_back({"option_mss", e});
    Segment f;
    f.src_port = 7;
    f.options.push_back(Option{2, 4, {1, 2, 3, 4}});
    f.options.push_back(Option{1, 0, {}});
    f.options.push_back(Option{0, 0, {}});
    for (int i = 0; i < 37; ++i) f.data.push_back((uint8_t)i);
    cases.push_back({"options_mss_noop_eol", f});
    const uint8_t src[4] = {192, 168, 0, 1}, dst[4] = {192, 168, 0, 2};
    for (auto& [name, s] : cases) {
        if (name != "TestSegmentComputeChecksum") s.offset = s.compute_offset();  // tcp_test.go:27 leaves it 0
        const std::vector<uint8_t> bytes = s.bytes();
        const std::vector<uint8_t> pseudo = nsx::tcp::ipv4_pseudo_header(src, dst, 6, (uint16_t)bytes.size());
        std::printf("%s %u %s %u %u\n", name.c_str(), s.offset, hex(bytes).c_str(), s.compute_checksum(),
                    s.compute_checksum(pseudo));
    }
}

int main() {
    TestSegmentComputeOffset();
    TestSegmentComputeChecksum();
    TestSegmentCodec();
    TestCTLCodec();
    TestParseErrors();
    golden();
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("OK\n");
    return 0;
}
