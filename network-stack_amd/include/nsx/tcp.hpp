// nsx/tcp.hpp — C++ mirror of the reference's TCP segment model over the C ABI.
//
// Mirrors transport/tcp/tcp.go (oneee-playground/network-stack):
//   segment          tcp.go:39-54     → nsx::tcp::Segment
//   computeOffset    tcp.go:59-66     → Segment::compute_offset
//   computeChecksum  tcp.go:72-95     → Segment::compute_checksum (nsx_csum16)
//   bytes            tcp.go:98-128    → Segment::bytes
//   parseSegment     tcp.go:130-185   → parse_segment
//   ctl, ctlFromByte tcp.go:188-216   → Ctl::byte, Ctl::from_byte
//   option.bytes     tcp.go:225-231   → Option::bytes
// Same field meanings and byte layout, including the reference's quirks that
// decide which bytes get checksummed: `offset` is stored as the whole byte 12
// (tcp.go:106, :142) and options are padded with `remainder` zero bytes rather
// than 4-remainder (tcp.go:118-121).
//
// Error behaviour: computeChecksum cannot fail in Go, and compute_checksum
// never throws. parseSegment returns an error for a short or over-long header
// (tcp.go:131-152) and parse_segment does the same; where the Go code would
// loop forever (unknown option kind, tcp.go:160-179) or panic on an
// out-of-range MSS slice (tcp.go:172-175), parse_segment returns an error.
//
// Header-only; link against libnsx_csum.so.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/nsx_csum.h"

namespace nsx::tcp {

constexpr int kMinSegmentLength = 20;  // tcp.go:56
constexpr int kOffsetMultiplier = 4;   // tcp.go:57

enum OptionKind : uint8_t { kOptionEOL = 0, kOptionNoOp = 1, kOptionMSS = 2 };  // tcp.go:236-238

struct Ctl {  // tcp.go:188-190; bit 7 = cwr … bit 0 = fin
    bool cwr = false, ece = false, urg = false, ack = false, psh = false, rst = false, syn = false, fin = false;

    uint8_t byte() const {  // tcp.go:192-203
        const bool f[8] = {cwr, ece, urg, ack, psh, rst, syn, fin};
        uint8_t b = 0;
        for (int i = 0; i < 8; ++i)
            if (f[i]) b |= (uint8_t)(1u << (7 - i));
        return b;
    }
    static Ctl from_byte(uint8_t b) {  // tcp.go:205-216
        Ctl c;
        bool* f[8] = {&c.cwr, &c.ece, &c.urg, &c.ack, &c.psh, &c.rst, &c.syn, &c.fin};
        for (int i = 0; i < 8; ++i) *f[i] = (b & (1u << (7 - i))) != 0;
        return c;
    }
    bool operator==(const Ctl& o) const { return byte() == o.byte(); }
};

struct Option {  // tcp.go:218-222
    uint8_t kind = 0;
    uint8_t length = 0;
    std::vector<uint8_t> data;

    std::vector<uint8_t> bytes() const {  // tcp.go:225-231
        if (kind == kOptionMSS) {
            std::vector<uint8_t> b{kind, length};
            b.insert(b.end(), data.begin(), data.end());
            return b;
        }
        return {kind};
    }
    bool operator==(const Option& o) const { return kind == o.kind && length == o.length && data == o.data; }
};

struct Segment {  // tcp.go:39-54
    uint16_t src_port = 0, dst_port = 0;
    uint32_t seq_num = 0, ack_num = 0;
    uint8_t offset = 0;  // data offset in 32-bit words, stored as the whole byte 12
    Ctl control;
    uint16_t window = 0;
    uint16_t checksum = 0;
    uint16_t urgent_ptr = 0;
    std::vector<Option> options;
    std::vector<uint8_t> data;

    uint8_t compute_offset() const {  // tcp.go:59-66
        int off = kMinSegmentLength;
        for (const Option& o : options) off += (int)o.bytes().size();
        return (uint8_t)((off + kOffsetMultiplier - 1) / kOffsetMultiplier);
    }

    std::vector<uint8_t> bytes() const {  // tcp.go:98-128
        std::vector<uint8_t> b;
        b.reserve(kMinSegmentLength + 44 + data.size());
        auto be16 = [&](uint16_t v) { b.push_back((uint8_t)(v >> 8)); b.push_back((uint8_t)v); };
        auto be32 = [&](uint32_t v) { for (int s = 24; s >= 0; s -= 8) b.push_back((uint8_t)(v >> s)); };
        be16(src_port);
        be16(dst_port);
        be32(seq_num);
        be32(ack_num);
        b.push_back(offset);
        b.push_back(control.byte());
        be16(window);
        be16(checksum);
        be16(urgent_ptr);
        if (!options.empty()) {
            for (const Option& o : options) {
                const std::vector<uint8_t> ob = o.bytes();
                b.insert(b.end(), ob.begin(), ob.end());
            }
            const size_t rem = b.size() % kOffsetMultiplier;
            b.insert(b.end(), rem, 0);  // the reference appends `remainder` zeros (tcp.go:118-121)
        }
        b.insert(b.end(), data.begin(), data.end());
        return b;
    }

    // The raw one's-complement sum over pseudo ‖ bytes() (tcp.go:72-95). The
    // sender stores ~sum in `checksum` with the field zero; a receiver accepts
    // iff the sum is 0xFFFF (tcp.go:68-71).
    uint16_t compute_checksum(const std::vector<uint8_t>& pseudo = {}) const {
        const std::vector<uint8_t> b = bytes();
        uint16_t sum = 0;
        (void)nsx_csum16(pseudo.empty() ? nullptr : pseudo.data(), pseudo.size(), b.empty() ? nullptr : b.data(),
                         b.size(), &sum);
        return sum;
    }

    bool operator==(const Segment& o) const {
        return src_port == o.src_port && dst_port == o.dst_port && seq_num == o.seq_num && ack_num == o.ack_num &&
               offset == o.offset && control == o.control && window == o.window && checksum == o.checksum &&
               urgent_ptr == o.urgent_ptr && options == o.options && data == o.data;
    }
};

// parseSegment (tcp.go:130-185). Returns false and sets err on failure.
inline bool parse_segment(const std::vector<uint8_t>& raw, Segment& s, std::string& err) {
    if (raw.size() < (size_t)kMinSegmentLength) {
        err = "segment too short";
        return false;
    }
    auto be16 = [&](size_t i) { return (uint16_t)((raw[i] << 8) | raw[i + 1]); };
    auto be32 = [&](size_t i) {
        return (uint32_t)raw[i] << 24 | (uint32_t)raw[i + 1] << 16 | (uint32_t)raw[i + 2] << 8 | raw[i + 3];
    };
    s = Segment{};
    s.src_port = be16(0);
    s.dst_port = be16(2);
    s.seq_num = be32(4);
    s.ack_num = be32(8);
    s.offset = raw[12];
    s.control = Ctl::from_byte(raw[13]);
    s.window = be16(14);
    s.checksum = be16(16);
    s.urgent_ptr = be16(18);
    const size_t data_at = (size_t)s.offset * kOffsetMultiplier;
    if (data_at > raw.size()) {
        err = "advertised data offset too long";
        return false;
    }
    if (s.offset > kMinSegmentLength / kOffsetMultiplier) {
        size_t i = kMinSegmentLength;
        while (i < data_at) {
            const uint8_t kind = raw[i];
            if (kind == kOptionEOL) break;
            Option o;
            o.kind = kind;
            if (kind == kOptionNoOp) {
                i++;
            } else if (kind == kOptionMSS) {
                if (i + 2 > raw.size() || i + 2 + raw[i + 1] > raw.size()) {
                    err = "option out of range";  // Go would panic on the slice (tcp.go:173)
                    return false;
                }
                o.length = raw[i + 1];
                o.data.assign(raw.begin() + i + 2, raw.begin() + i + 2 + o.length);
                i += 6;  // 1(kind) + 1(length) + 4(data), as tcp.go:175
            } else {
                err = "unknown option kind";  // Go would not advance and loop forever (tcp.go:160-179)
                return false;
            }
            s.options.push_back(o);
        }
    }
    s.data.assign(raw.begin() + data_at, raw.end());
    return true;
}

// IPv4 TCP pseudo-header (RFC 9293 §3.1) from ip.Addr.Raw() bytes
// (network/ip/v4/ipv4.go:15) and ip.NextProtoTCP = 6 (network/ip/protocols.go:8).
inline std::vector<uint8_t> ipv4_pseudo_header(const uint8_t src[4], const uint8_t dst[4], uint8_t proto,
                                               uint16_t tcp_len) {
    return {src[0], src[1], src[2], src[3], dst[0], dst[1], dst[2], dst[3],
            0,      proto,  (uint8_t)(tcp_len >> 8), (uint8_t)tcp_len};
}

// IPv6 pseudo-header (RFC 8200 §8.1) from ipv6 Addr.Raw() (network/ip/v6/ipv6.go:16).
inline std::vector<uint8_t> ipv6_pseudo_header(const uint8_t src[16], const uint8_t dst[16], uint8_t next_header,
                                               uint32_t upper_len) {
    std::vector<uint8_t> p(src, src + 16);
    p.insert(p.end(), dst, dst + 16);
    for (int s = 24; s >= 0; s -= 8) p.push_back((uint8_t)(upper_len >> s));
    p.insert(p.end(), {0, 0, 0, next_header});
    return p;
}

}  // namespace nsx::tcp
