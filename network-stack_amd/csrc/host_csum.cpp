// host_csum.cpp — single-segment host checksum and the shard planner.
//
// host_csum16 is the cgo-facing replacement of one computeChecksum call
// (transport/tcp/tcp.go:72-95): same result, without the reference's
// allocate-and-concatenate (tcp.go:73) or the serial compare-carry loop
// (tcp.go:80-92). It sums 8 bytes per step as four little-endian 16-bit lanes
// (two u64 accumulators of 32-bit lanes), folds, and converts the LE-domain sum
// to the big-endian word domain with one byte swap (256·256 ≡ 1 mod 0xFFFF).
#include "host_csum.h"

#include <algorithm>
#include <cstring>

namespace nsx {
namespace {

inline uint32_t fold32(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint32_t)s;
}

inline uint32_t bswap16(uint32_t s) { return ((s & 0xFFu) << 8) | (s >> 8); }

// Sum of the little-endian 16-bit halves of p[0..len): byte p[i] weighs 1 for
// even i and 256 for odd i. Result folded to [0, 0xFFFF], 0 iff all bytes zero.
uint32_t le_sum(const uint8_t* p, size_t len) {
    uint64_t total = 0;
    size_t i = 0;
    while (len - i >= 8) {
        // Each 32-bit lane of a/b accumulates 16-bit values: 2^16 steps cannot overflow.
        uint64_t a = 0, b = 0;
        const size_t steps = std::min<size_t>((len - i) / 8, 65535);
        for (size_t k = 0; k < steps; ++k, i += 8) {
            uint64_t x;
            std::memcpy(&x, p + i, 8);
            a += x & 0x0000FFFF0000FFFFull;
            b += (x >> 16) & 0x0000FFFF0000FFFFull;
        }
        total += (a & 0xFFFFFFFFu) + (a >> 32) + (b & 0xFFFFFFFFu) + (b >> 32);
    }
    for (; i + 1 < len; i += 2) total += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
    if (i < len) total += p[i];  // odd tail: its pad byte is zero
    return fold32(total);
}

// Raw BE one's-complement sum of bytes that start at stream position parity `odd`.
inline uint32_t be_sum(const uint8_t* p, size_t len, bool odd) {
    const uint32_t s = le_sum(p, len);
    return odd ? s : bswap16(s);
}

}  // namespace

uint16_t host_csum16(const uint8_t* prefix, size_t prefix_len, const uint8_t* seg, size_t seg_len) {
    uint32_t s = 0;
    if (prefix_len) s += be_sum(prefix, prefix_len, false);
    if (seg_len) s += be_sum(seg, seg_len, (prefix_len & 1) != 0);
    return (uint16_t)fold32(s);
}

void shard_plan(const uint64_t* offsets, uint64_t n, int parts, uint64_t* bounds) {
    bounds[0] = 0;
    bounds[parts] = n;
    if (!offsets || n == 0) {
        for (int g = 1; g < parts; ++g) bounds[g] = n * (uint64_t)g / (uint64_t)parts;
        return;
    }
    // Byte-balanced: shard g starts at the first segment whose start offset
    // reaches g/parts of the total bytes (lower_bound on the prefix sums).
    const uint64_t lo = offsets[0], total = offsets[n] - offsets[0];
    for (int g = 1; g < parts; ++g) {
        const uint64_t target = lo + (uint64_t)((unsigned __int128)total * (unsigned)g / (unsigned)parts);
        const uint64_t* it = std::lower_bound(offsets, offsets + n, target);
        uint64_t b = (uint64_t)(it - offsets);
        bounds[g] = std::max<uint64_t>(std::min<uint64_t>(b, n), bounds[g - 1]);
    }
}

}  // namespace nsx
