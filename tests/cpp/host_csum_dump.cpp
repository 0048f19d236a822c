// Reads checksum cases from argv[1] (each: u32 prefix_len, u32 seg_len, u32 align, prefix bytes, seg bytes) and
// prints host_csum16 (network-stack_amd/csrc/host_csum.cpp, the cgo-facing computeChecksum of tcp.go:72-95) of
// each, with the segment copied to an exactly-sized heap buffer at `align` bytes past a 16-aligned start, so
// AddressSanitizer sees any read past either span. Then argv[2] (u64 n, u32 parts, n+1 u64 offsets) through
// shard_plan, printing the bounds.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <memory>
#include <vector>

#include "../../network-stack_amd/csrc/host_csum.h"

template <class T>
static T take(const std::vector<uint8_t>& b, size_t& at) {
    T v;
    std::memcpy(&v, b.data() + at, sizeof v);
    at += sizeof v;
    return v;
}

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    std::ifstream f(argv[1], std::ios::binary);
    const std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    for (size_t at = 0; at < b.size();) {
        const uint32_t pl = take<uint32_t>(b, at), sl = take<uint32_t>(b, at), al = take<uint32_t>(b, at);
        std::unique_ptr<uint8_t[]> pre(pl ? new uint8_t[pl] : nullptr);
        if (pl) std::memcpy(pre.get(), b.data() + at, pl);
        at += pl;
        std::unique_ptr<uint8_t[]> mem(new uint8_t[al + sl]);  // the segment ends exactly at the allocation's end
        if (sl) std::memcpy(mem.get() + al, b.data() + at, sl);
        at += sl;
        std::printf("%u\n", (unsigned)nsx::host_csum16(pre.get(), pl, mem.get() + al, sl));
    }
    std::ifstream g(argv[2], std::ios::binary);
    const std::vector<uint8_t> s((std::istreambuf_iterator<char>(g)), std::istreambuf_iterator<char>());
    size_t at = 0;
    const uint64_t n = take<uint64_t>(s, at);
    const uint32_t parts = take<uint32_t>(s, at);
    std::vector<uint64_t> offs(n + 1);
    for (auto& o : offs) o = take<uint64_t>(s, at);
    std::vector<uint64_t> bounds(parts + 1);
    nsx::shard_plan(offs.data(), n, (int)parts, bounds.data());
    for (auto v : bounds) std::printf("b %llu\n", (unsigned long long)v);
    return 0;
}
