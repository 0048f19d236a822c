// host_csum.h — host-side pieces of the C ABI that need no GPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace nsx {

// computeChecksum (transport/tcp/tcp.go:72-95) over prefix ‖ seg on the host CPU:
// the single-segment entry point nsx_csum16. Not used by any batch/device path.
uint16_t host_csum16(const uint8_t* prefix, size_t prefix_len, const uint8_t* seg, size_t seg_len);

// Contiguous shard boundaries (parts+1 entries): equal counts when offsets is
// null, equal byte counts over the prefix-sum offsets otherwise.
void shard_plan(const uint64_t* offsets, uint64_t n, int parts, uint64_t* bounds);

}  // namespace nsx
