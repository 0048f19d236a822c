// csum_kernels.h — internal launcher interface between the C ABI (csum_api.cpp)
// and the gfx950 kernels (csum_kernels.hip). Not a public header.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nsx {

struct LaunchCfg {
    uint32_t max_blocks;  // persistent grid cap = CUs × blocks per CU
    int segs_per_wave;    // fixed path: segments per wave pass (1, 2, 4)
    int nontemporal;      // 1 = nt loads
    int xcd_map;          // 1 = XCD-contiguous task deal
    bool block_mode;      // one segment per 256-thread block (few long segments)
};

hipError_t launch_fixed(const LaunchCfg& c, const void* d_base, uint64_t stride, uint32_t seg_len,
                        uint64_t n, const uint32_t* partial, uint16_t* out, hipStream_t st);
hipError_t launch_ragged(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st);
hipError_t launch_pseudo_ipv4(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t proto,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st);
hipError_t launch_fill_splitmix64(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                                  uint32_t max_blocks, hipStream_t st);

}  // namespace nsx
