// csum_kernels.h — internal launcher interface between the C ABI (csum_api.cpp,
// host_batch.cpp) and the gfx950 kernels (csum_kernels.hip). Not a public header.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

struct nsx_tune;  // include/nsx_tune.h

namespace nsx {

// Per-call launch configuration: the device's CU count plus the optional
// overrides of include/nsx_tune.h (0 = the per-path default measured best on
// MI355X). Built per call from the caller's nsx_tune (or none);
// there is no process-wide tuning state.
struct LaunchCfg {
    int cus = 0;              // compute units of the device
    int blocks_per_cu = 0;    // persistent grid = cus × blocks_per_cu blocks of 256 threads
    int segs_per_wave = 0;    // fixed short-segment paths: segments per wave task (1, 2, 4, 8)
    int block_mode = 0;       // 0 auto (a block per segment when n < 4·cus), 1 never, 2 always
    int rows = 0;             // ragged scan kernel: 1 KiB rows per batch (4, 8, 16)
    int run_segs = 0;         // ragged scan kernel: segments per wave task (1..63)
    int xcd_chunk = 0;        // XCD deal: 0 auto, 1..20 = chunks of 2^k tasks, else contiguous eighths
    int64_t window_bytes = 0; // fixed short-segment path: back-to-back launches of ≤ this many bytes (0 auto, -1 one)
    int kernel = 0;           // force an alternative code path (nsx_tune.h NSX_TUNE_KERNEL_*); 0 = by layout
    int deal = 0;             // -1: equal static shares (no dealt runs) for this call
};

// The LaunchCfg of one call on a device with `cus` compute units; t nullable (csum_api.cpp).
LaunchCfg launch_cfg(int cus, const nsx_tune* t);

// Kernel launches nsx_csum_fixed_dev makes for this batch (its back-to-back windows).
uint64_t fixed_launch_count(const LaunchCfg& c, uintptr_t base, uint64_t stride, uint32_t seg_len, uint64_t n);
// Launches one IPv4 header call makes (the packed 20 B kernel's windows).
uint64_t ipv4_hdr_launch_count(const LaunchCfg& c, uintptr_t base, uint64_t stride, uint32_t hdr_off, uint64_t n);

hipError_t launch_fixed(const LaunchCfg& c, const void* d_base, uint64_t stride, uint32_t seg_len,
                        uint64_t n, const uint32_t* partial, uint16_t* out, hipStream_t st);
hipError_t launch_ragged(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st);
// Fused receive pass: IPv4 (ipver 4: header + pseudo-header + TCP checksum) or IPv6 (ipver 6: pseudo-header +
// TCP checksum) per frame into a validity bitmask (ceil(n/64) words); ip_raw (IPv4 only) / tcp_raw nullable.
// false for overrides that name no shape of the receive kernels (segs_per_wave outside {0, 1, 2, 5-9}, or 5-9 off the
// default grid): NSX_EINVAL
bool rx_tune_valid(const LaunchCfg& c);
bool ragged_tune_valid(const LaunchCfg& c);
hipError_t launch_rx_tcp(const LaunchCfg& c, int ipver, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         uint64_t* mask, uint16_t* ip_raw, uint16_t* tcp_raw, hipStream_t st);
hipError_t launch_pseudo_ipv4(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t proto,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st);
hipError_t launch_pseudo_ipv6(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t nh,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st);
hipError_t launch_verify_mask(const uint16_t* raw, uint64_t n, uint64_t* mask, uint32_t max_blocks,
                              hipStream_t st);
struct TcpHdrSoA {  // device arrays, one entry per segment (tcp.go:39-54 field order)
    const uint16_t* src_port;
    const uint16_t* dst_port;
    const uint32_t* seq;
    const uint32_t* ack;
    const uint8_t* offset;
    const uint8_t* ctl;
    const uint16_t* window;
    const uint16_t* urgent;
};
hipError_t launch_tcp_build(const LaunchCfg& c, const TcpHdrSoA& h, const uint8_t* opts, const uint64_t* opt_off,
                            const uint8_t* data, const uint64_t* data_off, uint64_t data_bytes,
                            const uint32_t* partial, uint64_t n, uint8_t* out, const uint64_t* out_off,
                            uint16_t* raw, hipStream_t st);
struct TcpParsedSoA {  // device arrays, one entry per segment; every member nullable
    uint16_t* src_port;
    uint16_t* dst_port;
    uint32_t* seq;
    uint32_t* ack;
    uint8_t* offset;
    uint8_t* ctl;
    uint16_t* window;
    uint16_t* checksum;
    uint16_t* urgent;
    uint64_t* data_off;
    uint8_t* n_options;
    uint8_t* status;
};
// parseSegment (tcp.go:130-185) over segments d_base[d_offsets[i], d_offsets[i+1]).
hipError_t launch_tcp_parse(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                            const TcpParsedSoA& o, hipStream_t st);
// mode 0 verify (out), 1 fill (out nullable), 2 verify into the bitmask `mask` (ceil(n/64) words)
hipError_t launch_ipv4_hdr(const LaunchCfg& c, uint8_t* base, uint64_t stride, uint32_t hdr_off, uint64_t n,
                           int mode, uint16_t* out, uint64_t* mask, hipStream_t st);
// The per-stream deal counter sets (csum_kernels.hip deal_heads): return stream st's for reuse; sets given out.
void deal_release(hipStream_t st);
uint32_t deal_sets_in_use(int dev);
hipError_t launch_fill_splitmix64(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                                  uint32_t max_blocks, hipStream_t st);

}  // namespace nsx
