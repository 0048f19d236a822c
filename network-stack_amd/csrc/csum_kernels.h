// csum_kernels.h — internal launcher interface between the C ABI (csum_api.cpp)
// and the gfx950 kernels (csum_kernels.hip). Not a public header.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nsx {

constexpr int kKernelRowStream = 1;  // csum_stream_kernel
constexpr int kKernelPerSegment = 2; // csum_fixed_kernel / csum_wave_kernel
constexpr int kKernelPipelined = 3;  // buffer-load kernels: csum_fixed_buf_kernel / csum_ragged_buf_kernel
constexpr int kKernelScan = 4;       // csum_ragged_scan_kernel (ragged; the default there)
constexpr int kKernelSwPipe = 5;     // csum_fixed_swp_kernel: software-pipelined fixed-stride buffer kernel
constexpr int kKernelScanPipe = 6;   // csum_ragged_scan_kernel, software-pipelined row batches (nt loads)
constexpr int kKernelLongSwp = 7;    // csum_long_swp_kernel: long aligned fixed-stride segments, pipelined rows

// Raw NSX_PARAM_* values (0 = "default for this path"); the launchers resolve
// them per path (fixed short / fixed long / ragged) to the defaults measured
// best on MI355X by tools/sweep.py.
struct LaunchCfg {
    int cus;             // compute units of the device
    int blocks_per_cu;   // persistent grid = cus × blocks_per_cu blocks of 256 threads
    int segs_per_wave;   // per-segment fixed kernel: 1, 2, 4
    int nontemporal;     // 1 nt loads, 2 default policy
    int block_mode;      // 1 never, 2 always, 0 auto (n < 4·cus)
    int xcd_map;         // 1 XCD-contiguous deal, 2 grid-stride, 3 contiguous range per wave
    int kernel;          // kKernelRowStream / kKernelPerSegment
    int rows;            // row-stream rows per batch: 4, 8, 16
    int run_segs;        // ragged scan kernel: segments per wave task, 1..63
    int xcd_chunk;       // XCD deal: interleaved chunks of 2^k tasks (0 = auto, 1..20 fixed, else contiguous eighths)
    int64_t window_bytes = 0;  // fixed short-segment path: back-to-back launches of ≤ this many bytes (0 auto, -1 one launch)
};

// Launch configuration from the process-wide NSX_PARAM_* knobs (csum_api.cpp).
LaunchCfg default_launch_cfg(int cus, uint64_t n);

hipError_t launch_fixed(const LaunchCfg& c, const void* d_base, uint64_t stride, uint32_t seg_len,
                        uint64_t n, const uint32_t* partial, uint16_t* out, hipStream_t st);
hipError_t launch_ragged(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st);
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
hipError_t launch_tcp_build(const TcpHdrSoA& h, const uint8_t* opts, const uint64_t* opt_off, const uint8_t* data,
                            const uint64_t* data_off, uint64_t data_bytes, const uint32_t* partial, uint64_t n,
                            uint8_t* out, const uint64_t* out_off, uint16_t* raw, uint32_t max_blocks, int policy,
                            int xchunk, int kernel, int spw, hipStream_t st);
// bpc / unroll: raw NSX_PARAM_BLOCKS_PER_CU / NSX_PARAM_SEGS_PER_WAVE (0 = per-kernel default);
// mode 0 verify (out), 1 fill (out nullable), 2 verify into the bitmask `mask` (ceil(n/64) words)
hipError_t launch_ipv4_hdr(uint8_t* base, uint64_t stride, uint32_t hdr_off, uint64_t n, int mode, uint16_t* out,
                           uint64_t* mask, int cus, int bpc, int kernel, int unroll, int xchunk, hipStream_t st);
hipError_t launch_fill_splitmix64(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                                  uint32_t max_blocks, hipStream_t st);

}  // namespace nsx
