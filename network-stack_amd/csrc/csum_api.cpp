// csum_api.cpp — C ABI (include/nsx_csum.h) over the gfx950 checksum kernels.
//
// Boundary for transport/tcp/tcp.go:72-95 (computeChecksum). Device entry points
// validate arguments, pick the kernel variant and launch asynchronously on the
// caller's stream; host entry points shard a host-resident batch over GPUs and
// pipeline pinned H2D → kernel → D2H per GPU. Nothing here computes a batch
// checksum on the CPU: with no GPU the batch calls return NSX_ENODEV.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nsx_csum.h"
#include "../../include/nsx_tune.h"
#include "csum_kernels.h"
#include "host_csum.h"

namespace {

constexpr int kMaxDevices = 64;

struct DevInfo {
    int cus = 0;
    bool ok = false;
};
DevInfo g_dev[kMaxDevices];
std::once_flag g_dev_once[kMaxDevices];

int device_count_raw() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

const DevInfo* dev_info(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    std::call_once(g_dev_once[dev], [dev] {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
            g_dev[dev].cus = cus;
            g_dev[dev].ok = true;
        } else {
            (void)hipGetLastError();
        }
    });
    return g_dev[dev].ok ? &g_dev[dev] : nullptr;
}

// Current device of the calling thread, or -1 when there is no usable GPU.
int current_device() {
    if (device_count_raw() <= 0) return -1;
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return dev_info(d) ? d : -1;
}

int map_err(hipError_t e);

}  // namespace

namespace nsx {

// Launch configuration of one call: the device's CU count + the caller's overrides (nsx_tune.h).
LaunchCfg launch_cfg(int cus, const nsx_tune* t) {
    LaunchCfg c;
    c.cus = cus;
    if (t) {
        c.blocks_per_cu = t->blocks_per_cu;
        c.segs_per_wave = t->segs_per_wave;
        c.block_mode = t->block_mode;
        c.rows = t->rows;
        c.run_segs = t->run_segs;
        c.xcd_chunk = t->xcd_chunk;
        c.window_bytes = t->window_bytes;
        c.kernel = t->kernel;
        c.deal = t->deal;
    }
    return c;
}

}  // namespace nsx

namespace {

nsx::LaunchCfg make_cfg(int dev, const nsx_tune* t) { return nsx::launch_cfg(dev_info(dev)->cus, t); }

int map_err(hipError_t e) {
    if (e == hipSuccess) return NSX_OK;
    (void)hipGetLastError();
    if (e == hipErrorOutOfMemory) return NSX_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return NSX_ENODEV;
    return NSX_EIO;
}

}  // namespace

extern "C" {

int nsx_abi_version(void) { return NSX_ABI_VERSION; }

int nsx_device_count(int* out_count) {
    if (!out_count) return NSX_EINVAL;
    *out_count = device_count_raw();
    return NSX_OK;
}

const char* nsx_strerror(int code) {
    switch (code) {
        case NSX_OK: return "ok";
        case NSX_EIO: return "HIP runtime or kernel launch failure";
        case NSX_ENOMEM: return "out of memory";
        case NSX_ENODEV: return "no usable GPU";
        case NSX_EINVAL: return "invalid argument";
        default: return "unknown error";
    }
}

// ------------------------------------------------------------ single segment
int nsx_csum16(const uint8_t* prefix, size_t prefix_len, const uint8_t* seg, size_t seg_len,
               uint16_t* out_raw_sum) {
    if (!out_raw_sum || (prefix_len && !prefix) || (seg_len && !seg)) return NSX_EINVAL;
    *out_raw_sum = nsx::host_csum16(prefix, prefix_len, seg, seg_len);
    return NSX_OK;
}

// ------------------------------------------------------------ device batches
// Each product entry point is its *_tuned twin (include/nsx_tune.h) with no overrides.
int nsx_csum_fixed_dev(const void* d_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                       const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream) {
    return nsx_csum_fixed_dev_tuned(d_base, stride, seg_len, n, d_prefix_partial, d_out, stream, nullptr);
}

int nsx_csum_fixed_dev_tuned(const void* d_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                             const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream,
                             const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_out || (seg_len && !d_base)) return NSX_EINVAL;
    // stride 0 with n > 1 is allowed: every segment aliases the first
    if (n > ((uint64_t)1 << 40)) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    return map_err(nsx::launch_fixed(make_cfg(dev, tune), d_base, stride, seg_len, n, d_prefix_partial, d_out,
                                     static_cast<hipStream_t>(stream)));
}

int nsx_fixed_launch_count(uint64_t stride, uint32_t seg_len, uint64_t n, const nsx_tune* tune, uint64_t* out_count) {
    if (!out_count) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    *out_count = nsx::fixed_launch_count(make_cfg(dev, tune), 0, stride, seg_len, n);
    return NSX_OK;
}

int nsx_ipv4_hdr_launch_count(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, const nsx_tune* tune,
                              uint64_t* out_count) {
    if (!out_count) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    *out_count = nsx::ipv4_hdr_launch_count(make_cfg(dev, tune), (uintptr_t)d_base, stride, hdr_off, n);
    return NSX_OK;
}

int nsx_csum_ragged_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                        const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream) {
    return nsx_csum_ragged_dev_tuned(d_base, d_offsets, n, d_prefix_partial, d_out, stream, nullptr);
}

int nsx_csum_ragged_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                              const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream,
                              const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_out || !d_offsets || !d_base) return NSX_EINVAL;
    if (n > ((uint64_t)1 << 40)) return NSX_EINVAL;
    if (!nsx::ragged_tune_valid(nsx::launch_cfg(1, tune))) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    return map_err(nsx::launch_ragged(make_cfg(dev, tune), d_base, d_offsets, n, d_prefix_partial, d_out, nullptr,
                                      static_cast<hipStream_t>(stream)));
}

int nsx_verify_ragged_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                          const uint32_t* d_prefix_partial, uint8_t* d_ok, uint16_t* d_raw,
                          nsx_stream_t stream) {
    return nsx_verify_ragged_dev_tuned(d_base, d_offsets, n, d_prefix_partial, d_ok, d_raw, stream, nullptr);
}

int nsx_verify_ragged_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                                const uint32_t* d_prefix_partial, uint8_t* d_ok, uint16_t* d_raw,
                                nsx_stream_t stream, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_ok || !d_offsets || !d_base) return NSX_EINVAL;
    if (n > ((uint64_t)1 << 40)) return NSX_EINVAL;
    if (!nsx::ragged_tune_valid(nsx::launch_cfg(1, tune))) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    return map_err(nsx::launch_ragged(make_cfg(dev, tune), d_base, d_offsets, n, d_prefix_partial, d_raw, d_ok,
                                      static_cast<hipStream_t>(stream)));
}

int nsx_rx_ipv4_tcp_verify_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                               uint16_t* d_ip_raw, uint16_t* d_tcp_raw, nsx_stream_t stream) {
    return nsx_rx_ipv4_tcp_verify_dev_tuned(d_base, d_offsets, n, d_mask, d_ip_raw, d_tcp_raw, stream, nullptr);
}

int nsx_rx_ipv4_tcp_verify_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                                     uint16_t* d_ip_raw, uint16_t* d_tcp_raw, nsx_stream_t stream,
                                     const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_base || !d_offsets || !d_mask) return NSX_EINVAL;
    if (n > ((uint64_t)1 << 40)) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const nsx::LaunchCfg cfg = make_cfg(dev, tune);
    if (!nsx::rx_tune_valid(cfg)) return NSX_EINVAL;
    return map_err(nsx::launch_rx_tcp(cfg, 4, d_base, d_offsets, n, d_mask, d_ip_raw, d_tcp_raw,
                                      static_cast<hipStream_t>(stream)));
}

int nsx_rx_ipv6_tcp_verify_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                               uint16_t* d_tcp_raw, nsx_stream_t stream) {
    return nsx_rx_ipv6_tcp_verify_dev_tuned(d_base, d_offsets, n, d_mask, d_tcp_raw, stream, nullptr);
}

int nsx_rx_ipv6_tcp_verify_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                                     uint16_t* d_tcp_raw, nsx_stream_t stream, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_base || !d_offsets || !d_mask) return NSX_EINVAL;
    if (n > ((uint64_t)1 << 40)) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const nsx::LaunchCfg cfg = make_cfg(dev, tune);
    if (!nsx::rx_tune_valid(cfg)) return NSX_EINVAL;
    return map_err(nsx::launch_rx_tcp(cfg, 6, d_base, d_offsets, n, d_mask, nullptr, d_tcp_raw,
                                      static_cast<hipStream_t>(stream)));
}

int nsx_pseudo_ipv4_partial_dev(const uint8_t* d_src, const uint8_t* d_dst, const uint32_t* d_len,
                                uint8_t proto, uint64_t n, uint32_t* d_partial, nsx_stream_t stream) {
    if (n == 0) return NSX_OK;
    if (!d_src || !d_dst || !d_len || !d_partial) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const DevInfo* di = dev_info(dev);
    return map_err(nsx::launch_pseudo_ipv4(d_src, d_dst, d_len, proto, n, d_partial, (uint32_t)di->cus * 8,
                                           static_cast<hipStream_t>(stream)));
}

int nsx_pseudo_ipv6_partial_dev(const uint8_t* d_src, const uint8_t* d_dst, const uint32_t* d_len,
                                uint8_t next_header, uint64_t n, uint32_t* d_partial, nsx_stream_t stream) {
    if (n == 0) return NSX_OK;
    if (!d_src || !d_dst || !d_len || !d_partial) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const DevInfo* di = dev_info(dev);
    return map_err(nsx::launch_pseudo_ipv6(d_src, d_dst, d_len, next_header, n, d_partial, (uint32_t)di->cus * 8,
                                           static_cast<hipStream_t>(stream)));
}

int nsx_verify_mask_dev(const uint16_t* d_raw, uint64_t n, uint64_t* d_mask, nsx_stream_t stream) {
    if (n == 0) return NSX_OK;
    if (!d_raw || !d_mask) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const DevInfo* di = dev_info(dev);
    return map_err(nsx::launch_verify_mask(d_raw, n, d_mask, (uint32_t)di->cus * 8, static_cast<hipStream_t>(stream)));
}

uint64_t nsx_tcp_wire_len(uint64_t opt_len, uint64_t data_len) {
    return 20u + opt_len + (opt_len ? (20u + opt_len) % 4u : 0u) + data_len;
}

int nsx_tcp_layout_host(const uint64_t* h_opt_off, const uint64_t* h_data_off, uint64_t n, uint64_t* h_out_off) {
    if (!h_out_off || (n && !h_data_off)) return NSX_EINVAL;
    uint64_t at = 0;
    for (uint64_t i = 0; i < n; ++i) {
        h_out_off[i] = at;
        const uint64_t ol = h_opt_off ? h_opt_off[i + 1] - h_opt_off[i] : 0;
        at += (nsx_tcp_wire_len(ol, h_data_off[i + 1] - h_data_off[i]) + 3) & ~3ull;
    }
    h_out_off[n] = at;
    return NSX_OK;
}

int nsx_tcp_build_dev(const nsx_tcp_hdr_soa* hdr, const uint8_t* d_opts, const uint64_t* d_opt_off,
                      const uint8_t* d_data, const uint64_t* d_data_off, uint64_t data_bytes,
                      const uint32_t* d_prefix_partial, uint64_t n, uint8_t* d_out, const uint64_t* d_out_off,
                      uint16_t* d_raw, nsx_stream_t stream) {
    return nsx_tcp_build_dev_tuned(hdr, d_opts, d_opt_off, d_data, d_data_off, data_bytes, d_prefix_partial, n, d_out,
                                   d_out_off, d_raw, stream, nullptr);
}

int nsx_tcp_build_dev_tuned(const nsx_tcp_hdr_soa* hdr, const uint8_t* d_opts, const uint64_t* d_opt_off,
                            const uint8_t* d_data, const uint64_t* d_data_off, uint64_t data_bytes,
                            const uint32_t* d_prefix_partial, uint64_t n, uint8_t* d_out, const uint64_t* d_out_off,
                            uint16_t* d_raw, nsx_stream_t stream, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!hdr || !hdr->src_port || !hdr->dst_port || !hdr->seq_num || !hdr->ack_num ||
        !hdr->control || !hdr->window || !hdr->urgent_ptr || !d_data_off || !d_out || !d_out_off ||
        (d_opt_off && !d_opts) || (data_bytes && !d_data))
        return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const nsx::TcpHdrSoA h{hdr->src_port, hdr->dst_port, hdr->seq_num, hdr->ack_num,
                           hdr->offset,   hdr->control,  hdr->window,  hdr->urgent_ptr};
    return map_err(nsx::launch_tcp_build(make_cfg(dev, tune), h, d_opts, d_opt_off, d_data, d_data_off, data_bytes,
                                         d_prefix_partial, n, d_out, d_out_off, d_raw,
                                         static_cast<hipStream_t>(stream)));
}

int nsx_tcp_parse_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, const nsx_tcp_parsed_soa* out,
                      nsx_stream_t stream) {
    if (n == 0) return NSX_OK;
    if (!d_base || !d_offsets || !out) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const nsx::TcpParsedSoA o{out->src_port, out->dst_port, out->seq_num,    out->ack_num,
                              out->offset,   out->control,  out->window,     out->checksum,
                              out->urgent_ptr, out->data_off, out->n_options, out->status};
    return map_err(nsx::launch_tcp_parse(make_cfg(dev, nullptr), d_base, d_offsets, n, o,
                                         static_cast<hipStream_t>(stream)));
}

static int ipv4_args_ok(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n) {
    if (!d_base) return NSX_EINVAL;
    if (n > 1 && stride == 0) return NSX_EINVAL;
    if (stride > ((uint64_t)1 << 22) || hdr_off > ((uint32_t)1 << 22)) return NSX_EINVAL;  // 32-bit block offsets
    return NSX_OK;
}

int nsx_ipv4_hdr_csum_dev(void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, int mode,
                          uint16_t* d_out_raw, nsx_stream_t stream) {
    return nsx_ipv4_hdr_csum_dev_tuned(d_base, stride, hdr_off, n, mode, d_out_raw, stream, nullptr);
}

int nsx_ipv4_hdr_csum_dev_tuned(void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, int mode,
                                uint16_t* d_out_raw, nsx_stream_t stream, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if ((mode != 0 && mode != 1) || (mode == 0 && !d_out_raw)) return NSX_EINVAL;
    if (int rc = ipv4_args_ok(d_base, stride, hdr_off, n)) return rc;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    return map_err(nsx::launch_ipv4_hdr(make_cfg(dev, tune), static_cast<uint8_t*>(d_base), stride, hdr_off, n, mode,
                                        d_out_raw, nullptr, static_cast<hipStream_t>(stream)));
}

int nsx_ipv4_hdr_verify_mask_dev(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, uint64_t* d_mask,
                                 nsx_stream_t stream) {
    return nsx_ipv4_hdr_verify_mask_dev_tuned(d_base, stride, hdr_off, n, d_mask, stream, nullptr);
}

int nsx_ipv4_hdr_verify_mask_dev_tuned(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n,
                                       uint64_t* d_mask, nsx_stream_t stream, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!d_mask) return NSX_EINVAL;
    if (int rc = ipv4_args_ok(d_base, stride, hdr_off, n)) return rc;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    // mode 2 only reads the headers (the kernels take a non-const base for fill mode)
    return map_err(nsx::launch_ipv4_hdr(make_cfg(dev, tune), static_cast<uint8_t*>(const_cast<void*>(d_base)), stride,
                                        hdr_off, n, 2, nullptr, d_mask, static_cast<hipStream_t>(stream)));
}

int nsx_fill_splitmix64_dev(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                            nsx_stream_t stream) {
    if (nbytes == 0) return NSX_OK;
    if (!d_buf) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    const DevInfo* di = dev_info(dev);
    return map_err(nsx::launch_fill_splitmix64(d_buf, byte_off, nbytes, seed, (uint32_t)di->cus * 8,
                                               static_cast<hipStream_t>(stream)));
}

// ------------------------------------------------------------ sharding plan
int nsx_shard_plan(const uint64_t* h_offsets, uint64_t n, int parts, uint64_t* out_bounds) {
    if (parts < 1 || !out_bounds) return NSX_EINVAL;
    nsx::shard_plan(h_offsets, n, parts, out_bounds);
    return NSX_OK;
}

// ------------------------------------------------------------ per-stream deal counters
int nsx_stream_release(nsx_stream_t stream) {
    nsx::deal_release(static_cast<hipStream_t>(stream));
    return NSX_OK;
}

int nsx_deal_sets_in_use(uint32_t* out_count) {
    if (!out_count) return NSX_EINVAL;
    const int dev = current_device();
    if (dev < 0) return NSX_ENODEV;
    *out_count = nsx::deal_sets_in_use(dev);
    return NSX_OK;
}

// ------------------------------------------------------------ pinned memory
int nsx_alloc_pinned(size_t bytes, void** out) {
    if (!out) return NSX_EINVAL;
    *out = nullptr;
    if (bytes == 0) return NSX_OK;
    if (device_count_raw() <= 0) return NSX_ENODEV;
    hipError_t e = hipHostMalloc(out, bytes, hipHostMallocPortable);
    if (e != hipSuccess) {
        *out = nullptr;
        return map_err(e);
    }
    return NSX_OK;
}

int nsx_free_pinned(void* p) {
    if (!p) return NSX_OK;
    return map_err(hipHostFree(p));
}

}  // extern "C"
