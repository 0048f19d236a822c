/*
 * nsx_csum.h — C ABI of the MI355X-native Internet checksum (RFC 1071) path.
 *
 * This is the drop-in boundary for the reference's one checksum function,
 *   transport/tcp/tcp.go:72-95  func (s segment) computeChecksum(ipPseudoHeader []byte) uint16
 * (reference: oneee-playground/network-stack, pure Go). A Go caller reaches it
 * through the cgo shim in network-stack_amd/go/transport/tcp/ (INTEGRATION.md).
 *
 * Semantics shared by every entry point (tcp.go:68-95):
 *   - the checksummed stream is prefix ‖ segment (tcp.go:73); an odd total is
 *     zero-padded (tcp.go:74-77);
 *   - 16-bit big-endian words are added with end-around carry (tcp.go:79-92);
 *   - the RAW one's-complement sum is returned, NOT complemented (tcp.go:94).
 *     0x0000 only for an all-zero input; a nonzero input whose sum is
 *     ≡ 0 mod 0xFFFF gives 0xFFFF. The sender stores nsx_field(raw) = ~raw
 *     (tcp_test.go:28); a receiver accepts iff raw == 0xFFFF (tcp.go:70).
 *
 * Conventions:
 *   - Return 0 (NSX_OK) or a negative errno-style code; never abort or print.
 *   - The caller owns every buffer. No pointer is retained after the stream
 *     work completes (device calls) or after return (host calls).
 *   - Device calls are asynchronous on `stream` (a hipStream_t; NULL = the
 *     default stream of the current device). Device pointers must belong to the
 *     device current on the calling thread. No host synchronisation, no
 *     allocation inside device calls (hipGraph-capturable).
 *   - Re-entrant; no global mutable state on the data path.
 *   - A device call on a host with no usable GPU returns NSX_ENODEV. There is no
 *     CPU fallback for the batch/device entry points.
 */
#ifndef NSX_CSUM_H
#define NSX_CSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NSX_OK      0
#define NSX_EIO    (-5)   /* a HIP runtime call or kernel launch failed */
#define NSX_ENOMEM (-12)  /* host or device allocation failed */
#define NSX_ENODEV (-19)  /* no usable GPU / bad device ordinal */
#define NSX_EINVAL (-22)  /* null pointer with nonzero length, bad sizes */

#define NSX_ABI_VERSION 2  /* 2: process-wide tuning knobs removed (nsx_tune.h) */

typedef void* nsx_stream_t; /* hipStream_t, opaque to C/Go callers */

/* ----------------------------------------------------------------------------
 * Single segment, host CPU.
 * Replaces: transport/tcp/tcp.go:72-95 computeChecksum (called from
 * tcp_test.go:28,30). Exactly its semantics over prefix ‖ seg, without the
 * reference's allocation/copy of the concatenation (tcp.go:73) and without
 * writing into the prefix's spare capacity. For per-segment cgo calls; never
 * touches the GPU (a per-segment cgo call must not drive the device).
 * prefix may be NULL iff prefix_len == 0; likewise seg.
 */
int nsx_csum16(const uint8_t* prefix, size_t prefix_len,
               const uint8_t* seg, size_t seg_len, uint16_t* out_raw_sum);

/* ----------------------------------------------------------------------------
 * Device-resident batches (the hot path). One result (raw sum) per segment.
 *
 * d_prefix_partial (nullable): per-segment integer sum of the prefix's
 * big-endian 16-bit words (e.g. an IPv4/IPv6 TCP pseudo-header, whose length is
 * even), folded or not; result[i] = raw sum over prefix_i ‖ segment_i.
 * Produce it with nsx_pseudo_ipv4_partial_dev or nsx_csum_fixed_dev on the
 * pseudo-headers themselves.
 */

/* Fixed stride: segment i occupies d_base[i*stride, i*stride + seg_len).
 * The span [d_base, d_base + (n-1)*stride + seg_len) must be readable.
 * Replaces a Go loop of computeChecksum over equal-size segments (tcp.go:72). */
int nsx_csum_fixed_dev(const void* d_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                       const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream);

/* Ragged: segment i occupies d_base[d_offsets[i], d_offsets[i+1]); d_offsets
 * has n+1 non-decreasing entries; segments may start at any byte (dense packing,
 * odd starts). The span [d_base + d_offsets[0], d_base + d_offsets[n]) must be
 * readable. */
int nsx_csum_ragged_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                        const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream);

/* Receive-side verify (tcp.go:70): d_ok[i] = (raw_i == 0xFFFF), where raw_i is
 * the ragged-batch raw sum with the optional prefix partial. d_raw (nullable)
 * also receives the raw sums. */
int nsx_verify_ragged_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                          const uint32_t* d_prefix_partial, uint8_t* d_ok, uint16_t* d_raw,
                          nsx_stream_t stream);

/* IPv4 TCP pseudo-header partials (RFC 9293 §3.1: src(4) dst(4) 0 proto len(2))
 * for n segments: d_src/d_dst are n×4 address bytes as ip.Addr.Raw()
 * (network/ip/v4/ipv4.go:15), d_len the TCP length of each segment, proto e.g.
 * ip.NextProtoTCP = 6 (network/ip/protocols.go:8). Writes the integer BE-word
 * sum to d_partial[i] (the d_prefix_partial convention above). */
int nsx_pseudo_ipv4_partial_dev(const uint8_t* d_src, const uint8_t* d_dst,
                                const uint32_t* d_len, uint8_t proto, uint64_t n,
                                uint32_t* d_partial, nsx_stream_t stream);

/* IPv6 TCP pseudo-header partials (RFC 8200 §8.1: src(16) dst(16) len(4)
 * zero(3) next_header(1)) for n segments: d_src/d_dst are n×16 address bytes as
 * ip.Addr.Raw() (network/ip/v6/ipv6.go:16), d_len the upper-layer length, and
 * next_header e.g. ip.NextProtoTCP = 6. Same d_partial convention as above. */
int nsx_pseudo_ipv6_partial_dev(const uint8_t* d_src, const uint8_t* d_dst,
                                const uint32_t* d_len, uint8_t next_header, uint64_t n,
                                uint32_t* d_partial, nsx_stream_t stream);

/* Receive-side verify as a bitmask (tcp.go:70): bit (i % 64) of d_mask[i / 64]
 * is set iff d_raw[i] == 0xFFFF; bits past n in the last word are 0. d_mask
 * holds ceil(n/64) words. Pairs with nsx_csum_fixed_dev / nsx_csum_ragged_dev. */
int nsx_verify_mask_dev(const uint16_t* d_raw, uint64_t n, uint64_t* d_mask, nsx_stream_t stream);

/* Fused sender path: segment.bytes() + computeChecksum +
 * field write in one GPU pass (transport/tcp/tcp.go:98-128, :68-71). For each
 * segment i it writes the wire image — the 20-byte big-endian header built from
 * the fields below (checksum field = ~raw), the option bytes
 * d_opts[d_opt_off[i], d_opt_off[i+1]) followed by the reference's padding of
 * `remainder` zero bytes (tcp.go:118-121), then the payload
 * d_data[d_data_off[i], d_data_off[i+1]) — to d_out + d_out_off[i], where raw is
 * the sum over prefix_i ‖ image with the field zero. d_out_off[i] must be a
 * multiple of 4 and leave room for nsx_tcp_wire_len bytes; up to 3 bytes after
 * each image are zero-filled (use nsx_tcp_layout_host). d_opt_off nullable (no
 * options); data_bytes = size of the d_data buffer. d_raw (nullable) receives
 * the raw sums. All nsx_tcp_hdr_soa members are device arrays of n entries;
 * `offset` is the whole byte 12, as the reference stores it (tcp.go:106); a
 * NULL `offset` computes it on the device as computeOffset() does (tcp.go:59-66):
 * uint8((20 + option bytes + 3) / 4).
 * Each wire image must be shorter than 2^31 bytes (TCP segments are ≤ 64 KiB;
 * TSO super-segments ≤ 256 KiB). */
typedef struct {
    const uint16_t* src_port;
    const uint16_t* dst_port;
    const uint32_t* seq_num;
    const uint32_t* ack_num;
    const uint8_t* offset;
    const uint8_t* control;  /* ctl.byte() (tcp.go:192-203) */
    const uint16_t* window;
    const uint16_t* urgent_ptr;
} nsx_tcp_hdr_soa;

int nsx_tcp_build_dev(const nsx_tcp_hdr_soa* hdr, const uint8_t* d_opts, const uint64_t* d_opt_off,
                      const uint8_t* d_data, const uint64_t* d_data_off, uint64_t data_bytes,
                      const uint32_t* d_prefix_partial, uint64_t n, uint8_t* d_out, const uint64_t* d_out_off,
                      uint16_t* d_raw, nsx_stream_t stream);

/* Receive-side parse (parseSegment, transport/tcp/tcp.go:130-185) of n TCP
 * segments d_base[d_offsets[i], d_offsets[i+1]) (any alignment, d_offsets as
 * for nsx_csum_ragged_dev) into device arrays of n entries; every member of
 * *out is nullable. Fields as the reference reads them (offset = the whole byte
 * 12, control = ctl.byte(), checksum = bytes 16-17); data_off[i] = d_offsets[i]
 * + offset*4 (the payload, s.data = raw[dataAt:]); n_options = the options the
 * reference appends (NOP and MSS; EOL ends the walk). status[i]:
 *   NSX_TCP_PARSE_OK            parsed;
 *   NSX_TCP_PARSE_SHORT         fewer than 20 bytes ("segment too short", :131);
 *   NSX_TCP_PARSE_OFFSET        offset*4 > length ("advertised data offset too
 *                               long", :152);
 *   NSX_TCP_PARSE_OPTION_RANGE  an MSS option whose length runs past the segment
 *                               (the reference's slice panics or reads past the
 *                               segment, :173-174);
 *   NSX_TCP_PARSE_OPTION_KIND   an option kind other than 0-2 before dataAt (the
 *                               reference's loop never advances, :160-179).
 * On any status but OK the fields, data_off and n_options are 0 (the reference
 * returns segment{}). */
#define NSX_TCP_PARSE_OK 0
#define NSX_TCP_PARSE_SHORT 1
#define NSX_TCP_PARSE_OFFSET 2
#define NSX_TCP_PARSE_OPTION_RANGE 3
#define NSX_TCP_PARSE_OPTION_KIND 4
typedef struct {
    uint16_t* src_port;
    uint16_t* dst_port;
    uint32_t* seq_num;
    uint32_t* ack_num;
    uint8_t* offset;
    uint8_t* control;
    uint16_t* window;
    uint16_t* checksum;
    uint16_t* urgent_ptr;
    uint64_t* data_off;
    uint8_t* n_options;
    uint8_t* status;
} nsx_tcp_parsed_soa;

int nsx_tcp_parse_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, const nsx_tcp_parsed_soa* out,
                      nsx_stream_t stream);

/* Wire length of segment.bytes() with opt_len option bytes (tcp.go:98-128). */
uint64_t nsx_tcp_wire_len(uint64_t opt_len, uint64_t data_len);

/* 4-byte-aligned output offsets for nsx_tcp_build_dev (host arrays; h_opt_off
 * nullable): h_out_off[i] = Σ_{j<i} round_up4(wire_len_j), h_out_off[n] = total. */
int nsx_tcp_layout_host(const uint64_t* h_opt_off, const uint64_t* h_data_off, uint64_t n, uint64_t* h_out_off);

/* IPv4 header checksums (RFC 791 §3.1; SURVEY.md §8 f3 — the reference has no
 * IPv4 header codec, network/ip/v4/ipv4.go holds addresses only). Packet i's
 * header starts at d_base + i*stride + hdr_off (any alignment) and is IHL*4
 * bytes, IHL = low nibble of its first byte.
 *   mode 0 (receive): d_out_raw[i] = raw sum over the header as it stands;
 *          the header is valid iff it is 0xFFFF.
 *   mode 1 (send):    d_out_raw[i] (nullable) = raw sum with bytes 10-11 taken
 *          as zero, and ~raw is written big-endian into bytes 10-11 in place.
 * A malformed header (IHL < 5, or hdr_off + IHL*4 > stride) yields 0 and is
 * left untouched. At least 20 bytes must be readable at every header start;
 * stride and hdr_off ≤ 2^22 (NSX_EINVAL otherwise). */
int nsx_ipv4_hdr_csum_dev(void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, int mode,
                          uint16_t* d_out_raw, nsx_stream_t stream);

/* IPv4 header verify straight into a bitmask (the receive side of f3 fused with
 * the f2 mask convention, tcp.go:70 rule applied to RFC 791 headers): bit
 * (i % 64) of d_mask[i / 64] is set iff header i is well-formed and its raw sum
 * is 0xFFFF (= nsx_ipv4_hdr_csum_dev mode 0 followed by nsx_verify_mask_dev,
 * one pass, 1 bit written per header instead of 16); bits past n in the last
 * word are 0. d_mask holds ceil(n/64) words. Same layout rules and limits as
 * nsx_ipv4_hdr_csum_dev; the headers are only read. */
int nsx_ipv4_hdr_verify_mask_dev(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n,
                                 uint64_t* d_mask, nsx_stream_t stream);

/* Fused receive pass (SURVEY.md §8 f2 + f3 in one launch): n received IPv4
 * datagrams carrying TCP, densely packed — frame i = d_base[d_offsets[i],
 * d_offsets[i+1]), any alignment, d_offsets as for nsx_csum_ragged_dev. Bit
 * (i % 64) of d_mask[i / 64] is set iff frame i
 *   - is a well-formed, unfragmented IPv4 datagram carrying TCP: version 4,
 *     IHL >= 5, IHL*4 <= frame length, total length (bytes 2-3) == frame
 *     length, MF clear and fragment offset 0 (a fragment's TCP checksum covers
 *     bytes it does not hold), protocol 6 (ip.NextProtoTCP,
 *     network/ip/protocols.go:8), and a TCP segment (total − IHL*4 bytes) of at
 *     least 20 bytes (tcp.go:131, minSegmentLength);
 *   - has a valid header checksum: the raw sum over its IHL*4 header bytes is
 *     0xFFFF (RFC 791 §3.1);
 *   - has a valid TCP checksum: the raw sum over the pseudo-header built from
 *     the header's own source and destination (ip.Addr.Raw(),
 *     network/ip/v4/ipv4.go:15), 0, 6, TCP length ‖ the segment is 0xFFFF
 *     (tcp.go:70 receiver rule over computeChecksum, tcp.go:72-95).
 * Bits past n in the last word are 0; d_mask holds ceil(n/64) words.
 * d_ip_raw (nullable): the header's raw sum (0 when IHL < 5 or IHL*4 exceeds the
 * frame). d_tcp_raw (nullable): the raw sum over pseudo-header ‖ segment (0
 * unless the frame is well-formed as above). One pass over the frame bytes.
 * Work split: the batch's last eighth of frames is dealt to the GPU's waves as
 * they finish, from counters the library keeps per stream (64 streams per
 * device, in the library's own device memory; every launch leaves them at zero
 * for the stream's next, so launches sharing them must run one after another).
 * Only a handle that is one ordered queue of the current device gets counters:
 * a stream the caller created, or the null stream. hipStreamPerThread (one
 * handle, a different stream per host thread), a stream of another device, a
 * stream being captured into a graph, and streams past the 64th split the
 * batch statically instead; results are the same either way. See
 * nsx_stream_release. */
int nsx_rx_ipv4_tcp_verify_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                               uint16_t* d_ip_raw, uint16_t* d_tcp_raw, nsx_stream_t stream);

/* The same receive pass for IPv6 (the IPv6 pseudo-header of
 * ip.Addr.Raw(), network/ip/v6/ipv6.go:16): frame i is an IPv6 packet whose
 * fixed 40-byte header (RFC 8200 §3) is followed directly by a TCP segment.
 * Bit (i % 64) of d_mask[i / 64] is set iff frame i
 *   - is well-formed: at least 40 bytes, version 6, 40 + payload length (bytes
 *     4-5) == frame length, Next Header (byte 6) == 6 (ip.NextProtoTCP; a
 *     packet with extension headers is not walked and does not verify), and a
 *     payload of at least 20 bytes (tcp.go:131);
 *   - has a valid TCP checksum: the raw sum over the RFC 8200 §8.1 pseudo-header
 *     src(16) dst(16) payload length(4) 0 0 0 6 from the header's own addresses
 *     ‖ the segment is 0xFFFF (tcp.go:70 over computeChecksum, tcp.go:72-95).
 * IPv6 has no header checksum. d_tcp_raw (nullable): that raw sum, 0 unless the
 * frame is well-formed. Layout rules and work split as
 * nsx_rx_ipv4_tcp_verify_dev. */
int nsx_rx_ipv6_tcp_verify_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                               uint16_t* d_tcp_raw, nsx_stream_t stream);

/* ----------------------------------------------------------------------------
 * Host-resident batches: pinned staging, H2D → kernel → D2H double-buffered
 * over two streams per GPU, segments sharded contiguously across num_gpus
 * devices (0 = auto: one GPU per 64 MiB of batch, up to all visible). No
 * collective: shards are independent.
 * h_prefix_partial nullable.
 */
int nsx_csum_fixed_host(const uint8_t* h_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                        const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus);

int nsx_csum_ragged_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n,
                         const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus);

/* The fused receive pass (nsx_rx_ipv4_tcp_verify_dev) over host-resident
 * datagrams: h_mask receives ceil(n/64) words. Shards and chunks start on
 * 64-frame mask words. */
int nsx_rx_ipv4_tcp_verify_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                int num_gpus);
int nsx_rx_ipv6_tcp_verify_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                int num_gpus);

/* The fused sender pass (nsx_tcp_build_dev) over host-resident segments: the
 * header fields (nsx_tcp_hdr_soa members here are HOST arrays of n entries;
 * `offset` nullable as for the device call), options (h_opt_off nullable),
 * payloads, partials (nullable) and the output are in host memory, pageable or
 * pinned (nsx_alloc_pinned; pinned data and output are DMA'd directly). Writes
 * each wire image to h_out + h_out_off[i] with the device call's layout rule
 * (h_out_off[i] a multiple of 4, room for the image rounded up to 4 bytes, the
 * up to 3 bytes after it zero-filled; nsx_tcp_layout_host makes such offsets;
 * bytes between a padded image and the next offset are left as they are) and
 * the raw sums to h_raw (nullable). Offsets must be non-decreasing and every
 * image shorter than 2^31 bytes (NSX_EINVAL otherwise, checked before any copy).
 * Sharded by image bytes over num_gpus devices like the calls above (0 = auto),
 * chunks of <= 64 MiB of images double-buffered per device.
 * Replaces a Go send loop over bytes() + computeChecksum + the field store
 * (transport/tcp/tcp.go:98-128, :110, :68-71) whose images then go into the
 * transport's pipe or socket buffers (transport/pipe/pipe.go:92-124). */
int nsx_tcp_build_host(const nsx_tcp_hdr_soa* h_hdr, const uint8_t* h_opts, const uint64_t* h_opt_off,
                       const uint8_t* h_data, const uint64_t* h_data_off, const uint32_t* h_prefix_partial,
                       uint64_t n, uint8_t* h_out, const uint64_t* h_out_off, uint16_t* h_raw, int num_gpus);

/* The host batch calls keep per-device streams and grow-only device/pinned
 * staging buffers across calls (a transport calls them once per batch). This
 * frees the cached buffers; the next call re-allocates. Safe to call at any
 * time; concurrent host batch calls on a device wait for each other. */
int nsx_host_cache_release(void);

/* Return the per-stream work-deal counters the device calls above gave
 * `stream` (nsx_rx_ipv4_tcp_verify_dev and friends) before the caller destroys
 * it: call after the stream has drained (hipStreamSynchronize) and before
 * hipStreamDestroy. The counters go to the next new stream; without this, a
 * process that creates and destroys streams in a loop keeps the first 64 on the
 * dealt path and splits every later one statically (correct, ~2% slower). */
int nsx_stream_release(nsx_stream_t stream);

/* Pinned (DMA-registered) host memory for zero-copy staging from Go via
 * unsafe.Slice (cgo forbids C retaining Go pointers; runtime.Pinner does not
 * DMA-register). */
int nsx_alloc_pinned(size_t bytes, void** out);
int nsx_free_pinned(void* p);

/* ----------------------------------------------------------------------------
 * Sharding plan (host logic, no GPU): split n segments over `parts` shards.
 * Fixed stride (h_offsets NULL): contiguous index ranges of near-equal count.
 * Ragged: contiguous index ranges of near-equal BYTE count using the prefix-sum
 * offsets. Writes parts+1 boundaries to out_bounds (out_bounds[0]=0,
 * out_bounds[parts]=n).
 */
int nsx_shard_plan(const uint64_t* h_offsets, uint64_t n, int parts, uint64_t* out_bounds);

/* ----------------------------------------------------------------------------
 * Synthetic batches (bench/test data): byte j of the stream is
 * byte j%8 of the little-endian word splitmix64(seed, j/8); writes stream bytes
 * [byte_off, byte_off + nbytes) to d_buf. Counter-based, so any range can be
 * regenerated on the host. */
int nsx_fill_splitmix64_dev(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                            nsx_stream_t stream);

/* ----------------------------------------------------------------------------
 * Introspection. (Benchmark/test launch overrides are per call, in
 * include/nsx_tune.h — not part of this boundary.)
 */
int nsx_abi_version(void);
int nsx_device_count(int* out_count);        /* NSX_OK with 0 when no GPU */
const char* nsx_strerror(int code);

/* Receiver/sender helpers (tcp.go:68-71, tcp_test.go:28-31). */
static inline uint16_t nsx_field(uint16_t raw_sum) { return (uint16_t)~raw_sum; }
static inline int nsx_verify(uint16_t raw_sum) { return raw_sum == 0xFFFF; }

#ifdef __cplusplus
}
#endif
#endif /* NSX_CSUM_H */
