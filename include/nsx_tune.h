/*
 * nsx_tune.h — per-call launch overrides for benchmarks and tests.
 *
 * NOT part of the drop-in boundary (include/nsx_csum.h): a transport never
 * needs these. Every product entry point uses the per-path defaults measured
 * best on MI355X; the *_tuned twins below take an explicit
 * nsx_tune per call — there is no process-wide tuning state, so concurrent
 * callers with different settings cannot interfere. A NULL tune, or a field
 * left 0, means the default. Every setting is bit-exact; they change only the
 * launch shape (grid, work split, windows) or force one of the code paths the
 * defaults pick by layout, so the parity tests can reach each path on every
 * layout.
 */
#ifndef NSX_TUNE_H
#define NSX_TUNE_H

#include "nsx_csum.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NSX_TUNE_KERNEL_AUTO          0  /* the path the layout selects */
#define NSX_TUNE_KERNEL_HDR_THREAD    1  /* IPv4 headers: one thread per header (any stride) */
#define NSX_TUNE_KERNEL_HDR_DENSE     2  /* IPv4 headers: LDS-staged 64-header spans (stride <= 64) */
#define NSX_TUNE_KERNEL_BUILD_PLAIN   2  /* TCP build: no software pipelining */
#define NSX_TUNE_KERNEL_BUILD_GENERAL 3  /* TCP build: the general pipelined composition for every layout */
#define NSX_TUNE_KERNEL_SCAN_PLAIN    2  /* ragged scan: single row batches (rows 4, 8 or 16) */

typedef struct nsx_tune {
    int32_t blocks_per_cu;     /* persistent grid: 1..8 blocks of 256 threads per CU. Default of the ragged
                                  scan and receive kernels: 4 per CU, of which a streamed batch uses 3
                                  (a ragged batch of segments averaging >= 2048 B: 2; the rest return at
                                  once); a value
                                  here launches exactly that grid. A shape that may take an LDS form (the
                                  ragged scan's and receive pass's small-unit forms: ~34 KB of LDS per
                                  block) has at most 4 of its blocks resident per CU at a time (160 KB of
                                  LDS); above 4 blocks/CU forced streamed shapes allocate no LDS */
    int32_t segs_per_wave;     /* fixed batches of <= 4 KiB segments: segments per wave task (1, 2, 4, 8).
                                  Ragged scan: 0 auto (a batch whose segments average < 128 B: the small-
                                  segment mode — the LDS form on two waves per block, results parked and
                                  written 8 KiB at a time; otherwise per wave: the LDS form in waves whose
                                  segments average < 128 B, else streamed runs of two 63-segment sets
                                  < 256 B, else of one, on 3 blocks/CU, 2 from a 2048 B mean), 1 = runs
                                  of one set on the uncapped single-set kernel, 2 = the small-segment mode,
                                  3 = the LDS form in every wave (four per block, results stored per run),
                                  5 = runs of two sets in every wave; any other value is NSX_EINVAL (4,
                                  runs of four sets, was removed in round 4). Only the default pipelined
                                  2-row shape has two sets: with kernel = SCAN_PLAIN or rows != 2 a 5
                                  gives runs of one set. Grids of <= 4 blocks/CU park the streamed
                                  forms' results in LDS and write them 8 KiB at a time.
                                  Receive kernels: 0 auto = the default grid (4 blocks/CU) choosing by the
                                  batch's mean frame and frame count: < 112 B the LDS form for whole runs
                                  of <= 256 B frames that fit 8 KiB, switching at the first other run to
                                  the hybrid loop (such runs as prefix-form pieces of <= 7 KiB); below the
                                  streaming threshold (448 B in batches of < 2.5M frames, 768 B from 2.5M)
                                  the prefix form with 15 KiB slots on two waves per block, else streamed
                                  runs on 3 blocks/CU; 5 / 6 / 7 / 8 / 9 force the small-frame mode / the two-wave prefix
                                  form / the hybrid loop throughout / the streamed runs (3 blocks/CU) / the small-frame
                                  mode fed by LDS-DMA through a ring on that grid (NSX_EINVAL with rows
                                  other than 0 / 2 or with blocks_per_cu set). With rows or blocks_per_cu set (the
                                  pre-prefix shapes): 0 = per wave the LDS form (mean < 128 B) or streamed
                                  runs, 1 = streamed runs, 2 = the LDS form. (A run that does not fit the
                                  LDS form's 8 KiB slot, or a piece whose first 8 frames exceed the prefix
                                  form's slot, is streamed.) */
    int32_t block_mode;        /* 0 auto (a block per segment when n < 4 * CUs), 1 never, 2 always */
    int32_t rows;              /* ragged scan / receive kernels: 1 KiB rows per load batch (4, 8, 16) */
    int32_t run_segs;          /* segments per wave task: ragged scan kernel 1..63, TCP build 1..64 */
    int32_t xcd_chunk;         /* XCD deal: 0 auto, 1..20 = chunks of 2^k wave tasks, -1 contiguous eighths */
    int64_t window_bytes;      /* fixed <= 4 KiB segments: back-to-back launches of <= this many bytes;
                                  0 auto (batches >= 3.2 GB as ~1.6 GB windows), -1 one launch */
    int32_t kernel;            /* NSX_TUNE_KERNEL_* */
    int32_t shards_per_device; /* host batch calls: contiguous shards per GPU, each with its own host thread,
                                  streams and staging (default 1) */
    int32_t deal;              /* the ragged small-segment mode and the receive passes: 0 = the batch's last
                                  eighth dealt to the waves from the stream's counters where the stream allows
                                  it (nsx_csum.h, nsx_rx_ipv4_tcp_verify_dev), -1 = equal static shares
                                  throughout (A/B; replaces round 5's NSX_NO_DEAL build) */
    int32_t reserved[5];
} nsx_tune;

int nsx_csum_fixed_dev_tuned(const void* d_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                             const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream,
                             const nsx_tune* tune);
int nsx_csum_ragged_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                              const uint32_t* d_prefix_partial, uint16_t* d_out, nsx_stream_t stream,
                              const nsx_tune* tune);
int nsx_verify_ragged_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                                const uint32_t* d_prefix_partial, uint8_t* d_ok, uint16_t* d_raw,
                                nsx_stream_t stream, const nsx_tune* tune);
int nsx_tcp_build_dev_tuned(const nsx_tcp_hdr_soa* hdr, const uint8_t* d_opts, const uint64_t* d_opt_off,
                            const uint8_t* d_data, const uint64_t* d_data_off, uint64_t data_bytes,
                            const uint32_t* d_prefix_partial, uint64_t n, uint8_t* d_out, const uint64_t* d_out_off,
                            uint16_t* d_raw, nsx_stream_t stream, const nsx_tune* tune);
int nsx_ipv4_hdr_csum_dev_tuned(void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, int mode,
                                uint16_t* d_out_raw, nsx_stream_t stream, const nsx_tune* tune);
int nsx_ipv4_hdr_verify_mask_dev_tuned(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n,
                                       uint64_t* d_mask, nsx_stream_t stream, const nsx_tune* tune);
int nsx_rx_ipv4_tcp_verify_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                                     uint16_t* d_ip_raw, uint16_t* d_tcp_raw, nsx_stream_t stream,
                                     const nsx_tune* tune);
int nsx_rx_ipv6_tcp_verify_dev_tuned(const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_mask,
                                     uint16_t* d_tcp_raw, nsx_stream_t stream, const nsx_tune* tune);
int nsx_csum_fixed_host_tuned(const uint8_t* h_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                              const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus,
                              const nsx_tune* tune);
int nsx_csum_ragged_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n,
                               const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus,
                               const nsx_tune* tune);
int nsx_rx_ipv4_tcp_verify_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                      int num_gpus, const nsx_tune* tune);
int nsx_rx_ipv6_tcp_verify_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                      int num_gpus, const nsx_tune* tune);
int nsx_tcp_build_host_tuned(const nsx_tcp_hdr_soa* h_hdr, const uint8_t* h_opts, const uint64_t* h_opt_off,
                             const uint8_t* h_data, const uint64_t* h_data_off, const uint32_t* h_prefix_partial,
                             uint64_t n, uint8_t* h_out, const uint64_t* h_out_off, uint16_t* h_raw, int num_gpus,
                             const nsx_tune* tune);

/* Kernel launches one nsx_csum_fixed_dev(_tuned) call makes for this batch on the current device (its
 * back-to-back windows; 1 for most batches), for per-launch timing in benchmarks. */
int nsx_fixed_launch_count(uint64_t stride, uint32_t seg_len, uint64_t n, const nsx_tune* tune, uint64_t* out_count);
/* The same for nsx_ipv4_hdr_csum_dev / nsx_ipv4_hdr_verify_mask_dev(_tuned) (d_base only for its alignment):
 * packed 20 B headers of at least 2^26 go out as back-to-back windows of about 2^25. */
int nsx_ipv4_hdr_launch_count(const void* d_base, uint64_t stride, uint32_t hdr_off, uint64_t n, const nsx_tune* tune,
                              uint64_t* out_count);

/* Per-stream deal counter sets currently given out on the current device (tests: a stream returned with
 * nsx_stream_release gives its set to the next stream instead of taking a fresh one). */
int nsx_deal_sets_in_use(uint32_t* out_count);

#ifdef __cplusplus
}
#endif
#endif /* NSX_TUNE_H */
