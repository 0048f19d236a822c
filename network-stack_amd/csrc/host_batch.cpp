// host_batch.cpp — host-resident batches: shard over GPUs, pipeline per GPU.
//
// The reference's checksum input lives in transport buffers in host memory
// (transport/pipe/pipe.go:73-124 hands []byte slices between goroutines), so the
// end-to-end path is host → HBM → kernel → host. Each GPU gets a contiguous
// shard (no collective: segments are independent) and a host thread that
// double-buffers fixed-size chunks over two HIP streams: chunk k+1's H2D copy
// overlaps chunk k's kernel and D2H. Caller memory that is already pinned
// (nsx_alloc_pinned) is DMA'd directly; pageable memory is bounced through
// pinned staging buffers (multi-threaded copy, stage_copy). Streams and buffers
// persist per device (DevCtx).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nsx_csum.h"
#include "../../include/nsx_tune.h"
#include "csum_kernels.h"
#include "host_csum.h"

namespace {

constexpr uint64_t kChunkBytes = 64ull << 20;

// Pageable caller memory is bounced through pinned staging; one thread's memcpy (~10-25 GB/s) would
// then, not PCIe, set the end-to-end rate. Large copies are split over up to kCopyThreads threads
// (NSX_HOST_COPY_THREADS overrides; 1 = serial).
constexpr int kCopyThreads = 8;
constexpr uint64_t kCopySplitMin = 4ull << 20;

int copy_threads() {
    static const int n = [] {
        const char* e = std::getenv("NSX_HOST_COPY_THREADS");
        int v = e ? std::atoi(e) : 0;
        if (v < 1) v = std::min<int>(kCopyThreads, (int)std::max(1u, std::thread::hardware_concurrency()));
        return std::min(v, 64);
    }();
    return n;
}

void stage_copy(void* dst, const void* src, uint64_t bytes) {
    const int nt = bytes >= kCopySplitMin ? copy_threads() : 1;
    if (nt <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const uint64_t part = ((bytes + nt - 1) / nt + 4095) & ~4095ull;  // page-sized pieces
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const uint64_t lo = part * t;
        if (lo >= bytes) break;
        th.emplace_back([=] { std::memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, std::min(part, bytes - lo)); });
    }
    std::memcpy(dst, src, std::min(part, bytes));
    for (auto& x : th) x.join();
}

bool is_pinned(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

int map_err(hipError_t e) {
    if (e == hipSuccess) return NSX_OK;
    (void)hipGetLastError();
    return e == hipErrorOutOfMemory ? NSX_ENOMEM : NSX_EIO;
}

#define NSX_TRY(expr)                          \
    do {                                       \
        hipError_t e_ = (expr);                \
        if (e_ != hipSuccess) {                \
            rc = map_err(e_);                  \
            goto done;                         \
        }                                      \
    } while (0)

nsx::LaunchCfg cfg_for(int dev, const nsx_tune* tune) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        (void)hipGetLastError();
        cus = 256;
    }
    return nsx::launch_cfg(cus, tune);
}

// One chunk = segments [c0, c1) of the shard.
struct Chunk {
    uint64_t c0, c1;
    uint64_t byte_lo, byte_hi;  // host span copied for the chunk
};

struct Job {
    // inputs (shard-relative views)
    const uint8_t* h_base;
    uint64_t stride;
    uint32_t seg_len;
    const uint64_t* h_offsets;  // null → fixed stride; else absolute offsets into h_base
    uint64_t lo, hi;            // segment index range of the shard
    const uint32_t* h_partial;
    uint16_t* h_out;            // checksum mode: one raw sum per segment
    uint64_t* h_mask;           // receive mode (nsx_rx_ipv*_tcp_verify_host): one validity bit per frame
    int ipver;                  // receive mode: 4 or 6
    int dev;
    int slot;  // shard slot on the device (its own DevCtx: streams + staging)
    const nsx_tune* tune;
    int rc;
};

std::vector<Chunk> plan_chunks(const Job& j) {
    std::vector<Chunk> v;
    if (j.h_mask) {  // receive mode: chunks of whole 64-frame mask words (the shard starts on one)
        uint64_t c0 = j.lo;
        while (c0 < j.hi) {
            uint64_t c1 = c0 + 1;
            while (c1 < j.hi && j.h_offsets[c1 + 1] - j.h_offsets[c0] <= kChunkBytes) ++c1;
            if (c1 < j.hi) c1 = std::min(j.hi, c0 + std::max<uint64_t>(64, (c1 - c0) / 64 * 64));
            v.push_back({c0, c1, j.h_offsets[c0], j.h_offsets[c1]});
            c0 = c1;
        }
    } else if (!j.h_offsets) {
        const uint64_t span = std::max<uint64_t>(std::max<uint64_t>(j.stride, j.seg_len), 1);
        const uint64_t per = std::max<uint64_t>(1, kChunkBytes / span);
        for (uint64_t c0 = j.lo; c0 < j.hi; c0 += per) {
            const uint64_t c1 = std::min(j.hi, c0 + per);
            v.push_back({c0, c1, c0 * j.stride, (c1 - 1) * j.stride + j.seg_len});
        }
    } else {
        uint64_t c0 = j.lo;
        while (c0 < j.hi) {
            uint64_t c1 = c0 + 1;
            while (c1 < j.hi && j.h_offsets[c1 + 1] - j.h_offsets[c0] <= kChunkBytes) ++c1;
            v.push_back({c0, c1, j.h_offsets[c0], j.h_offsets[c1]});
            c0 = c1;
        }
    }
    return v;
}

// Per-device resources reused across calls: the transport calls the host
// batch API once per received batch (tools/loopback.cpp), so stream creation,
// hipMalloc and hipHostMalloc (page registration) must not sit on every call —
// they cost milliseconds against a ~100 KB batch's tens of microseconds.
// Buffers only grow; nsx_host_cache_release() frees them. Calls on the same
// device serialise on the context's mutex (each call already fills the GPU's
// copy engines with its own double-buffered chunks).
template <bool kHost>
struct Grow {
    void* p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap) return hipSuccess;
        release();
        uint64_t c = 4096;
        while (c < bytes) c <<= 1;
        const hipError_t e = kHost ? hipHostMalloc(&p, c, hipHostMallocPortable) : hipMalloc(&p, c);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        cap = c;
        return hipSuccess;
    }
    void release() {
        if (p) (void)(kHost ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct DevCtx {
    std::mutex mu;
    hipStream_t st[2] = {nullptr, nullptr};
    Grow<false> d_data[2], d_out[2], d_part[2], d_off[2];
    Grow<true> h_stage[2], h_ostage[2], h_pstage[2], h_offstage[2];
    // the sender pass (nsx_tcp_build_host) also stages header fields, options and raw sums
    Grow<false> d_fields[2], d_opts[2], d_raw[2];
    Grow<true> h_fstage[2], h_optstage[2], h_rawstage[2];
    void release() {
        for (int s = 0; s < 2; ++s) {
            d_data[s].release(), d_out[s].release(), d_part[s].release(), d_off[s].release();
            h_stage[s].release(), h_ostage[s].release(), h_pstage[s].release(), h_offstage[s].release();
            d_fields[s].release(), d_opts[s].release(), d_raw[s].release();
            h_fstage[s].release(), h_optstage[s].release(), h_rawstage[s].release();
        }
    }
};

constexpr int kMaxDevices = 64;
constexpr int kMaxSlots = 8;  // nsx_tune.shards_per_device ≤ this
std::mutex g_ctx_mu;
DevCtx* g_ctx[kMaxDevices][kMaxSlots] = {};  // never destroyed: HIP may be torn down before static destructors run

DevCtx* dev_ctx(int dev, int slot) {
    if (dev < 0 || dev >= kMaxDevices || slot < 0 || slot >= kMaxSlots) return nullptr;
    std::lock_guard<std::mutex> g(g_ctx_mu);
    if (!g_ctx[dev][slot]) g_ctx[dev][slot] = new DevCtx;
    return g_ctx[dev][slot];
}

void run_job(Job* j) {
    int rc = NSX_OK;
    const std::vector<Chunk> chunks = plan_chunks(*j);
    uint64_t max_span = 0, max_segs = 0;
    for (const Chunk& c : chunks) {
        max_span = std::max(max_span, c.byte_hi - c.byte_lo);
        max_segs = std::max(max_segs, c.c1 - c.c0);
    }
    const bool rx = j->h_mask != nullptr;
    // results of chunk segments [c0, c1): raw sums, or mask words (receive mode; c0 is a multiple of 64)
    auto out_bytes = [rx](uint64_t cn) { return rx ? (cn + 63) / 64 * 8 : cn * sizeof(uint16_t); };
    auto out_host = [j, rx](uint64_t c0) {
        return rx ? reinterpret_cast<uint8_t*>(j->h_mask + c0 / 64) : reinterpret_cast<uint8_t*>(j->h_out + c0);
    };
    const bool in_pinned = is_pinned(j->h_base);
    const bool out_pinned = is_pinned(out_host(j->lo));
    const bool ragged = j->h_offsets != nullptr;
    const int nslots = chunks.size() > 1 ? 2 : 1;
    DevCtx* ctx = dev_ctx(j->dev, j->slot);
    if (!ctx) {
        j->rc = NSX_EINVAL;
        return;
    }
    std::lock_guard<std::mutex> hold(ctx->mu);
    hipStream_t* st = ctx->st;
    nsx::LaunchCfg cfg;
    const Chunk* pending[2] = {nullptr, nullptr};

    NSX_TRY(hipSetDevice(j->dev));
    cfg = cfg_for(j->dev, j->tune);
    for (int s = 0; s < nslots; ++s) {
        if (!st[s]) NSX_TRY(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
        NSX_TRY(ctx->d_data[s].ensure(std::max<uint64_t>(max_span, 16)));
        NSX_TRY(ctx->d_out[s].ensure(std::max<uint64_t>(out_bytes(max_segs), 8)));
        if (j->h_partial) {
            NSX_TRY(ctx->d_part[s].ensure(max_segs * sizeof(uint32_t)));
            NSX_TRY(ctx->h_pstage[s].ensure(max_segs * sizeof(uint32_t)));
        }
        if (ragged) {
            NSX_TRY(ctx->d_off[s].ensure((max_segs + 1) * sizeof(uint64_t)));
            NSX_TRY(ctx->h_offstage[s].ensure((max_segs + 1) * sizeof(uint64_t)));
        }
        if (!in_pinned) NSX_TRY(ctx->h_stage[s].ensure(std::max<uint64_t>(max_span, 16)));
        if (!out_pinned) NSX_TRY(ctx->h_ostage[s].ensure(std::max<uint64_t>(out_bytes(max_segs), 8)));
    }

    for (size_t k = 0; k < chunks.size(); ++k) {
        const int s = (int)(k % nslots);
        const Chunk& c = chunks[k];
        const uint64_t cn = c.c1 - c.c0, span = c.byte_hi - c.byte_lo;
        uint8_t* d_data = ctx->d_data[s].as<uint8_t>();
        uint16_t* d_out = ctx->d_out[s].as<uint16_t>();
        uint32_t* d_part = j->h_partial ? ctx->d_part[s].as<uint32_t>() : nullptr;
        uint8_t* h_ostage = ctx->h_ostage[s].as<uint8_t>();
        if (pending[s]) {  // slot reuse: finish chunk k-2
            NSX_TRY(hipStreamSynchronize(st[s]));
            if (!out_pinned)
                std::memcpy(out_host(pending[s]->c0), h_ostage, out_bytes(pending[s]->c1 - pending[s]->c0));
            pending[s] = nullptr;
        }
        const uint8_t* src = j->h_base + c.byte_lo;
        if (!in_pinned) {
            stage_copy(ctx->h_stage[s].p, src, span);
            src = ctx->h_stage[s].as<uint8_t>();
        }
        if (span) NSX_TRY(hipMemcpyAsync(d_data, src, span, hipMemcpyHostToDevice, st[s]));
        if (j->h_partial) {
            uint32_t* h_pstage = ctx->h_pstage[s].as<uint32_t>();
            std::memcpy(h_pstage, j->h_partial + c.c0, cn * sizeof(uint32_t));
            NSX_TRY(hipMemcpyAsync(d_part, h_pstage, cn * sizeof(uint32_t), hipMemcpyHostToDevice, st[s]));
        }
        uint8_t* out_dst = out_pinned ? out_host(c.c0) : h_ostage;
        hipError_t e;
        if (ragged) {
            uint64_t* h_offstage = ctx->h_offstage[s].as<uint64_t>();
            uint64_t* d_off = ctx->d_off[s].as<uint64_t>();
            for (uint64_t i = 0; i <= cn; ++i) h_offstage[i] = j->h_offsets[c.c0 + i] - c.byte_lo;
            NSX_TRY(hipMemcpyAsync(d_off, h_offstage, (cn + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st[s]));
            e = rx ? nsx::launch_rx_tcp(cfg, j->ipver, d_data, d_off, cn, reinterpret_cast<uint64_t*>(d_out),
                                        nullptr, nullptr, st[s])
                   : nsx::launch_ragged(cfg, d_data, d_off, cn, d_part, d_out, nullptr, st[s]);
        } else {
            e = nsx::launch_fixed(cfg, d_data, j->stride, j->seg_len, cn, d_part, d_out, st[s]);
        }
        NSX_TRY(e);
        NSX_TRY(hipMemcpyAsync(out_dst, d_out, out_bytes(cn), hipMemcpyDeviceToHost, st[s]));
        pending[s] = &c;
    }
    for (int s = 0; s < nslots; ++s) {
        NSX_TRY(hipStreamSynchronize(st[s]));
        if (pending[s] && !out_pinned)
            std::memcpy(out_host(pending[s]->c0), ctx->h_ostage[s].p, out_bytes(pending[s]->c1 - pending[s]->c0));
        pending[s] = nullptr;
    }

done:
    if (rc != NSX_OK)  // leave the streams idle for the next call
        for (int s = 0; s < 2; ++s)
            if (st[s]) (void)hipStreamSynchronize(st[s]);
    j->rc = rc;
}

// Shards: num_gpus × shards_per_device contiguous ranges (byte-balanced for ragged batches); shard g runs on
// device g / shards_per_device in slot g % shards_per_device, one host thread per shard.
int run_sharded(const uint8_t* h_base, uint64_t stride, uint32_t seg_len, const uint64_t* h_offsets, uint64_t n,
                const uint32_t* h_partial, uint16_t* h_out, uint64_t* h_mask, int ipver, int num_gpus,
                const nsx_tune* tune) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        count = 0;
    }
    if (count <= 0) return NSX_ENODEV;
    if (num_gpus <= 0) {  // auto: all GPUs, but no shard smaller than one chunk
        const uint64_t bytes = h_offsets ? h_offsets[n] - h_offsets[0] : n * std::max<uint64_t>(stride, seg_len);
        const uint64_t want = std::max<uint64_t>(1, (bytes + kChunkBytes - 1) / kChunkBytes);
        num_gpus = (int)std::min<uint64_t>(want, (uint64_t)count);
    }
    if (num_gpus > count) return NSX_ENODEV;
    const int spd = (tune && tune->shards_per_device > 1) ? std::min(tune->shards_per_device, kMaxSlots) : 1;
    int caller_dev = 0;
    (void)hipGetDevice(&caller_dev);
    const int parts = (int)std::min<uint64_t>((uint64_t)num_gpus * spd, n);
    std::vector<uint64_t> bounds(parts + 1);
    nsx::shard_plan(h_offsets, n, parts, bounds.data());
    if (h_mask)  // receive mode: every shard starts on a 64-frame mask word
        for (int g = 1; g < parts; ++g) bounds[g] = std::min<uint64_t>(n, (bounds[g] + 63) / 64 * 64);
    std::vector<Job> jobs(parts);
    for (int g = 0; g < parts; ++g)
        jobs[g] = Job{h_base,  stride, seg_len, h_offsets, bounds[g], bounds[g + 1], h_partial, h_out, h_mask, ipver,
                      g / spd, g % spd, tune,    NSX_OK};
    std::vector<std::thread> th;
    for (int g = 1; g < parts; ++g)
        if (jobs[g].hi > jobs[g].lo) th.emplace_back(run_job, &jobs[g]);
    if (jobs[0].hi > jobs[0].lo) run_job(&jobs[0]);
    for (auto& t : th) t.join();
    (void)hipSetDevice(caller_dev);
    for (const Job& j : jobs)
        if (j.rc != NSX_OK) return j.rc;
    return NSX_OK;
}

// ---- the fused sender pass over host-resident segments (nsx_tcp_build_host) ----
// A Go transport's send loop builds segments (tcp.go:98-128), stores ^sum at bytes 16-17 (tcp.go:110, :68-71) and
// writes the images into its pipe or socket buffers (transport/pipe/pipe.go:92-124): header fields, options and
// payloads start in host memory and the wire images end there. Per chunk of segments (≤ 64 MiB of images): the
// fields (18 B per segment, one pinned block of 8 sub-arrays), the rebased offsets, the option and payload spans
// and the partials go H2D, nsx_tcp_build_dev's kernel runs, and the image span and raw sums come back, double-
// buffered over the shard's two streams like the checksum chunks above. The staged payload keeps its byte offset
// mod 256 and sits ≥ 256 B into its buffer, and the image span keeps its offset mod 256, so every segment takes the
// kernel path it would take in a device-resident batch at a 256-aligned base.
struct BuildJob {
    const nsx_tcp_hdr_soa* h;  // host arrays
    const uint8_t* opts;
    const uint64_t* opt_off;  // nullable
    const uint8_t* data;
    const uint64_t* data_off;
    const uint32_t* partial;  // nullable
    uint8_t* out;
    const uint64_t* out_off;
    uint16_t* raw;  // nullable
    bool gaps;      // some image slot is longer than its 4-padded image: the caller's bytes there are preserved
    uint64_t lo, hi;
    int dev, slot;
    const nsx_tune* tune;
    int rc;
};

constexpr uint64_t kFieldAlign = 256;

uint64_t field_block_bytes(uint64_t cn) {  // 8 sub-arrays of cn entries, each 256 B-aligned
    const uint64_t a = kFieldAlign - 1;
    return 2 * ((2 * cn + a) & ~a) + 2 * ((4 * cn + a) & ~a) + 2 * ((2 * cn + a) & ~a) + 2 * ((cn + a) & ~a);
}

void run_build_job(BuildJob* j) {
    int rc = NSX_OK;
    std::vector<Chunk> chunks;  // byte_lo/byte_hi: the chunk's image span
    for (uint64_t c0 = j->lo; c0 < j->hi;) {
        uint64_t c1 = c0 + 1;
        while (c1 < j->hi && j->out_off[c1 + 1] - j->out_off[c0] <= kChunkBytes &&
               j->data_off[c1 + 1] - j->data_off[c0] <= kChunkBytes)
            ++c1;
        chunks.push_back({c0, c1, j->out_off[c0], j->out_off[c1]});
        c0 = c1;
    }
    uint64_t max_out = 0, max_data = 0, max_opt = 0, max_segs = 0;
    for (const Chunk& c : chunks) {
        max_out = std::max(max_out, c.byte_hi - c.byte_lo);
        max_data = std::max(max_data, j->data_off[c.c1] - j->data_off[c.c0]);
        if (j->opt_off) max_opt = std::max(max_opt, j->opt_off[c.c1] - j->opt_off[c.c0]);
        max_segs = std::max(max_segs, c.c1 - c.c0);
    }
    const bool in_pinned = is_pinned(j->data), out_pinned = is_pinned(j->out);
    const int nslots = chunks.size() > 1 ? 2 : 1;
    DevCtx* ctx = dev_ctx(j->dev, j->slot);
    if (!ctx) {
        j->rc = NSX_EINVAL;
        return;
    }
    std::lock_guard<std::mutex> hold(ctx->mu);
    hipStream_t* st = ctx->st;
    nsx::LaunchCfg cfg;
    const Chunk* pending[2] = {nullptr, nullptr};
    const uint64_t noffs = j->opt_off ? 3 : 2;  // rebased data_off, out_off (, opt_off), cn + 1 entries each
    auto finish = [&](int s) {  // chunk pending[s] is complete on the device: hand its results to the caller
        const Chunk* c = pending[s];
        const uint64_t lead_o = c->byte_lo & 255;
        // the images back into pageable caller memory: the same multi-threaded copy as the payloads' way in (one
        // thread's memcpy held the pageable build at 31.7 GB/s of PCIe traffic against 54.3 pinned)
        if (!out_pinned) stage_copy(j->out + c->byte_lo, ctx->h_ostage[s].as<uint8_t>() + lead_o, c->byte_hi - c->byte_lo);
        if (j->raw) std::memcpy(j->raw + c->c0, ctx->h_rawstage[s].p, (c->c1 - c->c0) * sizeof(uint16_t));
        pending[s] = nullptr;
    };

    NSX_TRY(hipSetDevice(j->dev));
    cfg = cfg_for(j->dev, j->tune);
    for (int s = 0; s < nslots; ++s) {
        if (!st[s]) NSX_TRY(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
        NSX_TRY(ctx->d_data[s].ensure(512 + max_data + 16));
        NSX_TRY(ctx->d_out[s].ensure(256 + max_out + 16));
        NSX_TRY(ctx->d_fields[s].ensure(field_block_bytes(max_segs)));
        NSX_TRY(ctx->h_fstage[s].ensure(field_block_bytes(max_segs)));
        NSX_TRY(ctx->d_off[s].ensure(noffs * (max_segs + 1) * sizeof(uint64_t)));
        NSX_TRY(ctx->h_offstage[s].ensure(noffs * (max_segs + 1) * sizeof(uint64_t)));
        NSX_TRY(ctx->d_raw[s].ensure(std::max<uint64_t>(max_segs * sizeof(uint16_t), 16)));
        NSX_TRY(ctx->h_rawstage[s].ensure(std::max<uint64_t>(max_segs * sizeof(uint16_t), 16)));
        if (j->partial) {
            NSX_TRY(ctx->d_part[s].ensure(max_segs * sizeof(uint32_t)));
            NSX_TRY(ctx->h_pstage[s].ensure(max_segs * sizeof(uint32_t)));
        }
        if (j->opt_off) {
            NSX_TRY(ctx->d_opts[s].ensure(max_opt + 16));
            NSX_TRY(ctx->h_optstage[s].ensure(max_opt + 16));
        }
        if (!in_pinned) NSX_TRY(ctx->h_stage[s].ensure(max_data + 16));
        if (!out_pinned) NSX_TRY(ctx->h_ostage[s].ensure(256 + max_out + 16));
    }

    for (size_t k = 0; k < chunks.size(); ++k) {
        const int s = (int)(k % nslots);
        const Chunk& c = chunks[k];
        const uint64_t cn = c.c1 - c.c0, span_o = c.byte_hi - c.byte_lo;
        const uint64_t d0 = j->data_off[c.c0], span_d = j->data_off[c.c1] - d0;
        const uint64_t lead_d = 256 + (d0 & 255), lead_o = c.byte_lo & 255;
        if (pending[s]) {  // slot reuse: finish chunk k-2
            NSX_TRY(hipStreamSynchronize(st[s]));
            finish(s);
        }
        // header fields: 8 sub-arrays in one pinned block, one copy
        uint8_t* hf = ctx->h_fstage[s].as<uint8_t>();
        uint8_t* df = ctx->d_fields[s].as<uint8_t>();
        const void* src_f[8] = {j->h->src_port, j->h->dst_port, j->h->seq_num, j->h->ack_num,
                                j->h->window,   j->h->urgent_ptr, j->h->offset, j->h->control};
        const uint64_t esz[8] = {2, 2, 4, 4, 2, 2, 1, 1};
        const void* dev_f[8];
        uint64_t at = 0;
        for (int f = 0; f < 8; ++f) {
            dev_f[f] = src_f[f] ? df + at : nullptr;
            if (src_f[f]) std::memcpy(hf + at, (const uint8_t*)src_f[f] + c.c0 * esz[f], cn * esz[f]);
            at += (cn * esz[f] + kFieldAlign - 1) & ~(kFieldAlign - 1);
        }
        NSX_TRY(hipMemcpyAsync(df, hf, at, hipMemcpyHostToDevice, st[s]));
        // offsets, rebased to the staged spans
        uint64_t* ho = ctx->h_offstage[s].as<uint64_t>();
        uint64_t* dofs = ctx->d_off[s].as<uint64_t>();
        for (uint64_t i = 0; i <= cn; ++i) {
            ho[i] = j->data_off[c.c0 + i] - d0 + lead_d;
            ho[cn + 1 + i] = j->out_off[c.c0 + i] - c.byte_lo + lead_o;
            if (j->opt_off) ho[2 * (cn + 1) + i] = j->opt_off[c.c0 + i] - j->opt_off[c.c0];
        }
        NSX_TRY(hipMemcpyAsync(dofs, ho, noffs * (cn + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st[s]));
        const uint8_t* d_opts = nullptr;
        if (j->opt_off) {
            const uint64_t ospan = j->opt_off[c.c1] - j->opt_off[c.c0];
            uint8_t* hos = ctx->h_optstage[s].as<uint8_t>();
            if (ospan) {
                std::memcpy(hos, j->opts + j->opt_off[c.c0], ospan);
                NSX_TRY(hipMemcpyAsync(ctx->d_opts[s].p, hos, ospan, hipMemcpyHostToDevice, st[s]));
            }
            d_opts = ctx->d_opts[s].as<uint8_t>();
        }
        // payloads
        uint8_t* d_data = ctx->d_data[s].as<uint8_t>();
        const uint8_t* src = j->data + d0;
        if (!in_pinned && span_d) {
            stage_copy(ctx->h_stage[s].p, src, span_d);
            src = ctx->h_stage[s].as<uint8_t>();
        }
        if (span_d) NSX_TRY(hipMemcpyAsync(d_data + lead_d, src, span_d, hipMemcpyHostToDevice, st[s]));
        uint32_t* d_part = nullptr;
        if (j->partial) {
            uint32_t* hp = ctx->h_pstage[s].as<uint32_t>();
            std::memcpy(hp, j->partial + c.c0, cn * sizeof(uint32_t));
            d_part = ctx->d_part[s].as<uint32_t>();
            NSX_TRY(hipMemcpyAsync(d_part, hp, cn * sizeof(uint32_t), hipMemcpyHostToDevice, st[s]));
        }
        uint8_t* d_out = ctx->d_out[s].as<uint8_t>();
        uint8_t* out_dst = out_pinned ? j->out + c.byte_lo : ctx->h_ostage[s].as<uint8_t>() + lead_o;
        if (j->gaps && span_o) {  // the caller's bytes between images stay as they are
            if (!out_pinned) stage_copy(out_dst, j->out + c.byte_lo, span_o);
            NSX_TRY(hipMemcpyAsync(d_out + lead_o, out_dst, span_o, hipMemcpyHostToDevice, st[s]));
        }
        const nsx::TcpHdrSoA h{(const uint16_t*)dev_f[0], (const uint16_t*)dev_f[1], (const uint32_t*)dev_f[2],
                               (const uint32_t*)dev_f[3], (const uint8_t*)dev_f[6],  (const uint8_t*)dev_f[7],
                               (const uint16_t*)dev_f[4], (const uint16_t*)dev_f[5]};
        uint16_t* d_raw = ctx->d_raw[s].as<uint16_t>();
        NSX_TRY(nsx::launch_tcp_build(cfg, h, d_opts, j->opt_off ? dofs + 2 * (cn + 1) : nullptr, d_data, dofs,
                                      lead_d + span_d, d_part, cn, d_out, dofs + cn + 1, j->raw ? d_raw : nullptr, st[s]));
        if (span_o) NSX_TRY(hipMemcpyAsync(out_dst, d_out + lead_o, span_o, hipMemcpyDeviceToHost, st[s]));
        if (j->raw)
            NSX_TRY(hipMemcpyAsync(ctx->h_rawstage[s].p, d_raw, cn * sizeof(uint16_t), hipMemcpyDeviceToHost, st[s]));
        pending[s] = &c;
    }
    for (int s = 0; s < nslots; ++s) {
        NSX_TRY(hipStreamSynchronize(st[s]));
        if (pending[s]) finish(s);
    }

done:
    if (rc != NSX_OK)
        for (int s = 0; s < 2; ++s)
            if (st[s]) (void)hipStreamSynchronize(st[s]);
    j->rc = rc;
}

int run_build_sharded(const BuildJob& proto, uint64_t n, int num_gpus, const nsx_tune* tune) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        count = 0;
    }
    if (count <= 0) return NSX_ENODEV;
    if (num_gpus <= 0) {  // auto: all GPUs, but no shard smaller than one chunk of images
        const uint64_t bytes = proto.out_off[n] - proto.out_off[0];
        const uint64_t want = std::max<uint64_t>(1, (bytes + kChunkBytes - 1) / kChunkBytes);
        num_gpus = (int)std::min<uint64_t>(want, (uint64_t)count);
    }
    if (num_gpus > count) return NSX_ENODEV;
    const int spd = (tune && tune->shards_per_device > 1) ? std::min(tune->shards_per_device, kMaxSlots) : 1;
    int caller_dev = 0;
    (void)hipGetDevice(&caller_dev);
    const int parts = (int)std::min<uint64_t>((uint64_t)num_gpus * spd, n);
    std::vector<uint64_t> bounds(parts + 1);
    nsx::shard_plan(proto.out_off, n, parts, bounds.data());  // balanced by image bytes
    std::vector<BuildJob> jobs(parts, proto);
    for (int g = 0; g < parts; ++g) {
        jobs[g].lo = bounds[g], jobs[g].hi = bounds[g + 1];
        jobs[g].dev = g / spd, jobs[g].slot = g % spd, jobs[g].tune = tune, jobs[g].rc = NSX_OK;
    }
    std::vector<std::thread> th;
    for (int g = 1; g < parts; ++g)
        if (jobs[g].hi > jobs[g].lo) th.emplace_back(run_build_job, &jobs[g]);
    if (jobs[0].hi > jobs[0].lo) run_build_job(&jobs[0]);
    for (auto& t : th) t.join();
    (void)hipSetDevice(caller_dev);
    for (const BuildJob& j : jobs)
        if (j.rc != NSX_OK) return j.rc;
    return NSX_OK;
}

}  // namespace

extern "C" {

int nsx_csum_fixed_host(const uint8_t* h_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                        const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus) {
    return nsx_csum_fixed_host_tuned(h_base, stride, seg_len, n, h_prefix_partial, h_out, num_gpus, nullptr);
}

int nsx_csum_fixed_host_tuned(const uint8_t* h_base, uint64_t stride, uint32_t seg_len, uint64_t n,
                              const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus,
                              const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!h_out || (seg_len && !h_base)) return NSX_EINVAL;
    return run_sharded(h_base, stride, seg_len, nullptr, n, h_prefix_partial, h_out, nullptr, 0, num_gpus, tune);
}

int nsx_csum_ragged_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n,
                         const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus) {
    return nsx_csum_ragged_host_tuned(h_base, h_offsets, n, h_prefix_partial, h_out, num_gpus, nullptr);
}

int nsx_csum_ragged_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n,
                               const uint32_t* h_prefix_partial, uint16_t* h_out, int num_gpus,
                               const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!h_out || !h_offsets || !h_base) return NSX_EINVAL;
    if (!nsx::ragged_tune_valid(nsx::launch_cfg(1, tune))) return NSX_EINVAL;
    for (uint64_t i = 0; i < n; ++i)
        if (h_offsets[i + 1] < h_offsets[i]) return NSX_EINVAL;
    return run_sharded(h_base, 0, 0, h_offsets, n, h_prefix_partial, h_out, nullptr, 0, num_gpus, tune);
}

int nsx_rx_ipv4_tcp_verify_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                int num_gpus) {
    return nsx_rx_ipv4_tcp_verify_host_tuned(h_base, h_offsets, n, h_mask, num_gpus, nullptr);
}

static int rx_host(int ipver, const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                   int num_gpus, const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!h_mask || !h_offsets || !h_base) return NSX_EINVAL;
    if (!nsx::rx_tune_valid(nsx::launch_cfg(1, tune))) return NSX_EINVAL;
    for (uint64_t i = 0; i < n; ++i)
        if (h_offsets[i + 1] < h_offsets[i]) return NSX_EINVAL;
    return run_sharded(h_base, 0, 0, h_offsets, n, nullptr, nullptr, h_mask, ipver, num_gpus, tune);
}

int nsx_rx_ipv4_tcp_verify_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                      int num_gpus, const nsx_tune* tune) {
    return rx_host(4, h_base, h_offsets, n, h_mask, num_gpus, tune);
}

int nsx_rx_ipv6_tcp_verify_host(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                int num_gpus) {
    return rx_host(6, h_base, h_offsets, n, h_mask, num_gpus, nullptr);
}

int nsx_rx_ipv6_tcp_verify_host_tuned(const uint8_t* h_base, const uint64_t* h_offsets, uint64_t n, uint64_t* h_mask,
                                      int num_gpus, const nsx_tune* tune) {
    return rx_host(6, h_base, h_offsets, n, h_mask, num_gpus, tune);
}

int nsx_tcp_build_host(const nsx_tcp_hdr_soa* h_hdr, const uint8_t* h_opts, const uint64_t* h_opt_off,
                       const uint8_t* h_data, const uint64_t* h_data_off, const uint32_t* h_prefix_partial, uint64_t n,
                       uint8_t* h_out, const uint64_t* h_out_off, uint16_t* h_raw, int num_gpus) {
    return nsx_tcp_build_host_tuned(h_hdr, h_opts, h_opt_off, h_data, h_data_off, h_prefix_partial, n, h_out,
                                    h_out_off, h_raw, num_gpus, nullptr);
}

int nsx_tcp_build_host_tuned(const nsx_tcp_hdr_soa* h_hdr, const uint8_t* h_opts, const uint64_t* h_opt_off,
                             const uint8_t* h_data, const uint64_t* h_data_off, const uint32_t* h_prefix_partial,
                             uint64_t n, uint8_t* h_out, const uint64_t* h_out_off, uint16_t* h_raw, int num_gpus,
                             const nsx_tune* tune) {
    if (n == 0) return NSX_OK;
    if (!h_hdr || !h_hdr->src_port || !h_hdr->dst_port || !h_hdr->seq_num || !h_hdr->ack_num || !h_hdr->control ||
        !h_hdr->window || !h_hdr->urgent_ptr || !h_data_off || !h_out || !h_out_off || (h_opt_off && !h_opts))
        return NSX_EINVAL;
    // every span the chunks copy must be well-formed: non-decreasing offsets, 4-aligned image slots that hold
    // their image and its zero padding (nsx_tcp_build_dev's layout rule), images shorter than 2^31 bytes
    if (h_data_off[n] > h_data_off[0] && !h_data) return NSX_EINVAL;
    bool gaps = false;
    for (uint64_t i = 0; i < n; ++i) {
        if (h_data_off[i + 1] < h_data_off[i] || (h_opt_off && h_opt_off[i + 1] < h_opt_off[i]) ||
            h_out_off[i + 1] < h_out_off[i] || (h_out_off[i] & 3))
            return NSX_EINVAL;
        const uint64_t ol = h_opt_off ? h_opt_off[i + 1] - h_opt_off[i] : 0;
        const uint64_t slot = (nsx_tcp_wire_len(ol, h_data_off[i + 1] - h_data_off[i]) + 3) & ~3ull;
        if (slot >= (1ull << 31) || h_out_off[i + 1] - h_out_off[i] < slot) return NSX_EINVAL;
        gaps |= h_out_off[i + 1] - h_out_off[i] > slot;
    }
    const BuildJob proto{h_hdr, h_opts, h_opt_off, h_data, h_data_off, h_prefix_partial, h_out, h_out_off, h_raw,
                         gaps,  0,      0,         0,      0,          tune,             NSX_OK};
    return run_build_sharded(proto, n, num_gpus, tune);
}

int nsx_host_cache_release(void) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    int dev0 = 0;
    const bool restore = hipGetDevice(&dev0) == hipSuccess;
    for (int d = 0; d < kMaxDevices; ++d) {
        for (int s = 0; s < kMaxSlots; ++s) {
            if (!g_ctx[d][s]) continue;
            std::lock_guard<std::mutex> hold(g_ctx[d][s]->mu);
            if (hipSetDevice(d) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            g_ctx[d][s]->release();  // streams stay: they are cheap and reused
        }
    }
    if (restore) (void)hipSetDevice(dev0);
    return NSX_OK;
}

}  // extern "C"
