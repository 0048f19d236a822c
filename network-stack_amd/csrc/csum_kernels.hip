// csum_kernels.hip — gfx950 (CDNA4) kernels for the RFC 1071 Internet checksum.
//
// Replaces the hot loop of transport/tcp/tcp.go:72-95 (computeChecksum) for
// batches of segments resident in HBM. The arithmetic identity used, checked
// against the serial Go loop by the oracle tests (tests/test_oracle.py):
//
//   Go: 16-bit BIG-endian words of prefix‖segment (odd tail zero-padded), added
//       with end-around carry (tcp.go:79-92).
//   Here: every 4-byte-aligned LITTLE-endian dword of the segment's memory
//       window (bytes outside the segment masked to 0) contributes its two LE
//       16-bit halves (v_sad_u16 x,0,acc = acc + lo16 + hi16); the wave total is
//       folded to 16 bits (2^16 ≡ 1 mod 0xFFFF), then byte-swapped to the BE
//       domain iff the segment starts at an EVEN address (a byte at an even
//       address is the low half of its LE word but must weigh as the high half
//       of a BE word when the segment itself starts even; 256·256 ≡ 1).
//       Zero-padding an odd tail is the masking itself. fold() never turns a
//       nonzero sum into 0, so 0x0000 ↔ all-zero input and 0xFFFF for a nonzero
//       multiple of 0xFFFF, exactly as the serial loop.
//
// Work decomposition (HBM-bound streaming reduction, no MFMA, no LDS needed on
// the fast path): one wave64 owns a segment; a "row" is one wave-wide 16-B/lane
// load = 1 KiB of the segment window, fully coalesced. Persistent grid of
// 256-thread blocks; tasks are dealt to the 8 XCDs in interleaved chunks, each
// XCD walking its chunks in order (their 2-byte result stores then fill whole
// lines in one XCD's L2 instead of being split across XCDs; see chunk_deal).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "csum_kernels.h"

namespace nsx {
namespace {

constexpr uint32_t kWave = 64;
constexpr uint32_t kRow = 1024;        // bytes per wave-wide 16 B/lane load
constexpr uint32_t kBlock = 256;       // 4 waves
constexpr uint32_t kWavesPerBlock = kBlock / kWave;

// 16 bytes at a 4-byte-aligned address: hipcc emits one global_load_dwordx4
// (gfx950 serves dword-aligned multi-dword global loads in hardware).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}

// 16-byte LDS chunks with their natural alignment (u32x4 is only 4-aligned, which splits LDS accesses into
// ds_read2_b32 / ds_write2_b32; a slot chunk is always 16-aligned, so ds_read_b128 / ds_write_b128)
typedef uint32_t lds16 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 lds_get(const lds16* slot, uint32_t c) {
    const lds16 v = slot[c];
    return u32x4{v.x, v.y, v.z, v.w};
}

// Only at the very end of the readable span: load the whole dwords below
// safe_end (a 4-aligned dword holding a readable byte never crosses a page).
__device__ __forceinline__ u32x4 ld16_guarded(const uint8_t* p, const uint8_t* safe_end) {
    u32x4 v = {0u, 0u, 0u, 0u};
    const uint32_t* d = reinterpret_cast<const uint32_t*>(p);
    if (p + 4 <= safe_end) v.x = d[0];
    if (p + 8 <= safe_end) v.y = d[1];
    if (p + 12 <= safe_end) v.z = d[2];
    if (p + 16 <= safe_end) v.w = d[3];
    return v;
}

// Low `b` bytes of a dword set (b clamped to [0,4]).
__device__ __forceinline__ uint32_t low_bytes(int64_t b) {
    int s = b <= 0 ? 0 : (b >= 4 ? 32 : (int)b * 8);
    return s == 0 ? 0u : (0xFFFFFFFFu >> (32 - s));
}

// Keep only the bytes of the 16-B chunk at window offset q that fall in [lo, hi).
__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int64_t q, int64_t lo, int64_t hi) {
    v.x &= low_bytes(hi - q) & ~low_bytes(lo - q);
    v.y &= low_bytes(hi - q - 4) & ~low_bytes(lo - q - 4);
    v.z &= low_bytes(hi - q - 8) & ~low_bytes(lo - q - 8);
    v.w &= low_bytes(hi - q - 12) & ~low_bytes(lo - q - 12);
    return v;
}

__device__ __forceinline__ const uint8_t* align_up4(const uint8_t* p) {
    return reinterpret_cast<const uint8_t*>(((uintptr_t)p + 3) & ~(uintptr_t)3);
}

__device__ __forceinline__ uint32_t sad4(u32x4 v, uint32_t acc) {
    acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.w, 0u, acc);
    return acc;
}

__device__ __forceinline__ uint32_t fold32(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

// Wave-wide sum of a per-lane value < 2^26: DPP row_ror inside each 16-lane
// row (4 fused v_add_u32_dpp), then the 4 row totals via v_readlane into SGPRs.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xF, 0xF, false);  // row_ror:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xF, 0xF, false);  // row_ror:1
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
           __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

// Wave-wide maximum (DPP row_ror inside each row, then the 4 row maxima via v_readlane): a scalar.
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false));  // row_ror:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x122, 0xF, 0xF, false));  // row_ror:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x121, 0xF, 0xF, false));  // row_ror:1
    return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// Wave total of LE half-sums → raw BE one's-complement sum, plus the prefix partial.
__device__ __forceinline__ uint32_t finish(uint32_t le_total, bool start_even, uint32_t partial) {
    uint32_t s = fold32(le_total);
    if (start_even) s = ((s & 0xFFu) << 8) | (s >> 8);
    return fold32(s + fold32(partial));
}

// Task range of this block under the XCD-contiguous deal (or plain grid-stride).
struct TaskIter {
    uint64_t next, end, step;
};

// XCD-interleaved deal: the batch is cut into chunks of 2^clog tasks and XCD x takes chunks x, x+8,
// x+16, ...; its waves walk their chunks' tasks in order. i = the wave's local sequence index (start
// slot*4 + wave, step per*4). Set up by chunk_deal below; chunk sizes by deal_clog (launchers).
struct ChunkDeal {
    uint32_t x, clog;  // clog = 0: off (task = i)
    __device__ __forceinline__ uint32_t task(uint32_t i) const {
        return clog ? ((((i >> clog) << 3) + x) << clog) | (i & ((1u << clog) - 1u)) : i;
    }
};

// Each XCD's blocks stream one contiguous eighth of the batch, dealt round-robin inside it (kernels that
// take a chunk size then switch to the interleaved chunks with chunk_deal); grids that are not a multiple
// of the 8 XCDs fall back to a plain grid-stride deal.
__device__ __forceinline__ TaskIter task_iter(uint64_t ntasks, uint32_t wave) {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    TaskIter it;
    if (nb >= 16 && (nb & 7) == 0) {
        // blocks b, b+8, ... share an XCD (observed round-robin dispatch; speed only).
        const uint32_t x = b & 7, slot = b >> 3, per = nb >> 3;
        const uint64_t lo = ntasks * x / 8, hi = ntasks * (x + 1) / 8;
        it.next = lo + (uint64_t)slot * kWavesPerBlock + wave;
        it.end = hi;
        it.step = (uint64_t)per * kWavesPerBlock;
    } else {
        it.next = (uint64_t)b * kWavesPerBlock + wave;
        it.end = ntasks;
        it.step = (uint64_t)nb * kWavesPerBlock;
    }
    return it;
}

// Switch a wave's task_iter iteration to the XCD-interleaved chunk deal when clog > 0 and the grid
// allows it; the wave then walks i = it.next, it.next + it.step, ... < it.end with task cd.task(i),
// stopping at the first task ≥ ntasks (task(i) increases with i). With clog = 0 nothing changes
// (task(i) = i < it.end ≤ ntasks).
__device__ __forceinline__ ChunkDeal chunk_deal(TaskIter& it, uint32_t wave, uint32_t clog, uint64_t ntasks) {
    ChunkDeal cd{0u, 0u};
    if (clog && gridDim.x >= 16 && (gridDim.x & 7) == 0 && ntasks < (1ull << 31)) {
        cd.x = blockIdx.x & 7;
        cd.clog = clog;
        it.next = (blockIdx.x >> 3) * kWavesPerBlock + wave;
        it.step = (gridDim.x >> 3) * kWavesPerBlock;
        it.end = 0xFFFFFFFFu;
    }
    return cd;
}

// ---------------------------------------------------------------------------
// Software-pipelined fixed-stride kernel on buffer loads. Same work split as
// csum_fixed_kernel (U segments × NROWS rows per wave task), but task t+1's
// loads are issued before task t is reduced, so every wave keeps a task's worth
// of loads in flight while it computes. All memory operations are
// unconditional buffer ops: a lane that must not load gets an out-of-range
// offset (the hardware returns 0 and moves no data), so hipcc can count
// vmcnt exactly across the two register buffers instead of draining to 0.
// Range checking on gfx950 is per dword (tools/probes/buffer_oob.hip): with
// num_records ending at the 4-aligned end of the batch, a 16-byte load that
// straddles the end returns exactly its in-range dwords, so no tail path.
// ---------------------------------------------------------------------------
// Mask for the chunk of lane byte offset ql inside a row whose segment bytes are
// [lo_r, hi_r) relative to the row start (both clamped, 32-bit).
__device__ __forceinline__ uint32_t keep_mask(int32_t lo_r, int32_t hi_r, int32_t d) {
    const int32_t e = min(max(hi_r - d, 0), 4), s = min(max(lo_r - d, 0), 4);
    const uint32_t me = e >= 4 ? 0xFFFFFFFFu : ((1u << (8 * e)) - 1u);
    const uint32_t ms = s >= 4 ? 0xFFFFFFFFu : ((1u << (8 * s)) - 1u);
    return me & ~ms;
}

constexpr uint32_t kOOB = 0x80000000u;  // voffset that is always out of range (num_records < 2^31)
// s_waitcnt operand (gfx9 encoding): vmcnt(0), expcnt and lgkmcnt left at their maxima (no wait)
constexpr int kWaitVm0 = 0x0F70;
// Cache-policy operand of a buffer store on gfx950: sc1 (bit 4) = write-through, the line leaves the XCD's L2.
constexpr int kStoreSc1 = 16;

// Wave w of this block's wpb in a grid of nb blocks, numbered XCD by XCD (blocks b, b + 8, ... run on one XCD).
__device__ __forceinline__ uint32_t wave_number(uint32_t nb, uint32_t wpb, uint32_t w) {
    const uint32_t b = blockIdx.x;
    return (nb >= 16 && (nb & 7) == 0) ? ((b & 7) * (nb >> 3) + (b >> 3)) * wpb + w : b * wpb + w;
}

// Per-wave timing stamps, the one diagnostic hook in the product kernels (the fixed-stride, receive-pass and
// packed-header kernels): entry(), ready() once the wave's range is known, done(wave number, work) at its end. The product build's
// WaveStamps records nothing and every call compiles away (the code object is byte-identical to one without the
// calls). `make stamps` builds lib_stamps/ with the recording policy of tools/probes/wave_stamps.h instead, read back
// by tools/probes/rx_wave_times.py and f3_wave_times.py.
#ifdef NSX_WAVE_STAMPS
#include "../../tools/probes/wave_stamps.h"
#else
struct WaveStamps {
    __device__ __forceinline__ void entry() {}
    __device__ __forceinline__ void ready() {}
    __device__ __forceinline__ void done(uint32_t g, uint64_t work, uint32_t lane) {}
};
#endif

// The deal's shape: the pool is a batch's last 1/2^kDealPoolShift, dealt from kDealHeads counters, each on its own
// 64 B line (kDealStride dwords); kDealSlots streams per device hold a set of heads at once (deal_heads).
#ifndef NSX_DEAL_POOL_SHIFT
#define NSX_DEAL_POOL_SHIFT 3
#endif
constexpr uint32_t kDealPoolShift = NSX_DEAL_POOL_SHIFT;
#ifndef NSX_DEAL_HEADS
#define NSX_DEAL_HEADS 32
#endif
constexpr uint32_t kDealHeads = NSX_DEAL_HEADS;
constexpr uint32_t kDealStride = 16;
constexpr uint32_t kDealSlots = 64;

// ---- Work dealt through a block's LDS ring (round 6) ----
// A batch's last units are dealt to the waves as they finish, without any streaming wave waiting on a ticket's round
// trip: one dealer wave per block pulls tickets (device-scope atomics on the stream's heads, 1-3 µs each) for the
// entries its block's streaming waves have claimed and posts them in an LDS ring; a streaming wave claims entries
// ahead (an LDS atomic) and reads them from LDS when it gets there. vmcnt retires in issue order, so a ticket pulled
// by a streaming wave itself would hold up every load issued after it (§7 step 72). The receive pass's streamed
// modes (rx_runs_ring) and the fixed-stride kernel (csum_fixed_swp_kernel<·, ·, true>) use it.
constexpr uint32_t kPieceRing = 64;        // ring entries per block
constexpr uint32_t kPieceFree = ~0u;       // an entry read by its consumer (or never written)

struct PieceRing {
    uint32_t claim;     // entries claimed by the streaming waves (LDS atomic add)
    uint32_t produced;  // entries the dealer has written, in order
    uint32_t end_at;    // the dealer's final entry count once its head's share ran out (~0 until then)
    uint32_t pad;
    uint32_t e[kPieceRing];  // entry p at e[p % kPieceRing]: a piece's first frame; kPieceFree once read
};

// A streaming wave's side of the block's ring: claim an entry (an LDS atomic), read a claimed entry (waiting for the
// dealer only if it has not posted it yet; `end` past the share) and free its slot for the dealer.
struct RingClient {
    PieceRing* rg;
    uint32_t lane;
    __device__ __forceinline__ uint32_t claim() const {
        uint32_t v = 0u;
        if (lane == 0u) v = __hip_atomic_fetch_add(&rg->claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_amdgcn_readfirstlane(v);
    }
    __device__ __forceinline__ uint32_t read(uint32_t idx, uint32_t end) const {  // entry idx's value, or end
        for (;;) {
            const uint32_t p = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&rg->produced, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (idx < p) {
                uint32_t* slot = &rg->e[idx % kPieceRing];
                const uint32_t v = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (lane == 0u) __hip_atomic_store(slot, kPieceFree, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return v;
            }
            const uint32_t e = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&rg->end_at, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (idx >= e) return end;
            __builtin_amdgcn_s_sleep(1);
        }
    }
};

// The dealer wave of a block: for every entry its streaming waves claim, a ticket t from the block's head (at most
// 4 pulls in flight), posted to the ring as the piece's first unit pb + t·unit; past the head's share it posts the end. The head's dword 0 is the ticket
// counter (shared with DealtRuns, which leaves it at 0), dword 1 counts the head's dealers that have finished: the
// last one to finish resets both to 0 for the stream's next launch (a dealer may pull up to 4 tickets past the
// share, so the pull count cannot mark the last pull as in DealtRuns).
__device__ __forceinline__ void ring_dealer(PieceRing* rg, uint32_t* head, uint32_t pb, uint32_t unit, uint32_t qh,
                                            uint32_t dealers, uint32_t ahead, uint32_t lane) {
    uint32_t p = 0u;
    bool live = true;
    while (live) {
        // entries to post: every claimed one, plus `ahead` more, up to 16 per round trip
        const uint32_t c = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&rg->claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        const uint32_t k = min(c + ahead - p, 16u);
        if (k == 0u || (int32_t)(c + ahead - p) <= 0) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        // k tickets in one pull: base .. base + k − 1, of which those below qh are the head's share
        uint32_t t = 0u;
        if (lane == 0u) t = __hip_atomic_fetch_add(head, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t base = __builtin_amdgcn_readfirstlane(t);
        const uint32_t v = base < qh ? min(k, qh - base) : 0u;
        // lane j < v posts entry p + j; its slot's previous entry must have been read (rarely waits)
        uint32_t* slot = &rg->e[(p + lane) % kPieceRing];
        while (__builtin_amdgcn_ballot_w64(lane < v && __hip_atomic_load(slot, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP) != kPieceFree))
            __builtin_amdgcn_s_sleep(1);
        if (lane < v) __hip_atomic_store(slot, pb + (base + lane) * unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        p += v;
        live = v == k;
        if (lane == 0u) __hip_atomic_store(&rg->produced, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (lane == 0u) {
        __hip_atomic_store(&rg->end_at, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t done = __hip_atomic_fetch_add(head + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done + 1u == dealers) {
            __hip_atomic_store(head, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(head + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint64_t bytes) {
    // Wave-uniform inputs only, so no waterfall loop (guide T20); clamp without a
    // 64-bit unsigned compare (SALU has none: hipcc would borrow VGPRs for it).
    const uint32_t nr = (bytes >> 31) ? kOOB - 1 : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)nr, 0x00020000);
}

template <bool NT>
__device__ __forceinline__ u32x4 bld16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, NT ? 2 : 0);
    return u32x4{x.x, x.y, x.z, x.w};
}

// Byte mask keeping the low `keep` bytes of a dword (keep in 1..3).
__device__ __forceinline__ uint32_t low_keep(uint32_t keep) { return (1u << (8 * keep)) - 1u; }

// Segment window descriptor: base = the segment start rounded down to 4 B,
// num_records = head + len rounded UP to 4 B. The per-dword range check then
// returns 0 for every dword outside the segment's window (and moves no data
// for them), so only the partial first dword (head bytes of the previous
// segment) and the partial last dword (bytes past the end) need a byte mask.
struct SegWin {
    __amdgpu_buffer_rsrc_t r;
    uint32_t head;  // 0..3 bytes before the segment in its first dword
    uint32_t end;   // head + len: window bytes that belong to the segment
    bool even;      // segment starts at an even address (byte-swap rule)
};

__device__ __forceinline__ SegWin seg_win(const uint8_t* p, uint32_t len, bool live) {
    SegWin w;
    w.head = (uint32_t)((uintptr_t)p & 3u);
    w.end = w.head + len;
    w.even = ((uintptr_t)p & 1u) == 0;
    w.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p - w.head), 0,
                                            live ? (int)((w.end + 3u) & ~3u) : 0, 0x00020000);
    return w;
}

// Apply the two partial-dword masks to row k's chunk of this lane.
__device__ __forceinline__ u32x4 edge_mask(u32x4 x, const SegWin& w, uint32_t k, uint32_t lane) {
    if (w.head && k == 0 && lane == 0) x.x &= ~low_keep(w.head);
    const uint32_t keep = w.end & 3u;
    if (keep) {
        const uint32_t ld = (w.end - 1u) >> 2;  // dword holding the last byte
        if ((ld >> 8) == k && ((ld & 255u) >> 2) == lane) {
            const uint32_t m = low_keep(keep), c = ld & 3u;
            x.x &= c == 0 ? m : 0xFFFFFFFFu;
            x.y &= c == 1 ? m : 0xFFFFFFFFu;
            x.z &= c == 2 ? m : 0xFFFFFFFFu;
            x.w &= c == 3 ? m : 0xFFFFFFFFu;
        }
    }
    return x;
}

template <int U>
__device__ __forceinline__ void fixed_flush(uint32_t res, uint32_t first, uint32_t step, uint32_t count, uint32_t n,
                                            __amdgpu_buffer_rsrc_t ors, uint32_t lane, const ChunkDeal& cd) {
    const uint32_t j = lane / U;
    const uint32_t seg = cd.task(first + j * step) * U + lane % U;
    const uint32_t off = (j < count && seg < n) ? seg * 2 : kOOB;
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)res, ors, off, 0, 0);
}

// Fixed stride on buffer loads, any alignment (batches whose base, stride or length is not a multiple of
// 4; 4-aligned batches take csum_fixed_swp_kernel): a wave task = U consecutive segments × NROWS rows,
// every load unconditional (lanes past a segment's window read 0 and move no data), only the partial
// first and last dword of a segment masked (edge_mask). Results are parked one per lane and flushed with
// a single scattered 2-byte store per 64/U tasks.
template <int U, int NROWS>
__global__ __launch_bounds__(kBlock) void csum_fixed_buf_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t seg_len, uint32_t n,
    const uint32_t* __restrict__ partial, uint16_t* __restrict__ out, uint32_t chunk_log2) {
    constexpr uint32_t G = kWave / U;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t ntasks = (n + U - 1) / U;
    TaskIter it = task_iter(ntasks, wave);
    const ChunkDeal cd = chunk_deal(it, wave, chunk_log2, ntasks);
    const uint32_t end = (uint32_t)it.end, step = (uint32_t)it.step;
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out, (uint64_t)n * 2);
    const __amdgpu_buffer_rsrc_t prs = make_rsrc(partial, partial ? (uint64_t)n * 4 : 0);
    uint32_t res = 0, k = 0, first = (uint32_t)it.next;
    for (uint32_t i = (uint32_t)it.next; i < end; i += step) {
        const uint32_t t = cd.task(i);
        if (t >= ntasks) break;
        const uint32_t s0 = t * U;
        u32x4 v[U][NROWS];
        SegWin w[U];
        const uint8_t* p = base + (uint64_t)s0 * stride;
#pragma unroll
        for (int u = 0; u < U; ++u, p += stride) {
            w[u] = seg_win(p, seg_len, s0 + u < n);
#pragma unroll
            for (int r = 0; r < NROWS; ++r) v[u][r] = bld16<true>(w[u].r, r * kRow + lane * 16);
        }
        const uint32_t part =
            __builtin_amdgcn_raw_buffer_load_b32(prs, lane < (uint32_t)U ? (s0 + lane) * 4 : kOOB, 0, 0);
        // All U*NROWS loads are issued before the first use: LLVM would otherwise
        // sink each (invariant) load next to its consumer and serialise the wave
        // on memory. An in/out operand pins each load above this point.
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < NROWS; ++r) asm volatile("" : "+v"(v[u][r]));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t acc = 0;
#pragma unroll
            for (int r = 0; r < NROWS; ++r) acc = sad4(edge_mask(v[u][r], w[u], r, lane), acc);
            const uint32_t rr = finish(wave_sum(fold32(acc)), w[u].even, __builtin_amdgcn_readlane(part, u));
            res = lane == k * U + u ? rr : res;
        }
        if (++k == G) {
            fixed_flush<U>(res, first, step, k, n, ors, lane, cd);
            k = 0;
            first = i + step;
        }
    }
    if (k) fixed_flush<U>(res, first, step, k, n, ors, lane, cd);
}

// Fixed stride, 4-aligned batches (base, stride and seg_len ≡ 0 mod 4 — config 2's 1500 B): every segment
// starts 4-aligned and even, so there are no edge masks, the descriptor size is a constant, and the finish
// (byte swap + prefix partial) is done vector-wide for a whole group of parked results at flush time (the
// group's partials load when the group starts, so their latency hides under 64/U tasks). Software-
// pipelined: two register sets of one task each (U segments × NROWS rows); the next task's loads are issued
// before the current task is reduced, so a wave keeps its loads in flight through its own reduce/park/flush
// phases instead of leaving them to other waves.
//
// DEAL (round 6): the batch's last 1/2^kDealPoolShift of the tasks are not split statically
// but dealt through the block's LDS ring (ring_dealer) to the four streaming waves as they finish: a fifth wave per
// block pulls the tickets from the stream's heads. With equal static shares the launch waited ~12 µs (5%) for its
// last waves — the XCDs and CUs run at different speeds (tools/probes/f3_wave_times.py --config 2,
// profiles/r06_fixed_wave_times_c2.txt). A dealt task's 8 results are finished with their own partials and stored
// at once (16 B).
#ifndef NSX_FIXED_AHEAD
#define NSX_FIXED_AHEAD 4
#endif
constexpr uint32_t kFixedAhead = NSX_FIXED_AHEAD;  // ring entries the dealer posts beyond the claimed ones
#ifndef NSX_FIXED_POOL_SHIFT
#define NSX_FIXED_POOL_SHIFT 3
#endif
constexpr uint32_t kFixedPoolShift = NSX_FIXED_POOL_SHIFT;  // the dealt pool: the last 1/2^k of the tasks
#ifndef NSX_FIXED_DEAL_MODE
#define NSX_FIXED_DEAL_MODE 0
#endif
constexpr int kFixedDealMode = NSX_FIXED_DEAL_MODE;  // the aligned default shapes' deal: 0 none, 1 dealer wave, 2 in-wave
// DEAL 1: the dealer wave and ring above; DEAL 2: each wave pulls its own tickets from the heads, two tasks ahead
// (two ticket registers alternating with the two register sets, so no ticket is ever copied or selected — reading one
// waits only for its own pull, issued two task-loads earlier; round 6 A/B).
template <int U, int NROWS, int DEAL = 0>
__global__ __launch_bounds__(DEAL == 1 ? kBlock + kWave : kBlock) void csum_fixed_swp_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t seg_len, uint32_t n,
    const uint32_t* __restrict__ partial, uint16_t* __restrict__ out, uint32_t chunk_log2,
    uint32_t* __restrict__ deal) {
    constexpr uint32_t G = kWave / U;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    WaveStamps ws;
    ws.entry();
    uint32_t ntk = 0;  // tasks done (for the stamps)
    const uint32_t all_tasks = (n + U - 1) / U;
    uint32_t ntasks = all_tasks;  // the statically split tasks [0, ntasks)
    [[maybe_unused]] RingClient rc{nullptr, lane};
    [[maybe_unused]] uint32_t claim0 = 0, claim1 = 0;
    // DEAL 2: this wave's head (waves numbered XCD by XCD: every head has waves on all 8 XCDs), its share of the
    // pool, and the two tickets pulled at entry (held through the static part)
    [[maybe_unused]] uint32_t* shead = nullptr;
    [[maybe_unused]] uint32_t spb = 0, sq = 0, swaves = 0, tkx = 0, tky = 0;
    auto spull = [&]() {
        uint32_t t = 0u;
        if (lane == 0u) t = __hip_atomic_fetch_add(shead, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return t;
    };
    if constexpr (DEAL == 2) {
        ntasks = all_tasks - (all_tasks >> kFixedPoolShift);
        const uint32_t W = gridDim.x * kWavesPerBlock, H = min(kDealHeads, W);
        const uint32_t h = wave_number(gridDim.x, kWavesPerBlock, wave) % H;
        const uint32_t Q = all_tasks - ntasks;
        const uint32_t r0 = (uint32_t)((uint64_t)Q * h / H);
        sq = (uint32_t)((uint64_t)Q * (h + 1u) / H) - r0;
        spb = ntasks + r0;
        swaves = (W - h + H - 1u) / H;
        shead = deal + h * kDealStride;
    }
    if constexpr (DEAL == 1) {
        __shared__ PieceRing ring;
        ntasks = all_tasks - (all_tasks >> kFixedPoolShift);
        if (wave == kWavesPerBlock) {
            if (lane < kPieceRing) ring.e[lane] = kPieceFree;
            if (lane == 0u) ring.claim = 0u, ring.produced = 0u, ring.end_at = ~0u;
        }
        __syncthreads();
        if (wave == kWavesPerBlock) {  // the dealer: head h (blocks numbered XCD by XCD), its share of the pool
            const uint32_t nb = gridDim.x, H = min(kDealHeads, nb), h = wave_number(nb, 1u, 0u) % H;
            const uint32_t Q = all_tasks - ntasks;
            const uint32_t r0 = (uint32_t)((uint64_t)Q * h / H), qh = (uint32_t)((uint64_t)Q * (h + 1u) / H) - r0;
            ring_dealer(&ring, deal + h * kDealStride, ntasks + r0, 1u, qh, (nb - h + H - 1u) / H, kFixedAhead, lane);
            return;
        }
        rc.rg = &ring;
        claim0 = rc.claim();  // two pool entries claimed ahead from the start: posted by the time they are needed
        claim1 = rc.claim();
    }
    TaskIter it = task_iter(ntasks, wave);
    const ChunkDeal cd = chunk_deal(it, wave, chunk_log2, ntasks);
    const uint32_t end = (uint32_t)it.end, step = (uint32_t)it.step;
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out, (uint64_t)n * 2);
    const __amdgpu_buffer_rsrc_t prs = make_rsrc(partial, partial ? (uint64_t)n * 4 : 0);
    auto group_seg = [&](uint32_t first) { return cd.task(first + (lane / U) * step) * U + lane % U; };
    struct Set {
        u32x4 v[U][NROWS];
        bool ok;
    };
    auto issue = [&](uint32_t i, Set& S) {
        const uint32_t t = cd.task(i);
        S.ok = i < end && t < ntasks;
        const uint32_t s0 = (S.ok ? t : 0u) * U;
        const uint8_t* p = base + (uint64_t)s0 * stride;
#pragma unroll
        for (int u = 0; u < U; ++u, p += stride) {
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t*>(p), 0, (S.ok && s0 + u < n) ? (int)seg_len : 0, 0x00020000);
#pragma unroll
            for (int rr = 0; rr < NROWS; ++rr) S.v[u][rr] = bld16<true>(r, rr * kRow + lane * 16);
        }
    };
    uint32_t res = 0, k = 0, first = (uint32_t)it.next;
    uint32_t gpart;
    {
        const uint32_t sg = group_seg(first);
        gpart = __builtin_amdgcn_raw_buffer_load_b32(prs, sg < n ? sg * 4 : kOOB, 0, 0);
    }
    auto consume = [&](uint32_t i, Set& S) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int rr = 0; rr < NROWS; ++rr) asm volatile("" : "+v"(S.v[u][rr]));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t acc = 0;
#pragma unroll
            for (int rr = 0; rr < NROWS; ++rr) acc = sad4(S.v[u][rr], acc);
            const uint32_t tot = wave_sum(fold32(acc));
            res = lane == k * U + u ? tot : res;
        }
        ++ntk;
        if (++k == G) {
            res = finish(res, true, gpart);
            fixed_flush<U>(res, first, step, k, n, ors, lane, cd);
            k = 0;
            first = i + step;
            const uint32_t sg = group_seg(first);
            gpart = __builtin_amdgcn_raw_buffer_load_b32(prs, (first < end && sg < n) ? sg * 4 : kOOB, 0, 0);
        }
    };
    Set A, B;
    uint32_t i = (uint32_t)it.next;
    // DEAL 2: the two first tickets are pulled when the static stream has at most two tasks left, so that they are
    // in hand when the pool starts and the waves' pulls spread over their different end times (pulled at entry, the
    // 2048 pulls of a launch queued on 32 counters at once)
    [[maybe_unused]] bool pulled = false;
    auto pull_late = [&](uint32_t inext) {
        if constexpr (DEAL == 2) {
            if (!pulled && !(inext < end && cd.task(inext) < ntasks)) {
                tkx = spull();
                tky = spull();
                pulled = true;
            }
        }
    };
    issue(i, A);
    while (A.ok) {
        const uint32_t i1 = i + step;
        pull_late(i1 + step);
        issue(i1, B);
        consume(i, A);
        if (!B.ok) break;
        i = i1 + step;
        pull_late(i + step);
        issue(i, A);
        consume(i1, B);
    }
    if constexpr (DEAL == 2) {
        if (!pulled) tkx = spull(), tky = spull();
    }
    if (k) {
        res = finish(res, true, gpart);
        fixed_flush<U>(res, first, step, k, n, ors, lane, cd);
    }
    if constexpr (DEAL != 0) {
        // The pool: tasks read from the ring (each claimed two tasks ahead), software-pipelined like the static
        // loop; a task's partials load with its rows, its results are finished and stored when it is summed.
        struct PSet {
            u32x4 v[U][NROWS];
            uint32_t t, part;
        };
        auto take = [&]() {
            const uint32_t t = rc.read(claim0, all_tasks);
            claim0 = claim1;
            if (t < all_tasks) claim1 = rc.claim();
            return t;
        };
        auto pissue = [&](uint32_t t, PSet& S) {
            S.t = t;
            const bool ok = t < all_tasks;
            const uint32_t s0 = (ok ? t : 0u) * U;
            const uint8_t* p = base + (uint64_t)s0 * stride;
#pragma unroll
            for (int u = 0; u < U; ++u, p += stride) {
                const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint8_t*>(p), 0, (ok && s0 + u < n) ? (int)seg_len : 0, 0x00020000);
#pragma unroll
                for (int rr = 0; rr < NROWS; ++rr) S.v[u][rr] = bld16<true>(r, rr * kRow + lane * 16);
            }
            S.part = __builtin_amdgcn_raw_buffer_load_b32(prs, ok && lane < (uint32_t)U && s0 + lane < n ? (s0 + lane) * 4
                                                                                                          : kOOB, 0, 0);
        };
        auto pconsume = [&](PSet& S) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int rr = 0; rr < NROWS; ++rr) asm volatile("" : "+v"(S.v[u][rr]));
            uint32_t r = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t acc = 0;
#pragma unroll
                for (int rr = 0; rr < NROWS; ++rr) acc = sad4(S.v[u][rr], acc);
                const uint32_t tot = wave_sum(fold32(acc));
                r = lane == (uint32_t)u ? tot : r;
            }
            r = finish(r, true, S.part);
            const uint32_t seg = S.t * U + lane;
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)r, ors, lane < (uint32_t)U && seg < n ? seg * 2 : kOOB, 0, 0);
            ++ntk;
        };
        PSet P0, P1;
        if constexpr (DEAL == 1) {
            pissue(take(), P0);
            while (P0.t < all_tasks) {
                pissue(take(), P1);
                pconsume(P0);
                if (P1.t >= all_tasks) break;
                pissue(take(), P0);
                pconsume(P1);
            }
        } else {
            // ticket register X feeds set P0, Y feeds P1; each is read two task-loads after its pull and refilled at
            // once while the share lasts. A wave stops at the first ticket past the share and then reads its other
            // outstanding pull too (a ticket is never dropped, whatever order the pulls executed in); the last wave of
            // the head to finish resets it (dword 0) and the finished count (dword 1) for the stream's next launch.
            auto tk_task = [&](uint32_t v) { return v < sq ? spb + v : all_tasks; };
            P1.t = all_tasks;
            uint32_t tx = tk_task(__builtin_amdgcn_readfirstlane(tkx));
            if (tx < all_tasks) tkx = spull();
            pissue(tx, P0);
            bool ymore = true;  // Y holds an unread pull
            while (P0.t < all_tasks) {
                const uint32_t ty = tk_task(__builtin_amdgcn_readfirstlane(tky));
                ymore = false;
                if (ty < all_tasks) tky = spull(), ymore = true;
                pissue(ty, P1);
                pconsume(P0);
                if (P1.t >= all_tasks) break;
                tx = tk_task(__builtin_amdgcn_readfirstlane(tkx));
                if (tx < all_tasks) tkx = spull();
                pissue(tx, P0);
                pconsume(P1);
            }
            // drain: P0 or P1 ended the loop with the end marker; the other ticket register may hold an unread pull
            // (X if the loop ended on P1, else Y) — a valid one is a task to do
            uint32_t last = all_tasks;
            if (P1.t >= all_tasks && P0.t < all_tasks) {  // ended on P1: X was refilled when P0 was issued
                last = tk_task(__builtin_amdgcn_readfirstlane(tkx));
            } else if (ymore) {
                last = tk_task(__builtin_amdgcn_readfirstlane(tky));
            }
            if (last < all_tasks) {  // rare: a pull executed out of order and returned inside the share; every pull
                pissue(last, P0);    // after the one already seen past it returns past it too (one counter)
                pconsume(P0);
            }
            if (lane == 0u) {
                const uint32_t done = __hip_atomic_fetch_add(shead + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (done + 1u == swaves) {
                    __hip_atomic_store(shead, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(shead + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    ws.done(blockIdx.x * kWavesPerBlock + wave, ntk, lane);
}

// ---------------------------------------------------------------------------
// One segment per wave, runtime row count, rows issued R at a time: fixed
// batches with long segments (> 4 KiB).
// ---------------------------------------------------------------------------
struct SegRef {
    const uint8_t* p;
    uint64_t len;
};

template <int R>
__device__ __forceinline__ uint32_t seg_lane_sum(const uint8_t* p, uint64_t len, uint32_t lane,
                                                 const uint8_t* safe_end, uint64_t row_first,
                                                 uint64_t row_step) {
    const uint32_t head = (uint32_t)((uintptr_t)p & 3u);
    const uint8_t* wb = p - head;
    const int64_t lo = head, hi = (int64_t)head + (int64_t)len;
    const uint64_t rows = (uint64_t)(hi + kRow - 1) / kRow;
    uint32_t acc = 0;
    for (uint64_t r0 = row_first; r0 < rows; r0 += R * row_step) {
        u32x4 v[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            v[j] = u32x4{0u, 0u, 0u, 0u};
            const uint64_t r = r0 + j * row_step;
            const int64_t q = (int64_t)(r * kRow) + lane * 16;
            if (q < hi) {
                const uint8_t* a = wb + q;
                if (wb + (r + 1) * kRow <= safe_end || a + 16 <= safe_end) v[j] = ld16<true>(a);
                else v[j] = ld16_guarded(a, safe_end);
            }
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int64_t rb = (int64_t)((r0 + j * row_step) * kRow);
            u32x4 x = v[j];
            if (rb < lo || rb + kRow > hi) x = mask_chunk(x, rb + lane * 16, lo, hi);
            acc = sad4(x, acc);
        }
        acc = fold32(acc);  // keeps acc < 2^17 for any segment length
    }
    return acc;
}

template <bool RAGGED>
__device__ __forceinline__ SegRef seg_ref(const uint8_t* base, const uint64_t* offsets, uint64_t stride,
                                          uint32_t seg_len, uint64_t i) {
    if constexpr (RAGGED) {
        const uint64_t o0 = offsets[i], o1 = offsets[i + 1];
        return SegRef{base + o0, o1 > o0 ? o1 - o0 : 0};
    } else {
        return SegRef{base + i * stride, seg_len};
    }
}

template <int R>
__global__ __launch_bounds__(kBlock) void csum_wave_kernel(const uint8_t* __restrict__ base, uint64_t stride,
                                                           uint32_t seg_len, uint64_t n,
                                                           const uint32_t* __restrict__ partial,
                                                           uint16_t* __restrict__ out, const uint8_t* safe_end,
                                                           uint32_t clog) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    TaskIter it = task_iter(n, wave);
    const ChunkDeal cd = chunk_deal(it, wave, clog, n);
    for (uint64_t k = it.next; k < it.end; k += it.step) {
        const uint64_t i = cd.clog ? cd.task((uint32_t)k) : k;
        if (i >= n) break;
        const SegRef s = seg_ref<false>(base, nullptr, stride, seg_len, i);
        const uint32_t tot = wave_sum(seg_lane_sum<R>(s.p, s.len, lane, safe_end, 0, 1));
        if (lane == 0) out[i] = (uint16_t)finish(tot, ((uintptr_t)s.p & 1u) == 0, partial ? partial[i] : 0u);
    }
}

// ---------------------------------------------------------------------------
// One segment per 256-thread block (few, very long segments): wave w takes rows
// w, w+4, ... so the block reads 4 KiB contiguous per step; cross-wave total
// through LDS.
// ---------------------------------------------------------------------------
template <bool RAGGED, int R, bool VERIFY>
__global__ __launch_bounds__(kBlock) void csum_block_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, uint64_t stride,
    uint32_t seg_len, uint64_t n, const uint32_t* __restrict__ partial, uint16_t* __restrict__ out,
    uint8_t* __restrict__ ok, const uint8_t* safe_end) {
    __shared__ uint32_t part[kWavesPerBlock];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if constexpr (RAGGED) safe_end = align_up4(base + offsets[n]);
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const SegRef s = seg_ref<RAGGED>(base, offsets, stride, seg_len, i);
        const uint32_t w = wave_sum(seg_lane_sum<R>(s.p, s.len, lane, safe_end, wave, kWavesPerBlock));
        if (lane == 0) part[wave] = fold32(w);
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = part[0] + part[1] + part[2] + part[3];
            const uint32_t res = finish(tot, ((uintptr_t)s.p & 1u) == 0, partial ? partial[i] : 0u);
            if (out) out[i] = (uint16_t)res;
            if constexpr (VERIFY) ok[i] = res == 0xFFFFu;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t k) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, k);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), k);
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------
// Ragged prefix-scan kernel (the default ragged kernel).
//
// With byte weights w(a) = 1 at even and 256 at odd addresses, let
// S(x) = Σ_{a<x} b_a·w(a). For a segment [s, e) the raw checksum is
// fold(S(e) − S(s)), byte-swapped iff s is even (the rule of finish()); the
// difference is an exact integer, 0 iff every byte is 0. So a densely packed
// run of segments is one contiguous byte range, and its checksums are the
// differences of S sampled at the segment boundaries.
//
// A wave owns a run of up to kScanRun consecutive segments (run+1 boundaries,
// one per lane). It streams the run's bytes as 1 KiB rows
// through one buffer descriptor (full rows aligned to 128-byte lines, no
// per-segment windows, R rows in flight), and per row does: lane half-sums (v_sad_u16), an inclusive wave
// scan (DPP), and — only in rows that hold a boundary — each boundary lane
// fetches the chunk and exclusive prefix of the lane its boundary falls in
// (ds_bpermute) and adds the partial chunk below the boundary. Work per byte
// no longer depends on how many segments the bytes are cut into.
// ---------------------------------------------------------------------------
constexpr uint32_t kScanRun = 63;

// Keep bytes [lo, hi) (0 ≤ lo ≤ hi ≤ 16) of a 16-byte chunk.
__device__ __forceinline__ u32x4 keep_bytes(u32x4 x, int32_t lo, int32_t hi) {
    x.x &= keep_mask(lo, hi, 0);
    x.y &= keep_mask(lo, hi, 4);
    x.z &= keep_mask(lo, hi, 8);
    x.w &= keep_mask(lo, hi, 12);
    return x;
}

// Inclusive prefix sum over the 64 lanes (DPP row shifts, then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4), (int)v);
}

__device__ __forceinline__ uint64_t ld_off(__amdgpu_buffer_rsrc_t ofs, uint32_t i) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, i * 8, 0, 0);
    return ((uint64_t)x.y << 32) | x.x;
}

// Two lower bounds over offsets[0..n] at once (first i with offsets[i] >= t[k]; n if
// none), 64-ary: every round each lane probes one index per search, both loads in
// flight together, and a ballot keeps the sub-range that holds the answer
// (n = 1M: 1M → 16K → 256 → 4 → exact, four dependent rounds).
__device__ __forceinline__ void seg_lower_bound2(__amdgpu_buffer_rsrc_t ofs, uint32_t n, uint64_t t0, uint64_t t1,
                                                 uint32_t lane, uint32_t s[2]) {
    uint32_t lo[2] = {0u, 0u}, hi[2] = {n, n};
    const uint64_t t[2] = {t0, t1};
    while (hi[0] - lo[0] > kWave || hi[1] - lo[1] > kWave) {
        uint32_t step[2], idx[2];
        uint64_t v[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            step[k] = (hi[k] - lo[k] + kWave - 1) / kWave;
            idx[k] = min(lo[k] + lane * step[k], hi[k]);
            v[k] = ld_off(ofs, idx[k]);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            // probes lo + j·step (j = 0..63) are monotone: c of them lie below t
            const uint32_t c = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(v[k] < t[k]));
            const uint32_t l = c ? lo[k] + (c - 1) * step[k] + 1 : lo[k];
            hi[k] = min(lo[k] + c * step[k], hi[k]);
            lo[k] = min(l, hi[k]);
        }
    }
    uint64_t v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) v[k] = lo[k] + lane < hi[k] ? ld_off(ofs, lo[k] + lane) : ~0ull;
#pragma unroll
    for (int k = 0; k < 2; ++k)
        s[k] = lo[k] + (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(v[k] < t[k]));
}

// The units [a0, a_end) of wave g of W (a0, a_end multiples of `align`, except a_end = n for the last wave), and the
// wave's bytes. Byte-balanced — wave g owns the units that start in the g-th of W equal byte slices, found by two
// interleaved 64-ary searches over the offsets — unless the batch's mean unit is under small_mean bytes: then equal
// unit counts, no search (§7 step 51). On batches of small frames the search's third round touches ~8 KB of
// offsets lines per wave that are evicted again before the wave's runs read them (5-7% of the batch's bytes,
// FETCH_SIZE), and its four dependent round trips hold every wave at the start; small units of similar size
// balance well by count.
struct WaveRange {
    uint32_t a0, a_end;
    uint64_t bytes;
};
// count_align (nonzero): the alignment of equal-count ranges instead of `align`.
// Weighted form: the wave's share is the slice [lo, hi) of a total weight T (the unweighted form: g, g + 1, W).
// (T < 2^32: the slices are scaled 32-bit weights; a 64-bit T — a full 64 / 64-bit division here — gave some waves of
// the streamed receive pass wrong ranges in round 6's first slot-share build, with the same partition in exact
// arithmetic, and is not used.)
__device__ __forceinline__ WaveRange wave_range_w(__amdgpu_buffer_rsrc_t ofs, uint32_t n, uint32_t lo, uint32_t hi,
                                                  uint32_t T, uint32_t lane, uint32_t small_mean, uint32_t align,
                                                  uint32_t count_align = 0) {
    const uint64_t o_lo = ld_off(ofs, 0), o_hi = ld_off(ofs, n);
    const uint64_t tot = o_hi - o_lo;
    uint32_t s[2];
    const bool by_count = tot < (uint64_t)small_mean * n;
    if (by_count && count_align) align = count_align;
    if (by_count) {
        s[0] = (uint32_t)((uint64_t)n * lo / T);
        s[1] = (uint32_t)((uint64_t)n * hi / T);
    } else {
        seg_lower_bound2(ofs, n, o_lo + tot * lo / T, o_lo + tot * hi / T, lane, s);
    }
    WaveRange r;
    r.a0 = lo == 0 ? 0u : min((s[0] + align - 1u) / align * align, n);
    r.a_end = hi == T ? n : min((s[1] + align - 1u) / align * align, n);
    r.bytes = by_count ? ld_off(ofs, r.a_end) - ld_off(ofs, r.a0) : tot * hi / T - tot * lo / T;
    return r;
}

__device__ __forceinline__ WaveRange wave_range(__amdgpu_buffer_rsrc_t ofs, uint32_t n, uint32_t g, uint32_t W,
                                                uint32_t lane, uint32_t small_mean, uint32_t align,
                                                uint32_t count_align = 0) {
    return wave_range_w(ofs, n, g, g + 1u, W, lane, small_mean, align, count_align);
}

// Byte shares by the block's slot on its CU (round 6). A CU's blocks are dispatched
// breadth-first (the first CUs/8 blocks of an XCD each go to their own CU, the next CUs/8 take the second place on
// the same CUs, ...), and the CU issues its oldest waves first: in the streamed receive pass (3 blocks of 4 waves
// per CU) the waves of a CU's first block ended 4.1 µs before the launch's median wave and those of its third 4.6 µs
// after (workload 10; 14: −6.7 / +6.8 µs, tools/probes/rx_wave_times.py, profiles/r06_rx_wave_times_slots.txt) —
// the launch's tail. So a wave's byte share is weighted by its block's slot (1/1024s; slots past the third weigh as
// the third). The measured rates alone (1059 / 1024 / 989) halved the slots' spread; the weights were then tuned on
// workloads 10, 11, 14 (1080 / 1024 / 968; 1100 / 1024 / 950 was better on 10 only) and, for the ragged scan's two
// active slots, on config 3 (1059 / 1024; 1050 and 1070 slower) — profiles/r06_slot_tune_libab.txt,
// r06_scan_slot_tune_libab.txt. Wave g = XCD-major as wave_number(nb, wpb, w).
#ifndef NSX_SLOT_WEIGHTS
#define NSX_SLOT_WEIGHTS 1
#endif
constexpr bool kSlotWeights = NSX_SLOT_WEIGHTS;
#ifndef NSX_SCAN_SLOT_WEIGHTS
#define NSX_SCAN_SLOT_WEIGHTS 1
#endif
constexpr bool kScanSlotWeights = NSX_SCAN_SLOT_WEIGHTS;  // the ragged scan's streamed forms (A/B builds)
#ifndef NSX_SLOT_W0
#define NSX_SLOT_W0 1080
#define NSX_SLOT_W1 1024
#define NSX_SLOT_W2 968
#endif
#ifndef NSX_SCAN_W0
#define NSX_SCAN_W0 1059
#define NSX_SCAN_W1 1024
#endif
// the streamed receive pass (3 active blocks per CU) and the ragged scan's streamed forms (2 or 3)
struct SlotWeights {
    uint32_t w0, w1, w2;
};
constexpr SlotWeights kRxSlotW{NSX_SLOT_W0, NSX_SLOT_W1, NSX_SLOT_W2};
constexpr SlotWeights kScanSlotW{NSX_SCAN_W0, NSX_SCAN_W1, NSX_SLOT_W2};
struct SlotShare {
    uint32_t lo, hi, T;  // T = 8 · (an XCD's weight) · wpb < 2^32 for any grid this library launches
};
__device__ __forceinline__ SlotShare slot_share(uint32_t nb, uint32_t wpb, uint32_t w, uint32_t cus_per_xcd,
                                                const SlotWeights sw) {
    const uint32_t b = blockIdx.x, per = nb >> 3;  // blocks per XCD (nb a multiple of 8)
    const uint32_t x = b & 7u, j = b >> 3;        // XCD, place in the XCD's dispatch order
    const uint32_t c = cus_per_xcd;
    // the weight of the first k blocks of an XCD: slots 0 and 1 of c blocks each, then slot 2 and later (closed form:
    // round 6's first build summed the slots in a loop, and its first slot's waves got wrong ranges on the GPU)
    auto below = [&](uint32_t k) {
        const uint32_t k0 = min(k, c), k1 = min(k - k0, c), k2 = k - k0 - k1;
        return k0 * sw.w0 + k1 * sw.w1 + k2 * sw.w2;
    };
    const uint32_t me = j < c ? sw.w0 : j < 2u * c ? sw.w1 : sw.w2;
    const uint32_t xw = below(per);
    const uint32_t lo = x * xw * wpb + below(j) * wpb + w * me;
    return SlotShare{lo, lo + me, 8u * xw * wpb};
}

// Stream the bytes [rbase + head, rbase + span) as 1 KiB rows of one wave (rbase 128-byte aligned, so a row
// touches exactly 8 lines), R rows per load batch, and sample S (the weighted byte sum of the ragged scan
// kernel, relative to rbase) at every lane's boundaries brel[k] (−1: none), k < NS: bval[k] = S(brel[k]). A
// boundary at or past the last row gets the total; carry = S(span) on return. Bytes before head and past span
// count as 0. NS boundary slots per lane let one pass cover NS sets of 64 boundaries: the per-span costs (the
// pipeline filling at its start and draining at its end, the caller's setup and results) are paid once per NS
// sets — with frames of a few hundred bytes a span of 64 is ~50 KB and those costs were ~7% of the time.
// PIPE: two register sets — batch r0 + R loads while batch r0 is scanned.
template <int R, bool PIPE = false, int NS = 1>
__device__ __forceinline__ void scan_span(const uint8_t* rbase, uint64_t span, uint32_t head,
                                          const int64_t (&brel)[NS], uint32_t lane, uint64_t (&bval)[NS],
                                          uint64_t& carry) {
    const uint64_t nrows = (span + kRow - 1) / kRow;
    // Batch r0 = rows [r0, r0 + R), one descriptor based at its first row (rows past the run read 0).
    auto issue = [&](uint64_t r0, u32x4 (&v)[R]) {
        const uint8_t* bb = rbase + r0 * kRow;
        const uint64_t rem = r0 < nrows ? span - r0 * kRow : 0;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(bb, (rem + 3) & ~3ull);
#pragma unroll
        for (int j = 0; j < R; ++j) v[j] = bld16<true>(rs, j * kRow + lane * 16);
    };
    auto process = [&](uint64_t r0, u32x4 (&v)[R]) {
#pragma unroll
        for (int j = 0; j < R; ++j) asm volatile("" : "+v"(v[j]));
        // Phase 1: edge masks (first/last row of the run only), lane half-sums
        // and the R row scans as independent chains (ILP across rows).
        uint32_t sl[R], incl[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint64_t r = r0 + j;
            const int64_t rowrel = (int64_t)(r * kRow);
            if (r == 0 && head) {  // bytes before the run's first segment
                const int32_t h = (int32_t)head - (int32_t)lane * 16;
                v[j] = keep_bytes(v[j], min(max(h, 0), 16), 16);
            }
            if (r < nrows && rowrel + (int64_t)kRow > (int64_t)span) {  // bytes past the run's end
                const int32_t e = (int32_t)((int64_t)span - rowrel) - (int32_t)lane * 16;
                v[j] = keep_bytes(v[j], 0, min(max(e, 0), 16));
            }
            sl[j] = sad4(v[j], 0u);
        }
#pragma unroll
        for (int j = 0; j < R; ++j) incl[j] = wave_incl_scan(sl[j]);
        uint64_t crow[R];  // S at the start of row j
        uint64_t c = carry;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            crow[j] = c;
            c += __builtin_amdgcn_readlane(incl[j], 63);
        }
        // Phase 2: boundaries that fall in this batch (rows past nrows hold zeros).
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const int64_t qb = brel[k] - (int64_t)(r0 * kRow);
            const bool in_batch = qb >= 0 && qb < (int64_t)R * kRow;
            if (__builtin_amdgcn_ballot_w64(in_batch)) {
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int64_t q = qb - (int64_t)j * kRow;  // boundary position inside row j
                    const bool here = q >= 0 && q < (int64_t)kRow;
                    if (__builtin_amdgcn_ballot_w64(here)) {
                        const uint32_t src = here ? (uint32_t)(q >> 4) : lane;
                        const uint32_t pre = bperm(incl[j] - sl[j], src);
                        u32x4 y;
                        y.x = bperm(v[j].x, src);
                        y.y = bperm(v[j].y, src);
                        y.z = bperm(v[j].z, src);
                        y.w = bperm(v[j].w, src);
                        const uint32_t part = sad4(keep_bytes(y, 0, (int32_t)(q & 15)), 0u);
                        if (here) bval[k] = crow[j] + pre + part;
                    }
                }
            }
        }
        carry = c;
    };
    if constexpr (PIPE) {
        u32x4 A[R], B[R];
        issue(0, A);
        for (uint64_t r0 = 0; r0 < nrows; r0 += 2 * R) {
            issue(r0 + R, B);  // past the rows: an empty descriptor, the loads move nothing
            process(r0, A);
            if (r0 + R >= nrows) break;
            issue(r0 + 2 * R, A);
            process(r0 + R, B);
        }
    } else {
        for (uint64_t r0 = 0; r0 < nrows; r0 += R) {
            u32x4 v[R];
            issue(r0, v);
            process(r0, v);
        }
    }
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if (brel[k] >= (int64_t)(nrows * kRow)) bval[k] = carry;  // boundary at the very end of the rows
}

// Ragged scan forms by mean segment size (profiles/r04_ragged_form_sweep.txt): per batch, the small-segment mode
// under kScanLdsSeg; else per wave the LDS form under kScanLdsSeg (runs of 63 such segments fit its 8 KiB slot),
// else streamed runs of two 63-segment sets under kScanTwoSetSeg, else of one set, on 3 blocks/CU under
// kScanBigMean, else 2.
constexpr uint32_t kScanLdsSeg = 128;
constexpr uint32_t kScanTwoSetSeg = 256;
constexpr uint32_t kScanBigMean = 2048;

// Blocks of this launch that take work. The persistent grids of the ragged scan and the receive pass are sized for
// small units (4 blocks/CU: every wave's rows in flight count when each unit costs a header check or an LDS
// sum); a batch whose mean unit is at least `big_mean` bytes streams best on fewer waves (config 3 at 2 blocks/CU
// 3% faster than at 4, workload 10 at 3 blocks/CU 2.9% faster), so only its first
// ⌊gridDim·keep/4⌋ blocks (rounded to the 8 XCDs) take byte ranges and the rest return at once. keep = 0: every
// block. (Blocks are dealt to CUs breadth-first, so the first 3/4 of a 4-per-CU grid is 3 per CU: workload 10 ran
// within 0.4% of a 3-per-CU launch.)
__device__ __forceinline__ uint32_t active_blocks(__amdgpu_buffer_rsrc_t ofs, uint32_t n, uint32_t big_mean,
                                                  uint32_t keep) {
    const uint32_t nb = gridDim.x;
    if (keep == 0 || nb < 64) return nb;
    const uint64_t tot = ld_off(ofs, n) - ld_off(ofs, 0);
    if (tot < (uint64_t)big_mean * n) return nb;
    const uint32_t k = (nb / 4u * keep) & ~7u;
    return k ? k : nb;
}

// Results parked in LDS and written in bulk. A 2-byte raw sum (or a 1-byte verdict)
// per segment is a small write stream beside a large read stream, and written as it is produced (128 B per wave and
// run) it cost far more than its bytes: 12-14% of the small-segment LDS form's time, 5-16% of the streamed form's
// with frames of 160-620 B (profiles/r04_ragged_park_*, r04_rawstream_ab.txt). Parked, a wave's results go out up to
// 8 KiB at a time, 16 B per lane and store. T = the result type (uint16_t raw sums, uint8_t verdicts of the batch
// verify); buf[i] holds the result of segment base + i, base chosen so that out + base is 16 B aligned (al = the
// output's misalignment in results; base may wrap below 0: only differences of indices are compared); [lo, hi) is
// parked. A wave parks in increasing segment order and flushes when the next set is not contiguous or would not
// fit, and at its end. Off (buf null): stored directly.
template <typename T>
struct ResultPark {
    static constexpr uint32_t kPer = 16u / sizeof(T);    // results per 16 B block
    static constexpr uint32_t kCap = 8192u / sizeof(T);  // results per buffer: 8 KiB of a wave's 8.25 KiB LDS slot
    T* buf;
    __amdgpu_buffer_rsrc_t rs;  // the output
    uint32_t al, base, lo, hi;
    uint32_t cap;  // results the buffer holds (≤ kCap, a multiple of kPer)
    __device__ __forceinline__ void rebase(uint32_t a) {
        base = ((a + al) & ~(kPer - 1u)) - al;
        lo = hi = a;
    }
};

template <typename T>
__device__ __forceinline__ ResultPark<T> make_park(T* buf, __amdgpu_buffer_rsrc_t rs, const void* out, uint32_t a0,
                                                   uint32_t cap = ResultPark<T>::kCap) {
    ResultPark<T> pk{buf, rs, (uint32_t)((uintptr_t)out / sizeof(T)) & (ResultPark<T>::kPer - 1u), 0, 0, 0, cap};
    pk.rebase(a0);
    return pk;
}

template <typename T>
__device__ __forceinline__ void store_result(T v, __amdgpu_buffer_rsrc_t rs, uint32_t off) {
    if constexpr (sizeof(T) == 2) __builtin_amdgcn_raw_buffer_store_b16(v, rs, off, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b8(v, rs, off, 0, 0);
}

template <typename T>
__device__ __forceinline__ void park_flush(ResultPark<T>& pk, uint32_t lane) {
    constexpr uint32_t P = ResultPark<T>::kPer;
    if (!pk.buf || pk.hi == pk.lo) return;
    __builtin_amdgcn_wave_barrier();
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t l = pk.lo - pk.base, h = pk.hi - pk.base;  // parked: buf[l, h), 0 ≤ l < h ≤ cap
    const uint32_t b0 = l / P, b1 = (h + P - 1u) / P;           // the 16 B blocks touched
    const bool head_full = P * b0 == l, tail_full = P * b1 == h;
    for (uint32_t q = b0; q < b1; q += kWave) {  // whole blocks: one 16 B store each
        const uint32_t blk = q + lane;
        const bool full = blk < b1 && (blk != b0 || head_full) && (blk != b1 - 1u || tail_full);
        const lds16 v = reinterpret_cast<const lds16*>(pk.buf)[blk < pk.cap / P ? blk : 0u];
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, pk.rs,
                                               full ? (pk.base + P * blk) * (uint32_t)sizeof(T) : kOOB, 0, 0);
    }
    // the results of a partial first / last block, one lane each (lanes 0..P-1: block b0, P..2P-1: block b1 − 1
    // when it is another block; a block is partial when [l, h) does not cover it, as the full-block test above)
    const bool one = b1 - 1u == b0;
    const bool part0 = !head_full || (one && !tail_full), part1 = !one && !tail_full;
    const uint32_t i = (lane < P ? P * b0 : P * (b1 - 1u)) + (lane & (P - 1u));
    const bool st = lane < 2u * P && (lane < P ? part0 : part1) && i >= l && i < h;
    const T r = pk.buf[st ? i : 0u];
    store_result<T>(r, pk.rs, st ? (pk.base + i) * (uint32_t)sizeof(T) : kOOB);
    __builtin_amdgcn_wave_barrier();
    pk.rebase(pk.hi);
}

// Segment a + lane's result (lanes < cnt): parked, or stored directly when parking is off.
template <typename T>
__device__ __forceinline__ void park_put(ResultPark<T>& pk, uint32_t a, uint32_t cnt, uint32_t lane, uint32_t res) {
    if (!pk.buf) {
        store_result<T>((T)res, pk.rs, lane < cnt ? (a + lane) * (uint32_t)sizeof(T) : kOOB);
        return;
    }
    if (pk.hi != a || a + cnt - pk.base > pk.cap) {  // not contiguous, or would overflow: flush, rebase
        park_flush(pk, lane);
        pk.rebase(a);
    }
    if (lane < cnt) pk.buf[a + lane - pk.base] = (T)res;
    pk.hi = a + cnt;
}

// The outputs of segments [a, a + cnt) (lane l: segment a + l): the raw sum parked (checksum), or — the batch verify
// (VERIFY) — the 1-byte verdict parked and the raw sum, when asked for (raw), stored directly.
template <bool VERIFY>
using ScanPark = ResultPark<typename std::conditional<VERIFY, uint8_t, uint16_t>::type>;

template <bool VERIFY>
__device__ __forceinline__ void put_results(ScanPark<VERIFY>& pk, __amdgpu_buffer_rsrc_t ors, bool raw, uint32_t a,
                                            uint32_t cnt, uint32_t lane, uint32_t res) {
    if constexpr (VERIFY) {
        if (raw) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)res, ors, lane < cnt ? (a + lane) * 2u : kOOB, 0, 0);
        if (cnt) park_put(pk, a, cnt, lane, res == 0xFFFFu ? 1u : 0u);
    } else {
        (void)ors;
        (void)raw;
        if (cnt) park_put(pk, a, cnt, lane, res);
    }
}

// One run of NS sets of ≤ run segments in the streaming form: set k = segments [a + k·run, + cnt[k]), lane l ≤
// cnt[k] holds boundary my_off[k] = offsets[a + k·run + l] and (l < cnt[k]) the partial my_part[k]. Results into
// the wave's park (put_results).
template <int R, bool VERIFY, bool PIPE, int NS>
__device__ __forceinline__ void ragged_run_stream(const uint8_t* __restrict__ base, uint32_t a, uint32_t run,
                                                  const uint32_t (&cnt)[NS], const uint64_t (&my_off)[NS],
                                                  const uint32_t (&my_part)[NS], __amdgpu_buffer_rsrc_t ors,
                                                  bool raw, uint32_t lane, ScanPark<VERIFY>& pk) {
    int64_t brel[NS];
    uint64_t bval[NS];
    // the run's last boundary: set kl = the last set with segments, its lane cnt
    uint32_t kl = 0;
#pragma unroll
    for (int k = 1; k < NS; ++k) kl = cnt[k] ? (uint32_t)k : kl;
    uint64_t hi = 0;
#pragma unroll
    for (int k = 0; k < NS; ++k)
        if ((uint32_t)k == kl) hi = readlane64(my_off[k], cnt[k]);
    const uint64_t lo = readlane64(my_off[0], 0);
    // Rows start on a 128-byte line so a 1 KiB row touches exactly 8 lines.
    const uint8_t* rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + lo)) & ~(uintptr_t)127);
    const uint64_t span = (uint64_t)((base + hi) - rbase);           // bytes from rbase to the run's end
    const uint32_t head = (uint32_t)((uintptr_t)(base + lo) & 127u);  // bytes before the run in row 0
    // Boundary lane state: its position relative to rbase, and S there.
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        brel[k] = cnt[k] && lane <= cnt[k] ? (int64_t)((base + my_off[k]) - rbase) : -1;
        bval[k] = 0;
    }
    uint64_t carry = 0;
    scan_span<R, PIPE, NS>(rbase, span, head, brel, lane, bval, carry);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        // Segment `lane` of set k = [boundary lane, boundary lane+1).
        const uint64_t nb = ((uint64_t)__shfl_down((unsigned long long)bval[k], 1));
        const uint64_t d = nb - bval[k];
        const uint32_t le = fold32((uint32_t)(d & 0xFFFFFFFFu)) + fold32((uint32_t)(d >> 32));
        const bool even = (((uintptr_t)base + my_off[k]) & 1u) == 0;
        const uint32_t res = finish(le, even, my_part[k]);
        put_results<VERIFY>(pk, ors, raw, a + k * run, cnt[k], lane, res);
    }
}

// The wave's runs [a0, a_end) of NS sets of ≤ run segments (see csum_ragged_scan_kernel).
template <int R, bool VERIFY, bool PIPE, int NS>
__device__ __forceinline__ void ragged_runs(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                            __amdgpu_buffer_rsrc_t prs, __amdgpu_buffer_rsrc_t ors,
                                            __amdgpu_buffer_rsrc_t oks, uint32_t run, uint32_t a0, uint32_t a_end,
                                            uint32_t lane, void* park_buf, const void* out, bool raw) {
    using T = typename std::conditional<VERIFY, uint8_t, uint16_t>::type;
    ScanPark<VERIFY> pk = make_park<T>(static_cast<T*>(park_buf), VERIFY ? oks : ors, out, a0);
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const uint32_t a_step = run * NS;
    auto load_offs = [&](uint32_t a) -> uint64_t {  // lane l ≤ run length: offsets[a + l]
        const uint32_t voff = (a < a_end && lane <= run && a + lane <= n) ? (a + lane) * 8 : kOOB;
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, voff, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    uint64_t nxt_off[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) nxt_off[k] = load_offs(a0 + k * run);
    for (uint32_t a = a0; a < a_end; a += a_step) {
        uint64_t my_off[NS];  // set k: boundary `lane` (lanes 0..cnt_k)
        uint32_t cnt[NS], my_part[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const uint32_t ak = a + k * run;
            cnt[k] = ak < a_end ? min(run, a_end - ak) : 0u;
            my_off[k] = nxt_off[k];
            nxt_off[k] = load_offs(a + a_step + k * run);
            my_part[k] = __builtin_amdgcn_raw_buffer_load_b32(prs, lane < cnt[k] ? (ak + lane) * 4 : kOOB, 0, 0);
        }
        ragged_run_stream<R, VERIFY, PIPE, NS>(base, a, run, cnt, my_off, my_part, ors, raw, lane, pk);
    }
    park_flush(pk, lane);
}

// Sum of the bytes [p, e) of a wave's LDS slot for the lanes' consecutive ranges of one run (p, e slot positions;
// e - p < 2^15): lane l's range ends where lane l + 1's begins (e_l = p_{l+1}), lanes past the run have live =
// false, and the slot's bytes from the run's end up to the next 16 B boundary are 0 (lds_zero_tail). dq = the slot
// dword holding byte p. The weighted byte sum of the range (LE half-sums of its 4-aligned dwords, as in
// scan_span): the slot keeps every byte's address mod 128.
//
// The 16 B chunks [p/16, ceil(e/16)) are summed whole, eight reads in flight per lane, minus
//   head = the first chunk's bytes before p: the v_sad_u16 chain that sums that chunk yields its dword prefix
//          sums, so head = prefix(p/4 mod 4) + the low p mod 4 bytes of dq — no byte masks;
//   tail = the last chunk's bytes from e on = lane l + 1's first-chunk bytes from p_{l+1} = e on (one DPP shift
//          across the wave), or 0 when e is a multiple of 16; the last lane of the run gets 0 from a lane past
//          it (or past the wave), which is right because the bytes after the run's end are 0.
// (Round-3 first form: both ends masked byte-wise with keep_bytes, ~56 VALU per run)
__device__ __forceinline__ uint32_t lds_range_sum(const lds16* slot, uint32_t p, uint32_t e, uint32_t dq, bool live) {
    const uint32_t c0 = p >> 4, c1 = (e + 15u) >> 4, nch = c1 - c0;
    // A first block of 8 chunks, then blocks of 4 while the wave's longest range has more: a wave-uniform trip
    // count (an SGPR loop counter: a loop ending on a ballot left hipcc an undefined exit value that it read with
    // v_readfirstlane from a register still being loaded — a vmcnt wait that drained the next run's rows before this
    // run's sums began). A block reads its chunks from one address with immediate offsets and keeps those below nch.
    // The first block is always read (its first chunk gives head and the neighbour's tail even for an empty range);
    // it reads chunks c0 .. c0 + 7, at most 7 past the range's last chunk, which the slot's 256 B pad holds. Blocks
    // of 4 after it: 64-128 B segments span up to 9 chunks, and a second block of 8 read 7 chunks for nothing in
    // nearly every wave. A lane whose range has ended (j0 ≥ nch) reads its block from c0 again instead of c0 + j0,
    // so no lane reads more than 3 chunks past its range: in a run that mixes a several-KB unit with small ones, j0
    // runs up to the long unit's chunk count, and c0 + j0 would leave the slot.
    // Only a wave with a range past the first block pays for the wave maximum (round 5: 4 DPP + 4 v_readlane per run
    // on every run of small units before; one compare and a scalar test now).
    const bool more = __builtin_amdgcn_ballot_w64(nch > 8u) != 0;
    uint32_t acc;
    {
        u32x4 x[8];
        const lds16* blk = slot + c0;
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) x[j] = lds_get(blk, j);
        const uint32_t pre1 = __builtin_amdgcn_sad_u16(x[0].x, 0u, 0u);
        const uint32_t pre2 = __builtin_amdgcn_sad_u16(x[0].y, 0u, pre1);
        const uint32_t pre3 = __builtin_amdgcn_sad_u16(x[0].z, 0u, pre2);
        const uint32_t s0 = __builtin_amdgcn_sad_u16(x[0].w, 0u, pre3);
        const uint32_t q = (p >> 2) & 3u;
        const uint32_t pq = q == 0u ? 0u : q == 1u ? pre1 : q == 2u ? pre2 : pre3;
        const uint32_t head = __builtin_amdgcn_sad_u16(dq & ((1u << (8u * (p & 3u))) - 1u), 0u, pq);
        const uint32_t g = live ? s0 - head : 0u;  // this lane's first-chunk bytes from p on
        const uint32_t gn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)g, 0x130, 0xF, 0xF, false);  // wave_shl:1
        const uint32_t tail = (e & 15u) ? gn : 0u;
        acc = (nch ? s0 : 0u) - tail - head;  // an empty range (nch = 0) starts 16-aligned: head = tail = 0
#pragma unroll
        for (uint32_t j = 1; j < 8u; ++j) {
            const uint32_t s4 = sad4(x[j], 0u);
            acc += j < nch ? s4 : 0u;
        }
    }
    if (more) {
        const uint32_t nmax = wave_max(nch);
        for (uint32_t j0 = 8; j0 < nmax; j0 += 4u) {
            u32x4 x[4];
            const lds16* blk = slot + c0 + (j0 < nch ? j0 : 0u);
#pragma unroll
            for (uint32_t j = 0; j < 4u; ++j) x[j] = lds_get(blk, j);
#pragma unroll
            for (uint32_t j = 0; j < 4u; ++j) {
                const uint32_t s4 = sad4(x[j], 0u);
                acc += j0 + j < nch ? s4 : 0u;
            }
        }
    }
    return acc;
}

// Zero the slot's bytes [span, 4·ceil(span/4)) after lds_stage: the bytes of the run's last dword past its end (the
// row loads read whole dwords; from there on to the 16 B boundary they already read 0), so lds_range_sum's last
// range needs no tail.
__device__ __forceinline__ void lds_zero_tail(lds16* slot, uint64_t span, uint32_t lane) {
    const uint32_t z = (uint32_t)span, k = (4u - (z & 3u)) & 3u;
    if (lane < k) reinterpret_cast<uint8_t*>(slot)[z + lane] = 0;
    __builtin_amdgcn_wave_barrier();
}

// Stage the rows [0, span) of a run into the wave's slot (rows already loaded into V, all in flight; only the
// rows the run covers are written). The previous run's LDS reads come first: a wave's DS operations stay in
// order, and the wave barriers keep the compiler from moving reads or writes across.
template <uint32_t ROWS>
__device__ __forceinline__ void lds_stage(lds16* slot, u32x4 (&V)[ROWS], uint64_t span, uint32_t lane) {
#pragma unroll
    for (uint32_t r = 0; r < ROWS; ++r) asm volatile("" : "+v"(V[r]));
    __builtin_amdgcn_wave_barrier();
    const uint32_t rows = __builtin_amdgcn_readfirstlane((uint32_t)((span + kRow - 1) / kRow));  // ≤ ROWS (scalar)
#pragma unroll
    for (uint32_t r = 0; r < ROWS; ++r)
        if (r < rows) slot[r * (kRow / 16u) + lane] = lds16{V[r].x, V[r].y, V[r].z, V[r].w};
    __builtin_amdgcn_wave_barrier();
}

constexpr uint32_t kSeqRun = 64;
// Run sequences (round 5): the runs of kSeqRun units a wave takes, in order, named by their
// first unit. The run loops (pfx_runs, rx_runs_lds) read them two runs ahead — the next run's rows and the offsets of
// the run after it are loaded while one run is summed — and call next() exactly once per run, in order: a dealt
// sequence pulls from a shared counter there. cnt(a) = the units of run a; a value a with !live(a) ends the
// sequence (cnt 0).

// The units [a0, a_end) in runs of `run` from a0 (end: a_end).
struct StaticRuns {
    uint32_t a0, a_end, run = kSeqRun;
    __device__ __forceinline__ bool live(uint32_t a) const { return a < a_end; }
    __device__ __forceinline__ uint32_t first() const { return a0; }
    __device__ __forceinline__ uint32_t next(uint32_t a) const { return a + run < a_end ? a + run : a_end; }
    __device__ __forceinline__ uint32_t cnt(uint32_t a) const { return min(run, a_end - a); }
    __device__ __forceinline__ void refill() const {}
};

// A wave's static runs [a0, e_st), then runs dealt from a pool: the batch's last units [S, n), as runs from S, split
// into one share per counter ("head") — the share's runs pb + 64 t, t < q, go to the waves of this head in the order
// they ask (end: n). A wave always holds one ticket ahead (pulled one run before it is needed, so that the counter's
// round trip, ~1-3 µs under load, overlaps a run's work): the pull is a returning device-scope atomic add from lane
// 0, its value read (readfirstlane) only when the ticket is taken. Every wave of the head takes tickets until one is
// past its share, so the head sees exactly q + (its waves) pulls per launch: the wave that draws the last of them,
// `last`, resets the counter to 0 for the next launch that uses it — launches on one stream run one after another,
// and the host gives each stream its own heads (deal_heads).
struct DealtRuns {
    uint32_t a0, e_st, n;
    uint32_t pb, q, last;
    uint32_t* head;
    uint32_t lane;
    uint32_t tk;    // the reserved ticket (lane 0's VGPR until taken)
    bool dealing;   // false once a ticket past the share was taken (or without a head)
    bool want;      // a ticket was taken and the next is not yet pulled (refill)
    __device__ __forceinline__ uint32_t pull() const {
        uint32_t t = 0u;
        if (lane == 0u) t = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return t;
    }
    __device__ __forceinline__ void init() {
        tk = pull();
        dealing = true;
        want = false;
    }
    // The pull for the next ticket, issued by the run loops after a run's loads: vmcnt retires in issue order, so
    // loads issued behind the atomic would wait for its round trip too.
    __device__ __forceinline__ void refill() {
        if (want) tk = pull();
        want = false;
    }
    __device__ __forceinline__ uint32_t take() {
        if (!dealing) return n;
        refill();
        const uint32_t t = __builtin_amdgcn_readfirstlane(tk);
        if (t < q) {
            want = true;
            return pb + t * kSeqRun;
        }
        dealing = false;
        if (t == last && lane == 0u) __hip_atomic_store(head, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return n;
    }
    __device__ __forceinline__ bool live(uint32_t a) const { return a < n; }
    __device__ __forceinline__ uint32_t first() { return a0 < e_st ? a0 : take(); }
    // a static run's successor, else a dealt run (a pool run, or the end n: both ≥ e_st)
    __device__ __forceinline__ uint32_t next(uint32_t a) { return a + kSeqRun < e_st ? a + kSeqRun : take(); }
    __device__ __forceinline__ uint32_t cnt(uint32_t a) const { return min(kSeqRun, (a < e_st ? e_st : n) - a); }
};


// Wave g of W's runs: with heads for this launch (deal), its equal share (wave_range: small_mean, align,
// count_align) of the batch's first n − n/2^kDealPoolShift units (S, a multiple of kSeqRun), then runs of the pool
// [S, n) dealt from head g mod kDealHeads — the waves of a head spread over every XCD (heads per XCD left the XCDs'
// speed differences in place, §7 step 72); without, its equal share of the whole batch. wr_out: the static share.
__device__ __forceinline__ DealtRuns deal_runs(__amdgpu_buffer_rsrc_t ofs, uint32_t n, uint32_t g, uint32_t W,
                                               uint32_t lane, uint32_t small_mean, uint32_t align,
                                               uint32_t count_align, uint32_t* deal, WaveRange* wr_out = nullptr) {
    const uint32_t S = deal ? (n - (n >> kDealPoolShift)) & ~(kSeqRun - 1u) : n;
    DealtRuns q{0u, 0u, n, 0u, 0u, 0u, nullptr, lane, 0u, false, false};
    WaveRange wr{0u, 0u, 0u};
    if (S > 0u) wr = wave_range(ofs, S, g, W, lane, small_mean, align, count_align);
    q.a0 = wr.a0, q.e_st = wr.a_end;
    if (wr_out) *wr_out = wr;
    if (deal) {
        const uint32_t H = min(kDealHeads, W), h = g % H;
        const uint32_t Q = (n - S + kSeqRun - 1u) / kSeqRun;  // the pool's runs
        const uint32_t r0 = (uint32_t)((uint64_t)Q * h / H);
        const uint32_t qh = (uint32_t)((uint64_t)Q * (h + 1u) / H) - r0;
        q.pb = S + r0 * kSeqRun, q.q = qh, q.last = qh + (W - h + H - 1u) / H - 1u;  // + the head's waves g ≡ h
        q.head = deal + h * kDealStride;
        q.init();
    }
    return q;
}

// A run loop's state at a run boundary, handed from one loop to another (rx_runs_lds → the hybrid loop): run a with
// its offsets (lane l = unit a + l; c_end: a + l + 1), the next run an with its offsets.
struct RunHead {
    uint32_t a, an;
    uint64_t c_off, c_end, n_off, n_end;
};

// The LDS form of the ragged checksum for small segments, the receive pass's
// (rx_runs_lds) applied to runs of ≤ run segments: lane l sums segment a + l out of the wave's slot, both of its
// offsets loaded by the lane itself. A run too wide for the slot is streamed (as ≤ 63 + the rest).
//
// PARK (runs of 64, the default small-segment mode, §7 step 61): the runs' results are not stored run by run but
// parked in LDS beside the slot and written 64 runs at a time — 8 KiB contiguous per wave, 16 B per lane and store.
// A result store per run (128 B per wave every few microseconds, 2 B per segment: 1.8% of workload 15's bytes) cost
// this loop 12-14% of its time: the receive pass over the same frames ran 14% slower when it also wrote its 2 B raw
// sums, and parking 8 / 32 / 64 runs took the ragged form 2% / 6% / 12.6% faster (profiles/r04_ragged_park_*). The
// park buffer is the second of the block's four 8.25 KiB slots, so the mode runs two waves per block (8 per CU).
// The partial of each run is loaded only when the batch has partials. A wave's partial last run, and the runs before
// a streamed one, are flushed (and stored) as they come.
constexpr uint32_t kScanSlotRows = 8;
constexpr uint32_t kScanSlot = kScanSlotRows * kRow + 256;  // + pad: lds_range_sum's first chunk block reads past the end

template <int R, bool VERIFY, bool PIPE, bool PARK, typename Seq>
__device__ __forceinline__ void ragged_runs_lds(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                                __amdgpu_buffer_rsrc_t prs, __amdgpu_buffer_rsrc_t ors,
                                                __amdgpu_buffer_rsrc_t oks, uint32_t run, Seq& q, uint32_t lane,
                                                lds16* slot, bool has_part, const void* out, bool raw) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    auto ld64 = [&](uint32_t i, bool live) -> uint64_t {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, live ? i * 8 : kOOB, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    // lane l < run length: segment a + l = [offsets[a + l], offsets[a + l + 1])
    auto load_offs = [&](uint32_t a) { return ld64(a + lane, q.live(a) && lane < run && a + lane <= n); };
    auto load_ends = [&](uint32_t a) { return ld64(a + lane + 1u, q.live(a) && lane < run && a + lane + 1u <= n); };
    struct Run {
        const uint8_t* rbase;
        uint64_t span;
        uint32_t cnt;
        bool lds;
    };
    auto geo = [&](uint32_t a, uint64_t off, uint64_t end) {  // wave-uniform geometry of run a
        Run g{base, 0, q.cnt(a), false};
        if (g.cnt) {
            const uint64_t lo = readlane64(off, 0), hi = readlane64(end, g.cnt - 1u);
            g.rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + lo)) & ~(uintptr_t)127);
            g.span = (uint64_t)((base + hi) - g.rbase);
            g.lds = g.span <= (uint64_t)kScanSlotRows * kRow;
        }
        return g;
    };
    auto load_part = [&](uint32_t a, uint32_t cnt) {
        return has_part ? __builtin_amdgcn_raw_buffer_load_b32(prs, lane < cnt ? (a + lane) * 4 : kOOB, 0, 0) : 0u;
    };
    u32x4 V[kScanSlotRows];
    auto issue = [&](const Run& g) {  // rows past the run: out of the descriptor's range, 0, no traffic
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(g.rbase, (g.span + 3) & ~3ull);
#pragma unroll
        for (uint32_t r = 0; r < kScanSlotRows; ++r) V[r] = bld16<true>(rs, r * kRow + lane * 16u);
    };
    // As rx_runs_lds: the LDS loop runs while consecutive runs fit the slot; a run that does not is streamed on
    // its own in the outer loop, so the streaming form's loads in flight at its end never merge into the LDS
    // loop's wait counts. The next run and its offsets are carried across (a dealt sequence's next() is called once
    // per run).
    uint32_t a = q.first();
    uint64_t c_off = load_offs(a), c_end = load_ends(a);
    uint32_t an = q.next(a);
    uint64_t n_off = load_offs(an), n_end = load_ends(an);
    q.refill();
    // PARK: the results parked in the slot after the run's (the small-segment mode gives each wave two); a dealt run
    // that does not follow the parked ones flushes them (park_put)
    using T = typename std::conditional<VERIFY, uint8_t, uint16_t>::type;
    ScanPark<VERIFY> pk = make_park<T>(PARK ? reinterpret_cast<T*>(reinterpret_cast<uint8_t*>(slot) + kScanSlot) : nullptr,
                                       VERIFY ? oks : ors, out, q.live(a) ? a : 0u);
    while (q.live(a)) {
        Run cur = geo(a, c_off, c_end);
        if (!cur.lds) {  // too wide for the slot: streamed (boundaries in lanes 0..cnt: ≤ 63 segments, then the rest)
            const uint32_t part = load_part(a, cur.cnt);
            const uint32_t c1 = min(cur.cnt, kScanRun), c2 = cur.cnt - c1;
            const uint32_t cnt1[1] = {c1}, part1[1] = {part};
            const uint64_t o1[1] = {lane == c1 ? readlane64(c_end, c1 - 1u) : c_off};
            ragged_run_stream<R, VERIFY, PIPE, 1>(base, a, kScanRun, cnt1, o1, part1, ors, raw, lane, pk);
            if (c2) {
                const uint32_t cnt2[1] = {c2}, part2[1] = {(uint32_t)__shfl_down((int)part, c1)};
                const uint64_t o2[1] = {lane == 0 ? readlane64(c_off, c1) : readlane64(c_end, c1)};
                ragged_run_stream<R, VERIFY, PIPE, 1>(base, a + c1, kScanRun, cnt2, o2, part2, ors, raw, lane, pk);
            }
            a = an, c_off = n_off, c_end = n_end;
            an = q.next(a);
            n_off = load_offs(an), n_end = load_ends(an);
            q.refill();
            continue;
        }
        issue(cur);
        __builtin_amdgcn_s_waitcnt(kWaitVm0);  // as in rx_runs_lds: nothing in flight at the loop's entry
        for (;;) {
            const uint32_t part = load_part(a, cur.cnt);
            lds_stage<kScanSlotRows>(slot, V, cur.span, lane);
            lds_zero_tail(slot, cur.span, lane);
            Run nxt = geo(an, n_off, n_end);
            if (!nxt.lds) nxt.span = 0;  // a run that will be streamed is not staged: empty loads
            issue(nxt);
            const uint32_t an2 = q.next(an);
            const uint64_t p_off = load_offs(an2), p_end = load_ends(an2);
            q.refill();
            const bool mine = lane < cur.cnt;
            const uint32_t p = mine ? (uint32_t)((base + c_off) - cur.rbase) : 0u;
            const uint32_t e = mine ? (uint32_t)((base + c_end) - cur.rbase) : 0u;
            const uint32_t dq = reinterpret_cast<const uint32_t*>(slot)[p >> 2];
            const uint32_t res = finish(fold32(lds_range_sum(slot, p, e, dq, mine)), (p & 1u) == 0, part);
            put_results<VERIFY>(pk, ors, raw, a, cur.cnt, lane, res);
            a = an, an = an2;
            c_off = n_off, c_end = n_end;
            n_off = p_off, n_end = p_end;
            if (!nxt.lds) break;  // the end of the wave's runs, or a run for the outer loop
            cur = nxt;
        }
    }
    park_flush(pk, lane);
}

// ---------------------------------------------------------------------------
// The prefix form: per-unit work that does not grow with the unit. The LDS forms
// (ragged_runs_lds above, rx_runs_lds below) sum each unit chunk by chunk in its own lane, so a run holding one
// 1500 B frame among ACKs waits ~94 chunk reads for that lane, and a run wider than the 8 KiB slot is streamed. The
// receive pass uses this form (rx_runs_pfx); on the ragged checksum, whose streamed four-set runs hold 0.74-0.82 at
// every segment size, it measured 2-13% slower everywhere and is not built (§7 step 56). Here the staging pass also writes the run's chunk PREFIX SUMS: per staged row,
// each lane's 16 B chunk sum (v_sad_u16 ×4) and an inclusive wave scan (DPP) plus the rows before it give I[c] = the
// weighted sum of the slot's bytes below chunk c. A unit starting at slot position p then has S(p) = I[p/16] + the
// bytes of chunk p/16 below p (its dword prefix sums and the low p mod 4 bytes of the dword holding p — no byte
// masks), and its sum is S(end) − S(p) with S(end) = the next lane's S(start) (one DPP shift; the piece's last lane
// takes the staged total, the bytes past the piece's end being zeroed at staging). Per lane: one ds_read_b128 and
// two ds_read_b32 at any unit size. Sums of a slot's bytes stay below 2^32 (ROWS·512 halves of < 2^16).
//
// Pieces instead of runs: a piece is the units of a 64-unit run from lane s on whose bytes fit the slot, cut at a
// multiple of ALIGN units (the receive pass: 8, whole mask bytes) unless it reaches the run's end. A run of ACKs fits
// whole; a run holding large frames goes as 2-3 pieces, each still one pass of cheap lanes (cutting runs cost 28% in
// the LDS form, §7 step 52, only because a lane then summed a 1500 B frame alone). Only a piece whose first ALIGN
// units exceed the slot (units of several KB) is streamed. The next piece's rows are loaded while this one is summed.
//
// Slot per wave: ROWS rows of data + 64 B (a header window read past the data) + I[0 .. 64·ROWS] (I[0] = 0).
constexpr uint32_t kPfxRun = 64;
template <uint32_t ROWS>
struct PfxSlot {
    static constexpr uint32_t kData = ROWS * kRow;
    static constexpr uint32_t kPrefix = kData + 64u;  // byte offset of I
    static constexpr uint32_t kBytes = (kPrefix + (ROWS * kWave + 1u) * 4u + 15u) & ~15u;
};
// The default receive grid (4 blocks/CU, §7 step 55) holds four 7-row slots (9040 B) or two 15-row slots (19280 B)
// per block.
// The hybrid loop's direct pieces: a whole run in the LDS form's 8 rows (+ 256 B pad, kScanSlot = kRxSlot).
constexpr uint32_t kPfxDirectRows = 8;
constexpr uint32_t kPfxDirectSlot = kPfxDirectRows * kRow + 256;
// Units up to this long may be summed lane by lane in direct pieces: 17 chunks.
constexpr uint32_t kPfxDirectMax = 256;


// Stage a piece's rows [0, span) into the slot (the rows already in V, all loaded) with their chunk prefix sums;
// returns S(span), the weighted sum of the staged bytes. The chunk holding byte `span` keeps only its bytes below
// it (the row loads read whole dwords up to 4·ceil(span/4): up to 3 bytes of the next unit). I[0] = 0 is written
// every time: the hybrid loop's direct pieces stage whole 8 KiB runs over it.
template <uint32_t ROWS, uint32_t VR>
__device__ __forceinline__ uint32_t pfx_stage(lds16* slot, u32x4 (&V)[VR], uint32_t span, uint32_t lane) {
    static_assert(ROWS <= VR, "rows in registers");
    uint32_t* I = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(slot) + PfxSlot<ROWS>::kPrefix);
#pragma unroll
    for (uint32_t r = 0; r < VR; ++r) asm volatile("" : "+v"(V[r]));
    __builtin_amdgcn_wave_barrier();
    const uint32_t rows = __builtin_amdgcn_readfirstlane((span + kRow - 1u) / kRow);  // ≤ ROWS (scalar)
    const uint32_t zr = span / kRow, zc = (span / 16u) & (kWave - 1u);
    const int32_t zk = (int32_t)(span & 15u);
    if (lane == 0) I[0] = 0u;
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t r = 0; r < ROWS; ++r) {
        if (r < rows) {
            u32x4 v = V[r];
            if (r == zr) v = lane == zc ? keep_bytes(v, 0, zk) : v;
            slot[r * kWave + lane] = lds16{v.x, v.y, v.z, v.w};
            const uint32_t incl = wave_incl_scan(sad4(v, 0u));
            I[r * kWave + lane + 1u] = carry + incl;
            carry += __builtin_amdgcn_readlane(incl, 63);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return carry;
}

// A wave's runs (the sequence q; h: the state a loop handed over, else q's first run), as pieces of the prefix form
// with ROWS-row slots. Unit a + l = bytes [offsets[a + l], offsets[a + l + 1]), lanes holding both ends. HYB (the hybrid loop, §7 step 55): a whole run
// whose bytes fit 8 rows and whose units are all ≤ kPfxDirectMax bytes is a DIRECT piece instead — staged without
// prefix sums and summed lane by lane (lds_range_sum, the LDS form, 3-6% faster on runs of ACKs alone: no per-row
// scans); the slot (PfxSlot<7>, 9040 B) holds either layout.
//   out(F, p, d0, live, a, s, cnt, off, end)  the results of units [a + s, a + s + cnt) (lane l = unit a + l):
//                                      F = the unit's weighted sum (32-bit), p its slot position, d0 = the slot dword
//                                      at p/4;
//   stream(a, s, rem, off, end)        units [a + s, a + s + rem) of the run at a in the streaming form (lane l of
//                                      off / end = unit a + l).
template <uint32_t ROWS, bool HYB, uint32_t ALIGN, typename Seq, typename Out, typename Stream>
__device__ __forceinline__ void pfx_runs(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                         Seq& q, uint32_t lane, lds16* slot, Out&& out, Stream&& stream,
                                         const RunHead* h = nullptr) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    constexpr uint32_t kCap = ROWS * kRow;
    constexpr uint32_t VR = HYB && ROWS < kPfxDirectRows ? kPfxDirectRows : ROWS;  // rows in flight per piece
    static_assert(!HYB || PfxSlot<ROWS>::kBytes >= kPfxDirectSlot, "a direct piece's 8 rows + pad fit the slot");
    auto load_off = [&](uint32_t i, bool live) -> uint64_t {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, live ? i * 8 : kOOB, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    const uint32_t* sdw = reinterpret_cast<const uint32_t*>(slot);
    const uint32_t* I = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(slot) + PfxSlot<ROWS>::kPrefix);
    struct Piece {
        uint32_t a, s, cnt, rem;  // units [a + s, a + s + cnt) of the run at a; rem = the run's units from s on
        const uint8_t* rbase;     // 128-aligned, at or below the piece's first byte
        uint32_t span;            // bytes from rbase to the piece's end
        bool direct;              // HYB: a whole run summed lane by lane
    };
    // Wave-uniform geometry of the piece of run a from lane s (off/end: that run's offsets, lane l = unit a + l).
    auto geo = [&](uint32_t a, uint32_t s, uint64_t off, uint64_t end) {
        Piece g{a, s, 0u, 0u, base, 0u, false};
        const uint32_t rc = q.cnt(a);
        if (s < rc) {
            g.rem = rc - s;
            g.rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + readlane64(off, s))) & ~(uintptr_t)127);
            const uint64_t lim = (uint64_t)(g.rbase - base) + kCap;  // units ending at or below fit the slot
            if constexpr (HYB) {
                if (s == 0) {
                    const uint64_t span = (uint64_t)((base + readlane64(end, rc - 1u)) - g.rbase);
                    const bool big = __builtin_amdgcn_ballot_w64(lane < rc && end - off > kPfxDirectMax) != 0;
                    if (span <= (uint64_t)kPfxDirectRows * kRow && !big) {
                        g.cnt = rc, g.span = (uint32_t)span, g.direct = true;
                        return g;
                    }
                }
            }
            const uint64_t over = __builtin_amdgcn_ballot_w64(lane >= s && lane < rc && end > lim);
            uint32_t fit = over ? (uint32_t)__builtin_ctzll(over) - s : g.rem;
            if (fit < g.rem) fit &= ~(ALIGN - 1u);
            g.cnt = fit;
            if (fit) g.span = (uint32_t)((base + readlane64(end, s + fit - 1u)) - g.rbase);
        }
        return g;
    };
    u32x4 V[VR];
    auto issue = [&](const Piece& g) {  // rows past the piece: out of the descriptor's range, 0, no traffic
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(g.rbase, g.cnt ? (g.span + 3u) & ~3u : 0u);
#pragma unroll
        for (uint32_t r = 0; r < VR; ++r) V[r] = bld16<true>(rs, r * kRow + lane * 16u);
    };
    auto live_of = [&](const Piece& g) { return lane >= g.s && lane < g.s + g.cnt; };
    auto offs = [&](uint32_t a, uint32_t k) { return load_off(a + lane + k, q.live(a) && a + lane + k <= n); };
    uint32_t a, an;
    uint64_t c_off, c_end, n_off, n_end;
    if (h) {
        a = h->a, an = h->an;
        c_off = h->c_off, c_end = h->c_end, n_off = h->n_off, n_end = h->n_end;
    } else {
        a = q.first();
        c_off = offs(a, 0u), c_end = offs(a, 1u);
        an = q.next(a);
        n_off = offs(an, 0u), n_end = offs(an, 1u);
        q.refill();
    }
    Piece cur = geo(a, 0u, c_off, c_end);
    issue(cur);
    __builtin_amdgcn_s_waitcnt(kWaitVm0);  // nothing in flight at the loop's entry (rx_runs_lds, §7 step 50)
    while (cur.rem) {
        if (!cur.cnt) {
            // The first ALIGN units from s exceed the slot: stream the run's units from s on.
            stream(a, cur.s, cur.rem, c_off, c_end);
            a = an;
            c_off = n_off, c_end = n_end;
            an = q.next(a);
            n_off = offs(an, 0u), n_end = offs(an, 1u);
            q.refill();
            cur = geo(a, 0u, c_off, c_end);
            issue(cur);
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            continue;
        }
        uint32_t total = 0;
        if (HYB && cur.direct) {
            lds_stage<VR>(slot, V, cur.span, lane);
            lds_zero_tail(slot, cur.span, lane);
        } else {
            total = pfx_stage<ROWS, VR>(slot, V, cur.span, lane);
        }
        // The next piece: the rest of this run, or the next run (whose offsets are already loaded).
        const bool adv = cur.cnt == cur.rem;
        Piece nxt;
        if (adv) nxt = geo(an, 0u, n_off, n_end);
        else nxt = geo(a, cur.s + cur.cnt, c_off, c_end);
        issue(nxt);
        const uint32_t an2 = adv ? q.next(an) : an;  // the run after the next, once this run is done (else unused)
        const uint64_t p_off = offs(adv ? an2 : n, 0u), p_end = offs(adv ? an2 : n, 1u);
        q.refill();
        {
            const bool live = live_of(cur);
            const uint32_t p = live ? (uint32_t)((base + c_off) - cur.rbase) : 0u;
            const uint32_t d0 = sdw[p >> 2];
            uint32_t F;  // < 2^32: a slot's bytes
            if (HYB && cur.direct) {
                const uint32_t e = live ? (uint32_t)((base + c_end) - cur.rbase) : 0u;
                F = lds_range_sum(slot, p, e, d0, live);
            } else {
                const lds16 x = slot[p >> 4];
                const uint32_t pre1 = __builtin_amdgcn_sad_u16(x.x, 0u, 0u);
                const uint32_t pre2 = __builtin_amdgcn_sad_u16(x.y, 0u, pre1);
                const uint32_t pre3 = __builtin_amdgcn_sad_u16(x.z, 0u, pre2);
                const uint32_t q = (p >> 2) & 3u;
                const uint32_t pq = q == 0u ? 0u : q == 1u ? pre1 : q == 2u ? pre2 : pre3;
                const uint32_t sp = I[p >> 4] + __builtin_amdgcn_sad_u16(d0 & ((1u << (8u * (p & 3u))) - 1u), 0u, pq);
                const uint32_t sn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sp, 0x130, 0xF, 0xF, false);  // wave_shl:1
                F = (lane == cur.s + cur.cnt - 1u ? total : sn) - sp;
            }
            out(F, p, d0, live, a, cur.s, cur.cnt, c_off, c_end);
        }
        if (adv) {
            a = an, an = an2;
            c_off = n_off, c_end = n_end;
            n_off = p_off, n_end = p_end;
        }
        cur = nxt;
    }
}

// sets (nsx_tune.segs_per_wave): 0 = by the batch's mean segment (below), 1 = runs of one set, 2 = the small-segment
// mode (the LDS form with parked results, two waves per block), 3 = the LDS form in every wave of four per block
// without parking (the form a wave of small segments takes in a batch of larger mean), 5 = runs of NS sets (two in
// the default instantiation) in every wave. (Runs of four sets, round 2's form for small segments, §7 step 42, lost
// to one or two sets once results were parked, §7 step 64, and were removed.)
// run: segments per run (0 = default: 63 per boundary set, 64 per LDS run).
// The default instantiation (NS = 2) is register-capped for 4 waves per SIMD (the default grid's 4 blocks per CU
// must all be resident: their ranges are dealt assuming it); the forced single-set shapes are not.
template <int R, bool VERIFY, bool PIPE, int NS>
__global__ __launch_bounds__(kBlock, NS == 2 ? 4 : 1) void csum_ragged_scan_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, uint32_t n,
    const uint32_t* __restrict__ partial, uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t run, int sets,
    uint32_t big_keep, bool park, uint32_t* __restrict__ deal) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    WaveStamps ws;
    ws.entry();
    const __amdgpu_buffer_rsrc_t ofs = make_rsrc(offsets, ((uint64_t)n + 1) * 8);
    const __amdgpu_buffer_rsrc_t prs = make_rsrc(partial, partial ? (uint64_t)n * 4 : 0);
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out, out ? (uint64_t)n * 2 : 0);
    const __amdgpu_buffer_rsrc_t oks = make_rsrc(ok, VERIFY ? (uint64_t)n : 0);
    extern __shared__ lds16 lds_scan[];
    const uint32_t lds_run = run ? run : kWave, scan_run = run ? run : kScanRun;
    // the parked output (the raw sums; the batch verify's verdicts) and whether the verify also writes raw sums
    const void* pout = VERIFY ? static_cast<const void*>(ok) : static_cast<const void*>(out);
    const bool raw = out != nullptr;
    // XCD-contiguous numbering of the blocks, wpb of each block's waves taking ranges
    auto wave_no = [&](uint32_t nb, uint32_t wpb) {
        const uint32_t b = blockIdx.x;
        return (nb >= 16 && (nb & 7) == 0) ? ((b & 7) * (nb >> 3) + (b >> 3)) * wpb + wave : b * wpb + wave;
    };
    // The small-segment mode (§7 step 61): a batch whose mean segment is under kScanLdsSeg bytes is summed out of LDS
    // by waves 0-1 of every block (equal-count ranges cut at multiples of 64 segments), each with two of the block's
    // four slots — one for the run's rows, one for its parked results.
    if (sets == 2 || (NS == 2 && sets == 0 && run == 0 &&
                      ld_off(ofs, n) - ld_off(ofs, 0) < (uint64_t)kScanLdsSeg * n)) {
        if (wave >= 2u) return;
        const uint32_t nb = gridDim.x, W = nb * 2u, g = wave_no(nb, 2u);
        lds16* slot = lds_scan + wave * (2u * kScanSlot / 16u);
        if (lds_run == kWave) {
            // runs of 64, results parked: the batch's last eighth dealt to the waves as they finish (the receive
            // pass's DealtRuns), with heads for this launch
            DealtRuns q = deal_runs(ofs, n, g, W, lane, kScanLdsSeg, 1u, kWave, deal);
            ragged_runs_lds<R, VERIFY, PIPE, true>(base, ofs, n, prs, ors, oks, kWave, q, lane, slot,
                                                   partial != nullptr, pout, raw);
        } else {  // tune.run_segs (tests): shorter runs, stored run by run
            const WaveRange wr = wave_range(ofs, n, g, W, lane, kScanLdsSeg, 1u, kWave);
            StaticRuns q{wr.a0, wr.a_end, lds_run};
            ragged_runs_lds<R, VERIFY, PIPE, false>(base, ofs, n, prs, ors, oks, lds_run, q, lane, slot,
                                                    partial != nullptr, pout, raw);
        }
        return;
    }
    // The grid is sized for small segments (4 blocks/CU); on the default grid (big_keep ≠ 0) streamed batches take
    // 3 of them, batches averaging ≥ kScanBigMean bytes big_keep (2).
    const uint64_t tot = ld_off(ofs, n) - ld_off(ofs, 0);
    const uint32_t nb = active_blocks(ofs, n, 0u, big_keep == 0 ? 0u : tot >= (uint64_t)kScanBigMean * n ? big_keep : 3u);
    if (blockIdx.x >= nb) return;
    // The wave's tasks are runs of NS sets [a_k, a_k + cnt_k) of ≤ run segments each (a_k = a + k·run), a = a0,
    // a0 + NS·run, ... < a_end; a run never crosses a_end. Byte-balanced: wave g (XCD-contiguous numbering) owns
    // the segments that start in the g-th of W equal byte slices of the batch, so every wave streams the same
    // bytes (± one segment) and none is left running alone at the end of the launch.
    // byte shares weighted by the block's slot on its CU (slot_share; 2 or 3 of the 4 blocks per CU active), else
    // equal; one range search either way (a second instance of it cost the kernel ~4% more code)
    SlotShare sh;
    if (kScanSlotWeights && nb >= 64 && (gridDim.x & 31u) == 0 && nb * 4u > gridDim.x && nb % (gridDim.x / 4u) == 0) {
        sh = slot_share(nb, kWavesPerBlock, wave, gridDim.x >> 5, kScanSlotW);
    } else {
        const uint32_t g = wave_no(nb, kWavesPerBlock);
        sh = SlotShare{g, g + 1u, nb * kWavesPerBlock};
    }
    const WaveRange wr = wave_range_w(ofs, n, sh.lo, sh.hi, sh.T, lane, kScanLdsSeg, 1u);
    const uint32_t a0 = wr.a0, a_end = wr.a_end;
    const uint64_t wave_bytes = wr.bytes;
    ws.ready();
    // A wave whose own segments average under kScanLdsSeg bytes sums them out of LDS (§7 step 44); the others stream
    // runs of two 63-segment sets under kScanTwoSetSeg, else of one (§7 step 64: with results parked, one set beat
    // four at every mean from 160 B to 4.5 KB, by up to 9%, and two from ~400 B; two sets ran 3-5% faster at a
    // 160 B mean). The streamed forms park their results in the wave's unused LDS slot when the launch has one.
    void* pbuf = park ? static_cast<void*>(lds_scan + wave * (kScanSlot / 16u)) : nullptr;
    if (sets == 3 || (NS == 2 && sets == 0 && wave_bytes < (uint64_t)kScanLdsSeg * (a_end - a0))) {
        StaticRuns q{a0, a_end, lds_run};
        ragged_runs_lds<R, VERIFY, PIPE, false>(base, ofs, n, prs, ors, oks, lds_run, q, lane,
                                                lds_scan + wave * (kScanSlot / 16u), partial != nullptr, pout, raw);
    } else if (NS == 2 && (sets == 5 || (sets == 0 && wave_bytes < (uint64_t)kScanTwoSetSeg * (a_end - a0)))) {
        ragged_runs<R, VERIFY, PIPE, 2>(base, ofs, n, prs, ors, oks, scan_run, a0, a_end, lane, pbuf, pout, raw);
    } else {
        ragged_runs<R, VERIFY, PIPE, 1>(base, ofs, n, prs, ors, oks, scan_run, a0, a_end, lane, pbuf, pout, raw);
    }
    ws.done(wave_no(nb, kWavesPerBlock), wave_bytes, lane);
}

// ---------------------------------------------------------------------------
// Fused receive pass (SURVEY.md §8 f2 + f3 in one launch): a batch of received
// IPv4 datagrams carrying TCP, densely packed (frame i = base[offsets[i],
// offsets[i+1]), any alignment). Per frame: the IPv4 header checksum (RFC 791),
// the TCP pseudo-header built from that header's own src/dst (ip.Addr.Raw(),
// network/ip/v4/ipv4.go:15; protocol ip.NextProtoTCP = 6, network/ip/
// protocols.go:8; TCP length = total length − IHL·4) and the TCP checksum over
// pseudo ‖ segment with the receiver rule raw == 0xFFFF (tcp.go:70, :72-95),
// into one validity bit per frame.
//
// The frames of a run stream exactly like the ragged scan kernel's segments
// (scan_span: one pass over the bytes, S sampled at every frame start), so a
// frame's weighted sum is F = S(end) − S(start) — with double-buffered row
// batches (scan_span<R, true>): frames of a few hundred bytes put a boundary in
// nearly every row, and the extra scan work per row needs the next batch
// already in flight (a pipelined ragged scan over config 3's 4.5 KB segments
// measured 3.7% slower). Each lane also loads its own
// frame's first 20 header bytes (plus the option dwords when some lane has
// IHL > 5): H = the header's weighted sum, computed in registers — those lines
// are the run's own first bytes, read again from cache — and the TCP segment's
// sum is F − H, exact. Runs are 64 frames starting at a multiple of 8, so each
// run's ballot is whole mask bytes (rx_store_mask).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap16u(uint32_t v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }

constexpr uint32_t kRxRun = 64;

// The receive pass's outputs: the validity mask, and the optional IPv4 header / TCP raw sums. raw (wave-uniform):
// either raw output is present; without one the per-frame raw stores are not issued at all (a store to an empty
// descriptor is dropped, but still an instruction through the memory pipeline per frame set).
struct RxOuts {
    __amdgpu_buffer_rsrc_t mrs, irs, trs;
    bool raw;
    // The streamed form's raw sums parked in the wave's LDS slot (§7 step 67; buf null in the LDS, hybrid and prefix
    // forms, whose slots hold rows): IPv4 header sums and TCP sums, 2048 each (IPv6: TCP sums, 4096).
    mutable ResultPark<uint16_t> ipk, tpk;
};

__device__ __forceinline__ RxOuts rx_outs(uint64_t* mask, uint16_t* ip_raw, uint16_t* tcp_raw, uint32_t n) {
    const __amdgpu_buffer_rsrc_t irs = make_rsrc(ip_raw, ip_raw ? (uint64_t)n * 2 : 0);
    const __amdgpu_buffer_rsrc_t trs = make_rsrc(tcp_raw, tcp_raw ? (uint64_t)n * 2 : 0);
    return RxOuts{make_rsrc(mask, (((uint64_t)n + 63) / 64) * 8), irs, trs, ip_raw != nullptr || tcp_raw != nullptr,
                  make_park<uint16_t>(nullptr, irs, ip_raw, 0), make_park<uint16_t>(nullptr, trs, tcp_raw, 0)};
}

// A run's validity ballot (frames [a, a + cnt), a a multiple of 8) as mask bytes a/8 ..: one byte per lane
// (lanes 0-7), so wave ranges need only be cut at multiples of 8 frames, not at whole 64-bit words; the
// batch's last run also zero-fills the rest of the mask's last word.
// A piece of the run (the prefix form's frames [a + s, a + s + cnt), s a multiple of 8, bits still indexed by lane
// = frame − a) writes only its own bytes s/8 ...
__device__ __forceinline__ void rx_store_mask(__amdgpu_buffer_rsrc_t mrs, uint64_t bits, uint32_t a, uint32_t cnt,
                                              uint32_t n, uint32_t lane, uint32_t s = 0) {
    const uint32_t nbytes = (uint64_t)a + s + cnt >= n ? (uint32_t)((((uint64_t)n + 63u) / 64u) * 8u - a / 8u)
                                                       : (s + cnt + 7u) / 8u;
    const uint32_t v = lane < 8u ? (uint32_t)(bits >> (8u * lane)) & 0xFFu : 0u;
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, mrs, lane >= s / 8u && lane < nbytes ? a / 8u + lane : kOOB, 0, 0);
}

// V6: IPv6 packets (RFC 8200 §3: fixed 40-byte header, Next Header 6 = TCP directly). There is no header
// checksum, and the pseudo-header's addresses (RFC 8200 §8.1) are the header's own bytes 8-39, which the frame
// sum F already holds in the same word pairing as the pseudo-header ‖ segment sum; so TCP sum =
// fold(F − bytes 0-7) + payload length + 6 (the pseudo-header's length and next-header words), and the header
// window is only the first 8 bytes (one 16 B load per lane).
//
// NS: 64-frame sets per run (one stream, one boundary slot per set and lane). Runs of one set suit the bench's
// 40-1500 B frames (~50 KB per run; two sets ran 7.6% slower). A wave whose frames average
// under kRxSmallFrame bytes takes the LDS form instead (rx_runs_lds, §7 step 43), which replaced round 2's runs of
// four sets (§7 step 41).
constexpr uint32_t kRxSmallFrame = 128;
// The pre-prefix shapes (rows / blocks_per_cu set): 4 blocks/CU for batches whose mean frame is under kRxBigMean,
// else 3 (profiles/r03_grid_sweep.txt: 4 blocks 9% faster at a
// 170 B mean, 3.4% at 320 B, 0.4% at 520 B; 3 blocks 2.9% faster at workload 10's 770 B)
constexpr uint32_t kRxBigMean = 640;

// Per-frame verdict of the receive pass, shared by every form, in two halves: rx_hdr parses the frame's header
// window and sums its header (what a form must take while the window is at hand), rx_verdict takes the frame's
// weighted byte sum F (exact; weights 1 / 256 at even / odd addresses, the LE half-sum rule) and writes the run's
// mask bytes and the raw sums. d[0..5] = the dwords from the frame's start rounded down to 4 B (hd = start & 3;
// IPv6 reads d[0..2]); opt(o) fills the IPv4 option dwords 6..15, called only when some lane has IHL > 5.
//
// Everything is summed in F's own domain (round 5): F is the BE one's-complement sum for an
// odd start and its byte swap for an even one, and a byte swap is a multiplication by 256 modulo 0xFFFF (256·256 ≡ 1),
// so the pseudo-header words are added in that domain too — rotated by the frame's start parity like the header
// dwords, the length term shifted up a byte for an even start — and the receiver rule (raw == 0xFFFF, tcp.go:70)
// is checked on fold(F − header + pseudo) directly: 0xFFFF is its own byte swap and every sum here is nonzero (the
// pseudo part alone is ≥ 6), so the verdict equals the BE raw sum's. Only a caller asking for raw sums pays the
// swap back to BE (round 4 swapped and folded both sums per frame on every call). The IPv4 header check is
// fold(hs) == 0xFFFF, likewise swap-free.
struct RxHdr {
    uint32_t hs;   // the header's weighted sum (IPv6: bytes 0-7), subtracted from F when hdr_ok
    uint32_t aux;  // the pseudo-header's words not in F, in F's domain: IPv4 src + dst + 6 + TCP length; IPv6 payload
                   // length + 6
    bool hdr_ok, well;
};

// 16-bit byte swap of a value ≤ 0xFFFF: one v_perm_b32 (bytes 1, 0 of x; zeros above)
__device__ __forceinline__ uint32_t swap16(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0C0C0001u); }

// Frame lengths as the form has them: 64-bit in the streamed form (frames of any length), 32-bit where a frame lies
// in a wave's slot (the LDS, hybrid and prefix forms: e − p < 2^15), which keeps the parse's compares single-word.
template <bool V6, typename Len, typename OptFn>
__device__ __forceinline__ RxHdr rx_hdr(const uint32_t (&d)[6], uint32_t hd, Len flen, bool live, OptFn&& opt) {
    const uint32_t rot = hd & 1u;         // F's domain: the frame-relative dwords rotated one byte for an odd start
    const uint32_t sh = (rot ^ 1u) << 3;  // ... and a BE term shifted up a byte for an even one
    if constexpr (V6) {
        const uint32_t H0 = __builtin_amdgcn_alignbyte(d[1], d[0], hd);  // version, class, flow label
        const uint32_t H1 = __builtin_amdgcn_alignbyte(d[2], d[1], hd);  // payload length, next header
        const uint32_t plen = swap16(H1 & 0xFFFFu);
        const bool well = live && flen >= (Len)40 && (H0 & 0xF0u) == 0x60u && (Len)(plen + 40u) == flen &&
                          ((H1 >> 16) & 0xFFu) == 6u && plen >= 20u;  // tcp.go:131
        const uint32_t h8 = __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(H1, H1, rot), 0u,
                                                     __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(H0, H0, rot), 0u, 0u));
        return RxHdr{h8, (plen + 6u) << sh, true, well};  // F − h8 = addresses ‖ segment
    } else {
        // IPv4 header fields (RFC 791 §3.1): header dword m = bytes 4m..4m+3, little-endian view.
        const uint32_t H0 = __builtin_amdgcn_alignbyte(d[1], d[0], hd);
        const uint32_t H1 = __builtin_amdgcn_alignbyte(d[2], d[1], hd);
        const uint32_t H2 = __builtin_amdgcn_alignbyte(d[3], d[2], hd);
        const uint32_t H3 = __builtin_amdgcn_alignbyte(d[4], d[3], hd);
        const uint32_t H4 = __builtin_amdgcn_alignbyte(d[5], d[4], hd);
        const uint32_t ihl = H0 & 15u, hlen = ihl * 4u;
        const uint32_t total = swap16(H0 >> 16);
        const uint32_t frag = H1 >> 16;  // flags + fragment offset, byte-swapped: the 0x3FFF field is 0xFF3F here
        const uint32_t proto = (H2 >> 8) & 0xFFu;
        const bool hdr_ok = live && flen >= (Len)20 && ihl >= 5u && (Len)hlen <= flen;
        const bool well = hdr_ok && (H0 & 0xF0u) == 0x40u && (Len)total == flen && (frag & 0xFF3Fu) == 0u &&
                          proto == 6u && total - hlen >= 20u;  // tcp.go:131: a segment is at least 20 bytes
        // Header sum over bytes [start, start + hlen), hlen = 4·IHL: the frame-relative dwords H_j, j < IHL, whole.
        // F weights bytes by address parity (the LE half-sum rule), so for an odd start each H_j is rotated one
        // byte before its v_sad_u16 (the halves then pair byte 1 with 2 and 3 with 0): no byte masks (round 2's
        // keep_mask per window dword cost ~45 VALU per frame set).
        auto hsum = [&](uint32_t h, uint32_t acc) {
            return __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(h, h, rot), 0u, acc);
        };
        uint32_t hs = hsum(H4, hsum(H3, hsum(H2, hsum(H1, hsum(H0, 0u)))));
        if (__builtin_amdgcn_ballot_w64(hdr_ok && ihl > 5u)) {  // option dwords 6..15
            uint32_t o[10];
            opt(o);
            uint32_t lo = d[5];
#pragma unroll
            for (int j = 5; j < 15; ++j) {  // H_j = window bytes hd + 4j .. hd + 4j + 3
                const uint32_t hj = __builtin_amdgcn_alignbyte(o[j - 5], lo, hd);
                hs = (uint32_t)j < ihl ? hsum(hj, hs) : hs;
                lo = o[j - 5];
            }
        }
        // Pseudo-header source and destination (header dwords 3-4) and 0, 6, TCP length, in F's domain: the
        // address dwords rotated like the header's (BE words for an odd start, LE half-sums — the swapped words — for
        // an even one), the constant words shifted up a byte for an even start.
        const uint32_t pseudo = hsum(H4, hsum(H3, (6u + ((total - hlen) & 0xFFFFu)) << sh));
        return RxHdr{hs, pseudo, hdr_ok, well};
    }
}

template <bool V6, typename Sum>
__device__ __forceinline__ void rx_verdict(Sum F, const RxHdr& h, bool even, bool live, uint32_t ak, uint32_t cnt,
                                           uint32_t n, uint32_t lane, const RxOuts& ro, uint32_t s) {
    const Sum T = F - (Sum)(h.hdr_ok ? h.hs : 0u);  // the TCP segment's weighted sum (IPv6: addresses ‖ segment)
    uint32_t tle;
    if constexpr (sizeof(Sum) == 8) tle = fold32((uint32_t)T) + fold32((uint32_t)(T >> 32));
    else tle = fold32(T);
    const uint32_t tf = fold32(tle + h.aux);  // ≡ the raw TCP sum, in F's domain (≥ 1)
    const uint32_t ipf = fold32(h.hs);        // ≡ the IPv4 header's raw sum, in F's domain
    const uint64_t bits = __builtin_amdgcn_ballot_w64(h.well && (V6 || ipf == 0xFFFFu) && tf == 0xFFFFu);
    rx_store_mask(ro.mrs, bits, ak, cnt, n, lane, s);
    if (ro.raw) {  // the raw sums in BE (tcp.go:94): back out of F's domain
        const uint32_t tcpr = h.well ? (even ? swap16(tf) : tf) : 0u;
        const uint32_t ipr = h.hdr_ok ? (even ? swap16(ipf) : ipf) : 0u;
        if (ro.tpk.buf) {  // parked (the streamed form: frames [ak, ak + cnt), live = lane < cnt)
            if constexpr (!V6) park_put(ro.ipk, ak, cnt, lane, ipr);
            park_put(ro.tpk, ak, cnt, lane, tcpr);
        } else {
            if constexpr (!V6)
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)ipr, ro.irs, live ? (ak + lane) * 2u : kOOB, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)tcpr, ro.trs, live ? (ak + lane) * 2u : kOOB, 0, 0);
        }
    }
}

template <bool V6, typename Sum, typename Len, typename OptFn>
__device__ __forceinline__ void rx_frame_out(Sum F, const uint32_t (&d)[6], uint32_t hd, Len flen, bool even,
                                             bool live, uint32_t ak, uint32_t cnt, uint32_t n, uint32_t lane,
                                             const RxOuts& ro, OptFn&& opt, uint32_t s = 0) {
    rx_verdict<V6>(F, rx_hdr<V6>(d, hd, flen, live, opt), even, live, ak, cnt, n, lane, ro, s);
}

// One run of NS sets of ≤ 64 frames in the streaming form: frame a + 64k + lane = [my_off[k], my_end[k]) for
// lane < cnt[k]; kl = the last set with frames.
template <int R, bool V6, int NS>
__device__ __forceinline__ void rx_run_stream(const uint8_t* __restrict__ base, uint32_t a, const uint32_t (&cnt)[NS],
                                              const uint64_t (&my_off)[NS], const uint64_t (&my_end)[NS], uint32_t kl,
                                              uint32_t n, uint32_t lane, const RxOuts& ro) {
    {
        const uint64_t lo = readlane64(my_off[0], 0);
        uint64_t hi = 0;
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if ((uint32_t)k == kl) hi = readlane64(my_end[k], cnt[k] - 1);
        const uint8_t* rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + lo)) & ~(uintptr_t)127);
        const uint64_t span = (uint64_t)((base + hi) - rbase);
        const uint32_t head = (uint32_t)((uintptr_t)(base + lo) & 127u);
        // Header window: the 4-aligned dwords from the frame start, 24 bytes (a 16 B and an 8 B load per lane)
        // through one descriptor over the run (rbase is 128-aligned, so window offset = brel & ~3); dwords past
        // the run read 0, bytes past the frame or the header are masked below. Issued ahead of the stream:
        // nothing waits for them until the run's last header step. A run wider than a descriptor (2 GiB of
        // frames — only possible behind frames longer than any IPv4 datagram) loads per lane instead.
        constexpr int kWin = V6 ? 3 : 6;  // window dwords: bytes 0-7 (IPv6) / 0-19 (IPv4) at any hd
        const bool narrow = span < (1ull << 31);
        const __amdgpu_buffer_rsrc_t hrs = make_rsrc(rbase, narrow ? ((span + 3) & ~3ull) : 0);
        const uint32_t* last_dw =
            reinterpret_cast<const uint32_t*>((uintptr_t)(base + (hi > lo ? hi - 1 : lo)) & ~(uintptr_t)3);
        int64_t brel[NS];
        uint32_t hwo[NS], d[NS][6];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const bool live = lane < cnt[k];
            brel[k] = live ? (int64_t)((base + my_off[k]) - rbase) : -1;
            hwo[k] = live && narrow ? (uint32_t)brel[k] & ~3u : kOOB;
            typedef uint32_t v2x __attribute__((ext_vector_type(2)));
            const u32x4 q = bld16<false>(hrs, hwo[k]);
            d[k][0] = q.x, d[k][1] = q.y, d[k][2] = q.z, d[k][3] = q.w;
            d[k][4] = d[k][5] = 0u;
            if constexpr (!V6) {
                const v2x r = __builtin_amdgcn_raw_buffer_load_b64(hrs, hwo[k] == kOOB ? kOOB : hwo[k] + 16u, 0, 0);
                d[k][4] = r.x, d[k][5] = r.y;
            }
            if (!narrow && hi > lo) {  // clamped to the run's last readable dword: every lane loads unconditionally
                const uint8_t* fp = base + (live ? my_off[k] : lo);
                const uint32_t* hw = reinterpret_cast<const uint32_t*>(fp - ((uintptr_t)fp & 3u));
#pragma unroll
                for (int j = 0; j < kWin; ++j) d[k][j] = hw + j < last_dw ? hw[j] : *last_dw;
            }
        }
        // The run's bytes, S sampled at every frame start.
        uint64_t bval[NS], carry = 0;
#pragma unroll
        for (int k = 0; k < NS; ++k) bval[k] = 0;
        scan_span<R, true, NS>(rbase, span, head, brel, lane, bval, carry);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            if (cnt[k] == 0) break;  // wave-uniform
            const uint32_t ak = a + k * kRxRun;
            const bool live = lane < cnt[k];
            const uint8_t* fp = base + (live ? my_off[k] : lo);
            const uint32_t hd = (uint32_t)((uintptr_t)fp & 3u);
            // a frame ends where the next one starts: the next lane's boundary, the next set's first, or the run's
            // end (the carry)
            uint64_t nxt = (uint64_t)__shfl_down((unsigned long long)bval[k], 1);
            if (lane == cnt[k] - 1) {
                uint64_t e = carry;
#pragma unroll
                for (int j = 0; j < NS; ++j)
                    if (j == k + 1 && (uint32_t)k < kl) e = readlane64(bval[j], 0);
                nxt = e;
            }
            const uint64_t F = nxt - bval[k];  // the frame's weighted sum (exact)
            // IPv4 option dwords 6..15 (only when some lane has IHL > 5)
            auto opt = [&](uint32_t (&o)[10]) {
                if (narrow) {
                    typedef uint32_t v2x __attribute__((ext_vector_type(2)));
                    const uint32_t w = hwo[k] == kOOB ? kOOB : hwo[k] + 24u;
                    const u32x4 q0 = bld16<false>(hrs, w), q1 = bld16<false>(hrs, w == kOOB ? kOOB : w + 16u);
                    const v2x r = __builtin_amdgcn_raw_buffer_load_b64(hrs, w == kOOB ? kOOB : w + 32u, 0, 0);
                    o[0] = q0.x, o[1] = q0.y, o[2] = q0.z, o[3] = q0.w, o[4] = q1.x, o[5] = q1.y, o[6] = q1.z;
                    o[7] = q1.w, o[8] = r.x, o[9] = r.y;
                } else {
                    const uint32_t* hw = reinterpret_cast<const uint32_t*>(fp - hd);
#pragma unroll
                    for (int j = 6; j < 16; ++j) o[j - 6] = hw + j < last_dw ? hw[j] : *last_dw;
                }
            };
            rx_frame_out<V6>(F, d[k], hd, my_end[k] - my_off[k], ((uintptr_t)fp & 1u) == 0, live, ak, cnt[k], n, lane,
                             ro, opt);
        }
    }
}

template <int R, bool V6, int NS>
__device__ __forceinline__ void rx_runs(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                        uint32_t a0, uint32_t a_end, uint32_t lane, const RxOuts& ro) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    auto load_off = [&](uint32_t i, bool live) -> uint64_t {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, live ? i * 8 : kOOB, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    constexpr uint32_t kStep = kRxRun * NS;
    // lane l of set k: offsets[a + 64k + l] and offsets[a + 64k + l + 1] of the next run, prefetched one run ahead
    uint64_t nxt_off[NS], nxt_end[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const uint32_t an = a0 + k * kRxRun;
        nxt_off[k] = load_off(an + lane, an < a_end && an + lane <= n);
        nxt_end[k] = load_off(an + lane + 1, an < a_end && an + lane + 1 <= n);
    }
    for (uint32_t a = a0; a < a_end; a += kStep) {
        uint32_t cnt[NS];
        uint64_t my_off[NS], my_end[NS];  // frame a + 64k + lane = [my_off[k], my_end[k]) for lane < cnt[k]
        uint32_t kl = 0;                  // the last set with frames (only a wave's last run has fewer sets)
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const uint32_t ak = a + k * kRxRun;
            cnt[k] = ak < a_end ? min(kRxRun, a_end - ak) : 0u;
            kl = cnt[k] ? (uint32_t)k : kl;
            my_off[k] = nxt_off[k], my_end[k] = nxt_end[k];
            const uint32_t an = ak + kStep;
            nxt_off[k] = load_off(an + lane, an < a_end && an + lane <= n);
            nxt_end[k] = load_off(an + lane + 1, an < a_end && an + lane + 1 <= n);
        }
        rx_run_stream<R, V6, NS>(base, a, cnt, my_off, my_end, kl, n, lane, ro);
    }
}

// ---- The streamed modes' tail, dealt through the block's LDS (round 6) ----
// With equal static shares the streamed receive pass (workloads 10, 11, 14: 12 waves per CU, ~5 runs of 64 frames
// each, ~20 µs a run) waited 9-16 µs for its last waves — whole blocks run 3-4 µs apart (the waves of one block end
// within ~1 µs of each other, profiles/r05_rx_wave_times_streamed.txt) — and dealing whole runs from the per-stream
// heads (DealtRuns) would leave a tail of up to a run. Here the batch's last 1/2^kStreamPoolShift of frames is dealt
// in pieces of kStreamPiece frames (~12 KB, ~5 µs), and the ticket round trip (a device-scope atomic, 1-3 µs) is
// kept off the streaming waves altogether: each block runs three streaming waves and one dealer wave (4 blocks × 3
// streaming waves per CU = the 12 of the static layout). The dealer pulls tickets from the stream's heads for the
// pieces its waves have claimed and posts them in an LDS ring; a streaming wave claims its next piece one unit ahead
// (an LDS atomic) and reads it from the ring when it moves on, so no vector-memory wait of a streaming wave ever
// covers a ticket (vmcnt retires in issue order: loads issued behind an atomic wait for it too, §7 step 72).
#ifndef NSX_STREAM_PIECE
#define NSX_STREAM_PIECE 16
#endif
#ifndef NSX_STREAM_POOL_SHIFT
#define NSX_STREAM_POOL_SHIFT 3
#endif
constexpr uint32_t kStreamPiece = NSX_STREAM_PIECE;          // frames per dealt piece (a multiple of 8: whole mask bytes)
constexpr uint32_t kStreamPoolShift = NSX_STREAM_POOL_SHIFT;  // the pool: the batch's last eighth of frames
constexpr uint32_t kStreamWaves = 3;       // streaming waves per block (wave 3 deals)
#ifndef NSX_STREAM_AHEAD
#define NSX_STREAM_AHEAD 0
#endif
constexpr uint32_t kStreamAhead = NSX_STREAM_AHEAD;  // entries the dealer posts beyond the claimed ones
#ifndef NSX_STREAM_ROTATE
#define NSX_STREAM_ROTATE 0
#endif
constexpr bool kStreamRotate = NSX_STREAM_ROTATE;
#ifndef NSX_STREAM_DEAL
#define NSX_STREAM_DEAL 0
#endif
constexpr bool kStreamDeal = NSX_STREAM_DEAL;  // the dealt streamed layout (A/B builds; the default: slot shares)

// A streaming wave's units: its static runs [a0, e_st) of kRxRun frames, then dealt pieces until the share ends
// (n). The entry for the unit after next is claimed when next() hands out a unit whose successor is a piece, and
// read when next() moves on to it.
struct RingRuns {
    uint32_t a0, e_st, n;
    RingClient rc;
    uint32_t pend;  // the claimed entry not yet read (kPieceFree: none)
    __device__ __forceinline__ uint32_t claim() const { return rc.claim(); }
    __device__ __forceinline__ uint32_t read(uint32_t idx) const { return rc.read(idx, n); }
    // after handing out unit r: is its successor a piece? then claim that piece's entry now
    __device__ __forceinline__ uint32_t ahead(uint32_t r) {
        if (r < n && (r >= e_st || r + kRxRun >= e_st)) pend = claim();
        return r;
    }
    __device__ __forceinline__ uint32_t first() {
        if (a0 < e_st) return ahead(a0);
        return ahead(read(claim()));
    }
    __device__ __forceinline__ uint32_t next(uint32_t a) {
        uint32_t r;
        if (a + kRxRun < e_st) {
            r = a + kRxRun;
        } else {
            r = pend == kPieceFree ? n : read(pend);
            pend = kPieceFree;
        }
        return ahead(r);
    }
    __device__ __forceinline__ uint32_t cnt(uint32_t a) const {
        return a < e_st ? min(kRxRun, e_st - a) : min(kStreamPiece, n - a);
    }
};

// A streaming wave's units (RingRuns) in the streaming form, the offsets of the next unit loaded one unit ahead.
template <int R, bool V6>
__device__ __forceinline__ void rx_runs_ring(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                             RingRuns& q, uint32_t lane, const RxOuts& ro) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    auto load_off = [&](uint32_t i, bool live) -> uint64_t {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, live ? i * 8 : kOOB, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    uint32_t a = q.first();
    uint64_t no = load_off(a + lane, a < n && a + lane <= n), ne = load_off(a + lane + 1, a < n && a + lane + 1 <= n);
    while (a < n) {
        uint32_t cnt[1] = {q.cnt(a)};
        uint64_t my_off[1] = {no}, my_end[1] = {ne};
        const uint32_t an = q.next(a);
        no = load_off(an + lane, an < n && an + lane <= n);
        ne = load_off(an + lane + 1, an < n && an + lane + 1 <= n);
        rx_run_stream<R, V6, 1>(base, a, cnt, my_off, my_end, 0u, n, lane, ro);
        a = an;
    }
}

// The LDS form of the receive pass, for waves of small frames. A run of 64 frames whose
// bytes fit kRxSlotRows rows is staged whole into the wave's LDS slot — coalesced 16 B-per-lane row loads, issued
// one run ahead (the next run's rows are in flight while this one is summed), then ds_write_b128 — and each lane
// sums ITS OWN frame out of LDS: the frame's 16 B chunks (ds_read_b128, eight in flight per lane), minus the bytes
// of the first chunk before the frame and of the last chunk past it; its header window comes from the slot too
// (no second fetch of the header bytes). No boundary scan, no ds_bpermute, no per-row ballots: per frame the work
// is its own length. A run whose bytes do not fit (a large frame among small ones) takes the streaming form.
constexpr uint32_t kRxSlotRows = 8;
constexpr uint32_t kRxSlot = kRxSlotRows * kRow + 256;  // + pad: a header window or chunk block read past the end

// The receive pass in the prefix form (pfx_runs: pieces cut at whole mask bytes; the header window from the slot).
template <int R, bool V6, uint32_t ROWS, bool HYB, typename Seq>
__device__ __forceinline__ void rx_runs_pfx(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                            Seq& q, uint32_t lane, lds16* slot, const RxOuts& ro,
                                            const RunHead* h = nullptr) {
    static_assert(kPfxRun == kRxRun && kPfxDirectSlot == kRxSlot, "the receive pass's runs and direct slot");
    const uint32_t* sdw = reinterpret_cast<const uint32_t*>(slot);
    auto out = [&](uint32_t F, uint32_t p, uint32_t d0, bool live, uint32_t a, uint32_t s, uint32_t cnt, uint64_t off,
                   uint64_t end) {
        const uint32_t w0 = p >> 2;
        uint32_t d[6];
        d[0] = d0;
#pragma unroll
        for (int j = 1; j < (V6 ? 3 : 6); ++j) d[j] = sdw[w0 + j];
        if constexpr (V6) d[3] = d[4] = d[5] = 0u;
        auto opt = [&](uint32_t (&o)[10]) {
#pragma unroll
            for (int j = 6; j < 16; ++j) o[j - 6] = sdw[w0 + j];
        };
        // a live frame lies in the slot (< 2^15 bytes): its length from the offsets' low words
        rx_frame_out<V6>(F, d, p & 3u, (uint32_t)end - (uint32_t)off, (p & 1u) == 0, live, a, cnt, n, lane, ro, opt, s);
    };
    auto stream = [&](uint32_t a, uint32_t s, uint32_t rem, uint64_t off, uint64_t end) {  // lanes shifted by s
        uint32_t cnt1[1] = {rem};
        uint64_t o1[1] = {(uint64_t)__shfl_down((unsigned long long)off, s)};
        uint64_t e1[1] = {(uint64_t)__shfl_down((unsigned long long)end, s)};
        rx_run_stream<R, V6, 1>(base, a + s, cnt1, o1, e1, 0u, n, lane, ro);
    };
    pfx_runs<ROWS, HYB, 8u>(base, ofs, n, q, lane, slot, out, stream, h);
}

template <bool V6>
__device__ __forceinline__ void rx_run_lds(const uint8_t* __restrict__ base, const uint8_t* rbase, uint32_t a,
                                           uint32_t cnt, uint64_t my_off, uint64_t my_end, uint32_t n, uint32_t lane,
                                           const lds16* slot, const RxOuts& ro) {
    const uint32_t* sdw = reinterpret_cast<const uint32_t*>(slot);
    const bool live = lane < cnt;
    // frame position in the slot (rbase is 128-aligned, so the slot keeps every byte's address mod 128)
    const uint32_t p = live ? (uint32_t)((base + my_off) - rbase) : 0u;
    const uint32_t e = live ? (uint32_t)((base + my_end) - rbase) : 0u;
    const uint32_t hd = p & 3u, w0 = p >> 2;
    uint32_t d[6];
#pragma unroll
    for (int j = 0; j < (V6 ? 3 : 6); ++j) d[j] = sdw[w0 + j];
    if constexpr (V6) d[3] = d[4] = d[5] = 0u;
    const uint32_t F = lds_range_sum(slot, p, e, d[0], live);  // the frame's weighted sum (< 2^32: ≤ 8 KiB)
    auto opt = [&](uint32_t (&o)[10]) {
#pragma unroll
        for (int j = 6; j < 16; ++j) o[j - 6] = sdw[w0 + j];
    };
    rx_frame_out<V6>(F, d, hd, e - p, (p & 1u) == 0, live, a, cnt, n, lane, ro, opt);
}

// A wave's runs [a0, a_end) in the LDS form (runs of 64 frames from a multiple of 8, as rx_runs).
// SW (the default grid's small-frame mode, §7 step 59): a run that is not a direct run — too wide for the slot, or
// holding a frame over kPfxDirectMax bytes, which one lane would sum alone — hands the rest of the wave's range to the
// hybrid loop (rx_runs_pfx<·, 7, true>) instead of being streamed; waves of ACKs alone stay in this tighter loop.
template <int R, bool V6, bool SW = false, typename Seq>
__device__ __forceinline__ void rx_runs_lds(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                            Seq& q, uint32_t lane, lds16* slot, const RxOuts& ro) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    auto load_off = [&](uint32_t i, bool live) -> uint64_t {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(ofs, live ? i * 8 : kOOB, 0, 0);
        return ((uint64_t)x.y << 32) | x.x;
    };
    auto offs = [&](uint32_t a, uint32_t k) { return load_off(a + lane + k, q.live(a) && a + lane + k <= n); };
    struct Run {
        const uint8_t* rbase;
        uint64_t span;
        uint32_t cnt;
        bool lds;
    };
    auto geo = [&](uint32_t a, uint64_t off, uint64_t end) {  // wave-uniform geometry of run a
        Run g{base, 0, q.cnt(a), false};
        if (g.cnt) {
            const uint64_t lo = readlane64(off, 0), hi = readlane64(end, g.cnt - 1u);
            g.rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + lo)) & ~(uintptr_t)127);
            g.span = (uint64_t)((base + hi) - g.rbase);
            g.lds = g.span <= (uint64_t)kRxSlotRows * kRow;
            if constexpr (SW) g.lds = g.lds && !__builtin_amdgcn_ballot_w64(lane < g.cnt && end - off > kPfxDirectMax);
        }
        return g;
    };
    u32x4 V[kRxSlotRows];
    auto issue = [&](const Run& g) {  // rows past the run: out of the descriptor's range, 0, no traffic
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(g.rbase, (g.span + 3) & ~3ull);
#pragma unroll
        for (uint32_t r = 0; r < kRxSlotRows; ++r) V[r] = bld16<true>(rs, r * kRow + lane * 16u);
    };
    // The LDS loop runs while consecutive runs fit the slot; a run that does not is streamed on its own in the
    // outer loop. (Kept apart so that the streaming form's loads still in flight at its end — its pipeline issues
    // one empty batch past the run — never merge into the LDS loop's wait counts: at a merge hipcc waits
    // vmcnt(0) before reusing such a register, which drained the next run's rows right after their issue.)
    // The next run and its offsets are always known one run ahead (before a streamed run, or by the LDS loop), so
    // that a switch between the forms does not wait for them (§7 step 53); they are carried across the switch.
    uint32_t a = q.first();
    uint64_t c_off = offs(a, 0u), c_end = offs(a, 1u);
    uint32_t an = q.next(a);
    uint64_t n_off = offs(an, 0u), n_end = offs(an, 1u);
    q.refill();
    while (q.live(a)) {
        Run cur = geo(a, c_off, c_end);
        if (SW && !cur.lds) {
            const RunHead h{a, an, c_off, c_end, n_off, n_end};
            rx_runs_pfx<R, V6, 7, true>(base, ofs, n, q, lane, slot, ro, &h);
            return;
        }
        if (!cur.lds) {  // a run too wide for the slot: the streaming form
            uint32_t cnt1[1] = {cur.cnt};
            uint64_t o1[1] = {c_off}, e1[1] = {c_end};
            rx_run_stream<R, V6, 1>(base, a, cnt1, o1, e1, 0u, n, lane, ro);
            a = an, c_off = n_off, c_end = n_end;
            an = q.next(a);
            n_off = offs(an, 0u), n_end = offs(an, 1u);
            q.refill();
            continue;
        }
        issue(cur);
        // Enter the loop with nothing in flight (the first run's rows and offsets are read at its head anyway). With
        // them pending, hipcc's wait-count pass merged the entry edge into the loop head and waited vmcnt(0) in
        // every iteration before reading the next run's offsets — a wait on the previous run's result stores,
        // ahead of the next run's row loads.
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        for (;;) {
            lds_stage<kRxSlotRows>(slot, V, cur.span, lane);
            lds_zero_tail(slot, cur.span, lane);
            Run nxt = geo(an, n_off, n_end);
            if (!nxt.lds) nxt.span = 0;  // the rows of a run that will be streamed are not staged: empty loads
            issue(nxt);
            const uint32_t an2 = q.next(an);
            const uint64_t p_off = offs(an2, 0u), p_end = offs(an2, 1u);
            q.refill();
            rx_run_lds<V6>(base, cur.rbase, a, cur.cnt, c_off, c_end, n, lane, slot, ro);
            a = an, an = an2;
            c_off = n_off, c_end = n_end;
            n_off = p_off, n_end = p_end;
            if (!nxt.lds) break;  // the end of the wave's runs, or a run for the outer loop
            cur = nxt;
        }
    }
}


// ---- LDS-DMA: loads that write LDS directly (buffer_load_dwordx4 … lds), no VGPR destination ----
// Issued as inline asm, so that hipcc neither reorders other memory operations across them nor waits for them on its
// own: a wave that uses them counts its vector-memory operations itself and waits with an explicit vmcnt. M0 (the
// LDS destination base, wave-uniform) is set and restored inside the one statement (MI355X guides: M0 is
// compiler-reserved). One wave instruction writes 16 B per active lane at lds_byte + 16·lane.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds_byte) : "memory");
}

// Wait until at most n of this wave's vector-memory operations are outstanding (n wave-uniform; s_waitcnt takes an
// immediate, so n is rounded DOWN to one of the listed counts — waiting for more than asked is always safe).
__device__ __forceinline__ void wait_vm_le(uint32_t n) {
#define NSX_VMW(k) asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory")
    n = __builtin_amdgcn_readfirstlane(n);
    if (n >= 16u) {
        if (n >= 40u) {
            if (n >= 63u) NSX_VMW(63); else if (n >= 56u) NSX_VMW(56); else if (n >= 48u) NSX_VMW(48); else NSX_VMW(40);
        } else if (n >= 28u) {
            if (n >= 34u) NSX_VMW(34); else if (n >= 31u) NSX_VMW(31); else NSX_VMW(28);
        } else {
            if (n >= 25u) NSX_VMW(25); else if (n >= 22u) NSX_VMW(22); else if (n >= 19u) NSX_VMW(19); else NSX_VMW(16);
        }
    } else if (n >= 8u) {
        if (n >= 14u) NSX_VMW(14); else if (n >= 12u) NSX_VMW(12); else if (n >= 10u) NSX_VMW(10); else NSX_VMW(8);
    } else if (n >= 4u) {
        if (n >= 7u) NSX_VMW(7); else if (n >= 6u) NSX_VMW(6); else if (n >= 5u) NSX_VMW(5); else NSX_VMW(4);
    } else {
        if (n >= 3u) NSX_VMW(3); else if (n >= 2u) NSX_VMW(2); else if (n >= 1u) NSX_VMW(1); else NSX_VMW(0);
    }
#undef NSX_VMW
}

// The small-frame mode's LDS loop fed by LDS-DMA through a ring (round 5): rx_runs_lds keeps
// one run's rows in flight (in VGPRs) while it sums another, so its loads stop at every run. Here each run's rows go
// straight from HBM into a ring of LDS run regions packed back to back (a region is the run's span rounded up to 16 B;
// the last row's lanes past the span are masked off, so no region is written past its end), and a wave keeps up to
// two runs in flight beyond the one it sums, as many as the ring holds. Each run's 66 offsets come the same way,
// four runs ahead of the sum, into one of four 528 B areas; the run's geometry and each lane's frame bounds are read
// from there. The wave counts its own vector-memory operations (the DMAs and rx_run_lds's stores) and waits for a
// group with vmcnt(younger operations). The first run that is not a direct run (too wide for 8 rows, or holding a
// frame over kPfxDirectMax bytes) hands the rest of the range to the hybrid loop, after the ring has drained.
// region: the wave's LDS (kRingWave bytes); offsets areas first, then the ring, then a 128 B pad that the chunk and
// header-window reads of a run's last frames may reach.
constexpr uint32_t kRingOffArea = 528;  // 33 lanes × 16 B: offsets[a .. a + 65]
constexpr uint32_t kRingWave = 20480;   // per wave: the default grid's 40 KB blocks hold two
constexpr uint32_t kRingBegin = 4u * kRingOffArea, kRingEnd = kRingWave - 128u;
template <int R, bool V6>
__device__ __forceinline__ void rx_runs_ring(const uint8_t* __restrict__ base, __amdgpu_buffer_rsrc_t ofs, uint32_t n,
                                             uint32_t a0, uint32_t a_end, uint32_t lane, lds16* region,
                                             const RxOuts& ro) {
    const uint32_t reg = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)region);
    const uint8_t* rb8 = reinterpret_cast<const uint8_t*>(region);
    const uint32_t stores_per_run = 1u + (ro.raw ? (V6 ? 1u : 2u) : 0u);  // rx_run_lds: the mask byte (+ raw sums)
    uint32_t vmc = 0;      // this wave's vector-memory operations issued in this loop
    uint32_t om[4];        // vmc right after the offsets DMA of run k (slot k & 3)
    auto om_get = [&](uint32_t k) { k &= 3u; return k == 0 ? om[0] : k == 1 ? om[1] : k == 2 ? om[2] : om[3]; };
    auto om_set = [&](uint32_t k, uint32_t v) {
        k &= 3u;
        om[0] = k == 0 ? v : om[0], om[1] = k == 1 ? v : om[1], om[2] = k == 2 ? v : om[2], om[3] = k == 3 ? v : om[3];
    };
    auto issue_offs = [&](uint32_t r) {  // run index r (a = a0 + 64 r): offsets[a .. a + 65] into area r & 3
        const uint32_t a = a0 + r * kRxRun;
        if (lane < 33u) dma16(ofs, a < a_end ? (a + 2u * lane) * 8u : kOOB, reg + (r & 3u) * kRingOffArea);
        om_set(r, ++vmc);
    };
    auto area_off = [&](uint32_t r, uint32_t l) {  // offsets[a + l] of run r from its area
        return *reinterpret_cast<const uint64_t*>(rb8 + (r & 3u) * kRingOffArea + l * 8u);
    };
    struct Q {
        uint32_t r, cnt, pos, span, mark;
        const uint8_t* rbase;
    };
    const uint32_t nruns = (a_end - a0 + kRxRun - 1u) / kRxRun;
    for (uint32_t r = 0; r < 4u && r < nruns; ++r) issue_offs(r);
    Q q0{}, q1{}, q2{};
    uint32_t qlen = 0, u = 0, last_end = kRingBegin;
    bool stop = false;
    for (;;) {
        // fill: up to two runs in flight beyond the one to be summed, while the ring has room
        while (qlen < 3u && u < nruns && !stop) {
            wait_vm_le(vmc - om_get(u));
            const uint32_t a = a0 + u * kRxRun, cnt = min(kRxRun, a_end - a);
            const uint64_t off = area_off(u, lane), end = area_off(u, lane + 1u);
            const uint64_t lo = readlane64(off, 0), hi = readlane64(end, cnt - 1u);
            const uint8_t* rbase = reinterpret_cast<const uint8_t*>(((uintptr_t)(base + lo)) & ~(uintptr_t)127);
            const uint64_t span = (uint64_t)((base + hi) - rbase);
            if (span > (uint64_t)kRxSlotRows * kRow || __builtin_amdgcn_ballot_w64(lane < cnt && end - off > kPfxDirectMax)) {
                stop = true;  // not a direct run: the hybrid loop takes over from run u
                break;
            }
            const uint32_t f = ((uint32_t)span + 15u) & ~15u;
            uint32_t pos;
            if (qlen == 0u) {
                pos = last_end + f <= kRingEnd ? last_end : kRingBegin;
            } else if (last_end >= q0.pos) {
                if (last_end + f <= kRingEnd) pos = last_end;
                else if (kRingBegin + f <= q0.pos) pos = kRingBegin;
                else break;  // no room until the oldest run is summed
            } else {
                if (last_end + f <= q0.pos) pos = last_end;
                else break;
            }
            // the rows: whole 1 KiB rows, the last one's lanes past the span masked off
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(rbase, (span + 3) & ~3ull);
            const uint32_t rows = __builtin_amdgcn_readfirstlane(((uint32_t)span + kRow - 1u) / kRow);
            for (uint32_t rr = 0; rr + 1u < rows; ++rr) dma16(rs, rr * kRow + lane * 16u, reg + pos + rr * kRow);
            if (rows) {
                const uint32_t lr = rows - 1u;
                if (lr * kRow + lane * 16u < (uint32_t)span) dma16(rs, lr * kRow + lane * 16u, reg + pos + lr * kRow);
            }
            vmc += rows;
            const Q e{u, cnt, pos, (uint32_t)span, vmc, rbase};
            if (qlen == 0u) q0 = e; else if (qlen == 1u) q1 = e; else q2 = e;
            ++qlen;
            last_end = pos + f;
            ++u;
        }
        if (qlen == 0u) break;
        // sum the oldest run
        wait_vm_le(vmc - q0.mark);
        lds16* slot = reinterpret_cast<lds16*>(const_cast<uint8_t*>(rb8) + q0.pos);
        lds_zero_tail(slot, q0.span, lane);
        const uint64_t my_off = area_off(q0.r, lane), my_end = area_off(q0.r, lane + 1u);
        rx_run_lds<V6>(base, q0.rbase, a0 + q0.r * kRxRun, q0.cnt, my_off, my_end, n, lane, slot, ro);
        vmc += stores_per_run;
        // its offsets area is free: the offsets of the run four ahead
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this run's LDS reads are done before the area is refilled
        if (q0.r + 4u < nruns) issue_offs(q0.r + 4u);
        q0 = q1, q1 = q2;
        --qlen;
    }
    wait_vm_le(0u);  // nothing may still be landing in the region the hybrid loop stages into
    const uint32_t a_sw = a0 + u * kRxRun;
    StaticRuns rest{a_sw, a_end};
    if (stop && a_sw < a_end) rx_runs_pfx<R, V6, 7, true>(base, ofs, n, rest, lane, region, ro);
}


// The receive pass's grids by the batch's mean frame m: m <
// kRxPfxMean: two waves per block (§7 step 68), the LDS loop for runs of small frames that fit 8 KiB, handing over at the first
// other run to the hybrid loop (direct pieces for such runs, prefix pieces of ≤ 7 KiB otherwise; §7 step 59);
// kRxPfxMean ≤ m < the streaming threshold: the prefix form with 15-row slots on two waves per block (8 waves per
// CU, ~19 KB of LDS each); above it streamed runs on 3 blocks per CU.
// The streaming threshold depends on the batch's frame count as well as its mean (DESIGN.md §7 step 63,
// profiles/r04_rx_form_sweep.txt: n 1M-8M × means 200-900 B): in batches of up to 2M frames streamed runs win from
// a 500 B mean (by 2-6% at 500-900 B) and lose by 1-23% at 200-400 B; from 3M frames the prefix form wins up to
// a 750 B mean (by 1-3%), streamed runs from 800 B. Fitted per batch size, the prefix form's time has a fixed
// part of ~5-9 µs that large batches amortise (its source is not isolated); the streamed runs' rate is flat in n.
constexpr uint32_t kRxPfxMean = 112;
constexpr uint32_t kRxStreamMeanSmallN = 448;      // the streaming threshold below kRxStreamBigN frames
constexpr uint32_t kRxStreamMeanBigN = 768;        // ... and from kRxStreamBigN frames
constexpr uint32_t kRxStreamBigN = 5u << 19;       // 2.5M frames

// PF = -1: the default grid's kernel (4 blocks/CU, PfxSlot<15> × 2 of LDS per block): sets 0 = by the batch's mean
// frame and frame count (above), 1 = streamed runs on every block, 8 = streamed runs on 3 blocks per CU, 5 = the small-frame mode (LDS loop, then the hybrid
// loop), 6 = the 15-row prefix form on waves 0-1, 7 = the hybrid loop throughout. (The prefix form at 3 and 2 blocks per CU, forced by sets 3 in §7 step 54, was removed once
// the default grid held both of its slots.)
// PF = 0: the shapes set by rows / blocks_per_cu: sets 0 = by the wave's mean frame size (the LDS form below
// kRxSmallFrame, else streamed runs of one 64-frame set); 1 = force the streamed runs; 2 = force the LDS form.
// (Round 2's streamed runs of four sets for small frames, §7 step 41, were removed: the LDS form beat them by
// 30-40% on every small-frame mix, §7 step 43.)
// WPS: waves per SIMD the registers must allow (__launch_bounds__'s second argument): 1 = no constraint (158 VGPRs,
// 3 waves per SIMD at the default 3 blocks/CU); 4 = the 4-blocks/CU instantiations (≤ 128 VGPRs).

template <int R, bool V6, int WPS, int PF = 0>
__global__ __launch_bounds__(kBlock, WPS) void rx_tcp_kernel(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ offsets, uint32_t n,
                                                             uint64_t* __restrict__ mask,
                                                             uint16_t* __restrict__ ip_raw,
                                                             uint16_t* __restrict__ tcp_raw, int sets,
                                                             uint32_t big_keep, uint32_t* __restrict__ deal) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    WaveStamps ws;
    ws.entry();
    const __amdgpu_buffer_rsrc_t ofs = make_rsrc(offsets, ((uint64_t)n + 1) * 8);
    const RxOuts ro = rx_outs(mask, ip_raw, tcp_raw, n);
    extern __shared__ lds16 lds_rx[];
    // Byte-balanced wave ranges (as csum_ragged_scan_kernel), cut at multiples of 8 frames. Cut at whole mask
    // words (64 frames, ~50 KB) instead, a wave streamed up to one run more than the mean, and the launch
    // waited ~20 µs for those waves at any batch size.
    // XCD-contiguous numbering of the blocks; wpb of each block's waves take ranges.
    auto range = [&](uint32_t nb, uint32_t wpb, uint32_t w) {
        return wave_range(ofs, n, wave_number(nb, wpb, w), nb * wpb, lane, kRxSmallFrame, 8u);
    };
    if constexpr (PF < 0) {
        int mode = sets;
        if (sets == 0) {
            const uint64_t tot = ld_off(ofs, n) - ld_off(ofs, 0);
            const uint64_t stream_mean = n >= kRxStreamBigN ? kRxStreamMeanBigN : kRxStreamMeanSmallN;
            mode = tot >= stream_mean * n ? 1 : tot >= (uint64_t)kRxPfxMean * n ? 6 : 5;
        }
        if (mode == 9) {  // two waves per block: the LDS loop fed by LDS-DMA through a ring (§7 step 70)
            if (wave >= 2u) return;
            const WaveRange wr = range(gridDim.x, 2u, wave);
            rx_runs_ring<R, V6>(base, ofs, n, wr.a0, wr.a_end, lane, lds_rx + wave * (kRingWave / 16u), ro);
        } else if (mode == 5 || mode == 6 || mode == 7) {
            // Two waves per block. 5: the LDS loop until a run needs the hybrid loop; 7: the hybrid loop throughout
            // (four waves per block ran 2.5-4.4% slower on 40-120 B frames, workloads 13, 16; 17 −0.3%: with 8 waves
            // per CU the VALU-heavy LDS loop queues less for issue); 6: the prefix form with
            // 15-row slots (waves 0-1: as fast as 0-1 / 2-3 by block parity and as 2 blocks/CU of four waves, §7 step
            // 55).
            // The runs (§7 step 72, deal_runs): with heads for this launch (deal), each wave's equal share of the
            // batch's first 7/8, then runs of the last 1/8 dealt to the waves as they finish. With equal shares of the
            // whole batch the waves ran at speeds ±4% apart (by CU and XCD, not by data), and a launch waited 5-29 µs
            // for its last waves (tools/probes/rx_wave_times.py, profiles/r05_rx_wave_times_by_cu.txt).
            if (wave >= 2u) return;
            const uint32_t W2 = gridDim.x * 2u, g = wave_number(gridDim.x, 2u, wave);
            WaveRange wr;
            DealtRuns q = deal_runs(ofs, n, g, W2, lane, kRxSmallFrame, 8u, 0u, deal, &wr);
            ws.ready();
            if (mode == 6) {
                rx_runs_pfx<R, V6, 15, false>(base, ofs, n, q, lane, lds_rx + wave * (PfxSlot<15>::kBytes / 16u), ro);
            } else {
                lds16* slot = lds_rx + wave * (PfxSlot<7>::kBytes / 16u);
                if (mode == 5) rx_runs_lds<R, V6, true>(base, ofs, n, q, lane, slot, ro);
                else rx_runs_pfx<R, V6, 7, true>(base, ofs, n, q, lane, slot, ro);
            }
            ws.done(g, wr.bytes, lane);
        } else if (kStreamDeal && deal && (sets == 0 || sets == 8)) {
            // Streamed runs with the batch's last eighth dealt in pieces through the block's LDS ring (the auto
            // choice and mode 8 when the stream has heads; §7 step 75): waves 0-2 of every block stream, wave 3 deals.
            // the dealer: wave 3, or (NSX_STREAM_ROTATE builds) the wave of the block's slot on its CU, so that the 4
            // blocks of a CU put their dealers on different SIMDs
            const uint32_t dw = kStreamRotate ? (uint32_t)((uint64_t)blockIdx.x * kWavesPerBlock / gridDim.x) : kStreamWaves;
            PieceRing* rg = reinterpret_cast<PieceRing*>(lds_rx + dw * (PfxSlot<7>::kBytes / 16u));
            static_assert(sizeof(PieceRing) <= PfxSlot<7>::kBytes && kPieceRing <= kWave, "the ring in the dealer's slot");
            if (wave == dw) {
                if (lane < kPieceRing) rg->e[lane] = kPieceFree;
                if (lane == 0u) rg->claim = 0u, rg->produced = 0u, rg->end_at = ~0u;
            }
            __syncthreads();
            const uint32_t nb = gridDim.x;
            const uint32_t S = (n - (n >> kStreamPoolShift)) & ~(kRxRun - 1u);  // the static shares: frames [0, S)
            if (wave == dw) {
                // head h of the block (numbered XCD by XCD, so every head has blocks on all 8 XCDs), its share of the
                // pool's pieces and its dealers
                const uint32_t H = min(kDealHeads, nb), h = wave_number(nb, 1u, 0u) % H;
                const uint32_t Q = (n - S + kStreamPiece - 1u) / kStreamPiece;
                const uint32_t r0 = (uint32_t)((uint64_t)Q * h / H), qh = (uint32_t)((uint64_t)Q * (h + 1u) / H) - r0;
                ring_dealer(rg, deal + h * kDealStride, S + r0 * kStreamPiece, kStreamPiece, qh, (nb - h + H - 1u) / H,
                            kStreamAhead, lane);
                return;
            }
            const uint32_t g = wave_number(nb, kStreamWaves, wave < dw ? wave : wave - 1u);
            WaveRange wr{0u, 0u, 0u};
            if (S > 0u) wr = wave_range(ofs, S, g, nb * kStreamWaves, lane, kRxSmallFrame, 8u);
            RxOuts rp = ro;
            if (ro.raw) {  // parked in the wave's 7-row slot, as below
                uint16_t* pb = reinterpret_cast<uint16_t*>(lds_rx + wave * (PfxSlot<7>::kBytes / 16u));
                rp.tpk = make_park<uint16_t>(pb, ro.trs, tcp_raw, wr.a0, V6 ? 4096u : 2048u);
                if constexpr (!V6) rp.ipk = make_park<uint16_t>(pb + 2048, ro.irs, ip_raw, wr.a0, 2048u);
            }
            ws.ready();
            RingRuns q{wr.a0, wr.a_end, n, RingClient{rg, lane}, kPieceFree};
            rx_runs_ring<R, V6>(base, ofs, n, q, lane, rp);
            if (ro.raw) {
                park_flush(rp.tpk, lane);
                if constexpr (!V6) park_flush(rp.ipk, lane);
            }
            ws.done(g, wr.bytes, lane);
        } else {  // streamed runs on 3 of the 4 blocks per CU (the auto choice and mode 8, which forces it, on a
                  // stream without heads); mode 1: on every block
            const uint32_t nb = active_blocks(ofs, n, 0u, sets == 0 || sets == 8 ? 3u : 0u);
            if (blockIdx.x >= nb) return;
            // byte shares weighted by the block's slot on its CU (slot_share) on the default grid: 4 blocks per CU
            // launched (gridDim = 32 × CUs per XCD), the first 3/4 active
            SlotShare sh;
            if (kSlotWeights && nb >= 64 && (gridDim.x & 31u) == 0 && nb == gridDim.x / 4u * 3u) {
                sh = slot_share(nb, kWavesPerBlock, wave, gridDim.x >> 5, kRxSlotW);
            } else {
                const uint32_t g = wave_number(nb, kWavesPerBlock, wave);
                sh = SlotShare{g, g + 1u, nb * kWavesPerBlock};
            }
            const WaveRange wr = wave_range_w(ofs, n, sh.lo, sh.hi, sh.T, lane, kRxSmallFrame, 8u);
            // raw sums parked in the wave's (otherwise unused) 7-row slot, 8 KiB: IPv4 2 × 2048 results, IPv6 4096
            static_assert(PfxSlot<7>::kBytes >= 8192, "two 4 KiB parks per wave slot");
            RxOuts rp = ro;
            if (ro.raw) {
                uint16_t* pb = reinterpret_cast<uint16_t*>(lds_rx + wave * (PfxSlot<7>::kBytes / 16u));
                rp.tpk = make_park<uint16_t>(pb, ro.trs, tcp_raw, wr.a0, V6 ? 4096u : 2048u);
                if constexpr (!V6) rp.ipk = make_park<uint16_t>(pb + 2048, ro.irs, ip_raw, wr.a0, 2048u);
            }
            ws.ready();
            rx_runs<R, V6, 1>(base, ofs, n, wr.a0, wr.a_end, lane, rp);
            if (ro.raw) {
                park_flush(rp.tpk, lane);
                if constexpr (!V6) park_flush(rp.ipk, lane);
            }
            ws.done(wave_number(nb, kWavesPerBlock, wave), wr.bytes, lane);
        }
        return;
    }
    // The grid is sized for small frames (4 blocks/CU); a batch of large ones streams on big_keep of them.
    const uint32_t nb = active_blocks(ofs, n, kRxBigMean, big_keep);
    if (blockIdx.x >= nb) return;
    const WaveRange wr = range(nb, kWavesPerBlock, wave);
    const uint32_t a0 = wr.a0, a_end = wr.a_end;
    const bool small = sets == 2 || (sets == 0 && wr.bytes < (uint64_t)kRxSmallFrame * (a_end - a0));
    if (small) {
        StaticRuns q{a0, a_end};
        rx_runs_lds<R, V6>(base, ofs, n, q, lane, lds_rx + wave * (kRxSlot / 16u), ro);
    } else {
        rx_runs<R, V6, 1>(base, ofs, n, a0, a_end, lane, ro);
    }
}

// ---------------------------------------------------------------------------
// Fused sender path: segment.bytes() + computeChecksum +
// field write in one pass (transport/tcp/tcp.go:98-128 and :68-71). Each wire
// image — the 20-byte BE header built from SoA fields, options, the
// reference's `remainder` padding (tcp.go:118-121), the payload — is written as
// whole dwords at out + out_off[i] (4-aligned; up to 3 slack bytes after the
// image are zero-filled) while its dwords are summed with the checksum field
// at 0; ~raw then goes into bytes 16-17.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32u(uint32_t v) {
    return (v >> 24) | ((v >> 8) & 0xFF00u) | ((v << 8) & 0xFF0000u) | (v << 24);
}

// Wave task = a group of G ≤ 64 consecutive segments: lane j loads segment
// g0+j's header fields and offsets (coalesced, one round trip per group), and the
// wave then builds the group's segments one after another with the values
// broadcast by v_readlane. Per segment, each lane owns 16-byte chunks of the
// output (1 KiB rows). Payload source dwords come from one buffer descriptor
// with unconditional loads — offsets before the payload, past the data end, or
// of rows past the segment are out of range, read 0 and move nothing — so the
// R rows of a batch are all in flight with no branch between them; bytes are
// realigned by v_alignbyte with the segment-uniform shift. Row 0 (the header
// row) loads its 5 source dwords one by one so that lanes straddling the
// header/payload edge read correctly; only it and the row holding the wire end
// take byte masks. Output goes through a descriptor ending at the segment's
// last dword (per-dword range check, tools/probes/copy_ceiling.hip), so a tail
// chunk needs no mask or branch. Dword 4 (urgent pointer + checksum field) is
// written once, last, with the field.
constexpr uint32_t kBuildRows = 2;

__device__ __forceinline__ u32x4 realign(u32x4 lo, uint32_t hi, uint32_t sh) {
    return u32x4{__builtin_amdgcn_alignbyte(lo.y, lo.x, sh), __builtin_amdgcn_alignbyte(lo.z, lo.y, sh),
                 __builtin_amdgcn_alignbyte(lo.w, lo.z, sh), __builtin_amdgcn_alignbyte(hi, lo.w, sh)};
}

struct BuildSeg {  // wave-uniform description of one segment
    uint32_t D0, D1, D2, D3, D4;  // header dwords as stored (LE view), field = 0
    uint32_t optlen, hdr_end, wire, nb4, rows, sh;
    int32_t sh0;                  // payload source offset (from the descriptor base) = wire pos + sh0
    uint64_t ob, db;              // option / payload byte offsets
    bool fast;                    // no options, payload 4-aligned, whole dwords, ≥ 20 B into the data array
};

// Source row r: 4+1 dwords per lane. Row 0 (head) clamps each dword separately.
template <int LP>
__device__ __forceinline__ void build_load_head(__amdgpu_buffer_rsrc_t drs, const BuildSeg& S, uint32_t lane,
                                                u32x4& lo, uint32_t& hi) {
    const int32_t t = ((int32_t)(lane * 16u) + S.sh0) >> 2;
    uint32_t d[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        d[j] = __builtin_amdgcn_raw_buffer_load_b32(drs, t + j >= 0 ? (uint32_t)(t + j) * 4u : kOOB, 0, LP);
    lo = u32x4{d[0], d[1], d[2], d[3]};
    hi = d[4];
}

template <int LP>
__device__ __forceinline__ void build_load_body(__amdgpu_buffer_rsrc_t drs, const BuildSeg& S, uint32_t lane,
                                                uint32_t r, u32x4& lo, uint32_t& hi) {
    const bool live = r < S.rows;
    const uint32_t a = (uint32_t)((int32_t)(r * kRow + lane * 16u) + S.sh0) & ~3u;  // ≥ 0 (hdr_end ≤ 1008)
    lo = bld16<LP != 0>(drs, live ? a : kOOB);
    hi = __builtin_amdgcn_raw_buffer_load_b32(drs, live && S.sh ? a + 16u : kOOB, 0, LP);
}

// Option bytes of one 16 B image chunk at image byte pos0: image byte p in [20, 20 + optlen) is option byte
// p - 20 (tcp.go:103-107). One descriptor over the segment's options, based at ob rounded down to 4 B and
// ending at the last option dword; five dword loads per lane (index pos0/4 - 5 + j, negative or past the
// options: out of range, 0, no traffic), realigned by ob & 3 and masked to the option bytes, so the header
// padding (tcp.go:118-121) reads 0. Issue (opt_load) and compose (opt_fin) are split so that the loads go
// out with the payload's.
struct OptRaw {
    u32x4 lo;
    uint32_t hi;
};

__device__ __forceinline__ OptRaw opt_load(const uint8_t* __restrict__ opts, uint64_t ob, uint32_t optlen,
                                           uint32_t pos0) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(opts + (ob & ~3ull), ((ob & 3u) + optlen + 3u) & ~3u);
    const int32_t t = (int32_t)(pos0 >> 2) - 5;
    uint32_t d[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) d[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, t + j >= 0 ? (uint32_t)(t + j) * 4u : kOOB, 0, 0);
    return OptRaw{u32x4{d[0], d[1], d[2], d[3]}, d[4]};
}

__device__ __forceinline__ u32x4 opt_fin(OptRaw o, uint64_t ob, uint32_t optlen, uint32_t pos0) {
    const uint32_t sh = (uint32_t)ob & 3u;
    const u32x4 x = sh ? realign(o.lo, o.hi, sh) : o.lo;
    return keep_bytes(x, min(max(20 - (int32_t)pos0, 0), 16), min(max(20 + (int32_t)optlen - (int32_t)pos0, 0), 16));
}

// Staged options: when every segment of a wave's group has ≤ 40 option bytes (all valid TCP: data offset ≤ 15),
// lane j loads segment g0+j's option bytes once per group (the group's options are one contiguous run, so the
// 11 dword loads are dense), realigns them by its own ob & 3 and zeroes the bytes past optlen: od[m] = option
// dword m. Building segment k then takes option dword m to image dword 5 + m — lane (5+m)/4, component
// (5+m)%4 — by v_readlane + v_cndmask, with no per-segment memory access. REPLACE: overwrite image dwords
// [5, hdr/4) (4-aligned header, fast paths; pad dwords get od's zeros); else OR into a zeroed chunk.
constexpr int kOptDw = 10;

__device__ __forceinline__ void set_comp(u32x4& x, int c, uint32_t v, bool on) {
    if (c == 0) x.x = on ? v : x.x;
    if (c == 1) x.y = on ? v : x.y;
    if (c == 2) x.z = on ? v : x.z;
    if (c == 3) x.w = on ? v : x.w;
}

template <bool REPLACE>
__device__ __forceinline__ u32x4 staged_opts(const uint32_t (&od)[kOptDw], uint32_t k, uint32_t ndw, uint32_t lane,
                                             u32x4 x) {
    if (!REPLACE) x = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int m = 0; m < kOptDw; ++m) {
        if ((uint32_t)m < ndw) {  // wave-uniform
            const uint32_t v = __builtin_amdgcn_readlane(od[m], k);
            set_comp(x, (5 + m) & 3, v, lane == (uint32_t)((5 + m) >> 2));
        }
    }
    return x;
}

// Compose row r of the wire image (general composition); oc = the chunk's option bytes (opt_fin, 0 when none).
__device__ __forceinline__ u32x4 compose_row(const BuildSeg& S, u32x4 oc, uint32_t lane, uint32_t r, u32x4 lo,
                                             uint32_t hi) {
    const uint32_t pos0 = r * kRow + lane * 16u;
    u32x4 x = S.sh ? realign(lo, hi, S.sh) : lo;
    if (r * kRow < S.hdr_end || (r + 1) * kRow > S.wire)  // keep payload bytes [hdr_end, wire) only
        x = keep_bytes(x, min(max((int32_t)S.hdr_end - (int32_t)pos0, 0), 16),
                       min(max((int32_t)S.wire - (int32_t)pos0, 0), 16));
    if (r == 0) {  // header bytes 0-19
        x.x |= lane == 0 ? S.D0 : lane == 1 ? S.D4 : 0u;
        x.y |= lane == 0 ? S.D1 : 0u;
        x.z |= lane == 0 ? S.D2 : 0u;
        x.w |= lane == 0 ? S.D3 : 0u;
    }
    x.x |= oc.x, x.y |= oc.y, x.z |= oc.z, x.w |= oc.w;  // option bytes [20, 20 + optlen)
    return x;
}

// Images of more than 2 rows (unpipelined path): compose, sum and store row r as it goes; dword 4 (urgent
// pointer + checksum field) is held back and written with the field once the sum is known.
template <int SP>
__device__ __forceinline__ uint32_t build_row(const BuildSeg& S, __amdgpu_buffer_rsrc_t ors, u32x4 oc, uint32_t lane,
                                              uint32_t r, u32x4 lo, uint32_t hi, uint32_t acc) {
    const uint32_t pos0 = r * kRow + lane * 16u;
    const u32x4 x = compose_row(S, oc, lane, r, lo, hi);
    acc = sad4(x, acc);
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint32_t v3u __attribute__((ext_vector_type(3)));
    const bool d4 = r == 0 && lane == 1;  // this chunk holds dword 4: store its other three now
    __builtin_amdgcn_raw_buffer_store_b128(v4u{x.x, x.y, x.z, x.w}, ors, d4 ? kOOB : pos0, 0, SP);
    if (r == 0) __builtin_amdgcn_raw_buffer_store_b96(v3u{x.y, x.z, x.w}, ors, d4 ? 20u : kOOB, 0, SP);
    return acc;
}

// PS: segments per register set on the pipelined fast-group path; OPT: the batch has an option array (else
// every option branch compiles out: 61 VGPRs vs 120 at PS 2)
template <int LP, int SP, int PS, bool OPT>
__global__ __launch_bounds__(kBlock) void tcp_build_kernel(TcpHdrSoA h, const uint8_t* __restrict__ opts,
                                                           const uint64_t* __restrict__ opt_off,
                                                           const uint8_t* __restrict__ data,
                                                           const uint64_t* __restrict__ data_off, uint64_t data_bytes,
                                                           const uint32_t* __restrict__ partial, uint64_t n,
                                                           uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ out_off,
                                                           uint16_t* __restrict__ raw_out, uint32_t group,
                                                           uint32_t clog, int pipe) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint32_t v3u __attribute__((ext_vector_type(3)));
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t data_end4 = (data_bytes + 3) & ~3ull;  // the last payload dword reads whole
    const uint64_t ngroups = (n + group - 1) / group;
    TaskIter it = task_iter(ngroups, wave);
    const ChunkDeal cd = chunk_deal(it, wave, clog, ngroups);
    for (uint64_t q = it.next; q < it.end; q += it.step) {
        const uint64_t g = cd.clog ? cd.task((uint32_t)q) : q;
        if (g >= ngroups) break;
        const uint64_t g0 = g * group;
        const uint32_t cnt = (uint32_t)min((uint64_t)group, n - g0);
        // Per-lane metadata of segment g0 + lane (lanes past cnt repeat the last one).
        const uint64_t i = g0 + min(lane, cnt - 1);
        const uint32_t mD0 = bswap16u(h.src_port[i]) | (bswap16u(h.dst_port[i]) << 16);
        const uint32_t mD1 = bswap32u(h.seq[i]), mD2 = bswap32u(h.ack[i]);
        const uint64_t mob = OPT ? opt_off[i] : 0;
        const uint32_t moptlen = OPT ? (uint32_t)(opt_off[i + 1] - mob) : 0u;
        // byte 12: the caller's, or computeOffset() (tcp.go:59-66) over the serialized option bytes
        const uint32_t moff = h.offset ? (uint32_t)h.offset[i] : ((23u + moptlen) >> 2) & 0xFFu;
        const uint32_t mD3 = moff | ((uint32_t)h.ctl[i] << 8) | (bswap16u(h.window[i]) << 16);
        const uint32_t mD4 = bswap16u(h.urgent[i]) << 16;  // checksum field (bytes 16-17) = 0 for the sum
        const uint64_t mdb = data_off[i], mde = data_off[i + 1], moo = out_off[i];
        const uint32_t mpart = partial ? partial[i] : 0u;
        const uint32_t mhdr = 20u + moptlen + (moptlen ? (20u + moptlen) % 4u : 0u);  // tcp.go:118-121
        const uint32_t mwire = mhdr + (uint32_t)(mde - mdb);                             // < 2^31
        uint32_t od[kOptDw];
        bool staged = false;  // wave-uniform: the group's options are held in od (see staged_opts)
        if (OPT) {
            // every lane's option bytes inside [first segment's ob, last segment's end) (so the group descriptor
            // covers them and its range cannot wrap), at most 40 each
            const uint64_t gb = readlane64(mob, 0) & ~3ull;
            const uint64_t ge = readlane64(mob, cnt - 1u) + __builtin_amdgcn_readlane(moptlen, cnt - 1u);
            staged = __builtin_amdgcn_ballot_w64(moptlen > 4u * kOptDw || mob < gb || mob + moptlen > ge) == 0;
            if (staged && __builtin_amdgcn_ballot_w64(moptlen != 0) != 0) {
                const __amdgpu_buffer_rsrc_t rs = make_rsrc(opts + gb, ((ge - gb) + 3u) & ~3ull);
                const uint32_t sh = (uint32_t)mob & 3u, off = (uint32_t)((mob & ~3ull) - gb);
                uint32_t d[kOptDw + 1];
#pragma unroll
                for (int m = 0; m <= kOptDw; ++m)
                    d[m] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * m < sh + moptlen ? off + 4u * m : kOOB, 0, 0);
#pragma unroll
                for (int m = 0; m < kOptDw; ++m)
                    od[m] = __builtin_amdgcn_alignbyte(d[m + 1], d[m], sh) & keep_mask(0, (int32_t)moptlen, 4 * m);
            } else {
#pragma unroll
                for (int m = 0; m < kOptDw; ++m) od[m] = 0u;
            }
        }
        auto seg_at = [&](uint32_t k, BuildSeg& S, __amdgpu_buffer_rsrc_t& drs, __amdgpu_buffer_rsrc_t& ors) {
            S.D0 = __builtin_amdgcn_readlane(mD0, k);
            S.D1 = __builtin_amdgcn_readlane(mD1, k);
            S.D2 = __builtin_amdgcn_readlane(mD2, k);
            S.D3 = __builtin_amdgcn_readlane(mD3, k);
            S.D4 = __builtin_amdgcn_readlane(mD4, k);
            S.optlen = __builtin_amdgcn_readlane(moptlen, k);
            S.hdr_end = __builtin_amdgcn_readlane(mhdr, k);
            S.wire = __builtin_amdgcn_readlane(mwire, k);
            S.nb4 = (S.wire + 3u) & ~3u;
            S.rows = (S.nb4 + kRow - 1) / kRow;
            S.ob = readlane64(mob, k);
            const uint64_t db = readlane64(mdb, k);
            S.sh0 = (int32_t)(db & 3u) - (int32_t)S.hdr_end;
            S.sh = (uint32_t)S.sh0 & 3u;
            const uint64_t dbase = db & ~3ull;
            S.db = db;
            S.fast = (S.hdr_end & 3u) == 0 && S.hdr_end <= kRow && (db & 3u) == 0 && db >= S.hdr_end &&
                     (S.wire & 3u) == 0;
            drs = make_rsrc(data + dbase, data_end4 - dbase);
            ors = make_rsrc(out + readlane64(moo, k), S.nb4);
        };
        // Raw sums are parked one per lane (lane k = segment g0 + k) and leave as one 2-byte store per lane
        // when the group is done.
        uint32_t raws = 0;
        auto seg_raw = [&](uint32_t k, uint32_t acc) {
            const uint32_t raw = finish(wave_sum(acc), true, __builtin_amdgcn_readlane(mpart, k));  // images 4-aligned
            raws = lane == k ? raw : raws;
            return raw;
        };
        auto seg_done = [&](uint32_t k, const BuildSeg& S, __amdgpu_buffer_rsrc_t ors, uint32_t acc) {
            const uint32_t raw = seg_raw(k, acc);
            __builtin_amdgcn_raw_buffer_store_b32(S.D4 | bswap16u(~raw & 0xFFFFu), ors, lane == 0 ? 16u : kOOB, 0, SP);
        };
        auto flush_raws = [&]() {
            const __amdgpu_buffer_rsrc_t rrs = make_rsrc(raw_out + g0, raw_out ? (uint64_t)cnt * 2u : 0u);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)raws, rrs, lane < cnt ? lane * 2u : kOOB, 0, 0);
        };
        // Every segment of the group on the fast path and at most 2 rows long (the bench layouts): software-
        // pipelined — segment k+1's two rows are loaded before segment k is built, so the wave keeps its loads
        // in flight through its own header/sum/store phases (tools/probes/copy_layout.hip seg_swp vs seg).
        const bool mfast = (mhdr & 3u) == 0 && (mdb & 3u) == 0 && mdb >= mhdr && (mwire & 3u) == 0 &&
                           mwire <= 2u * kRow;
        if (pipe == 1 && (!OPT || staged) && __builtin_amdgcn_ballot_w64(!(mfast || lane >= cnt)) == 0) {
            struct Rows {
                u32x4 v[PS][2];
            };
            auto fload = [&](uint32_t k0, Rows& F) {  // kk ≥ cnt: an empty descriptor, the loads move nothing
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e) {
                    const uint32_t kk = k0 + e, kc = min(kk, cnt - 1u);
                    const uint64_t db = readlane64(mdb, kc);
                    const uint32_t nb4 = kk < cnt ? __builtin_amdgcn_readlane(mwire, kc) : 0u;
                    const __amdgpu_buffer_rsrc_t frs = make_rsrc(data + db - __builtin_amdgcn_readlane(mhdr, kc), nb4);
                    F.v[e][0] = bld16<LP != 0>(frs, lane * 16u);
                    F.v[e][1] = bld16<LP != 0>(frs, kRow + lane * 16u);
                }
            };
            auto fdone = [&](uint32_t k0, Rows& F) {
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e) asm volatile("" : "+v"(F.v[e][0]), "+v"(F.v[e][1]));
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e) {
                    const uint32_t kk = k0 + e;
                    if (kk >= cnt) break;  // wave-uniform
                    BuildSeg S;
                    const uint32_t nb4 = __builtin_amdgcn_readlane(mwire, kk);
                    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out + readlane64(moo, kk), nb4);
                    u32x4 x = F.v[e][0];
                    if (OPT)  // image dwords [5, hdr/4): options and padding, not the source bytes under them
                        x = staged_opts<true>(od, kk, (__builtin_amdgcn_readlane(mhdr, kk) - 20u) >> 2, lane, x);
                    // header dwords broadcast from lane kk (pulling D0-D3 with ds_bpermute instead measured equal,
                    // DESIGN.md §7 step 46)
                    S.D0 = __builtin_amdgcn_readlane(mD0, kk);
                    S.D1 = __builtin_amdgcn_readlane(mD1, kk);
                    S.D2 = __builtin_amdgcn_readlane(mD2, kk);
                    S.D3 = __builtin_amdgcn_readlane(mD3, kk);
                    S.D4 = __builtin_amdgcn_readlane(mD4, kk);
                    x.x = lane == 0 ? S.D0 : (lane == 1 ? S.D4 : x.x);
                    x.y = lane == 0 ? S.D1 : x.y;
                    x.z = lane == 0 ? S.D2 : x.z;
                    x.w = lane == 0 ? S.D3 : x.w;
                    const u32x4 y = F.v[e][1];  // row 1: zeros past the image (range check), stores clipped likewise
                    const uint32_t raw = seg_raw(kk, fold32(sad4(y, sad4(x, 0u))));
                    // both rows leave once the sum is known, one store each: dword 4 (lane 1's first) carries the
                    // field (tcp.go:110, ^sum) — no separate partial-chunk or field stores
                    x.x = lane == 1 ? S.D4 | bswap16u(~raw & 0xFFFFu) : x.x;
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{x.x, x.y, x.z, x.w}, ors, lane * 16u, 0, SP);
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{y.x, y.y, y.z, y.w}, ors, kRow + lane * 16u, 0, SP);
                }
            };
            Rows A, B;
            fload(0, A);
            for (uint32_t kk = 0; kk < cnt; kk += 2u * PS) {
                fload(kk + PS, B);
                fdone(kk, A);
                if (kk + PS >= cnt) break;
                fload(kk + 2u * PS, A);
                fdone(kk + PS, B);
            }
            flush_raws();
            continue;
        }
        // Any payload alignment, any header length, images ≤ 2 rows, at least hdr_end bytes of the data array
        // before the payload: the same pipelining over the general composition. Image byte p comes from
        // data + db - hdr_end + p, so one descriptor based at that address rounded down to 4 B serves both rows —
        // a 16 B load and the next dword per lane, realigned by v_alignbyte — and the bytes under the header read
        // from inside the data array and are masked away (build_row); no per-dword clamped head loads.
        const bool mgen = mdb >= mhdr && mwire <= 2u * kRow;
        if (pipe && (!OPT || staged) && __builtin_amdgcn_ballot_w64(!(mgen || lane >= cnt)) == 0) {
            struct GRows {
                u32x4 lo[PS][2];
                uint32_t hi[PS][2];
            };
            auto gload = [&](uint32_t k0, GRows& G) {  // kk ≥ cnt: an empty descriptor, the loads move nothing
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e) {
                    const uint32_t kk = k0 + e, kc = min(kk, cnt - 1u);
                    const uint64_t src = readlane64(mdb, kc) - __builtin_amdgcn_readlane(mhdr, kc);
                    const uint32_t sh = (uint32_t)src & 3u;
                    const uint32_t nb = kk < cnt ? (sh + __builtin_amdgcn_readlane(mwire, kc) + 3u) & ~3u : 0u;
                    const __amdgpu_buffer_rsrc_t grs = make_rsrc(data + (src & ~3ull), nb);
#pragma unroll
                    for (uint32_t r = 0; r < 2u; ++r) {
                        G.lo[e][r] = bld16<LP != 0>(grs, r * kRow + lane * 16u);
                        G.hi[e][r] = __builtin_amdgcn_raw_buffer_load_b32(grs, sh ? r * kRow + lane * 16u + 16u : kOOB,
                                                                           0, LP);
                    }
                }
            };
            auto gdone = [&](uint32_t k0, GRows& G) {
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e)
                    asm volatile("" : "+v"(G.lo[e][0]), "+v"(G.lo[e][1]), "+v"(G.hi[e][0]), "+v"(G.hi[e][1]));
#pragma unroll
                for (uint32_t e = 0; e < (uint32_t)PS; ++e) {
                    const uint32_t kk = k0 + e;
                    if (kk >= cnt) break;  // wave-uniform
                    BuildSeg S;
                    __amdgpu_buffer_rsrc_t drs, ors;
                    seg_at(kk, S, drs, ors);
                    u32x4 oc0{0u, 0u, 0u, 0u};
                    if (OPT && S.optlen) oc0 = staged_opts<false>(od, kk, (S.optlen + 3u) >> 2, lane, oc0);
                    u32x4 x = compose_row(S, oc0, lane, 0, G.lo[e][0], G.hi[e][0]);
                    const u32x4 y = compose_row(S, u32x4{0u, 0u, 0u, 0u}, lane, 1, G.lo[e][1], G.hi[e][1]);
                    const uint32_t raw = seg_raw(kk, fold32(sad4(y, sad4(x, 0u))));  // row 1 is 0 past the image
                    x.x = lane == 1 ? S.D4 | bswap16u(~raw & 0xFFFFu) : x.x;  // the field, dword 4
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{x.x, x.y, x.z, x.w}, ors, lane * 16u, 0, SP);
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{y.x, y.y, y.z, y.w}, ors, kRow + lane * 16u, 0, SP);
                }
            };
            GRows A, B;
            gload(0, A);
            for (uint32_t kk = 0; kk < cnt; kk += 2u * PS) {
                gload(kk + PS, B);
                gdone(kk, A);
                if (kk + PS >= cnt) break;
                gload(kk + 2u * PS, A);
                gdone(kk + PS, B);
            }
            flush_raws();
            continue;
        }
        uint32_t k = 0;
        while (k < cnt) {
            BuildSeg S;
            __amdgpu_buffer_rsrc_t drs, ors;
            seg_at(k, S, drs, ors);
            uint32_t acc = 0;
            if (S.fast) {
                // A 4-aligned header (no options, or options padded to a dword) and a 4-aligned payload of
                // whole dwords at data offset ≥ hdr_end: the image is the payload shifted by exactly hdr_end/4
                // dwords. One descriptor based hdr_end bytes before the payload (inside the data array) maps
                // image dword k to source dword k, so every row is one plain 16 B load per lane with no shift
                // and no byte mask; bytes [0, hdr_end) of row 0 are replaced by the built header and options,
                // dwords past the image read 0 (range check).
                // Double-buffered batches of R rows: batch b + 1 loads while batch b is built (rows past the
                // image are out of the descriptor's range: 0, no traffic).
                constexpr uint32_t R = kBuildRows;
                const __amdgpu_buffer_rsrc_t frs = make_rsrc(data + S.db - S.hdr_end, S.nb4);
                OptRaw o{};
                if (S.optlen && !staged) o = opt_load(opts, S.ob, S.optlen, lane * 16u);
                auto fl = [&](uint32_t r0, u32x4 (&v)[R]) {
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr) v[rr] = bld16<LP != 0>(frs, (r0 + rr) * kRow + lane * 16u);
                };
                auto fb = [&](uint32_t r0, u32x4 (&v)[R]) {
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr) asm volatile("" : "+v"(v[rr]));
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr) {
                        const uint32_t r = r0 + rr;
                        if (r >= S.rows) break;
                        u32x4 x = v[rr];
                        if (r == 0) {
                            if (S.optlen && staged) {
                                x = staged_opts<true>(od, k, (S.hdr_end - 20u) >> 2, lane, x);
                            } else if (S.optlen) {
                                const u32x4 oc = opt_fin(o, S.ob, S.optlen, lane * 16u);
                                x = keep_bytes(x, min(max((int32_t)S.hdr_end - (int32_t)(lane * 16u), 0), 16), 16);
                                x.x |= oc.x, x.y |= oc.y, x.z |= oc.z, x.w |= oc.w;
                            }
                            x.x = lane == 0 ? S.D0 : (lane == 1 ? S.D4 : x.x);
                            x.y = lane == 0 ? S.D1 : x.y;
                            x.z = lane == 0 ? S.D2 : x.z;
                            x.w = lane == 0 ? S.D3 : x.w;
                        }
                        acc = sad4(x, acc);
                        const uint32_t pos0 = r * kRow + lane * 16u;
                        const bool d4 = r == 0 && lane == 1;  // dword 4 waits for the field
                        __builtin_amdgcn_raw_buffer_store_b128(v4u{x.x, x.y, x.z, x.w}, ors, d4 ? kOOB : pos0, 0, SP);
                        if (r == 0)
                            __builtin_amdgcn_raw_buffer_store_b96(v3u{x.y, x.z, x.w}, ors, d4 ? 20u : kOOB, 0, SP);
                    }
                    acc = fold32(acc);
                };
                u32x4 VA[R], VB[R];
                fl(0, VA);
                for (uint32_t r0 = 0; r0 < S.rows; r0 += 2u * R) {
                    if (r0 + R < S.rows) fl(r0 + R, VB);
                    fb(r0, VA);
                    if (r0 + R >= S.rows) break;
                    if (r0 + 2u * R < S.rows) fl(r0 + 2u * R, VA);
                    fb(r0 + R, VB);
                }
            } else if (S.hdr_end <= kRow - 16u) {
                constexpr uint32_t R = kBuildRows;
                // batch 0: the header row + rows 1..R-1, all loads in flight
                u32x4 lo[R];
                uint32_t hi[R];
                OptRaw o{};
                if (S.optlen && !staged) o = opt_load(opts, S.ob, S.optlen, lane * 16u);  // hdr_end ≤ 1008: row 0
                build_load_head<LP>(drs, S, lane, lo[0], hi[0]);
#pragma unroll
                for (uint32_t rr = 1; rr < R; ++rr) build_load_body<LP>(drs, S, lane, rr, lo[rr], hi[rr]);
#pragma unroll
                for (uint32_t rr = 0; rr < R; ++rr)
                    asm volatile("" : "+v"(lo[rr].x), "+v"(lo[rr].y), "+v"(lo[rr].z), "+v"(lo[rr].w), "+v"(hi[rr]));
                const u32x4 oc0 = !S.optlen ? u32x4{0u, 0u, 0u, 0u}
                                  : staged  ? staged_opts<false>(od, k, (S.optlen + 3u) >> 2, lane, u32x4{0u, 0u, 0u, 0u})
                                            : opt_fin(o, S.ob, S.optlen, lane * 16u);
#pragma unroll
                for (uint32_t rr = 0; rr < R; ++rr)
                    if (rr < S.rows)
                        acc = build_row<SP>(S, ors, rr == 0 ? oc0 : u32x4{0u, 0u, 0u, 0u}, lane, rr, lo[rr], hi[rr], acc);
                acc = fold32(acc);
                for (uint32_t r0 = R; r0 < S.rows; r0 += R) {  // long segments: further batches
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr) build_load_body<LP>(drs, S, lane, r0 + rr, lo[rr], hi[rr]);
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr)
                        asm volatile("" : "+v"(lo[rr].x), "+v"(lo[rr].y), "+v"(lo[rr].z), "+v"(lo[rr].w), "+v"(hi[rr]));
#pragma unroll
                    for (uint32_t rr = 0; rr < R; ++rr)
                        if (r0 + rr < S.rows)
                            acc = build_row<SP>(S, ors, u32x4{0u, 0u, 0u, 0u}, lane, r0 + rr, lo[rr], hi[rr], acc);
                    acc = fold32(acc);
                }
            } else {
                // options longer than ~1 KiB (not real TCP; the API allows it): every row clamps per dword
                for (uint32_t r = 0; r < S.rows; ++r) {
                    const uint32_t pos0 = r * kRow + lane * 16u;
                    const int32_t t = ((int32_t)pos0 + S.sh0) >> 2;
                    uint32_t d[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j)
                        d[j] = __builtin_amdgcn_raw_buffer_load_b32(drs, t + j >= 0 ? (uint32_t)(t + j) * 4u : kOOB, 0,
                                                                     2);
                    const u32x4 oc = r * kRow < 20u + S.optlen ? opt_fin(opt_load(opts, S.ob, S.optlen, pos0), S.ob,
                                                                         S.optlen, pos0)
                                                               : u32x4{0u, 0u, 0u, 0u};
                    acc = fold32(build_row<SP>(S, ors, oc, lane, r, u32x4{d[0], d[1], d[2], d[3]}, d[4], acc));
                }
            }
            seg_done(k, S, ors, acc);
            k += 1;
        }
        flush_raws();
    }
}

// ---------------------------------------------------------------------------
// IPv4 header checksum (RFC 791 §3.1 with the RFC 1071 sum), one thread per
// packet: headers are 20-60 bytes, too short for a wave each. Packet i's header
// starts at base + i*stride + hdr_off (any alignment, e.g. 14 behind an
// Ethernet header) and is IHL*4 bytes (IHL = low nibble of byte 0).
// A block takes 4 × 256 consecutive packets per iteration, each 256 through one
// buffer descriptor based at their first header (block-uniform, 32-bit per-lane
// offsets), with the loads of all four in flight together. Every lane issues
// the loads of its header's first 20 bytes unconditionally (5 aligned dwords,
// a 6th when the header is not dword-aligned); the dwords after those are loaded
// only when some lane of the wave has IHL > 5 (wave-uniform branch), each with
// an out-of-range offset beyond its own header, so no exec-masked load stalls
// the wave. Then the LE-half-sum / byte-swap rule of the segment kernels.
// MODE 0: out = raw sum over the header as it stands (valid iff 0xFFFF).
// MODE 1: out = raw sum with bytes 10-11 taken as zero; writes ~raw there.
// MODE 2: receive-side verify as a bitmask: bit (i % 64) of mask[i / 64] set iff
//         header i is well-formed and its raw sum is 0xFFFF (one v_cmp + ballot
//         per wave; 1 bit written per header instead of 16).
// A malformed header (IHL < 5, or longer than the stride) gets out = 0 and is
// not written.
// ---------------------------------------------------------------------------
constexpr int kHdrUnroll = 4;  // 256-header chunks per block iteration, loads of all in flight

template <int MODE>
__global__ __launch_bounds__(kBlock) void ipv4_hdr_kernel(uint8_t* __restrict__ base, uint64_t stride,
                                                          uint32_t hdr_off, uint64_t n, uint16_t* __restrict__ out,
                                                          uint64_t* __restrict__ mask) {
    constexpr int U = kHdrUnroll;
    const uint32_t t = threadIdx.x;
    for (uint64_t c00 = (uint64_t)blockIdx.x * kBlock * U; c00 < n; c00 += (uint64_t)gridDim.x * kBlock * U) {
        __amdgpu_buffer_rsrc_t rs[U];
        uint8_t* cbase[U];
        uint32_t rel[U], head[U], a[U], len[U], nd[U];
        bool live[U], ok[U];
        uint32_t d[U][16];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // chunk u: packets [c0, c0 + 256), one descriptor each
            const uint64_t c0 = c00 + (uint64_t)u * kBlock;
            const uint32_t cnt = c0 < n ? (uint32_t)min((uint64_t)kBlock, n - c0) : 0u;
            uint8_t* first = base + min(c0, n - 1) * stride + hdr_off;
            cbase[u] = reinterpret_cast<uint8_t*>((uintptr_t)first & ~(uintptr_t)3);
            const uint32_t lead = (uint32_t)(first - cbase[u]);
            // the last header may run 60 bytes; per-lane offsets never pass their own header
            rs[u] = make_rsrc(cbase[u], cnt ? (uint64_t)(cnt - 1) * stride + lead + 64u : 0u);
            live[u] = t < cnt;
            rel[u] = (live[u] ? t : 0u) * (uint32_t)stride + lead;
            head[u] = rel[u] & 3u;
            a[u] = rel[u] - head[u];
            const u32x4 q = bld16<false>(rs[u], live[u] ? a[u] : kOOB);  // dword-aligned 16 B: one wide load
            d[u][0] = q.x, d[u][1] = q.y, d[u][2] = q.z, d[u][3] = q.w;
            d[u][4] = __builtin_amdgcn_raw_buffer_load_b32(rs[u], live[u] ? a[u] + 16u : kOOB, 0, 0);
            d[u][5] = __builtin_amdgcn_raw_buffer_load_b32(rs[u], live[u] && head[u] ? a[u] + 20u : kOOB, 0, 0);
        }
        bool opts = false;
        uint32_t acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            len[u] = ((d[u][0] >> (8 * head[u])) & 15u) * 4u;
            ok[u] = live[u] && len[u] >= 20u && (stride == 0 || hdr_off + len[u] <= stride);
            nd[u] = ok[u] ? (head[u] + len[u] + 3u) >> 2 : 0u;
            opts |= nd[u] > (head[u] ? 6u : 5u);
            acc[u] = 0;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                // keep window bytes [head, head+len), minus the field in fill mode
                uint32_t m = keep_mask((int32_t)head[u], (int32_t)(head[u] + len[u]), 4 * k);
                if (MODE == 1) m &= ~keep_mask((int32_t)head[u] + 10, (int32_t)head[u] + 12, 4 * k);
                acc[u] = __builtin_amdgcn_sad_u16(d[u][k] & m, 0u, acc[u]);
            }
        }
        if (__ballot(opts)) {  // options present somewhere in this wave: dwords 5 (aligned headers) .. 15
#pragma unroll
            for (int u = 0; u < U; ++u) {
                d[u][5] = __builtin_amdgcn_raw_buffer_load_b32(rs[u], !head[u] && 5u < nd[u] ? a[u] + 20u : kOOB, 0, 0);
#pragma unroll
                for (int k = 6; k < 16; ++k)
                    d[u][k] = __builtin_amdgcn_raw_buffer_load_b32(rs[u], (uint32_t)k < nd[u] ? a[u] + 4u * k : kOOB,
                                                                    0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int k = 5; k < 16; ++k) {  // dword 5 of an unaligned header was summed above: it reads 0 here
                    uint32_t m = keep_mask((int32_t)head[u], (int32_t)(head[u] + len[u]), 4 * k);
                    if (MODE == 1) m &= ~keep_mask((int32_t)head[u] + 10, (int32_t)head[u] + 12, 4 * k);
                    acc[u] = __builtin_amdgcn_sad_u16(d[u][k] & m, 0u, acc[u]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint8_t* p = cbase[u] + rel[u];
            const uint32_t raw = ok[u] ? finish(acc[u], ((uintptr_t)p & 1u) == 0, 0u) : 0u;
            if (out && live[u]) out[c00 + (uint64_t)u * kBlock + t] = (uint16_t)raw;
            if constexpr (MODE == 2) {  // the wave's 64 headers start at a multiple of 64
                const uint64_t bits = __builtin_amdgcn_ballot_w64(ok[u] && raw == 0xFFFFu);
                const uint64_t h0 = c00 + (uint64_t)u * kBlock + (t & ~(kWave - 1));
                if ((t & (kWave - 1)) == 0 && h0 < n) mask[h0 / kWave] = bits;
            }
            if (MODE == 1 && ok[u]) {
                const uint16_t f = (uint16_t)~raw;
                p[10] = (uint8_t)(f >> 8);
                p[11] = (uint8_t)f;
            }
        }
    }
}

// Dense header arrays (stride ≤ 64 B, e.g. a header-split ring): a wave takes
// 64 consecutive headers and streams their contiguous span — up to the last
// header's 20th byte — with full-width coalesced loads into its LDS slice
// (one round trip, every line fetched once), then each lane reads its header's
// dwords from LDS. Option dwords (IHL > 5) are loaded straight from memory,
// only when some lane of the wave has them. Same results as ipv4_hdr_kernel.
constexpr uint32_t kHdrDenseMaxStride = 64;

template <int MODE, int ROWS, int U>
__global__ __launch_bounds__(kBlock) void ipv4_hdr_dense_kernel(uint8_t* __restrict__ base, uint32_t stride,
                                                                uint32_t hdr_off, uint64_t n,
                                                                uint16_t* __restrict__ out,
                                                                uint64_t* __restrict__ mask) {
    extern __shared__ uint32_t lds_hdr[];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint32_t* my = lds_hdr + wave * (U * ROWS * (kRow / 4));
    const uint64_t ntasks = (n + kWave - 1) / kWave;
    const uint64_t wstep = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kWavesPerBlock + wave; t0 < ntasks; t0 += wstep * U) {
        // U tasks (64 headers each) per iteration: all their rows in flight at once
        uint8_t* fa[U];
        uint32_t cnt[U], lead[U], last[U], nb[U];
        u32x4 v[U][ROWS];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t task = t0 + (uint64_t)u * wstep;
            const uint64_t i0 = min(task, ntasks - 1) * kWave;
            cnt[u] = task < ntasks ? (uint32_t)min((uint64_t)kWave, n - i0) : 0u;
            uint8_t* first = base + i0 * stride + hdr_off;
            fa[u] = reinterpret_cast<uint8_t*>((uintptr_t)first & ~(uintptr_t)3);
            lead[u] = (uint32_t)(first - fa[u]);
            last[u] = (cnt[u] ? cnt[u] - 1 : 0u) * stride + lead[u];  // last header's offset from fa
            nb[u] = cnt[u] ? (last[u] + 20u + 3u) & ~3u : 0u;         // every header's first 20 bytes
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(fa[u], nb[u]);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) v[u][r] = bld16<true>(rs, r * kRow + lane * 16u);
        }
        __builtin_amdgcn_wave_barrier();  // the previous iteration's LDS reads are done
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
                *reinterpret_cast<u32x4*>(my + (u * ROWS + r) * (kRow / 4) + lane * 4) = v[u][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!cnt[u]) break;
            const uint32_t* mu = my + u * ROWS * (kRow / 4);
            const bool live = lane < cnt[u];
            const uint32_t rel = (live ? lane : 0u) * stride + lead[u];
            const uint32_t head = rel & 3u, w0 = rel >> 2;
            uint32_t d[16];
#pragma unroll
            for (int k = 0; k < 6; ++k) d[k] = mu[min(w0 + k, nb[u] / 4u - 1u)];
            const uint32_t len = ((d[0] >> (8 * head)) & 15u) * 4u;
            const bool ok = live && len >= 20u && hdr_off + len <= stride;
            const uint32_t nd = ok ? (head + len + 3u) >> 2 : 0u;
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                uint32_t m = keep_mask((int32_t)head, (int32_t)min(head + len, head + 20u), 4 * k);
                if (MODE == 1) m &= ~keep_mask((int32_t)head + 10, (int32_t)head + 12, 4 * k);
                acc = __builtin_amdgcn_sad_u16(d[k] & m, 0u, acc);
            }
            if (__ballot(nd > (head ? 6u : 5u))) {  // option bytes [20, len) of some header in this wave
                const __amdgpu_buffer_rsrc_t ro = make_rsrc(fa[u], (uint64_t)last[u] + 64u);
#pragma unroll
                for (int k = 5; k < 16; ++k)
                    d[k] = __builtin_amdgcn_raw_buffer_load_b32(ro, (uint32_t)k < nd ? (rel - head) + 4u * k : kOOB, 0,
                                                                 0);
#pragma unroll
                for (int k = 5; k < 16; ++k)
                    acc = __builtin_amdgcn_sad_u16(d[k] & keep_mask((int32_t)head + 20, (int32_t)(head + len), 4 * k),
                                                   0u, acc);
            }
            uint8_t* p = fa[u] + rel;
            const uint32_t raw = ok ? finish(acc, ((uintptr_t)p & 1u) == 0, 0u) : 0u;
            if (out && live) out[(t0 + (uint64_t)u * wstep) * kWave + lane] = (uint16_t)raw;
            if constexpr (MODE == 2) {  // task = 64 headers = one mask word
                const uint64_t bits = __builtin_amdgcn_ballot_w64(ok && raw == 0xFFFFu);
                if (lane == 0) mask[t0 + (uint64_t)u * wstep] = bits;
            }
            if (MODE == 1 && ok) {
                const uint16_t f = (uint16_t)~raw;
                p[10] = (uint8_t)(f >> 8);
                p[11] = (uint8_t)f;
            }
        }
    }
}

// Packed option-less headers (stride 20, hdr_off 0, 4-aligned base — a
// header-split ring): the array is one flat stream of whole dwords and every
// dword belongs to exactly one header. A wave task is 256 headers = 5 KiB = five
// full coalesced rows (16 B per lane, no idle lane); the rows go through the
// wave's 5 KiB LDS slice (ds_write_b128 lane-contiguous, then ds_read_b128 at an
// 80 B lane stride — conflict-free), so lane l ends up with headers 4l..4l+3 whole
// in registers: no byte masks, no per-header window. A 20-byte stride only fits
// IHL = 5, so any other IHL is malformed (out 0, header untouched), the rule of
// the general kernels. A lane's 4 results leave as one 8-byte store (512 B per
// wave); U tasks per register set, XCD-interleaved chunk deal.
constexpr uint32_t kHdr20Task = 256;
constexpr uint32_t kHdr20Lds = kHdr20Task * 20u;  // bytes of LDS per wave

// Software-pipelined: two register sets of U tasks; the loads of the next set are issued before the
// current set goes through LDS, so every wave keeps loads in flight while it computes and stores (one wave
// per SIMD at 1 block/CU has no other wave to cover those phases).
template <int MODE, int U>
__global__ __launch_bounds__(kBlock) void ipv4_hdr20_kernel(uint8_t* __restrict__ base, uint32_t n,
                                                            uint16_t* __restrict__ out, uint32_t clog,
                                                            uint64_t* __restrict__ mask) {
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    WaveStamps ws;
    ws.entry();
    uint32_t ntk = 0;  // tasks done (for the stamps)
    extern __shared__ u32x4 lds20[];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    u32x4* my = lds20 + wave * (kHdr20Lds / 16u);
    const uint32_t ntasks = (n + kHdr20Task - 1) / kHdr20Task;
    TaskIter it = task_iter(ntasks, wave);
    const ChunkDeal cd = chunk_deal(it, wave, clog, ntasks);
    const uint32_t end = (uint32_t)it.end, step = (uint32_t)it.step;
    const __amdgpu_buffer_rsrc_t ors = make_rsrc(out, out ? (uint64_t)n * 2 : 0);
    struct Set {
        __amdgpu_buffer_rsrc_t rs[U];
        uint32_t cnt[U], tk[U];
        u32x4 v[U][5];
    };
    auto live = [&](uint32_t t0) { return t0 < end && cd.task(t0) < ntasks; };
    auto issue = [&](uint32_t t0, Set& S) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ii = t0 + (uint32_t)u * step;
            const uint32_t task = cd.task(ii);
            S.tk[u] = task;
            S.cnt[u] = (ii < end && task < ntasks) ? min(kHdr20Task, n - task * kHdr20Task) : 0u;
            S.rs[u] = make_rsrc(base + (uint64_t)min(task, ntasks - 1) * kHdr20Lds, S.cnt[u] * 20u);
#pragma unroll
            for (int j = 0; j < 5; ++j) S.v[u][j] = bld16<true>(S.rs[u], j * kRow + lane * 16u);
        }
    };
    auto consume = [&](Set& S) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 5; ++j) asm volatile("" : "+v"(S.v[u][j]));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!S.cnt[u]) break;  // wave-uniform
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < 5; ++j) my[j * kWave + lane] = S.v[u][j];
            __builtin_amdgcn_wave_barrier();
            u32x4 q[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) q[j] = my[lane * 5 + j];
            const uint32_t d[20] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w, q[2].x, q[2].y,
                                    q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w, q[4].x, q[4].y, q[4].z, q[4].w};
            uint32_t res[4];
            bool ok[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t* w = d + 5 * h;
                ok[h] = (w[0] & 15u) == 5u;
                uint32_t acc = __builtin_amdgcn_sad_u16(w[0], 0u, 0u);
                acc = __builtin_amdgcn_sad_u16(w[1], 0u, acc);
                acc = __builtin_amdgcn_sad_u16(MODE == 1 ? (w[2] & 0xFFFFu) : w[2], 0u, acc);
                acc = __builtin_amdgcn_sad_u16(w[3], 0u, acc);
                acc = __builtin_amdgcn_sad_u16(w[4], 0u, acc);
                res[h] = ok[h] ? finish(acc, true, 0u) : 0u;
            }
            const uint32_t i0 = S.tk[u] * kHdr20Task + lane * 4u;
            if constexpr (MODE == 2) {
                // lane l holds headers 4l..4l+3 of the task, so word k (headers 64k..64k+63) is the 16 nibbles of
                // DPP row k: each lane shifts its nibble into place (lanes 0-7 of a row the low dword, 8-15 the
                // high), a 4-step row_shr sum (disjoint bits: sum = OR) leaves the word in the row's last lane.
                // Headers past n read as zeros (IHL 0: malformed, bit 0).
                const uint32_t nib = (uint32_t)(ok[0] && res[0] == 0xFFFFu) | ((uint32_t)(ok[1] && res[1] == 0xFFFFu) << 1) |
                                     ((uint32_t)(ok[2] && res[2] == 0xFFFFu) << 2) |
                                     ((uint32_t)(ok[3] && res[3] == 0xFFFFu) << 3);
                const uint32_t j = lane & 15u;
                uint32_t lo = j < 8u ? nib << (4u * j) : 0u, hi = j >= 8u ? nib << (4u * (j - 8u)) : 0u;
                lo += __builtin_amdgcn_update_dpp(0u, lo, 0x111, 0xF, 0xF, false);  // row_shr:1
                hi += __builtin_amdgcn_update_dpp(0u, hi, 0x111, 0xF, 0xF, false);
                lo += __builtin_amdgcn_update_dpp(0u, lo, 0x112, 0xF, 0xF, false);  // row_shr:2
                hi += __builtin_amdgcn_update_dpp(0u, hi, 0x112, 0xF, 0xF, false);
                lo += __builtin_amdgcn_update_dpp(0u, lo, 0x114, 0xF, 0xF, false);  // row_shr:4
                hi += __builtin_amdgcn_update_dpp(0u, hi, 0x114, 0xF, 0xF, false);
                lo += __builtin_amdgcn_update_dpp(0u, lo, 0x118, 0xF, 0xF, false);  // row_shr:8
                hi += __builtin_amdgcn_update_dpp(0u, hi, 0x118, 0xF, 0xF, false);
                const uint32_t wi = S.tk[u] * (kHdr20Task / kWave) + (lane >> 4);  // < 2^22 (n < 2^28 per launch)
                if (j == 15u && wi * kWave < n) mask[wi] = ((uint64_t)hi << 32) | lo;
            } else if (S.cnt[u] == kHdr20Task) {
                // sc1 (write-through): a task's 512 B of sums are whole lines; sent on at once instead of sitting
                // dirty in L2 until evicted among the reads, they cost 4.7% less time
                __builtin_amdgcn_raw_buffer_store_b64(v2u{res[0] | (res[1] << 16), res[2] | (res[3] << 16)}, ors,
                                                      i0 * 2u, 0, kStoreSc1);
            } else {
#pragma unroll
                for (int h = 0; h < 4; ++h)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)res[h], ors, i0 + h < n ? (i0 + h) * 2u : kOOB, 0,
                                                          kStoreSc1);
            }
            if constexpr (MODE == 1) {
#pragma unroll
                for (int h = 0; h < 4; ++h)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)bswap16u(~res[h] & 0xFFFFu), S.rs[u],
                                                          ok[h] ? lane * 80u + h * 20u + 10u : kOOB, 0, 0);
            }
        }
    };
    Set A, B;
    uint32_t t0 = (uint32_t)it.next;
    issue(t0, A);
    while (live(t0)) {
        const uint32_t t1 = t0 + step * U;
        issue(t1, B);
        consume(A);
        ntk += U;
        if (!live(t1)) break;
        t0 = t1 + step * U;
        issue(t0, A);
        consume(B);
        ntk += U;
    }
    ws.done(blockIdx.x * kWavesPerBlock + wave, ntk, lane);
}

// ---------------------------------------------------------------------------
// IPv4 pseudo-header partials: src(4) dst(4) 0 proto len16 (RFC 9293 §3.1).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void pseudo_ipv4_kernel(const uint8_t* __restrict__ src,
                                                             const uint8_t* __restrict__ dst,
                                                             const uint32_t* __restrict__ len,
                                                             uint32_t proto, uint64_t n,
                                                             uint32_t* __restrict__ partial) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* s = src + 4 * i;
        const uint8_t* d = dst + 4 * i;
        uint32_t sum = ((uint32_t)s[0] << 8 | s[1]) + ((uint32_t)s[2] << 8 | s[3]) +
                       ((uint32_t)d[0] << 8 | d[1]) + ((uint32_t)d[2] << 8 | d[3]) + proto +
                       (len[i] & 0xFFFFu);
        partial[i] = sum;
    }
}

// ---------------------------------------------------------------------------
// IPv6 pseudo-header partials: src(16) dst(16) len32 zero(3) nh (RFC 8200
// §8.1). Addresses are 16-byte records, so a dwordx4 load per address when the
// arrays are 4-aligned; byte loads otherwise.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t be_words_sum16(const uint8_t* a, bool aligned) {
    uint32_t s = 0;
    if (aligned) {
        const uint4 v = *reinterpret_cast<const uint4*>(a);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)  // LE dword b0 b1 b2 b3 → BE words b0b1 + b2b3
            s += ((w[k] & 0xFFu) << 8 | (w[k] >> 8 & 0xFFu)) + ((w[k] >> 16 & 0xFFu) << 8 | w[k] >> 24);
    } else {
#pragma unroll
        for (int k = 0; k < 16; k += 2) s += (uint32_t)a[k] << 8 | a[k + 1];
    }
    return s;
}

__global__ __launch_bounds__(kBlock) void pseudo_ipv6_kernel(const uint8_t* __restrict__ src,
                                                             const uint8_t* __restrict__ dst,
                                                             const uint32_t* __restrict__ len,
                                                             uint32_t nh, uint64_t n, bool aligned,
                                                             uint32_t* __restrict__ partial) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t l = len[i];
        partial[i] = be_words_sum16(src + 16 * i, aligned) + be_words_sum16(dst + 16 * i, aligned) + (l >> 16) +
                     (l & 0xFFFFu) + nh;
    }
}

// ---------------------------------------------------------------------------
// Receive-side parse (parseSegment, transport/tcp/tcp.go:130-185) of a batch of
// TCP segments, d_base[offsets[i], offsets[i+1]), any alignment, into SoA
// fields. One thread per segment (the work is the 20-byte header, not the
// payload): the header's dwords are loaded from the 4-aligned address below its
// start — only those holding segment bytes, so nothing past the segment's last
// dword is read — and realigned with v_alignbyte. Fields are the reference's:
// offset is the whole byte 12 (tcp.go:142), dataAt = offset·4 (:150). Options
// (offset > 5) are walked byte by byte exactly as the reference does — EOL ends
// the walk, NOP advances 1, MSS reads its length and advances 6 whatever the
// length (:160-179) — and counted. Where the reference fails the segment comes
// back zero with a status: too short (:131), data offset past the end (:152);
// where its MSS slice runs past the segment (:173-174: raw[optIdx+1] past the
// end panics; a data slice past len(raw) panics, or reads the caller's bytes
// beyond the segment when the slice has spare capacity — not a property of the
// bytes) or it would loop forever on another option kind (:162-178, optIdx
// never advances), the status says so and the walk stops.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void tcp_parse_kernel(const uint8_t* __restrict__ base,
                                                           const uint64_t* __restrict__ offsets, uint64_t n,
                                                           TcpParsedSoA o) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s0 = offsets[i], s1 = offsets[i + 1];
        const uint64_t len = s1 > s0 ? s1 - s0 : 0;
        const uint8_t* p = base + s0;
        uint32_t status = 0, nopt = 0;
        uint32_t H[5] = {0u, 0u, 0u, 0u, 0u};
        if (len < 20) {
            status = 1;  // "segment too short"
        } else {
            const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
            const uint32_t* pa = reinterpret_cast<const uint32_t*>((uintptr_t)p - sh);
            uint32_t w[6];
#pragma unroll
            for (int k = 0; k < 6; ++k)  // dword k holds segment bytes iff it starts before the segment's end
                w[k] = (uint64_t)(4 * k) < len + sh ? pa[k] : 0u;
#pragma unroll
            for (int k = 0; k < 5; ++k) H[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
            const uint32_t off = H[3] & 0xFFu;
            const uint64_t data_at = (uint64_t)off * 4u;
            if (data_at > len) {
                status = 2;  // "advertised data offset too long"
            } else if (off > 5u) {
                uint64_t idx = 20;
                while (idx < data_at) {
                    const uint32_t kind = p[idx];
                    if (kind == 0u) break;  // EOL: the rest is padding
                    if (kind == 1u) {
                        ++idx;
                    } else if (kind == 2u) {
                        if (idx + 2 > len || idx + 2 + p[idx + 1] > len) {
                            status = 3;  // the MSS slice would run past the segment
                            break;
                        }
                        idx += 6;  // 1(kind) + 1(length) + 4(data), as tcp.go:175
                    } else {
                        status = 4;  // unknown kind: the reference's loop never advances
                        break;
                    }
                    ++nopt;
                }
            }
            if (o.data_off) o.data_off[i] = status ? 0u : s0 + data_at;
        }
        if (status) {
            nopt = 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) H[k] = 0u;  // the reference returns segment{}
            if (len < 20 && o.data_off) o.data_off[i] = 0u;
        }
        if (o.src_port) o.src_port[i] = (uint16_t)bswap16u(H[0] & 0xFFFFu);
        if (o.dst_port) o.dst_port[i] = (uint16_t)bswap16u(H[0] >> 16);
        if (o.seq) o.seq[i] = bswap32u(H[1]);
        if (o.ack) o.ack[i] = bswap32u(H[2]);
        if (o.offset) o.offset[i] = (uint8_t)H[3];
        if (o.ctl) o.ctl[i] = (uint8_t)(H[3] >> 8);
        if (o.window) o.window[i] = (uint16_t)bswap16u(H[3] >> 16);
        if (o.checksum) o.checksum[i] = (uint16_t)bswap16u(H[4] & 0xFFFFu);
        if (o.urgent) o.urgent[i] = (uint16_t)bswap16u(H[4] >> 16);
        if (o.n_options) o.n_options[i] = (uint8_t)min(nopt, 255u);
        if (o.status) o.status[i] = (uint8_t)status;
    }
}

// ---------------------------------------------------------------------------
// Receive-side verify as a bitmask (tcp.go:70): bit i of the mask is
// (raw[i] == 0xFFFF). One wave covers 64 sums and its ballot is one u64 word.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void verify_mask_kernel(const uint16_t* __restrict__ raw, uint64_t n,
                                                             uint64_t* __restrict__ mask) {
    const uint64_t words = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64; w < words;
         w += (uint64_t)gridDim.x * blockDim.x / 64) {
        const uint64_t i = w * 64 + lane;
        const bool ok = i < n && raw[i] == 0xFFFFu;
        const uint64_t bits = __ballot(ok);
        if (lane == 0) mask[w] = bits;
    }
}

// ---------------------------------------------------------------------------
// splitmix64 synthetic stream (bench/test data).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void fill_words_kernel(uint64_t* __restrict__ dst, uint64_t w0,
                                                            uint64_t nwords, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
         i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = splitmix64_at(seed, w0 + i);
}

__global__ __launch_bounds__(kBlock) void fill_bytes_kernel(uint8_t* __restrict__ dst, uint64_t byte_off,
                                                            uint64_t nbytes, uint64_t seed) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nbytes;
         j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t pos = byte_off + j;
        dst[j] = (uint8_t)(splitmix64_at(seed, pos >> 3) >> (8 * (pos & 7)));
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit). Per-path defaults, measured
// best on MI355X; a caller's nsx_tune may override them.
// ---------------------------------------------------------------------------
// XCD-interleaved chunk deal (chunk_deal): log2 of the tasks per chunk. param = nsx_tune.xcd_chunk:
// 1..20 fixed, 0 auto, anything else off (contiguous eighths). Auto: chunks of at most 24 MiB of batch
// (capped so that there are at least 64 chunks); off when that
// leaves < 4 tasks a chunk. Contiguous eighths ran 8% slow on some allocations on some boxes; 2^10-2^14-task
// chunks never did (round 1 allocation study).
static uint32_t deal_clog(int param, uint64_t ntasks, uint64_t task_bytes) {
    if (param >= 1 && param <= 20) return (uint32_t)param;
    if (param != 0) return 0u;
    uint32_t k = 0;
    while (k < 20 && (task_bytes << (k + 1)) <= (24ull << 20)) ++k;
    while (k > 0 && (ntasks >> k) < 64) --k;
    // XCD x takes chunks x, x + 8, ...: when the chunk count is not a multiple of 8, some XCDs hold one chunk
    // more than others and the launch waits for them. Halve the chunks until the busiest XCD holds at most
    // 2% more tasks than the mean (no change for the power-of-two bench batches).
    while (k > 2) {
        const uint64_t chunks = (ntasks + (1ull << k) - 1) >> k;
        if (((chunks + 7) / 8) * 8 * (1ull << k) * 100 <= ntasks * 102) break;
        --k;
    }
    return k >= 2 ? k : 0u;
}

static uint32_t grid_for(uint64_t wave_tasks, uint32_t max_blocks) {
    const uint64_t want = (wave_tasks + kWavesPerBlock - 1) / kWavesPerBlock;
    return (uint32_t)(want < max_blocks ? want : max_blocks);
}

static uint32_t max_blocks_of(const LaunchCfg& c, int default_bpc) {
    const int bpc = (c.blocks_per_cu >= 1 && c.blocks_per_cu <= 8) ? c.blocks_per_cu : default_bpc;
    return (uint32_t)(c.cus * bpc);
}

static bool use_block_mode(const LaunchCfg& c, uint64_t n) {
    return c.block_mode == 2 || (c.block_mode == 0 && n < (uint64_t)c.cus * 4);
}

// Auto window of the fixed short-segment path (window_bytes = 0): batches of at least twice this size are
// launched as back-to-back windows of about this many bytes. One launch over config 5's 25 GB span runs
// ~5% slower per byte than 1.6 GB windows of it.
constexpr uint64_t kAutoWindow = 1600ull * 1000 * 1000;
// Buffer descriptors address < 2^31 bytes of results / partials / offsets: batches are cut into launches
// of at most this many segments.
constexpr uint64_t kFixedChunk = 1ull << 28;
constexpr uint64_t kRaggedChunk = 1ull << 27;

static uint64_t fixed_rows(uint32_t seg_len) { return ((uint64_t)seg_len + 3 + kRow - 1) / kRow; }

// Segments per launch of the fixed short-segment path.
static uint64_t fixed_window(const LaunchCfg& c, uint64_t stride, uint64_t n) {
    if (stride == 0) return kFixedChunk;  // every segment aliases the first: one launch per chunk
    if (c.window_bytes > 0) {
        const uint64_t w = (uint64_t)c.window_bytes / stride;
        return w < 1 ? 1 : (w < kFixedChunk ? w : kFixedChunk);
    }
    if (c.window_bytes == 0 && n * stride >= 2 * kAutoWindow) {
        const uint64_t nw = (n * stride + kAutoWindow - 1) / kAutoWindow;  // config 5: 16 windows of 1M segments
        const uint64_t win = (n + nw - 1) / nw;
        return win < kFixedChunk ? win : kFixedChunk;
    }
    return kFixedChunk;
}

uint64_t fixed_launch_count(const LaunchCfg& c, uintptr_t /*base*/, uint64_t stride, uint32_t seg_len, uint64_t n) {
    if (n == 0) return 0;
    if (use_block_mode(c, n) || fixed_rows(seg_len) > 4) return 1;
    const uint64_t win = fixed_window(c, stride, n);
    return (n + win - 1) / win;
}

// One launch of the short-segment fixed path: U segments per wave task, NR rows per segment.
static uint32_t* deal_heads(const LaunchCfg& c, hipStream_t st);  // below: the stream's work-deal counters

static hipError_t launch_fixed_short(const LaunchCfg& c, const uint8_t* base, uint64_t stride, uint32_t seg_len,
                                     uint64_t n, const uint32_t* partial, uint16_t* out, int nrows, bool aligned,
                                     hipStream_t st) {
    // Aligned (config 2): the software-pipelined kernel, 8-segment tasks at one block per CU — two register
    // sets of 8 × 2 KiB per wave, a wave per SIMD (config 2 0.2222 → 0.2184 ms, config 5 3.712 → 3.626 ms
    // against 4-segment tasks at 2 blocks/CU). Unaligned: 4-segment tasks, 2 blocks/CU.
    int u = (c.segs_per_wave == 1 || c.segs_per_wave == 2 || c.segs_per_wave == 4 || c.segs_per_wave == 8)
                ? c.segs_per_wave : (aligned ? 8 : 4);
    if (nrows == 4 && u > 4) u = 4;
    const uint64_t ntasks = (n + u - 1) / u;
    const uint32_t grid = grid_for(ntasks, max_blocks_of(c, aligned ? 1 : 2));
    const uint32_t clog = deal_clog(c.xcd_chunk, ntasks, (uint64_t)u * stride);
    // The default aligned shapes deal their last tasks through each block's ring (a fifth, dealer wave per block;
    // §7 step 77) when the stream has heads and the batch has at least 64 tasks per block.
    if (kFixedDealMode != 0 && aligned && c.segs_per_wave == 0 && ntasks >= 64ull * grid) {
        if (uint32_t* deal = deal_heads(c, st)) {
#define NSX_FIXED_DEAL(U_, NR_)                                                                                  \
    if (u == U_ && nrows == NR_) {                                                                               \
        hipLaunchKernelGGL((csum_fixed_swp_kernel<U_, NR_, kFixedDealMode>), dim3(grid),                          \
                           dim3(kFixedDealMode == 1 ? kBlock + kWave : kBlock), 0, st, base, stride, seg_len,     \
                           (uint32_t)n, partial, out, clog, deal);                                               \
        return hipGetLastError();                                                                                \
    }
            NSX_FIXED_DEAL(8, 1) NSX_FIXED_DEAL(8, 2) NSX_FIXED_DEAL(4, 4)
#undef NSX_FIXED_DEAL
        }
    }
#define NSX_FIXED(U_, NR_)                                                                                    \
    if (u == U_ && nrows == NR_) {                                                                             \
        if (aligned)                                                                                           \
            hipLaunchKernelGGL((csum_fixed_swp_kernel<U_, NR_, 0>), dim3(grid), dim3(kBlock), 0, st, base, stride, \
                               seg_len, (uint32_t)n, partial, out, clog, nullptr);                             \
        else                                                                                                   \
            hipLaunchKernelGGL((csum_fixed_buf_kernel<U_, NR_>), dim3(grid), dim3(kBlock), 0, st, base, stride, \
                               seg_len, (uint32_t)n, partial, out, clog);                                      \
        return hipGetLastError();                                                                              \
    }
    NSX_FIXED(1, 1) NSX_FIXED(2, 1) NSX_FIXED(4, 1) NSX_FIXED(8, 1)
    NSX_FIXED(1, 2) NSX_FIXED(2, 2) NSX_FIXED(4, 2) NSX_FIXED(8, 2)
    NSX_FIXED(1, 4) NSX_FIXED(2, 4) NSX_FIXED(4, 4)
#undef NSX_FIXED
    return hipErrorInvalidValue;
}

hipError_t launch_fixed(const LaunchCfg& c, const void* d_base, uint64_t stride, uint32_t seg_len,
                        uint64_t n, const uint32_t* partial, uint16_t* out, hipStream_t st) {
    const uint8_t* base = static_cast<const uint8_t*>(d_base);
    const uint8_t* end = base + (n - 1) * stride + seg_len;
    const uint8_t* safe_end = reinterpret_cast<const uint8_t*>(((uintptr_t)end + 3) & ~(uintptr_t)3);
    if (use_block_mode(c, n)) {
        const uint32_t grid = (uint32_t)std::min<uint64_t>(n, max_blocks_of(c, 8));
        hipLaunchKernelGGL((csum_block_kernel<false, 4, false>), dim3(grid), dim3(kBlock), 0, st, base, nullptr, stride,
                           seg_len, n, partial, out, nullptr, safe_end);
        return hipGetLastError();
    }
    const uint64_t rows = fixed_rows(seg_len);  // a segment window starts up to 3 bytes early
    if (rows <= 4) {
        const int nrows = rows <= 1 ? 1 : (rows <= 2 ? 2 : 4);
        const bool aligned = ((uintptr_t)base & 3u) == 0 && (stride & 3u) == 0 && (seg_len & 3u) == 0;
        const uint64_t win = fixed_window(c, stride, n);
        for (uint64_t c0 = 0; c0 < n; c0 += win) {
            const uint64_t cn = n - c0 < win ? n - c0 : win;
            const hipError_t e = launch_fixed_short(c, base + c0 * stride, stride, seg_len, cn,
                                                    partial ? partial + c0 : nullptr, out + c0, nrows, aligned, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // Long segments (config 4's 64 KiB): one wave per segment, rows 4 at a time, 2 blocks/CU.
    const uint32_t grid = grid_for(n, max_blocks_of(c, 2));
    const uint32_t clog = deal_clog(c.xcd_chunk, n, std::max<uint64_t>(stride, 1));
    hipLaunchKernelGGL((csum_wave_kernel<4>), dim3(grid), dim3(kBlock), 0, st, base, stride, seg_len, n, partial, out,
                       safe_end, clog);
    return hipGetLastError();
}

// The deal counters (§7 step 72) of the receive pass and the ragged checksum's small-segment mode: kDealSlots sets
// of kDealHeads heads per device, zero at load; every launch leaves its heads at 0 (DealtRuns), so a set can serve
// one stream's launches one after another, whichever kernel they are.
__device__ uint32_t g_deal_heads[kDealSlots * kDealHeads * kDealStride];

// Which streams get a set. The deal is correct only if the launches sharing a set run one after another: the wave
// that draws a head's last pull resets it for the next launch (DealtRuns). So a set is given only to a handle that
// names ONE ordered queue of the current device:
// - a stream the caller created (hipStreamCreate*), on the current device;
// - the device's null stream (nullptr, and hipStreamLegacy, its explicit name; keyed together).
// Every other launch takes equal static shares (nullptr), bit-exact as well:
// - hipStreamPerThread: one handle value that stands for a different stream on every host thread, so launches from
//   two threads on it may run at once;
// - a stream of another device (g_deal_heads is per device: the set would be device A's memory under a kernel on B);
// - a stream being captured into a graph (a graph's launches could replay on several streams at once);
// - tune.deal = -1 (the A/B switch that replaced round 5's NSX_NO_DEAL build), or every set given out.
// A set stays with its stream for the process unless the stream is returned (nsx_stream_release, before the caller
// destroys it): returned sets are given out again first, so streams created and destroyed in a loop do not use up
// the 64 sets.
struct DealSets {
    uint32_t* base = nullptr;    // the device's g_deal_heads
    uint32_t fresh = 0;          // sets never given out start here
    std::vector<uint32_t> free;  // returned sets (their heads are 0: every launch that used them has completed)
};
static std::mutex g_deal_mu;
static std::map<std::pair<int, hipStream_t>, uint32_t> g_deal_slot;  // (device, stream) → set
static std::map<int, DealSets> g_deal_dev;

static hipStream_t deal_key(hipStream_t st) { return st == hipStreamLegacy ? nullptr : st; }

static uint32_t* deal_heads(const LaunchCfg& c, hipStream_t st) {
    if (c.deal < 0 || st == hipStreamPerThread) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
        (void)hipGetLastError();  // a refused query (e.g. the legacy stream while another captures) is not the launch's error
        return nullptr;
    }
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    int dev = 0, sdev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipStreamGetDevice(st, &sdev) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (sdev != dev) return nullptr;
    const hipStream_t key = deal_key(st);
    std::lock_guard<std::mutex> lock(g_deal_mu);
    DealSets& ds = g_deal_dev[dev];
    if (!ds.base) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_deal_heads)) != hipSuccess || !p) {
            (void)hipGetLastError();
            return nullptr;
        }
        ds.base = static_cast<uint32_t*>(p);
    }
    uint32_t slot;
    auto it = g_deal_slot.find({dev, key});
    if (it != g_deal_slot.end()) {
        slot = it->second;
    } else if (!ds.free.empty()) {
        slot = ds.free.back();
        ds.free.pop_back();
        g_deal_slot[{dev, key}] = slot;
    } else {
        if (ds.fresh >= kDealSlots) return nullptr;
        slot = ds.fresh++;
        g_deal_slot[{dev, key}] = slot;
    }
    return ds.base + (size_t)slot * kDealHeads * kDealStride;
}

// Return stream st's sets (on every device) for reuse: the caller has synchronised st and is about to destroy it.
void deal_release(hipStream_t st) {
    const hipStream_t key = deal_key(st);
    std::lock_guard<std::mutex> lock(g_deal_mu);
    for (auto it = g_deal_slot.begin(); it != g_deal_slot.end();) {
        if (it->first.second == key) {
            g_deal_dev[it->first.first].free.push_back(it->second);
            it = g_deal_slot.erase(it);
        } else {
            ++it;
        }
    }
}

// Sets given out on the current device (tests: a released stream's set is reused, not a fresh one).
uint32_t deal_sets_in_use(int dev) {
    std::lock_guard<std::mutex> lock(g_deal_mu);
    auto it = g_deal_dev.find(dev);
    return it == g_deal_dev.end() ? 0u : it->second.fresh - (uint32_t)it->second.free.size();
}

template <bool VERIFY>
static hipError_t launch_ragged_scan(const LaunchCfg& c, const uint8_t* base, const uint64_t* offsets, uint64_t n,
                                     const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st) {
    // Default: double-buffered batches of 2 rows, 63-segment runs, 2 blocks/CU (tools/ab.py --config 3, same
    // process on three boxes: 0.680 ms against 0.691 for single batches of 8 rows, 0.702-0.713 for pipelined
    // batches of 3 or 4 rows, 0.93 for 1 row). kernel 2 (NSX_TUNE_KERNEL_SCAN_PLAIN):
    // single batches of 4, 8 (default) or 16 rows.
    const bool pipe = c.kernel != 2;
    const int rows = pipe ? (c.rows == 2 || c.rows == 4 || c.rows == 8 ? c.rows : 2)
                          : (c.rows == 4 || c.rows == 8 || c.rows == 16 ? c.rows : 8);
    const uint32_t run = (c.run_segs >= 1 && c.run_segs <= (int)kScanRun) ? (uint32_t)c.run_segs : 0u;  // 0: default
    const uint32_t task = run ? run : kScanRun;
    // The default shape's kernel (NS = 2: register-capped for 4 blocks/CU) holds every form: the small-segment mode,
    // the LDS form, and streamed runs of one set (the default since §7 step 64) or two (segs_per_wave 5; the round-2
    // default, §7 step 33). segs_per_wave = 1 runs the uncapped single-set instantiation.
    const int ns = (pipe && rows == 2 && c.segs_per_wave != 1) ? 2 : 1;
    // force the small-segment mode (2), the four-wave LDS form (3) or runs of two sets (5); 0: by mean segment size
    // (ragged_tune_valid rejects any other value but 1)
    const int sets = c.segs_per_wave == 2 || c.segs_per_wave == 3 || c.segs_per_wave == 5 ? c.segs_per_wave : 0;
    // the LDS slots (four per block: the LDS forms' rows, the streamed forms' parked results; the small-segment mode
    // gives two to each of its two waves) whenever the kernel may choose an LDS form, and on grids of up to 4 blocks
    // per CU (33.8 KB of LDS per block caps a launch at 4 resident blocks per CU): forced streamed shapes above 4
    // blocks per CU allocate none and store their results directly
    const bool lds_form = sets == 2 || sets == 3 || (ns == 2 && sets == 0) || c.blocks_per_cu <= 4;
    const size_t lds = lds_form ? (size_t)kScanSlot * kWavesPerBlock : 0;
    // Default grid: 4 blocks/CU, of which a batch of segments averaging ≥ kScanBigMean uses 2 (active_blocks;
    // config 3 keeps its 2 blocks/CU) and a batch averaging < kScanLdsSeg two waves per block (§7 step 61). A
    // blocks_per_cu override runs exactly that grid.
    const bool pick = c.blocks_per_cu == 0 && pipe && rows == 2;
    const uint32_t mb = pick ? (uint32_t)c.cus * 4u : max_blocks_of(c, 2);
    const uint32_t keep = pick ? 2u : 0u;
    uint32_t* deal = deal_heads(c, st);  // the small-segment mode's dealt runs
    for (uint64_t c0 = 0; c0 < n; c0 += kRaggedChunk) {
        const uint32_t cn = (uint32_t)(n - c0 < kRaggedChunk ? n - c0 : kRaggedChunk);
        const uint32_t grid = grid_for((cn + task * ns - 1) / (task * ns), mb);
        const uint32_t* pc = partial ? partial + c0 : nullptr;
        uint16_t* oc = out ? out + c0 : nullptr;
        uint8_t* kc = ok ? ok + c0 : nullptr;
#define NSX_RSCAN(R_, P_, NS_)                                                                                 \
        if (rows == R_ && pipe == P_ && ns == NS_)                                                              \
            hipLaunchKernelGGL((csum_ragged_scan_kernel<R_, VERIFY, P_, NS_>), dim3(grid), dim3(kBlock), lds, st,\
                               base, offsets + c0, cn, pc, oc, kc, run, sets, keep, lds_form, deal);
        NSX_RSCAN(2, true, 1) NSX_RSCAN(4, true, 1) NSX_RSCAN(8, true, 1)
        NSX_RSCAN(4, false, 1) NSX_RSCAN(8, false, 1) NSX_RSCAN(16, false, 1)
        NSX_RSCAN(2, true, 2)
#undef NSX_RSCAN
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_ragged(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st) {
    if (!ragged_tune_valid(c)) return hipErrorInvalidValue;
    const uint8_t* base = static_cast<const uint8_t*>(d_base);
    if (use_block_mode(c, n)) {  // few segments: a block per segment
        const uint32_t grid = (uint32_t)std::min<uint64_t>(n, max_blocks_of(c, 8));
        if (ok)
            hipLaunchKernelGGL((csum_block_kernel<true, 4, true>), dim3(grid), dim3(kBlock), 0, st, base, d_offsets,
                               0, 0, n, partial, out, ok, nullptr);
        else
            hipLaunchKernelGGL((csum_block_kernel<true, 4, false>), dim3(grid), dim3(kBlock), 0, st, base, d_offsets,
                               0, 0, n, partial, out, nullptr, nullptr);
        return hipGetLastError();
    }
    if (ok) return launch_ragged_scan<true>(c, base, d_offsets, n, partial, out, ok, st);
    return launch_ragged_scan<false>(c, base, d_offsets, n, partial, out, nullptr, st);
}

bool ragged_tune_valid(const LaunchCfg& c) {
    // segs_per_wave: 0 auto, 1 the single-set kernel, 2 / 3 / 5 forced forms (4, runs of four sets, was removed in
    // round 4: NSX_EINVAL rather than silently running another form)
    const int s = c.segs_per_wave;
    return s == 0 || s == 1 || s == 2 || s == 3 || s == 5;
}

bool rx_tune_valid(const LaunchCfg& c) {
    // segs_per_wave: 0 auto, 1 / 2 forced per-wave forms of the rows / blocks_per_cu shapes, 5 / 6 / 7 / 8 / 9 a mode of
    // the default grid — which means nothing on the shapes rows / blocks_per_cu select (silently running
    // the auto shape there made fuzz cases test another form than they named); any other value names no form
    // (3, 4 or 9 used to run the automatic shape)
    const int s = c.segs_per_wave;
    if (!(s == 0 || s == 1 || s == 2 || (s >= 5 && s <= 9))) return false;
    const bool grid_mode = s >= 5;
    return !grid_mode || ((c.rows == 0 || c.rows == 2) && c.blocks_per_cu == 0);
}

hipError_t launch_rx_tcp(const LaunchCfg& c, int ipver, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         uint64_t* mask, uint16_t* ip_raw, uint16_t* tcp_raw, hipStream_t st) {
    if (!rx_tune_valid(c)) return hipErrorInvalidValue;
    // Double-buffered batches of 2 rows, 3 blocks/CU (tools/ab.py --config 10, same process: 0.1294 ms against
    // 0.1305 for batches of 4 rows, 0.1348 for single batches of 8 rows, 0.145 for 2 rows at 2 blocks/CU, 0.136
    // at 4); launches of ≤ 2^27 frames (a multiple of 64, so every launch starts on a mask word)
    const int rows = (c.rows == 2 || c.rows == 4 || c.rows == 8 || c.rows == 16) ? c.rows : 2;
    // Non-default shapes (below the default grid): per wave the LDS form or streamed runs of 64 frames, by each
    // wave's mean frame size or forced by segs_per_wave 1 / 2; blocks_per_cu runs exactly that grid (default 3;
    // the register-capped instantiation from 4 blocks/CU up).
    const int sets = c.segs_per_wave == 1 || c.segs_per_wave == 2 ? c.segs_per_wave : 0;
    // the LDS form's per-wave slots (3 blocks/CU: 100 KB), unless streamed runs are forced (sets 1)
    const size_t lds = sets == 1 ? 0 : (size_t)kRxSlot * kWavesPerBlock;
    const uint32_t mb = max_blocks_of(c, 3);
    const uint32_t keep = 0u;
    const bool w4 = rows == 2 && mb >= (uint32_t)c.cus * 4u;
    const uint8_t* base = static_cast<const uint8_t*>(d_base);
    // The default shape (and the forms it picks, forced by segs_per_wave 5 / 6 for tests and A/B): the
    // PF = -1 kernel at 4 blocks/CU, each block with two 15-row prefix slots of LDS (its four 7-row slots fit the
    // same 38.5 KB), the mode chosen in-kernel by the batch's mean frame.
    const bool auto_grid = rows == 2 && c.blocks_per_cu == 0 &&
                           (c.segs_per_wave == 0 || (c.segs_per_wave >= 5 && c.segs_per_wave <= 9));
    if (auto_grid) {
        // per block: two 15-row prefix slots or four 7-row slots (38.5 KB); forced mode 9, two DMA rings (kRingWave
        // each: 40 KB, 4 blocks per CU taking the CU's whole 160 KB)
        constexpr size_t la_def = (size_t)PfxSlot<15>::kBytes * 2, la_ring = (size_t)kRingWave * 2;
        static_assert(la_def >= (size_t)PfxSlot<7>::kBytes * kWavesPerBlock && la_def * 4 <= 163840 &&
                          la_ring * 4 <= 163840, "4 blocks per CU");
        const size_t la = c.segs_per_wave == 9 ? la_ring : la_def;
        uint32_t* deal = deal_heads(c, st);
        for (uint64_t c0 = 0; c0 < n; c0 += kRaggedChunk) {
            const uint32_t cn = (uint32_t)(n - c0 < kRaggedChunk ? n - c0 : kRaggedChunk);
            const uint32_t grid = grid_for((cn + kRxRun - 1) / kRxRun, (uint32_t)c.cus * 4u);
            uint16_t* ic = ip_raw ? ip_raw + c0 : nullptr;
            uint16_t* tc = tcp_raw ? tcp_raw + c0 : nullptr;
            if (ipver == 6)
                hipLaunchKernelGGL((rx_tcp_kernel<2, true, 4, -1>), dim3(grid), dim3(kBlock), la, st, base, d_offsets + c0,
                                   cn, mask + c0 / 64, nullptr, tc, c.segs_per_wave, 0u, deal);
            else
                hipLaunchKernelGGL((rx_tcp_kernel<2, false, 4, -1>), dim3(grid), dim3(kBlock), la, st, base,
                                   d_offsets + c0, cn, mask + c0 / 64, ic, tc, c.segs_per_wave, 0u, deal);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    for (uint64_t c0 = 0; c0 < n; c0 += kRaggedChunk) {
        const uint32_t cn = (uint32_t)(n - c0 < kRaggedChunk ? n - c0 : kRaggedChunk);
        const uint32_t grid = grid_for((cn + kRxRun - 1) / kRxRun, mb);
        uint16_t* ic = ip_raw ? ip_raw + c0 : nullptr;
        uint16_t* tc = tcp_raw ? tcp_raw + c0 : nullptr;
#define NSX_RX(R_, W_)                                                                                            \
        if (rows == R_ && w4 == (W_ == 4) && ipver == 6)                                                           \
            hipLaunchKernelGGL((rx_tcp_kernel<R_, true, W_>), dim3(grid), dim3(kBlock), lds, st, base, d_offsets + c0, \
                               cn, mask + c0 / 64, nullptr, tc, sets, keep, nullptr);                                    \
        if (rows == R_ && w4 == (W_ == 4) && ipver != 6)                                                           \
            hipLaunchKernelGGL((rx_tcp_kernel<R_, false, W_>), dim3(grid), dim3(kBlock), lds, st, base,                \
                               d_offsets + c0, cn, mask + c0 / 64, ic, tc, sets, keep, nullptr);
        NSX_RX(2, 1) NSX_RX(4, 1) NSX_RX(8, 1) NSX_RX(16, 1) NSX_RX(2, 4)
#undef NSX_RX
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pseudo_ipv4(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t proto,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st) {
    const uint64_t want = (n + kBlock - 1) / kBlock;
    const uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
    hipLaunchKernelGGL(pseudo_ipv4_kernel, dim3(grid), dim3(kBlock), 0, st, src, dst, len, (uint32_t)proto, n,
                       partial);
    return hipGetLastError();
}

hipError_t launch_pseudo_ipv6(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t nh,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st) {
    const uint64_t want = (n + kBlock - 1) / kBlock;
    const uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
    const bool aligned = (((uintptr_t)src | (uintptr_t)dst) & 3u) == 0;
    hipLaunchKernelGGL(pseudo_ipv6_kernel, dim3(grid), dim3(kBlock), 0, st, src, dst, len, (uint32_t)nh, n,
                       aligned, partial);
    return hipGetLastError();
}

hipError_t launch_tcp_parse(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                            const TcpParsedSoA& o, hipStream_t st) {
    const uint32_t grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((n + kBlock - 1) / kBlock, max_blocks_of(c, 4)));
    hipLaunchKernelGGL(tcp_parse_kernel, dim3(grid), dim3(kBlock), 0, st, static_cast<const uint8_t*>(d_base),
                       d_offsets, n, o);
    return hipGetLastError();
}

hipError_t launch_verify_mask(const uint16_t* raw, uint64_t n, uint64_t* mask, uint32_t max_blocks,
                              hipStream_t st) {
    const uint64_t want = (n + kBlock - 1) / kBlock;
    const uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
    hipLaunchKernelGGL(verify_mask_kernel, dim3(grid), dim3(kBlock), 0, st, raw, n, mask);
    return hipGetLastError();
}

constexpr uint64_t kBuildGroupBytes = 24576;  // images per TCP build wave task, about

hipError_t launch_tcp_build(const LaunchCfg& c, const TcpHdrSoA& h, const uint8_t* opts, const uint64_t* opt_off,
                            const uint8_t* data, const uint64_t* data_off, uint64_t data_bytes,
                            const uint32_t* partial, uint64_t n, uint8_t* out, const uint64_t* out_off,
                            uint16_t* raw, hipStream_t st) {
    // Path by layout: groups of ≤ 2-row images software-pipelined (the fast composition when every segment of
    // the group allows it, else the general one); longer images unpipelined. kernel 2 forces the unpipelined
    // path, kernel 3 the general pipelined composition (test coverage of those paths on every layout).
    // Group size: up to 16 segments per wave task (fewer when n would leave waves idle) at 2 blocks/CU — the
    // chip's waves then hold a compact window of the batch (2048 × 16 segments in flight instead of 4096 × 64):
    // same process, three boxes, workloads 6 / 8: 0.602 / 0.609 ms against 0.633 / 0.640 for 64-segment groups
    // at 4 blocks/CU (tools/ab.py).
    // Longer images take fewer segments per task, so that a task stays near 24 KiB of images: 256K jumbo builds
    // (8960 B images, workload 12) in groups of 3 ran 0.888 ms against 0.934 for 16 (2: 0.891, 1: 0.901, 32:
    // 0.946). The image size comes from the payload bytes per segment the caller passes.
    const uint32_t max_blocks = max_blocks_of(c, 2);
    const uint64_t waves = (uint64_t)max_blocks * kWavesPerBlock;
    const uint64_t wire = data_bytes / n + 20;  // mean image bytes (options aside)
    const uint64_t by_size = std::max<uint64_t>(1, (kBuildGroupBytes + wire / 2) / wire);
    uint32_t group = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(16, by_size), std::max<uint64_t>(1, (n + waves - 1) / waves));
    if (c.run_segs >= 1 && c.run_segs <= 64) group = (uint32_t)c.run_segs;
    const uint64_t tasks = (n + group - 1) / group;
    const uint32_t grid = grid_for(tasks, max_blocks);
    const uint32_t clog = deal_clog(c.xcd_chunk, tasks, (uint64_t)group * 2u * wire);  // payload + image per segment
    const int pipe = c.kernel == 2 ? 0 : c.kernel == 3 ? 2 : 1;
    if (opt_off)
        hipLaunchKernelGGL((tcp_build_kernel<0, 0, 2, true>), dim3(grid), dim3(kBlock), 0, st, h, opts, opt_off, data,
                           data_off, data_bytes, partial, n, out, out_off, raw, group, clog, pipe);
    else
        hipLaunchKernelGGL((tcp_build_kernel<0, 0, 2, false>), dim3(grid), dim3(kBlock), 0, st, h, opts, opt_off, data,
                           data_off, data_bytes, partial, n, out, out_off, raw, group, clog, pipe);
    return hipGetLastError();
}

// Headers per launch of the packed 20 B header kernel. Like the fixed path's windows (fixed_window), a batch
// of at least 2 × 2^25 headers (1.34 GB) goes out as equal back-to-back windows of about 2^25 headers: one launch
// over 64M headers ran 3.0% (bitmask) / 1.3% (raw sums) slower per byte than two of 32M, and 128M headers 3.3%
// slower than four. Windows are whole tasks (256 headers, a multiple of the 64-bit mask
// words). window_bytes > 0 sets the window, < 0 turns windows off.
constexpr uint64_t kHdrAutoWindow = 1ull << 25;

static uint64_t hdr20_window(const LaunchCfg& c, uint64_t n) {
    uint64_t win = kFixedChunk;
    if (c.window_bytes > 0) {
        win = std::max<uint64_t>(1, (uint64_t)c.window_bytes / 20u / kHdr20Task) * kHdr20Task;
    } else if (c.window_bytes == 0 && n >= 2 * kHdrAutoWindow) {
        const uint64_t nw = (n + kHdrAutoWindow - 1) / kHdrAutoWindow;
        win = ((n + nw - 1) / nw + kHdr20Task - 1) / kHdr20Task * kHdr20Task;
    }
    return std::min<uint64_t>(win, kFixedChunk);
}

static bool hdr20_path(const LaunchCfg& c, uintptr_t base, uint64_t stride, uint32_t hdr_off) {
    return stride == 20 && hdr_off == 0 && (base & 3u) == 0 && c.kernel == 0;
}

uint64_t ipv4_hdr_launch_count(const LaunchCfg& c, uintptr_t base, uint64_t stride, uint32_t hdr_off, uint64_t n) {
    if (n == 0) return 0;
    if (!hdr20_path(c, base, stride, hdr_off)) return 1;
    const uint64_t win = hdr20_window(c, n);
    return (n + win - 1) / win;
}

hipError_t launch_ipv4_hdr(const LaunchCfg& c, uint8_t* base, uint64_t stride, uint32_t hdr_off, uint64_t n,
                           int mode, uint16_t* out, uint64_t* mask, hipStream_t st) {
    // Kernel by layout: packed 20 B headers (stride 20, hdr_off 0, 4-aligned base) → the pipelined flat
    // kernel; other strides ≤ 64 → LDS-dense; else per-thread. kernel 1 forces per-thread, 2 LDS-dense.
    // mode: 0 verify (raw sums), 1 fill in place, 2 verify into the bitmask `mask`.
    auto by_mode = [&](auto launch) {
        switch (mode) {
            case 1: launch(std::integral_constant<int, 1>{}); break;
            case 2: launch(std::integral_constant<int, 2>{}); break;
            default: launch(std::integral_constant<int, 0>{}); break;
        }
    };
    if (hdr20_path(c, (uintptr_t)base, stride, hdr_off)) {
        // 1 block/CU with 2 tasks (10 KiB) in flight per wave = 40 KiB per CU (round 1 sweep: 0.220 ms vs
        // 0.232 at 2 blocks/CU, 0.284 at 1 task/wave); chunks keep each launch's results within one
        // descriptor (2^28 headers = 2^22 mask words)
        const uint32_t mb = max_blocks_of(c, 1);
        const uint64_t win = hdr20_window(c, n);
        for (uint64_t c0 = 0; c0 < n; c0 += win) {
            const uint32_t cn = (uint32_t)std::min<uint64_t>(win, n - c0);
            const uint64_t tasks = (cn + kHdr20Task - 1) / kHdr20Task;
            const uint32_t grid = grid_for(tasks, mb);
            uint8_t* b = base + c0 * 20u;
            uint16_t* o = out ? out + c0 : nullptr;
            uint64_t* mk = mask ? mask + c0 / kWave : nullptr;
            const size_t lds = (size_t)kHdr20Lds * kWavesPerBlock;
            const uint32_t clog = deal_clog(c.xcd_chunk, tasks, kHdr20Lds + kHdr20Task * 2u);
            by_mode([&](auto m) {
                constexpr int M = decltype(m)::value;
                hipLaunchKernelGGL((ipv4_hdr20_kernel<M, 2>), dim3(grid), dim3(kBlock), lds, st, b, cn, o, clog, mk);
            });
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const uint32_t max_blocks = max_blocks_of(c, 8);
    if (stride >= 1 && stride <= kHdrDenseMaxStride && (c.kernel == 0 || c.kernel == 2)) {
        // a wave's 64 headers span ≤ 63·stride + 3 + 20 bytes: ROWS 1 KiB rows per task in registers,
        // U tasks per iteration, an LDS slice of U·ROWS KiB per wave
        const uint32_t rows = (63u * (uint32_t)stride + 3u + 20u + 3u + kRow - 1) / kRow;
        const uint32_t grid = grid_for((n + kWave - 1) / kWave, max_blocks);
        by_mode([&](auto m) {
            constexpr int M = decltype(m)::value;
#define NSX_HDR(R, U)                                                                                              \
    hipLaunchKernelGGL((ipv4_hdr_dense_kernel<M, R, U>), dim3(grid), dim3(kBlock),                                 \
                       (size_t)(R) * (U) * kRow * kWavesPerBlock, st, base, (uint32_t)stride, hdr_off, n, out, mask)
            switch (rows) {
                case 1: NSX_HDR(1, 4); break;
                case 2: NSX_HDR(2, 2); break;
                case 3: NSX_HDR(3, 1); break;
                case 4: NSX_HDR(4, 1); break;
                default: NSX_HDR(5, 1); break;
            }
#undef NSX_HDR
        });
        return hipGetLastError();
    }
    const uint64_t want = (n + (uint64_t)kBlock * kHdrUnroll - 1) / ((uint64_t)kBlock * kHdrUnroll);
    const uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
    by_mode([&](auto m) {
        constexpr int M = decltype(m)::value;
        hipLaunchKernelGGL(ipv4_hdr_kernel<M>, dim3(grid), dim3(kBlock), 0, st, base, stride, hdr_off, n, out, mask);
    });
    return hipGetLastError();
}

hipError_t launch_fill_splitmix64(void* d_buf, uint64_t byte_off, uint64_t nbytes, uint64_t seed,
                                  uint32_t max_blocks, hipStream_t st) {
    uint8_t* dst = static_cast<uint8_t*>(d_buf);
    if ((byte_off & 7) == 0 && ((uintptr_t)dst & 7) == 0 && nbytes >= 8) {
        const uint64_t nwords = nbytes / 8;
        uint64_t want = (nwords + kBlock - 1) / kBlock;
        uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
        hipLaunchKernelGGL(fill_words_kernel, dim3(grid), dim3(kBlock), 0, st, reinterpret_cast<uint64_t*>(dst),
                           byte_off / 8, nwords, seed);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        dst += nwords * 8;
        byte_off += nwords * 8;
        nbytes -= nwords * 8;
    }
    if (nbytes) {
        uint64_t want = (nbytes + kBlock - 1) / kBlock;
        uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
        hipLaunchKernelGGL(fill_bytes_kernel, dim3(grid), dim3(kBlock), 0, st, dst, byte_off, nbytes, seed);
    }
    return hipGetLastError();
}

}  // namespace nsx
