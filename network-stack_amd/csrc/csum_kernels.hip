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
// 256-thread blocks; tasks are dealt so that the 8 XCDs each stream one
// contiguous region of the batch (their 2-byte result stores then fill whole
// lines in one XCD's L2 instead of being split across XCDs).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__device__ __forceinline__ TaskIter task_iter(uint64_t ntasks, uint32_t wave, int xcd_map) {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    TaskIter it;
    if (xcd_map && nb >= 16 && (nb & 7) == 0) {
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

// ---------------------------------------------------------------------------
// Fixed stride, U segments per wave pass, NROWS rows per segment (compile-time:
// every load of the pass is issued before the first is consumed).
// ---------------------------------------------------------------------------
template <int U, int NROWS, bool NT>
__global__ __launch_bounds__(kBlock) void csum_fixed_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t seg_len, uint64_t n,
    const uint32_t* __restrict__ partial, uint16_t* __restrict__ out, const uint8_t* safe_end,
    int xcd_map) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t ntasks = (n + U - 1) / U;
    TaskIter it = task_iter(ntasks, wave, xcd_map);

    for (uint64_t t = it.next; t < it.end; t += it.step) {
        const uint64_t s0 = t * U;
        const uint8_t* wb[U];
        uint32_t head[U];
        u32x4 v[U][NROWS];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint8_t* p = base + (s0 + u) * stride;
            head[u] = (uint32_t)((uintptr_t)p & 3u);
            wb[u] = p - head[u];
        }
        // Issue phase.
#pragma unroll
        for (int r = 0; r < NROWS; ++r) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                v[u][r] = u32x4{0u, 0u, 0u, 0u};
                const uint32_t q = r * kRow + lane * 16;
                if (s0 + u < n && q < head[u] + seg_len) {
                    const uint8_t* a = wb[u] + q;
                    if (wb[u] + (r + 1) * kRow <= safe_end || a + 16 <= safe_end) v[u][r] = ld16<NT>(a);
                    else v[u][r] = ld16_guarded(a, safe_end);
                }
            }
        }
        // Consume phase.
        uint32_t tot[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t acc = 0;
            const int64_t lo = head[u], hi = (int64_t)head[u] + seg_len;
#pragma unroll
            for (int r = 0; r < NROWS; ++r) {
                u32x4 x = v[u][r];
                const int64_t rb = (int64_t)r * kRow;
                if (rb < lo || rb + kRow > hi) x = mask_chunk(x, rb + lane * 16, lo, hi);
                acc = sad4(x, acc);
            }
            tot[u] = wave_sum(fold32(acc));
        }
        // Lane u writes segment s0+u: U contiguous u16 per wave.
        uint32_t mine = 0;
        bool mine_even = true;
        uint64_t my_seg = s0 + lane;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lane == (uint32_t)u) { mine = tot[u]; mine_even = ((uintptr_t)(wb[u] + head[u]) & 1u) == 0; }
        if (lane < (uint32_t)U && my_seg < n) {
            const uint32_t pp = partial ? partial[my_seg] : 0u;
            out[my_seg] = (uint16_t)finish(mine, mine_even, pp);
        }
    }
}

// ---------------------------------------------------------------------------
// One segment per wave, runtime row count, rows issued R at a time. Serves the
// ragged batch (offsets) and fixed batches with long segments.
// ---------------------------------------------------------------------------
struct SegRef {
    const uint8_t* p;
    uint64_t len;
};

template <int R, bool NT>
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
                if (wb + (r + 1) * kRow <= safe_end || a + 16 <= safe_end) v[j] = ld16<NT>(a);
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

template <bool RAGGED, int R, bool NT, bool VERIFY>
__global__ __launch_bounds__(kBlock) void csum_wave_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, uint64_t stride,
    uint32_t seg_len, uint64_t n, const uint32_t* __restrict__ partial, uint16_t* __restrict__ out,
    uint8_t* __restrict__ ok, const uint8_t* safe_end, int xcd_map) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if constexpr (RAGGED) safe_end = align_up4(base + offsets[n]);
    TaskIter it = task_iter(n, wave, xcd_map);
    for (uint64_t i = it.next; i < it.end; i += it.step) {
        const SegRef s = seg_ref<RAGGED>(base, offsets, stride, seg_len, i);
        const uint32_t tot = wave_sum(seg_lane_sum<R, NT>(s.p, s.len, lane, safe_end, 0, 1));
        if (lane == 0) {
            const uint32_t res = finish(tot, ((uintptr_t)s.p & 1u) == 0, partial ? partial[i] : 0u);
            if (out) out[i] = (uint16_t)res;
            if constexpr (VERIFY) ok[i] = res == 0xFFFFu;
        }
    }
}

// ---------------------------------------------------------------------------
// One segment per 256-thread block (few, very long segments): wave w takes rows
// w, w+4, ... so the block reads 4 KiB contiguous per step; cross-wave total
// through LDS.
// ---------------------------------------------------------------------------
template <bool RAGGED, int R, bool NT, bool VERIFY>
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
        const uint32_t w = wave_sum(seg_lane_sum<R, NT>(s.p, s.len, lane, safe_end, wave, kWavesPerBlock));
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
// Launchers (host side of this translation unit).
// ---------------------------------------------------------------------------
static hipError_t launch_fixed_rows(const LaunchCfg& c, const uint8_t* base, uint64_t stride,
                                    uint32_t seg_len, uint64_t n, const uint32_t* partial,
                                    uint16_t* out, const uint8_t* safe_end, int nrows, int u,
                                    hipStream_t st) {
    const uint64_t ntasks = (n + u - 1) / u;
    const uint64_t want = (ntasks + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t grid = (uint32_t)(want < c.max_blocks ? want : c.max_blocks);
#define NSX_FIXED(U_, NR_)                                                                          \
    if (u == U_ && nrows == NR_) {                                                                   \
        if (c.nontemporal)                                                                           \
            hipLaunchKernelGGL((csum_fixed_kernel<U_, NR_, true>), dim3(grid), dim3(kBlock), 0, st,  \
                               base, stride, seg_len, n, partial, out, safe_end, c.xcd_map);         \
        else                                                                                         \
            hipLaunchKernelGGL((csum_fixed_kernel<U_, NR_, false>), dim3(grid), dim3(kBlock), 0, st, \
                               base, stride, seg_len, n, partial, out, safe_end, c.xcd_map);         \
        return hipGetLastError();                                                                    \
    }
    NSX_FIXED(1, 1) NSX_FIXED(2, 1) NSX_FIXED(4, 1)
    NSX_FIXED(1, 2) NSX_FIXED(2, 2) NSX_FIXED(4, 2)
    NSX_FIXED(1, 4) NSX_FIXED(2, 4)
#undef NSX_FIXED
    return hipErrorInvalidValue;
}

template <bool RAGGED, bool VERIFY>
static hipError_t launch_seg(const LaunchCfg& c, const uint8_t* base, const uint64_t* offsets,
                             uint64_t stride, uint32_t seg_len, uint64_t n, const uint32_t* partial,
                             uint16_t* out, uint8_t* ok, const uint8_t* safe_end, bool block_mode,
                             hipStream_t st) {
    if (block_mode) {
        const uint32_t grid = (uint32_t)(n < c.max_blocks ? n : c.max_blocks);
        if (c.nontemporal)
            hipLaunchKernelGGL((csum_block_kernel<RAGGED, 4, true, VERIFY>), dim3(grid), dim3(kBlock), 0,
                               st, base, offsets, stride, seg_len, n, partial, out, ok, safe_end);
        else
            hipLaunchKernelGGL((csum_block_kernel<RAGGED, 4, false, VERIFY>), dim3(grid), dim3(kBlock), 0,
                               st, base, offsets, stride, seg_len, n, partial, out, ok, safe_end);
    } else {
        const uint64_t want = (n + kWavesPerBlock - 1) / kWavesPerBlock;
        const uint32_t grid = (uint32_t)(want < c.max_blocks ? want : c.max_blocks);
        if (c.nontemporal)
            hipLaunchKernelGGL((csum_wave_kernel<RAGGED, 4, true, VERIFY>), dim3(grid), dim3(kBlock), 0, st,
                               base, offsets, stride, seg_len, n, partial, out, ok, safe_end, c.xcd_map);
        else
            hipLaunchKernelGGL((csum_wave_kernel<RAGGED, 4, false, VERIFY>), dim3(grid), dim3(kBlock), 0,
                               st, base, offsets, stride, seg_len, n, partial, out, ok, safe_end,
                               c.xcd_map);
    }
    return hipGetLastError();
}

hipError_t launch_fixed(const LaunchCfg& c, const void* d_base, uint64_t stride, uint32_t seg_len,
                        uint64_t n, const uint32_t* partial, uint16_t* out, hipStream_t st) {
    const uint8_t* base = static_cast<const uint8_t*>(d_base);
    const uint8_t* end = base + (n - 1) * stride + seg_len;
    const uint8_t* safe_end = reinterpret_cast<const uint8_t*>(((uintptr_t)end + 3) & ~(uintptr_t)3);
    // Rows a segment window can span (the window starts up to 3 bytes early).
    const uint64_t rows = ((uint64_t)seg_len + 3 + kRow - 1) / kRow;
    if (rows <= 4 && !c.block_mode) {
        int nrows = rows <= 1 ? 1 : (rows <= 2 ? 2 : 4);
        int u = c.segs_per_wave;
        if (nrows == 4 && u > 2) u = 2;
        return launch_fixed_rows(c, base, stride, seg_len, n, partial, out, safe_end, nrows, u, st);
    }
    return launch_seg<false, false>(c, base, nullptr, stride, seg_len, n, partial, out, nullptr, safe_end,
                                    c.block_mode, st);
}

hipError_t launch_ragged(const LaunchCfg& c, const void* d_base, const uint64_t* d_offsets, uint64_t n,
                         const uint32_t* partial, uint16_t* out, uint8_t* ok, hipStream_t st) {
    const uint8_t* base = static_cast<const uint8_t*>(d_base);
    if (ok)
        return launch_seg<true, true>(c, base, d_offsets, 0, 0, n, partial, out, ok, nullptr, c.block_mode,
                                      st);
    return launch_seg<true, false>(c, base, d_offsets, 0, 0, n, partial, out, nullptr, nullptr, c.block_mode,
                                   st);
}

hipError_t launch_pseudo_ipv4(const uint8_t* src, const uint8_t* dst, const uint32_t* len, uint8_t proto,
                              uint64_t n, uint32_t* partial, uint32_t max_blocks, hipStream_t st) {
    const uint64_t want = (n + kBlock - 1) / kBlock;
    const uint32_t grid = (uint32_t)(want < max_blocks ? want : max_blocks);
    hipLaunchKernelGGL(pseudo_ipv4_kernel, dim3(grid), dim3(kBlock), 0, st, src, dst, len, (uint32_t)proto, n,
                       partial);
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
