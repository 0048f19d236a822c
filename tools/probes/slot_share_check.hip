// Device check of the slot-weighted wave ranges: every wave of a 4-blocks-per-CU grid
// computes its byte-weighted share (slot_share + wave_range_w) and its unweighted one (wave_range) over a batch of
// 300,007 frames of 40-100 B (equal-count split) and of 40-1500 B (byte-balanced search), exactly as the receive
// kernel's streamed branch does, and writes both; the host checks that each set of ranges tiles [0, n) in wave order,
// and that each unweighted range starts where the host's own lower bound of its byte target says. A third batch (40 B
// frames, then 1500 B ones; printed as "40--1 B") puts the byte targets far from a straight line through the offsets.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I network-stack_amd/csrc tools/probes/slot_share_check.hip \
//       -o tools/probes/slot_share_check && tools/probes/slot_share_check
#include "../../network-stack_amd/csrc/csum_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

namespace nsx {
namespace {
__global__ __launch_bounds__(kBlock) void slot_share_probe(const uint64_t* __restrict__ offsets, uint32_t n,
                                                           uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const __amdgpu_buffer_rsrc_t ofs = make_rsrc(offsets, ((uint64_t)n + 1) * 8);
    const uint32_t nb = gridDim.x / 4u * 3u;
    if (blockIdx.x >= nb) return;
    const SlotShare sh = slot_share(nb, kWavesPerBlock, wave, gridDim.x >> 5, kRxSlotW);
    const WaveRange a = wave_range_w(ofs, n, sh.lo, sh.hi, sh.T, lane, kRxSmallFrame, 8u);
    const uint32_t g = wave_number(nb, kWavesPerBlock, wave);
    const WaveRange b = wave_range(ofs, n, g, nb * kWavesPerBlock, lane, kRxSmallFrame, 8u);
    if (lane == 0) {
        out[g * 4 + 0] = a.a0, out[g * 4 + 1] = a.a_end, out[g * 4 + 2] = b.a0, out[g * 4 + 3] = b.a_end;
    }
}
}  // namespace
}  // namespace nsx

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t grid = (uint32_t)cus * 4u, W = grid / 4u * 3u * 4u;
    int bad_total = 0;
    for (int hi : {100, 1500, -1}) {  // -1: 40 B frames, then 1500 B ones (offsets far from a straight line)
        const uint32_t n = 300007;
        std::mt19937 rng(1234 + hi);
        std::vector<uint64_t> offs(n + 1, 0);
        for (uint32_t i = 0; i < n; ++i)
            offs[i + 1] = offs[i] + (hi < 0 ? (i < n / 2 ? 40u : 1500u) : 40 + rng() % (hi - 39));
        uint64_t* d_offs;
        uint32_t* d_out;
        (void)hipMalloc(&d_offs, offs.size() * 8);
        (void)hipMalloc(&d_out, (size_t)W * 16);
        (void)hipMemcpy(d_offs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice);
        (void)hipMemset(d_out, 0xFF, (size_t)W * 16);
        hipLaunchKernelGGL(nsx::slot_share_probe, dim3(grid), dim3(nsx::kBlock), 0, 0, d_offs, n, d_out);
        std::vector<uint32_t> o((size_t)W * 4);
        (void)hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
        for (int form = 0; form < 2; ++form) {
            int bad = 0;
            uint64_t lens_min = ~0ull, lens_max = 0;
            for (uint32_t g = 0; g < W; ++g) {
                const uint32_t a0 = o[g * 4 + 2 * form], a1 = o[g * 4 + 2 * form + 1];
                const uint32_t prev = g ? o[(g - 1) * 4 + 2 * form + 1] : 0u;
                if (a0 != prev || a1 < a0 || (g + 1 == W && a1 != n)) {
                    if (bad < 5) printf("  frames<=%d form %s wave %u: [%u, %u) after %u\n", hi,
                                        form ? "unweighted" : "slot", g, a0, a1, prev);
                    ++bad;
                }
                lens_min = std::min<uint64_t>(lens_min, a1 - a0), lens_max = std::max<uint64_t>(lens_max, a1 - a0);
                // the unweighted form against the host's own lower bound of the wave's byte target (byte-balanced
                // batches: mean frame >= kRxSmallFrame)
                const uint64_t tot = offs[n] - offs[0];
                if (form == 1 && tot >= (uint64_t)nsx::kRxSmallFrame * n && g > 0) {
                    const uint64_t tg = offs[0] + tot * g / W;
                    const uint32_t lb = (uint32_t)(std::lower_bound(offs.begin(), offs.end(), tg) - offs.begin());
                    const uint32_t want = std::min((lb + 7u) / 8u * 8u, n);
                    if (a0 != want) {
                        if (bad < 5) printf("  frames<=%d wave %u: start %u, host lower bound gives %u\n", hi, g, a0, want);
                        ++bad;
                    }
                }
            }
            printf("frames 40-%d B, %s ranges: %d waves out of place; frames per wave %llu-%llu\n", hi,
                   form ? "unweighted" : "slot-weighted", bad, (unsigned long long)lens_min,
                   (unsigned long long)lens_max);
            bad_total += bad;
        }
        (void)hipFree(d_offs);
        (void)hipFree(d_out);
    }
    return bad_total ? 1 : 0;
}
