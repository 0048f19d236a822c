// north_star's "segment staged through LDS" measured on config 2's own layout, beside the
// product kernel. Config 2: 1M TCP segments of 1500 B at a 1500 B stride (4-aligned), one raw checksum each.
// Three forms of one wave per packet (each wave takes U = 8 packets per iteration, all their loads in flight,
// 2 blocks/CU — the product's task size), identical arithmetic (v_sad_u16 half-sums, DPP wave sum, fold,
// byte swap for an even start):
//   vgpr  — rows loaded into VGPRs and summed there (what the product kernels do);
//   lds   — rows loaded into VGPRs, written to the wave's LDS slot (ds_write_b128), read back (ds_read_b128)
//           and summed: the packet staged through LDS;
//   dma   — rows loaded straight into LDS (buffer_load_dwordx4 ... lds, the gfx950 LDS-DMA path), then read
//           back and summed.
// and the product's nsx_csum_fixed_dev (csum_fixed_swp_kernel<8,2>) on the same buffer. Every form's results
// are compared with the product's on all 1M packets. Median of 5 × 20 launches after 200 settle launches.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/lds_stage.hip -Inetwork-stack_amd/../include
//        -Lnetwork-stack_amd/lib -lnsx_csum -Wl,-rpath,$PWD/network-stack_amd/lib -o tools/probes/lds_stage
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "nsx_csum.h"

constexpr uint32_t kU = 8, kRows = 2, kRow = 1024, kLen = 1500, kStride = 1500;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t sad4(v4u v, uint32_t acc) {
    acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
    acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
    return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xF, 0xF, false);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ uint32_t fold32(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    return (s & 0xFFFFu) + (s >> 16);
}

// MODE 0 vgpr, 1 lds, 2 dma
template <int MODE>
__global__ __launch_bounds__(256) void probe(const uint8_t* __restrict__ base, uint32_t n, uint16_t* __restrict__ out) {
    extern __shared__ v4u lds[];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    v4u* slot = lds + wave * (kU * kRows * (kRow / 16u));
    const uint32_t ntasks = (n + kU - 1) / kU, wstep = gridDim.x * 4u;
    for (uint32_t t = blockIdx.x * 4u + wave; t < ntasks; t += wstep) {
        v4u v[kU][kRows];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t i = t * kU + u;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t*>(base + (uint64_t)min(i, n - 1) * kStride), 0, i < n ? (int)kLen : 0, 0x00020000);
#pragma unroll
            for (uint32_t r = 0; r < kRows; ++r) {
                if constexpr (MODE == 2) {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rs, (__attribute__((address_space(3))) void*)(slot + (u * kRows + r) * (kRow / 16u)), 16,
                        r * kRow + lane * 16u, 0, 0, 0);
                } else {
                    v[u][r] = __builtin_amdgcn_raw_buffer_load_b128(rs, r * kRow + lane * 16u, 0, 2);
                }
            }
        }
        if constexpr (MODE == 1) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u)
#pragma unroll
                for (uint32_t r = 0; r < kRows; ++r) slot[(u * kRows + r) * (kRow / 16u) + lane] = v[u][r];
            __builtin_amdgcn_wave_barrier();
        }
        if constexpr (MODE == 2) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the LDS-DMA writes have landed
            __builtin_amdgcn_wave_barrier();
        }
        if constexpr (MODE != 0) {
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u)
#pragma unroll
                for (uint32_t r = 0; r < kRows; ++r) v[u][r] = slot[(u * kRows + r) * (kRow / 16u) + lane];
        }
        uint32_t res = 0;
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            uint32_t acc = 0;
#pragma unroll
            for (uint32_t r = 0; r < kRows; ++r) acc = sad4(v[u][r], acc);
            uint32_t s = fold32(wave_sum(fold32(acc)));
            s = ((s & 0xFFu) << 8) | (s >> 8);  // every packet starts at an even (4-aligned) address
            s = fold32(s);
            res = lane == u ? s : res;
        }
        if (lane < kU && t * kU + lane < n) out[t * kU + lane] = (uint16_t)res;
        if constexpr (MODE != 0) __builtin_amdgcn_wave_barrier();
    }
}

template <typename F>
static float timed(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(a);
        for (int k = 0; k < 20; ++k) launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

int main() {
    const uint32_t n = 1u << 20;
    const uint64_t bytes = (uint64_t)n * kStride;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t* buf = nullptr;
    uint16_t *ref = nullptr, *got = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&ref, n * 2) != hipSuccess ||
        hipMalloc(&got, n * 2) != hipSuccess)
        return 1;
    if (nsx_fill_splitmix64_dev(buf, 0, bytes, 0x1071, nullptr) != NSX_OK) return 1;
    const size_t lds = (size_t)4 * kU * kRows * kRow;  // 64 KiB per block: 2 blocks/CU fit
    const dim3 grid(cus * 2), blk(256);
    auto product = [&] { nsx_csum_fixed_dev(buf, kStride, kLen, n, nullptr, ref, nullptr); };
    auto f0 = [&] { hipLaunchKernelGGL(probe<0>, grid, blk, 0, 0, buf, n, got); };
    auto f1 = [&] { hipLaunchKernelGGL(probe<1>, grid, blk, lds, 0, buf, n, got); };
    auto f2 = [&] { hipLaunchKernelGGL(probe<2>, grid, blk, lds, 0, buf, n, got); };
    for (int k = 0; k < 200; ++k) product();
    (void)hipDeviceSynchronize();
    std::vector<uint16_t> want(n), have(n);
    (void)hipMemcpy(want.data(), ref, n * 2, hipMemcpyDeviceToHost);
    const char* names[4] = {"product csum_fixed_swp_kernel<8,2>", "vgpr (one wave per packet)",
                            "lds (staged: ds_write_b128 + ds_read_b128)", "dma (buffer_load ... lds + ds_read_b128)"};
    for (int round = 0; round < 2; ++round) {
        float ms[4] = {timed(product), timed(f0), timed(f1), timed(f2)};
        for (int m = 0; m < 4; ++m) {
            bool ok = true;
            if (m > 0) {
                (void)hipMemset(got, 0, n * 2);
                if (m == 1) f0();
                else if (m == 2) f1();
                else f2();
                (void)hipMemcpy(have.data(), got, n * 2, hipMemcpyDeviceToHost);
                ok = have == want;
            }
            printf("round %d %-44s %.4f ms  %.0f GB/s  frac %.3f  bit-exact vs product: %s\n", round, names[m], ms[m],
                   (bytes + 2.0 * n) / ms[m] / 1e6, (bytes + 2.0 * n) / ms[m] / 1e6 / 8000.0, ok ? "yes" : "NO");
        }
        fflush(stdout);
    }
    return 0;
}
