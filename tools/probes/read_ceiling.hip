// Practical read-bandwidth ceiling on this MI355X: a flat
// grid-stride dwordx4 read-and-sum over the same byte counts as config 2
// (1.5 GB) and config 4 (16 GiB), with no segment logic. Variants: loads in
// flight per lane (1/2/4/8), nt vs default policy, grid size (blocks per CU).
// Steady-state timing: 200 settle launches, then median of 5 × 20 launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int L, bool NT>
__global__ __launch_bounds__(256) void read_sum(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nth = (uint64_t)gridDim.x * 256;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (L - 1) * nth < n16; i += L * nth) {
        u32x4 v[L];
#pragma unroll
        for (int k = 0; k < L; ++k) v[k] = NT ? __builtin_nontemporal_load(p + i + k * nth) : p[i + k * nth];
#pragma unroll
        for (int k = 0; k < L; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    }
    for (; i < n16; i += nth) acc += p[i].x;
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

template <int L, bool NT>
float run(const u32x4* p, uint64_t n16, uint32_t* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        for (int k = 0; k < 20; ++k) hipLaunchKernelGGL((read_sum<L, NT>), dim3(blocks), dim3(256), 0, 0, p, n16, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

// Usage: read_ceiling [bytes ...]  (default: config 2's and config 4's byte counts)
int main(int argc, char** argv) {
    std::vector<uint64_t> sizes = {1572864000ull, 17179869184ull};
    if (argc > 1) {
        sizes.clear();
        for (int i = 1; i < argc; ++i) sizes.push_back(strtoull(argv[i], nullptr, 10) & ~15ull);
    }
    const uint64_t maxb = *std::max_element(sizes.begin(), sizes.end());
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, maxb) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x5A, maxb);
    const u32x4* p = (const u32x4*)buf;
    for (int k = 0; k < 200; ++k) hipLaunchKernelGGL((read_sum<4, true>), dim3(cus * 4), dim3(256), 0, 0, p, std::min(maxb, sizes[0]) / 16, out);
    (void)hipDeviceSynchronize();
    for (uint64_t bytes : sizes) {
        const uint64_t n16 = bytes / 16;
        for (int bpc : {2, 4, 8}) {
            const int blocks = cus * bpc;
            float r[8] = {run<1, true>(p, n16, out, blocks), run<2, true>(p, n16, out, blocks),
                          run<4, true>(p, n16, out, blocks), run<8, true>(p, n16, out, blocks),
                          run<1, false>(p, n16, out, blocks), run<2, false>(p, n16, out, blocks),
                          run<4, false>(p, n16, out, blocks), run<8, false>(p, n16, out, blocks)};
            printf("bytes=%llu blocks/CU=%d  GB/s  nt[L=1,2,4,8]: %.0f %.0f %.0f %.0f   plain[L=1,2,4,8]: %.0f %.0f %.0f %.0f\n",
                   (unsigned long long)bytes, bpc, bytes / r[0] / 1e6, bytes / r[1] / 1e6, bytes / r[2] / 1e6,
                   bytes / r[3] / 1e6, bytes / r[4] / 1e6, bytes / r[5] / 1e6, bytes / r[6] / 1e6, bytes / r[7] / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
