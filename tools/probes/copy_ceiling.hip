// Practical copy ceiling on this MI355X: the f1 fused build
// reads ~1.5 GB and writes ~1.5 GB per launch, so its roofline is a copy's, not
// a read's. Grid-stride dwordx4 copy of 1.5 GB with L loads in flight per lane,
// nt/plain policies, 2/4/8 blocks per CU; plus hipMemcpyDtoD for reference.
// Also checks how a raw buffer STORE that straddles num_records behaves
// (per-dword range check, as for loads?).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int L, bool NT>
__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n16) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nth = (uint64_t)gridDim.x * 256;
    uint64_t i = tid;
    for (; i + (L - 1) * nth < n16; i += L * nth) {
        u32x4 v[L];
#pragma unroll
        for (int k = 0; k < L; ++k) v[k] = NT ? __builtin_nontemporal_load(s + i + k * nth) : s[i + k * nth];
#pragma unroll
        for (int k = 0; k < L; ++k) {
            if (NT) __builtin_nontemporal_store(v[k], d + i + k * nth);
            else d[i + k * nth] = v[k];
        }
    }
    for (; i < n16; i += nth) d[i] = s[i];
}

__global__ void store_probe(uint32_t* base, uint32_t nrec, uint32_t voff) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nrec, 0x00020000);
    if (threadIdx.x == 0) __builtin_amdgcn_raw_buffer_store_b128(v4u{0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u}, r, voff, 0, 0);
}

template <int L, bool NT>
float run(const u32x4* s, u32x4* d, uint64_t n16, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        for (int k = 0; k < 20; ++k) hipLaunchKernelGGL((copy16<L, NT>), dim3(blocks), dim3(256), 0, 0, s, d, n16);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

int main() {
    const uint64_t bytes = 1572864000ull;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    void *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&dst, bytes) != hipSuccess) return 1;
    (void)hipMemset(src, 0x5A, bytes);
    // store straddling num_records: nrec = 24, store 16 B at offset 16 -> dwords 16..19, 20..23 in, 24..31 out
    uint32_t* sp = (uint32_t*)dst;
    (void)hipMemset(sp, 0, 64);
    hipLaunchKernelGGL(store_probe, dim3(1), dim3(64), 0, 0, sp, 24u, 16u);
    uint32_t h[12] = {0};
    (void)hipMemcpy(h, sp, 48, hipMemcpyDeviceToHost);
    printf("store straddle (nrec=24, voff=16): dwords 4..7 = %08x %08x %08x %08x  (per-dword check => 11111111 22222222 0 0)\n",
           h[4], h[5], h[6], h[7]);
    const u32x4* s = (const u32x4*)src;
    u32x4* d = (u32x4*)dst;
    const uint64_t n16 = bytes / 16;
    for (int k = 0; k < 100; ++k) hipLaunchKernelGGL((copy16<2, true>), dim3(cus * 4), dim3(256), 0, 0, s, d, n16);
    (void)hipDeviceSynchronize();
    for (int bpc : {2, 4, 8}) {
        const int blocks = cus * bpc;
        float r[6] = {run<1, true>(s, d, n16, blocks), run<2, true>(s, d, n16, blocks), run<4, true>(s, d, n16, blocks),
                      run<1, false>(s, d, n16, blocks), run<2, false>(s, d, n16, blocks),
                      run<4, false>(s, d, n16, blocks)};
        printf("copy 1.5GB blocks/CU=%d  read+write GB/s  nt[L=1,2,4]: %.0f %.0f %.0f   plain[L=1,2,4]: %.0f %.0f %.0f\n", bpc,
               2 * bytes / r[0] / 1e6, 2 * bytes / r[1] / 1e6, 2 * bytes / r[2] / 1e6, 2 * bytes / r[3] / 1e6,
               2 * bytes / r[4] / 1e6, 2 * bytes / r[5] / 1e6);
        fflush(stdout);
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        for (int k = 0; k < 20; ++k) (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    std::sort(t.begin(), t.end());
    printf("hipMemcpyDtoD 1.5GB: read+write %.0f GB/s\n", 2 * bytes / t[2] / 1e6);
    return 0;
}
