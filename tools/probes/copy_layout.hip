// Copy ceilings for the f1 build's memory layout: is the
// fused kernel's gap to the flat copy ceiling the layout's or the kernel's?
//   flat16   : grid-stride dwordx4 copy, both sides 16 B aligned (the ceiling probe)
//   flatmis  : the same copy from src+4 to dst+12 (4-aligned, not 16-aligned), buffer loads/stores
//   seg      : one wave per segment, 1480 B source rows at stride 1480 copied to 1500 B
//              images at stride 1500 (20 B header gap), 2 rows in flight: the build
//              kernel's access pattern with no header, no checksum
//   seg_al   : the same with source/destination strides rounded to 1536 (16 B aligned)
//   seg_swp  : seg, software-pipelined (the next segment's loads issue before this one's stores)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)n, 0x00020000);
}

__global__ __launch_bounds__(256) void flat_mis(const uint8_t* s, uint8_t* d, uint64_t n16, uint32_t soff,
                                                uint32_t doff) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nth = (uint64_t)gridDim.x * 256;
    for (uint64_t i = tid; i + nth < n16; i += 2 * nth) {
        const __amdgpu_buffer_rsrc_t rs0 = rsrc(s + soff + (i - threadIdx.x) * 16, 4096);
        const __amdgpu_buffer_rsrc_t rd0 = rsrc(d + doff + (i - threadIdx.x) * 16, 4096);
        const __amdgpu_buffer_rsrc_t rs1 = rsrc(s + soff + (i + nth - threadIdx.x) * 16, 4096);
        const __amdgpu_buffer_rsrc_t rd1 = rsrc(d + doff + (i + nth - threadIdx.x) * 16, 4096);
        v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs0, threadIdx.x * 16, 0, 2);
        v4u b = __builtin_amdgcn_raw_buffer_load_b128(rs1, threadIdx.x * 16, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(a, rd0, threadIdx.x * 16, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(b, rd1, threadIdx.x * 16, 0, 0);
    }
}

// one wave per segment, grid-stride over segments (contiguous per XCD not modelled)
template <int LP, int SP>
__global__ __launch_bounds__(256) void seg_copy(const uint8_t* s, uint8_t* d, uint32_t n, uint32_t sstride,
                                                uint32_t dstride, uint32_t plen, uint32_t gap) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t i = blockIdx.x * 4 + wave; i < n; i += nw) {
        const __amdgpu_buffer_rsrc_t rs = rsrc(s + (uint64_t)i * sstride, plen);
        const __amdgpu_buffer_rsrc_t rd = rsrc(d + (uint64_t)i * dstride + gap, plen);
        v4u a = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, LP);
        v4u b = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 + lane * 16, 0, LP);
        asm volatile("" : "+v"(a), "+v"(b));
        __builtin_amdgcn_raw_buffer_store_b128(a, rd, lane * 16, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(b, rd, 1024 + lane * 16 < plen ? 1024 + lane * 16 : kOOB, 0, SP);
    }
}

// the same per-segment copy, software-pipelined: segment i+nw's loads are issued before segment i is stored
template <int LP, int SP>
__global__ __launch_bounds__(256) void seg_copy_swp(const uint8_t* s, uint8_t* d, uint32_t n, uint32_t sstride,
                                                    uint32_t dstride, uint32_t plen, uint32_t gap) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * 4;
    auto ld = [&](uint32_t i, v4u& a, v4u& b) {
        const __amdgpu_buffer_rsrc_t rs = rsrc(s + (uint64_t)(i < n ? i : 0) * sstride, i < n ? plen : 0);
        a = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, LP);
        b = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 + lane * 16, 0, LP);
    };
    auto st = [&](uint32_t i, v4u& a, v4u& b) {
        asm volatile("" : "+v"(a), "+v"(b));
        const __amdgpu_buffer_rsrc_t rd = rsrc(d + (uint64_t)i * dstride + gap, plen);
        __builtin_amdgcn_raw_buffer_store_b128(a, rd, lane * 16, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(b, rd, 1024 + lane * 16 < plen ? 1024 + lane * 16 : kOOB, 0, SP);
    };
    uint32_t i = blockIdx.x * 4 + wave;
    v4u a0, b0, a1, b1;
    ld(i, a0, b0);
    while (i < n) {
        const uint32_t i1 = i + nw;
        ld(i1, a1, b1);
        st(i, a0, b0);
        if (i1 >= n) break;
        i = i1 + nw;
        ld(i, a0, b0);
        st(i1, a1, b1);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        for (int k = 0; k < 20; ++k) f();
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
    const uint32_t n = 1u << 20;
    const uint64_t bytes = (uint64_t)n * 1536 + 4096;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&dst, bytes) != hipSuccess) return 1;
    (void)hipMemset(src, 0x5A, bytes);
    (void)hipMemset(dst, 0, bytes);
    const uint64_t fb = (uint64_t)n * 1500;  // bytes per copy (the f1 image volume)
    const uint64_t n16 = fb / 16 - 64;
    for (int k = 0; k < 50; ++k) hipLaunchKernelGGL(flat_mis, dim3(cus * 4), dim3(256), 0, 0, src, dst, n16, 0u, 0u);
    (void)hipDeviceSynchronize();
    // which side's misalignment costs: flat copies with only the source, only the destination, or both 4 B off
    for (int bpc : {2, 4}) {
        const int g = cus * bpc;
        const double ab = 2.0 * n16 * 16;
        for (uint32_t so : {0u, 4u}) {
            for (uint32_t dof : {0u, 12u}) {
                const float t = timeit([&] { hipLaunchKernelGGL(flat_mis, dim3(g), dim3(256), 0, 0, src, dst, n16, so, dof); });
                printf("bpc=%d flat src+%u dst+%u %.4f ms %.0f GB/s\n", bpc, so, dof, t, ab / t / 1e6);
            }
        }
    }
    fflush(stdout);
    for (int bpc : {1, 2, 4, 8}) {
        const int g = cus * bpc;
        const float a = timeit([&] { hipLaunchKernelGGL(flat_mis, dim3(g), dim3(256), 0, 0, src, dst, n16, 0u, 0u); });
        const float b = timeit([&] { hipLaunchKernelGGL(flat_mis, dim3(g), dim3(256), 0, 0, src, dst, n16, 4u, 12u); });
        const float c = timeit([&] {
            hipLaunchKernelGGL((seg_copy<0, 0>), dim3(g), dim3(256), 0, 0, src, dst, n, 1480u, 1500u, 1480u, 20u);
        });
        const float c2 = timeit([&] {
            hipLaunchKernelGGL((seg_copy<2, 0>), dim3(g), dim3(256), 0, 0, src, dst, n, 1480u, 1500u, 1480u, 20u);
        });
        const float e = timeit([&] {
            hipLaunchKernelGGL((seg_copy<0, 0>), dim3(g), dim3(256), 0, 0, src, dst, n, 1536u, 1536u, 1480u, 32u);
        });
        const float f = timeit([&] {
            hipLaunchKernelGGL((seg_copy_swp<0, 0>), dim3(g), dim3(256), 0, 0, src, dst, n, 1480u, 1500u, 1480u, 20u);
        });
        const double ab = 2.0 * n16 * 16, sb = 2.0 * n * 1480.0;
        printf("bpc=%d seg_swp %.4f ms %.0f GB/s\n", bpc, f, sb / f / 1e6);
        printf("bpc=%d flat16 %.4f ms %.0f GB/s | flatmis %.4f ms %.0f GB/s | seg %.4f ms %.0f GB/s | seg(nt ld) %.4f ms "
               "%.0f GB/s | seg_al %.4f ms %.0f GB/s\n",
               bpc, a, ab / a / 1e6, b, ab / b / 1e6, c, sb / c / 1e6, c2, sb / c2 / 1e6, e, sb / e / 1e6);
    }
    return 0;
}
