// Read ceiling by stream layout (config 3 question): is 2048 waves each streaming
// its own contiguous slice of a 4.75 GB buffer slower than all waves sweeping one
// compact window? Every wave reads 1 KiB rows (16 B per lane), 8 rows per batch,
// two batches in flight (software-pipelined), and sums them.
//   slices : wave w reads rows [w*R/W, (w+1)*R/W) in order (the ragged kernel's byte-balanced ranges)
//   window : batch b of wave w is batch b*W + w (every wave within one W-batch window of the others)
//   rounds : K rounds; in round k wave w reads the w-th of W slices of the k-th of K equal parts
//   chunks : the product kernels' XCD chunk deal — chunks of 2^K batches, XCD x takes chunks x, x+8, ...,
//            its waves walk their chunks' batches in order (K passed as the chunk log2)
// Grid: 1 and 2 blocks of 4 waves per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kB = 8;  // rows per batch

__device__ __forceinline__ void ld_batch(const uint8_t* p, uint64_t row, uint64_t nrows, uint32_t lane, v4u (&v)[kB]) {
    const uint64_t left = row < nrows ? nrows - row : 0;
    const uint32_t n = (uint32_t)(left < kB ? left : kB);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p) + (row < nrows ? row : 0) * 1024,
                                                                        0, (int)(n * 1024), 0x00020000);
#pragma unroll
    for (int j = 0; j < kB; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * 1024 + lane * 16, 0, 2);
}

// MODE 0 slices, 1 window, 2 rounds (K parts)
template <int MODE>
__global__ __launch_bounds__(256) void stream(const uint8_t* p, uint64_t nrows, uint32_t K, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t W = gridDim.x * 4;
    // XCD-contiguous wave numbering (block b runs on XCD b % 8)
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t w = ((b & 7) * (nb >> 3) + (b >> 3)) * 4 + (threadIdx.x >> 6);
    const uint64_t nbatch = (nrows + kB - 1) / kB;
    // the wave's batch sequence: batch(i) for i = 0 .. cnt-1
    uint64_t cnt, b0 = 0;
    uint64_t per = 0;
    if (MODE == 0) {
        b0 = nbatch * w / W;
        cnt = nbatch * (w + 1) / W - b0;
    } else if (MODE == 1) {
        cnt = w < nbatch ? (nbatch - w + W - 1) / W : 0;
    } else if (MODE == 3) {
        // local index i = slot*4 + wave + k*per_x over the XCD's chunks; counted by walking (cheap: exit test)
        cnt = 0xFFFFFFFFull;
    } else {
        per = nbatch / K;  // batches per part (the tail part takes the remainder)
        cnt = 0;
        for (uint32_t k = 0; k < K; ++k) {
            const uint64_t pb = k * per, pn = (k + 1 == K ? nbatch : (k + 1) * per) - pb;
            cnt += pn * (w + 1) / W - pn * w / W;
        }
    }
    // rounds mode: walk part by part
    uint32_t k = 0;
    uint64_t kpos = 0, kend = 0;
    auto part_range = [&](uint32_t kk, uint64_t& s, uint64_t& e) {
        const uint64_t pb = kk * per, pn = (kk + 1 == K ? nbatch : (kk + 1) * per) - pb;
        s = pb + pn * w / W;
        e = pb + pn * (w + 1) / W;
    };
    if (MODE == 2) part_range(0, kpos, kend);
    const uint32_t cx = b & 7, cslot = b >> 3, cper = (nb >> 3) * 4;
    auto chunk_task = [&](uint64_t i) -> uint64_t {
        const uint64_t li = (uint64_t)cslot * 4 + (threadIdx.x >> 6) + i * cper;
        return ((((li >> K) << 3) + cx) << K) | (li & ((1ull << K) - 1));
    };
    auto next_batch = [&](uint64_t i) -> uint64_t {
        if (MODE == 3) return chunk_task(i);
        if (MODE == 0) return b0 + i;
        if (MODE == 1) return i * W + w;
        while (kpos >= kend && k + 1 < K) part_range(++k, kpos, kend);
        return kpos++;
    };
    uint32_t acc = 0;
    v4u A[kB], B[kB];
    uint64_t i = 0;
    if (MODE == 3) {  // chunks: the sequence ends at the first batch past the end (tasks increase with i)
        uint64_t lo = 0, hi = 1;
        while (chunk_task(hi) < nbatch) hi <<= 1;
        while (lo < hi) {  // first i with chunk_task(i) >= nbatch
            const uint64_t mid = (lo + hi) / 2;
            if (chunk_task(mid) < nbatch) lo = mid + 1; else hi = mid;
        }
        cnt = lo;
    }
    if (cnt) ld_batch(p, next_batch(0) * kB, nrows, lane, A);
    while (i < cnt) {
        const bool hb = i + 1 < cnt;
        ld_batch(p, hb ? next_batch(i + 1) * kB : nrows, nrows, lane, B);
#pragma unroll
        for (int j = 0; j < kB; ++j) asm volatile("" : "+v"(A[j]));
#pragma unroll
        for (int j = 0; j < kB; ++j) acc += A[j].x + A[j].y + A[j].z + A[j].w;
        if (!hb) break;
        const bool ha = i + 2 < cnt;
        ld_batch(p, ha ? next_batch(i + 2) * kB : nrows, nrows, lane, A);
#pragma unroll
        for (int j = 0; j < kB; ++j) asm volatile("" : "+v"(B[j]));
#pragma unroll
        for (int j = 0; j < kB; ++j) acc += B[j].x + B[j].y + B[j].z + B[j].w;
        i += 2;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a);
        for (int k = 0; k < 10; ++k) f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 10);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

int main(int argc, char** argv) {
    const uint64_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4752000000ull;  // default: config 3's volume
    const uint64_t nrows = bytes / 1024;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x5A, bytes);
    for (int k = 0; k < 30; ++k) hipLaunchKernelGGL((stream<1>), dim3(cus * 2), dim3(256), 0, 0, buf, nrows, 1u, out);
    (void)hipDeviceSynchronize();
    auto gbs = [&](float ms) { return bytes / ms / 1e6; };
    for (int round = 0; round < 2; ++round) {
        for (int bpc : {1, 2}) {
            const int g = cus * bpc;
            const float s = timeit([&] { hipLaunchKernelGGL((stream<0>), dim3(g), dim3(256), 0, 0, buf, nrows, 1u, out); });
            const float w = timeit([&] { hipLaunchKernelGGL((stream<1>), dim3(g), dim3(256), 0, 0, buf, nrows, 1u, out); });
            printf("bpc=%d slices %.4f ms %.0f GB/s | window %.4f ms %.0f GB/s", bpc, s, gbs(s), w, gbs(w));
            for (uint32_t K : {4u, 16u, 64u}) {
                const float r = timeit([&] { hipLaunchKernelGGL((stream<2>), dim3(g), dim3(256), 0, 0, buf, nrows, K, out); });
                printf(" | rounds K=%u %.4f ms %.0f GB/s", K, r, gbs(r));
            }
            for (uint32_t K : {8u, 11u, 14u}) {
                const float r = timeit([&] { hipLaunchKernelGGL((stream<3>), dim3(g), dim3(256), 0, 0, buf, nrows, K, out); });
                printf(" | chunks 2^%u %.4f ms %.0f GB/s", K, r, gbs(r));
            }
            printf("\n");
            fflush(stdout);
        }
    }
    return 0;
}
