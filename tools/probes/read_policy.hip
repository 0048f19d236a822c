// Read ceiling by cache policy: a 1.5 GB stream (config 2's bytes) read with
// buffer_load_dwordx4 under each cache-policy operand (aux bits of the raw buffer
// load builtin: sc0 / nt / sc1 on gfx950), 2 loads in flight per lane, software-
// pipelined (next pair issued before the current pair is summed), grid of
// 1/2/4 blocks per CU, XCD-interleaved 24 MiB chunks as in the product kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(256) void read_pol(const uint8_t* p, uint32_t nrows, uint32_t* out) {
    // a row = 4 KiB (one 256-thread block-wide 16 B/lane load); XCD x takes chunks x, x+8, ... of 6144 rows
    const uint32_t x = blockIdx.x & 7, slot = blockIdx.x >> 3, per = gridDim.x >> 3;
    constexpr uint32_t kChunkLog = 12;
    auto row_of = [&](uint32_t i) { return ((((i >> kChunkLog) << 3) + x) << kChunkLog) | (i & ((1u << kChunkLog) - 1)); };
    uint32_t acc = 0;
    auto ld = [&](uint32_t i, v4u& v) {
        const uint32_t r = row_of(i);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p) + (uint64_t)(r < nrows ? r : 0) * 4096, 0,
                                              r < nrows ? 4096 : 0, 0x00020000);
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, threadIdx.x * 16, 0, AUX);
    };
    uint32_t i = slot;
    v4u a0, a1, b0, b1;
    ld(i, a0);
    ld(i + per, a1);
    while (row_of(i) < nrows) {
        const uint32_t j = i + 2 * per;
        ld(j, b0);
        ld(j + per, b1);
        asm volatile("" : "+v"(a0), "+v"(a1));
        acc += a0.x + a0.y + a0.z + a0.w + a1.x + a1.y + a1.z + a1.w;
        if (row_of(j) >= nrows) break;
        i = j + 2 * per;
        ld(i, a0);
        ld(i + per, a1);
        asm volatile("" : "+v"(b0), "+v"(b1));
        acc += b0.x + b0.y + b0.z + b0.w + b1.x + b1.y + b1.z + b1.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int AUX>
float run(const uint8_t* p, uint32_t nrows, uint32_t* out, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a);
        for (int k = 0; k < 20; ++k) hipLaunchKernelGGL((read_pol<AUX>), dim3(blocks), dim3(256), 0, 0, p, nrows, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / 20);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

int main() {
    const uint64_t bytes = 1572864000ull;
    const uint32_t nrows = (uint32_t)(bytes / 4096);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0x5A, bytes);
    for (int k = 0; k < 200; ++k) hipLaunchKernelGGL((read_pol<2>), dim3(cus * 2), dim3(256), 0, 0, buf, nrows, out);
    (void)hipDeviceSynchronize();
    for (int bpc : {1, 2, 4}) {
        const int g = cus * bpc;
        const float t0 = run<0>(buf, nrows, out, g), t1 = run<1>(buf, nrows, out, g), t2 = run<2>(buf, nrows, out, g),
                    t3 = run<3>(buf, nrows, out, g), t16 = run<16>(buf, nrows, out, g),
                    t18 = run<18>(buf, nrows, out, g);
        auto gbs = [&](float ms) { return bytes / ms / 1e6; };
        printf("bpc=%d aux0 %.0f | aux1 %.0f | aux2(nt) %.0f | aux3 %.0f | aux16 %.0f | aux18 %.0f GB/s\n", bpc,
               gbs(t0), gbs(t1), gbs(t2), gbs(t3), gbs(t16), gbs(t18));
    }
    return 0;
}
