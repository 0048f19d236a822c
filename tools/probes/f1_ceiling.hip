// f1_ceiling — ONE copy ceiling for the fused TCP build's exact layout, measured in the same
// process and on the same buffers as the product build (nsx_tcp_build_dev, bench workload 6: 1M option-less
// segments, 1480 B payloads packed at 1480·i, 1500 B wire images packed at 1500·i, IPv4 pseudo-header partials).
//
//   build   : the product, nsx_tcp_build_dev (reads payload + 18 B fields + offsets + partial, writes the image
//             and a 2 B raw sum per segment)
//   layout  : the same byte movement with no header fields, offsets, partials or checksum: one wave per segment,
//             image-relative 16 B chunks (lane c stores image bytes [16c, 16c + 16) at out + 1500·i + 16c, loaded
//             from the payload 20 B earlier, the header dwords substituted) — the build's own store and load
//             pattern, 4 B-misaligned images included; groups of G consecutive segments per wave task, the next
//             segment's rows in flight while one is stored; best over grids and group sizes
//   flat    : the unconstrained copy of the same volume (n·1490 B read and written, 16 B aligned both sides,
//             grid-stride, K loads in flight per lane, plain or non-temporal stores); best over shapes
//   r02cp   : round 2's copy kernel (tools/probes/copy_ceiling.hip: flat pointer loads and stores, nt or plain,
//             L = 1-4 in flight; its nt L=1 at 4 blocks/CU read 5.976 TB/s in round 2) and the plain float4
//             grid-stride copy, over the same volume
//   memcpy  : hipMemcpyAsync device to device of the same volume
// The "layout" figure is circular as a ceiling — f1's own access shape with the arithmetic removed — so the
// SUMMARY reports the build against the best same-process copy of the volume (flat, r02cp, memcpy).
// Printed per variant: ms, TB/s of (payload read + image write), and the build's time as a fraction of it.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/probes/f1_ceiling.hip \
//          -L network-stack_amd/lib -lnsx_csum -Wl,-rpath,'$ORIGIN/../../network-stack_amd/lib' -o tools/probes/f1_ceiling
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "nsx_csum.h"

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;
constexpr uint32_t kPay = 1480, kImg = 1500, kHdr = 20;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)n, 0x00020000);
}

// flat copy, K chunks in flight per lane, SP = store cache policy (0 plain, 2 nt)
template <int K, int SP>
__global__ __launch_bounds__(256) void flat_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, uint64_t n16) {
    const uint64_t nth = (uint64_t)gridDim.x * 256;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < n16; i0 += nth * K) {
        v4u v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t c = i0 + (uint64_t)k * nth;
            const __amdgpu_buffer_rsrc_t r = rsrc(s + c * 16, c < n16 ? (uint32_t)std::min<uint64_t>(4096, (n16 - c) * 16) : 0);
            v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16, 0, 2);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) asm volatile("" : "+v"(v[k]));
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t c = i0 + (uint64_t)k * nth;
            const __amdgpu_buffer_rsrc_t r = rsrc(d + c * 16, c < n16 ? (uint32_t)std::min<uint64_t>(4096, (n16 - c) * 16) : 0);
            __builtin_amdgcn_raw_buffer_store_b128(v[k], r, threadIdx.x * 16, 0, SP);
        }
    }
}

// round 2's copy probe kernel (tools/probes/copy_ceiling.hip, profiles/r02_copy_ceiling.txt: nt, L = 1, 4 blocks/CU
// 5.976 TB/s over 1.5 GB): grid-stride over 16 B chunks with flat pointer loads and stores, consecutive lanes on
// consecutive chunks, L chunks in flight per lane, non-temporal loads and stores or plain ones — the plain form is
// the textbook float4 grid-stride copy
template <int L, bool NT>
__global__ __launch_bounds__(256) void copy16(const v4u* __restrict__ s, v4u* __restrict__ d, uint64_t n16) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, nth = (uint64_t)gridDim.x * 256;
    uint64_t i = tid;
    for (; i + (L - 1) * nth < n16; i += L * nth) {
        v4u v[L];
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

// f1's exact layout, no header fields / checksum: segments [t·G, t·G + G) per wave task, pipelined by segment;
// LP / SP = load / store cache policy (0 plain, 2 nt)
template <int G, int LP = 0, int SP = 0>
__global__ __launch_bounds__(256) void layout_copy(const uint8_t* __restrict__ data, uint8_t* __restrict__ out, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = gridDim.x * 4;
    const uint32_t ntask = (n + G - 1) / G;
    auto ld = [&](uint32_t i, v4u& a, v4u& b) {  // image-relative: dword k of the image ← payload dword k − 5
        const bool ok = i < n;
        const __amdgpu_buffer_rsrc_t r = rsrc(data + (uint64_t)(ok ? i : 1u) * kPay - kHdr, ok ? kImg : 0u);
        a = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, LP);
        b = __builtin_amdgcn_raw_buffer_load_b128(r, 1024 + lane * 16, 0, LP);
    };
    auto st = [&](uint32_t i, v4u a, v4u b) {
        asm volatile("" : "+v"(a), "+v"(b));
        if (lane == 0) a = v4u{i, i ^ 1u, i ^ 2u, i ^ 3u};  // header bytes 0-15
        if (lane == 1) a.x = i ^ 4u;                       // header bytes 16-19
        const __amdgpu_buffer_rsrc_t r = rsrc(out + (uint64_t)i * kImg, kImg);
        __builtin_amdgcn_raw_buffer_store_b128(a, r, lane * 16, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(b, r, 1024 + lane * 16, 0, SP);
    };
    for (uint32_t t = blockIdx.x * 4 + wave; t < ntask; t += nw) {
        const uint32_t s0 = t * G, s1 = std::min(n, s0 + G);
        v4u a0, b0, a1, b1;
        ld(s0, a0, b0);
        for (uint32_t i = s0; i < s1; i += 2) {
            ld(i + 1 < s1 ? i + 1 : n, a1, b1);
            st(i, a0, b0);
            if (i + 1 >= s1) break;
            ld(i + 2 < s1 ? i + 2 : n, a0, b0);
            st(i + 1, a1, b1);
        }
    }
}

template <typename F>
static float timeit(F f, int reps = 20) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) {
        (void)hipEventRecord(a);
        for (int k = 0; k < reps; ++k) f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms / reps);
    }
    std::sort(t.begin(), t.end());
    return t[3];
}

int main() {
    const uint32_t n = 1u << 20;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint64_t data_bytes = (uint64_t)n * kPay, out_bytes = (uint64_t)n * kImg;
    uint8_t *data0 = nullptr, *out = nullptr, *flat_dst = nullptr;
    // data starts 256 B into its allocation (the layout copy reads 20 B before payload 0)
    // (the flat copy reads n·1490 B from data's allocation)
    if (hipMalloc(&data0, (uint64_t)n * 1490 + 512) || hipMalloc(&out, out_bytes + 256) ||
        hipMalloc(&flat_dst, out_bytes + 256))
        return 1;
    uint8_t* data = data0 + 256;
    if (nsx_fill_splitmix64_dev(data, 0, data_bytes, 0x1074, nullptr) != NSX_OK) return 2;
    // the product's inputs: header fields (SoA), offsets, pseudo-header partials (bench workload 6's shape)
    std::vector<uint64_t> doff(n + 1), ooff(n + 1);
    for (uint32_t i = 0; i <= n; ++i) doff[i] = (uint64_t)i * kPay, ooff[i] = (uint64_t)i * kImg;
    uint64_t *d_doff, *d_ooff;
    uint8_t* fields;
    uint32_t* part;
    uint16_t* raw;
    if (hipMalloc(&d_doff, 8ull * (n + 1)) || hipMalloc(&d_ooff, 8ull * (n + 1)) || hipMalloc(&fields, 18ull * n + 64) ||
        hipMalloc(&part, 4ull * n) || hipMalloc(&raw, 2ull * n))
        return 1;
    (void)hipMemcpy(d_doff, doff.data(), 8ull * (n + 1), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ooff, ooff.data(), 8ull * (n + 1), hipMemcpyHostToDevice);
    (void)nsx_fill_splitmix64_dev(fields, 0, 18ull * n + 64, 0x1075, nullptr);
    (void)nsx_fill_splitmix64_dev(part, 0, 4ull * n, 0x1076, nullptr);
    (void)hipMemset(fields + 12ull * n, 5, n);  // offset = 5 (computeOffset of an option-less segment)
    nsx_tcp_hdr_soa h;
    h.src_port = reinterpret_cast<const uint16_t*>(fields);
    h.dst_port = reinterpret_cast<const uint16_t*>(fields + 2ull * n);
    h.seq_num = reinterpret_cast<const uint32_t*>(fields + 4ull * n);
    h.ack_num = reinterpret_cast<const uint32_t*>(fields + 8ull * n);
    h.offset = fields + 12ull * n;
    h.control = fields + 13ull * n;
    h.window = reinterpret_cast<const uint16_t*>(fields + 14ull * n);
    h.urgent_ptr = reinterpret_cast<const uint16_t*>(fields + 16ull * n);
    auto build = [&] {
        (void)nsx_tcp_build_dev(&h, nullptr, nullptr, data, d_doff, data_bytes, part, n, out, d_ooff, raw, nullptr);
    };
    for (int k = 0; k < 200; ++k) build();  // settle clocks
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    const double moved = (double)n * (kPay + kImg);  // payload read + image written (the copy volume)
    const double alg = (double)n * (kPay + 18 + 8 + 8 + 4 + kImg + 2) + 16;  // bench workload 6's algorithmic bytes
    std::vector<std::pair<const char*, float>> res;
    float t_build = timeit(build);
    printf("build (nsx_tcp_build_dev)       %.4f ms  %.3f TB/s copy volume  %.3f TB/s algorithmic (roofline %.3f)\n",
           t_build, moved / t_build / 1e9, alg / t_build / 1e9, alg / t_build / 1e9 / 8.0);
    fflush(stdout);
    float best_layout = 1e9, best_flat = 1e9, best_r02 = 1e9;
    const char* best_r02_name = "";
    char best_r02_buf[64];
    const uint64_t n16 = (uint64_t)n * 1490 / 16;
    for (int bpc : {1, 2, 4, 8}) {
        const uint32_t g = cus * bpc;
        auto L = [&](auto gc, auto lc, auto sc) {
            constexpr int G = decltype(gc)::value, LP = decltype(lc)::value, SP = decltype(sc)::value;
            const float t = timeit([&] { hipLaunchKernelGGL((layout_copy<G, LP, SP>), dim3(g), dim3(256), 0, 0, data, out, n); });
            printf("layout bpc=%d G=%-2d ld=%-5s st=%-5s %.4f ms  %.3f TB/s   build/this %.3f\n", bpc, G, LP ? "nt" : "plain",
                   SP ? "nt" : "plain", t, moved / t / 1e9, t / t_build);
            best_layout = std::min(best_layout, t);
        };
        using I0 = std::integral_constant<int, 0>;
        using I2 = std::integral_constant<int, 2>;
        L(std::integral_constant<int, 4>{}, I0{}, I0{});
        L(std::integral_constant<int, 16>{}, I0{}, I0{});
        L(std::integral_constant<int, 64>{}, I0{}, I0{});
        L(std::integral_constant<int, 16>{}, I2{}, I0{});
        L(std::integral_constant<int, 16>{}, I2{}, I2{});
        auto F = [&](auto kc, auto sc) {
            constexpr int K = decltype(kc)::value, SP = decltype(sc)::value;
            const float t = timeit([&] {
                hipLaunchKernelGGL((flat_copy<K, SP>), dim3(g), dim3(256), 0, 0, data, flat_dst, n16);
            });
            printf("flat   bpc=%d K=%d %-5s                %.4f ms  %.3f TB/s   build/this %.3f\n", bpc, K, SP ? "nt" : "plain", t,
                   moved / t / 1e9, t / t_build);
            best_flat = std::min(best_flat, t);
        };
        F(std::integral_constant<int, 1>{}, I0{});
        F(std::integral_constant<int, 2>{}, I0{});
        F(std::integral_constant<int, 4>{}, I0{});
        F(std::integral_constant<int, 1>{}, I2{});
        F(std::integral_constant<int, 2>{}, I2{});
        F(std::integral_constant<int, 4>{}, I2{});
        auto R = [&](auto lc, auto nc) {
            constexpr int LL = decltype(lc)::value;
            constexpr bool NT = decltype(nc)::value;
            const float t = timeit([&] {
                hipLaunchKernelGGL((copy16<LL, NT>), dim3(g), dim3(256), 0, 0, (const v4u*)data, (v4u*)flat_dst, n16);
            });
            printf("r02cp  bpc=%d L=%d %-5s                %.4f ms  %.3f TB/s   build/this %.3f\n", bpc, LL, NT ? "nt" : "plain",
                   t, moved / t / 1e9, t / t_build);
            if (t < best_r02) {
                best_r02 = t;
                snprintf(best_r02_buf, sizeof best_r02_buf, "bpc=%d L=%d %s", bpc, LL, NT ? "nt" : "plain");
                best_r02_name = best_r02_buf;
            }
        };
        R(std::integral_constant<int, 1>{}, std::true_type{});
        R(std::integral_constant<int, 2>{}, std::true_type{});
        R(std::integral_constant<int, 4>{}, std::true_type{});
        R(std::integral_constant<int, 1>{}, std::false_type{});
        R(std::integral_constant<int, 2>{}, std::false_type{});
        R(std::integral_constant<int, 4>{}, std::false_type{});
        fflush(stdout);
    }
    float t_dd;
    {
        t_dd = timeit([&] { (void)hipMemcpyAsync(flat_dst, data, n16 * 16, hipMemcpyDeviceToDevice, 0); });
        printf("hipMemcpyDtoD                          %.4f ms  %.3f TB/s   build/this %.3f\n", t_dd, moved / t_dd / 1e9,
               t_dd / t_build);
    }
    t_build = std::min(t_build, timeit(build));  // again after the probes (clock drift check)
    const float best_copy = std::min(std::min(best_flat, best_r02), t_dd);
    printf("SUMMARY build %.4f ms (%.3f TB/s copy volume) | best same-process copy of the volume %.4f ms (%.3f TB/s): "
           "build at %.3f of it | r02 copy kernel best %.4f ms (%.3f TB/s, %s) | buffer-load flat copy best %.4f ms | "
           "hipMemcpyDtoD %.4f ms | circular layout ceiling (f1's own access shape, arithmetic removed) %.4f ms: build "
           "at %.3f of it | build roofline %.3f\n",
           t_build, moved / t_build / 1e9, best_copy, moved / best_copy / 1e9, best_copy / t_build, best_r02,
           moved / best_r02 / 1e9, best_r02_name, best_flat, t_dd, best_layout, best_layout / t_build,
           alg / t_build / 1e9 / 8.0);
    return 0;
}
