// launch_cost — what one launch of a persistent grid costs when it does no work.
//
// A diagnostic build of the ragged checksum that returned at once still took ~8.3 µs per launch back to back
// (profiles/r04_fixed_cost_ab.txt). This probe separates the parts: an empty kernel (each wave exits at once, or
// after one 4 B load and one 2 B store per lane) at grids of 256-4096 blocks of 256 threads, with and without
// the ragged kernel's 33.8 KB of dynamic LDS per block, timed over 200 back-to-back launches with HIP events on
// one stream; then the same launches captured into one hipGraph and replayed.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/launch_cost.hip -o tools/probes/launch_cost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(256) void empty_kernel(uint32_t n) {
    if (n != 12345u) return;
}

__global__ __launch_bounds__(256) void touch_kernel(const uint32_t* __restrict__ in, uint16_t* __restrict__ out,
                                                     uint32_t n) {
    extern __shared__ uint32_t lds[];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint16_t)(in[i] + (n == 12345u ? lds[threadIdx.x] : 0u));
}

int main() {
    const int reps = 200;
    const size_t lds_big = 8 * 1024 * 4 + 256 * 4 + 1024;  // 33.8 KB, the ragged kernel's four slots
    uint32_t* in;
    uint16_t* out;
    CK(hipMalloc(&in, 4096 * 256 * 4));
    CK(hipMalloc(&out, 4096 * 256 * 2));
    CK(hipMemset(in, 0, 4096 * 256 * 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d; us per launch over %d back-to-back launches (stream) and in one hipGraph replay\n", cus, reps);
    printf("%-6s %-6s %-10s %10s %10s\n", "kind", "blocks", "lds", "stream_us", "graph_us");
    for (int kind = 0; kind < 2; ++kind)
        for (uint32_t blocks : {256u, 512u, 768u, 1024u, 2048u, 4096u})
            for (size_t lds : {(size_t)0, lds_big}) {
                auto launch = [&]() {
                    if (kind == 0)
                        hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), lds, st, 0u);
                    else
                        hipLaunchKernelGGL(touch_kernel, dim3(blocks), dim3(256), lds, st, in, out, blocks * 256u);
                };
                for (int i = 0; i < 20; ++i) launch();
                CK(hipStreamSynchronize(st));
                float best = 1e30f;
                for (int t = 0; t < 5; ++t) {
                    CK(hipEventRecord(e0, st));
                    for (int i = 0; i < reps; ++i) launch();
                    CK(hipEventRecord(e1, st));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms < best ? ms : best;
                }
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
                for (int i = 0; i < reps; ++i) launch();
                CK(hipStreamEndCapture(st, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGraphLaunch(ge, st));
                CK(hipStreamSynchronize(st));
                float bestg = 1e30f;
                for (int t = 0; t < 5; ++t) {
                    CK(hipEventRecord(e0, st));
                    CK(hipGraphLaunch(ge, st));
                    CK(hipEventRecord(e1, st));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    bestg = ms < bestg ? ms : bestg;
                }
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(g));
                printf("%-6s %-6u %-10zu %10.2f %10.2f\n", kind ? "touch" : "empty", blocks, lds, best * 1e3f / reps,
                       bestg * 1e3f / reps);
            }
    return 0;
}
