// Probe: gfx950 raw-buffer out-of-range semantics for partially out-of-range
// dwordx4 / dword loads (does the range check zero per dword, or the whole access?).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint32_t* buf, uint32_t num_records, uint32_t* out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, num_records, 0x00020000);
    const uint32_t lane = threadIdx.x;
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 4, 0, 0);
    out[lane * 5 + 0] = v.x; out[lane * 5 + 1] = v.y; out[lane * 5 + 2] = v.z; out[lane * 5 + 3] = v.w;
    out[lane * 5 + 4] = __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4 + 2, 0, 0);
}

int main() {
    uint32_t h[64];
    for (int i = 0; i < 64; ++i) h[i] = 0x11111111u * (uint32_t)((i % 15) + 1);
    uint32_t *d, *o;
    hipMalloc(&d, sizeof h); hipMalloc(&o, 8 * 5 * 4);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    for (uint32_t nr : {8u, 10u, 12u, 13u, 16u, 18u, 20u}) {
        hipMemset(o, 0xEE, 8 * 5 * 4);
        hipLaunchKernelGGL(probe, dim3(1), dim3(8), 0, 0, d, nr, o);
        uint32_t r[40];
        hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
        printf("num_records=%u\n", nr);
        for (int l = 0; l < 8; ++l)
            printf("  off %2d: x4 = %08x %08x %08x %08x | dword@%2d = %08x\n", l * 4, r[l*5], r[l*5+1], r[l*5+2], r[l*5+3], l * 4 + 2, r[l*5+4]);
    }
    return 0;
}
