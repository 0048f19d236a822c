// wave_stamps.h — the recording WaveStamps policy for per-wave timelines (diagnostic library only).
//
// csum_kernels.hip includes this instead of its empty WaveStamps when built with -DNSX_WAVE_STAMPS
// (`make -C network-stack_amd stamps` → lib_stamps/libnsx_csum.so); the product library never contains it.
// The receive pass (rx_tcp_kernel) and the packed-header kernel (ipv4_hdr20_kernel) call entry() at kernel entry,
// ready() once the wave knows its range and done(g, work, lane) at its end. Wave g of the last launch writes
//   g_wave_stamps[4g .. 4g+3] = {t_entry, t_ready (0 if never called), t_end, work (low 32 bits) | where << 32}
// with s_memrealtime times (100 MHz), work = the wave's bytes (receive pass) or tasks (packed headers), and where =
// XCC_ID << 16 | HW_ID's low half (wave, SIMD, CU, SH, SE). Read back (and cleared) with nsx_diag_wave_stamps;
// tools/probes/rx_wave_times.py and f3_wave_times.py print the timelines.
#pragma once

constexpr uint32_t kStampWaves = 8192;
__device__ uint64_t g_wave_stamps[kStampWaves * 4];

struct WaveStamps {
    uint64_t t_entry = 0, t_ready = 0;
    __device__ __forceinline__ void entry() {
        t_entry = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the stamp has landed
    }
    __device__ __forceinline__ void ready() {
        t_ready = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    __device__ __forceinline__ void done(uint32_t g, uint64_t work, uint32_t lane) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint64_t where = (uint64_t)((xcc & 0xFu) << 16 | (hw & 0xFFFFu)) << 32;
        const uint64_t v = lane == 0 ? t_entry : lane == 1 ? t_ready : lane == 2 ? t_end : (work & 0xFFFFFFFFu) | where;
        if (lane < 4u && g < kStampWaves) g_wave_stamps[(uint64_t)g * 4u + lane] = v;  // a vector store per lane
    }
};

// Copy min(count, 4·kStampWaves) stamp words to dst (host memory) and clear them on the device.
extern "C" __attribute__((visibility("default"))) int nsx_diag_wave_stamps(uint64_t* dst, uint64_t count) {
    const size_t bytes = (size_t)(count < (uint64_t)kStampWaves * 4 ? count : (uint64_t)kStampWaves * 4) * 8;
    if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wave_stamps), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess) return -5;
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_wave_stamps)) != hipSuccess) return -5;
    return hipMemset(p, 0, (size_t)kStampWaves * 32) == hipSuccess ? 0 : -5;
}
