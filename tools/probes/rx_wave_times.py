#!/usr/bin/env python3
"""Per-wave timeline of the receive pass (diagnostic library only: `make -C network-stack_amd stamps`, whose kernels'
WaveStamps hook records each wave's s_memrealtime stamps, tools/probes/wave_stamps.h, read back with
nsx_diag_wave_stamps). Loads network-stack_amd/lib_stamps, builds a bench workload, runs it many times back to back,
and prints
the distribution of wave start (relative to the launch's first wave), range-ready and end times, in µs, and how
the end times split over the hardware (the kernel also records each wave's HW_ID and XCC_ID): per XCD, per CU and
within a block — with the tail each level of balancing would leave (every CU's, or every block's, waves ending at
their mean).

    python tools/probes/rx_wave_times.py [--config 13] [--launches 20]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "network-stack_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=13)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--mode", type=int, default=5)
    ap.add_argument("--wpb", type=int, default=2, help="waves per block taking ranges (streamed modes: 4)")
    ap.add_argument("--lib", default="stamps", help="network-stack_amd/lib_<name>: a build with NSX_WAVE_STAMPS")
    ap.add_argument("--deal", type=int, default=0, help="nsx_tune.deal (-1: equal static shares)")
    ap.add_argument("--cus", type=int, default=256, help="CUs of the device (slot grouping)")
    a = ap.parse_args()
    import nsx
    nsx.LIB_PATH = os.path.join(ROOT, "network-stack_amd", f"lib_{a.lib}", "libnsx_csum.so")
    import torch
    import bench
    torch.cuda.set_device(0)
    cfg = dict(bench.WORKLOADS[a.config])
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    L = nsx.lib()
    L.nsx_diag_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    st = np.zeros(8192 * 4, np.uint64)
    rx = nsx.rx_ipv6_tcp_verify_dev if cfg.get("ipver") == 6 else nsx.rx_ipv4_tcp_verify_dev
    tune = dict(segs_per_wave=a.mode, deal=a.deal)
    for _ in range(200):
        rx(w["buf"], w["d_offs"], mask=w["out"], tune=tune)
    torch.cuda.synchronize()
    rows = []
    for _ in range(a.launches):
        assert L.nsx_diag_wave_stamps(st.ctypes.data, st.size) == 0  # clears
        for _ in range(3):
            rx(w["buf"], w["d_offs"], mask=w["out"], tune=tune)
        torch.cuda.synchronize()
        assert L.nsx_diag_wave_stamps(st.ctypes.data, st.size) == 0
        t = st
        nw = int(np.count_nonzero(t[2::4]))
        t = t[: nw * 4].reshape(nw, 4).astype(np.int64)
        t0 = t[:, 0].min()
        rows.append(((t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0, t[:, 3] & 0xFFFFFFFF,
                     t[:, 3] >> 32))
    for name, k in (("start", 0), ("range", 1), ("end", 2)):
        v = np.concatenate([r[k] for r in rows])
        print(f"{name:6s} us: min {v.min():7.2f} p10 {np.percentile(v, 10):7.2f} p50 {np.percentile(v, 50):7.2f} "
              f"p90 {np.percentile(v, 90):7.2f} p99 {np.percentile(v, 99):7.2f} max {v.max():7.2f}")
    # by XCD: waves are numbered XCD-major (g = xcd * W/8 + i), so the end time's mean per eighth of g
    nw = len(rows[0][0])
    for k, nm in ((2, "end"),):
        per = np.mean([[r[k][x * nw // 8:(x + 1) * nw // 8].mean() - np.median(r[k]) for x in range(8)] for r in rows], 0)
        print(f"{nm} minus median, mean per XCD (us): " + " ".join(f"{v:+.2f}" for v in per))
    # does a wave's end follow its frame bytes? (correlation over waves, median over launches)
    if rows[0][3].max() != rows[0][3].min():
        print(f"corr(end, bytes) {np.median([np.corrcoef(r[2], r[3])[0, 1] for r in rows]):.3f}; bytes per wave "
              f"p1 {np.percentile(rows[0][3], 1):.0f} p50 {np.median(rows[0][3]):.0f} p99 {np.percentile(rows[0][3], 99):.0f}")
    # where the spread lives: CU = (XCC_ID, HW_ID's SE/SH/CU bits); block = the wave pair g // 2
    def grouped_tail(r, key):
        end, med = r[2], np.median(r[2])
        _, inv = np.unique(key, return_inverse=True)
        means = np.bincount(inv, weights=end) / np.bincount(inv)
        within = end - means[inv]
        return means.max() - med, means.std(), within.std(), int(np.bincount(inv).mean())
    for nm, keyf in (("CU", lambda r: ((r[4] >> 16) << 8) | ((r[4] >> 8) & 0xFF)),
                     ("SIMD", lambda r: ((r[4] >> 16) << 10) | ((r[4] >> 4) & 0xFFF)),
                     ("block", lambda r: np.arange(len(r[2])) // a.wpb)):
        v = np.array([grouped_tail(r, keyf(r)) for r in rows])
        print(f"by {nm:5s}: waves per group {int(v[0, 3])}; std of group means {np.median(v[:, 1]):.2f} us, std within "
              f"groups {np.median(v[:, 2]):.2f} us; tail if each group's waves ended at their mean "
              f"{np.median(v[:, 0]):.2f} us")
    # by the block's slot on its CU: blocks are dealt to CUs breadth-first (block b on XCD b & 7; its CU's blocks
    # in order b >> 3 = 0, 32, 64, ... for 32 CUs per XCD), so a wave's slot = (b >> 3) // (CUs per XCD); the
    # waves are numbered XCD-major (g // wpb = (b & 7) * per + (b >> 3), per = active blocks / 8)
    nw = len(rows[0][2])
    per = nw // a.wpb // 8
    cus_per_xcd = max(1, a.cus // 8)
    slot = ((np.arange(nw) // a.wpb) % per) // cus_per_xcd
    for k in range(int(slot.max()) + 1):
        v = [np.median(r[2][slot == k]) - np.median(r[2]) for r in rows]
        print(f"slot {k}: waves {int((slot == k).sum())}, median end minus launch median {np.median(v):+.2f} us")
    print(f"end std over waves {np.median([r[2].std() for r in rows]):.2f} us")
    ends = np.array([r[2].max() for r in rows])
    med_end = np.array([np.median(r[2]) for r in rows])
    print(f"launch span (first start -> last end) us: median {np.median(ends):.2f}; median wave end {np.median(med_end):.2f}; "
          f"tail (last end - median end) {np.median(ends - med_end):.2f}; waves {len(rows[0][0])}")


if __name__ == "__main__":
    main()
