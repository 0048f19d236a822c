#!/usr/bin/env python3
"""Per-wave timeline of a stamped kernel (diagnostic library only) under one bench workload's step: the packed-header
kernel (ipv4_hdr20_kernel, workloads 7 and 9) or the fixed-stride kernel (csum_fixed_swp_kernel, configs 2 and 5; the
same stamps, work = tasks of 8 segments). Diagnostic library:
`make -C network-stack_amd stamps`, whose kernels' WaveStamps hook records each wave's s_memrealtime stamps at entry
and end, its task count and where it ran, tools/probes/wave_stamps.h, read back with nsx_diag_wave_stamps). Prints
the end-time spread over the launch's waves, by XCD and CU, and the tail (last end − median end), in µs.

    python tools/probes/f3_wave_times.py [--config 7] [--launches 20]
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
    ap.add_argument("--config", type=int, default=7)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--lib", default="stamps", help="network-stack_amd/lib_<name>: a build with NSX_WAVE_STAMPS")
    ap.add_argument("--wpb", type=int, default=4, help="waves per block that take work (slot grouping)")
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
    for _ in range(100):
        w["step"]()
    torch.cuda.synchronize()
    rows = []
    for _ in range(a.launches):
        assert L.nsx_diag_wave_stamps(st.ctypes.data, st.size) == 0  # clears
        w["step"]()
        torch.cuda.synchronize()
        assert L.nsx_diag_wave_stamps(st.ctypes.data, st.size) == 0
        t = st.reshape(-1, 4).astype(np.int64)
        t = t[t[:, 2] > 0]  # {entry, ready (0), end, tasks | where << 32}
        t0 = t[:, 0].min()
        rows.append(((t[:, 0] - t0) / 100.0, (t[:, 2] - t0) / 100.0, t[:, 3] & 0xFFFFFFFF, t[:, 3] >> 32))
    end = np.concatenate([r[1] for r in rows])
    print(f"waves {len(rows[0][0])}; tasks per wave p1 {np.percentile(rows[0][2], 1):.0f} p50 {np.median(rows[0][2]):.0f} "
          f"p99 {np.percentile(rows[0][2], 99):.0f}")
    print(f"start us: max {max(r[0].max() for r in rows):.2f}")
    print(f"end   us: min {end.min():.2f} p10 {np.percentile(end, 10):.2f} p50 {np.median(end):.2f} "
          f"p90 {np.percentile(end, 90):.2f} p99 {np.percentile(end, 99):.2f} max {end.max():.2f}")
    for nm, keyf in (("XCD", lambda r: r[3] >> 16), ("CU", lambda r: ((r[3] >> 16) << 8) | ((r[3] >> 8) & 0xFF))):
        v = []
        for r in rows:
            _, inv = np.unique(keyf(r), return_inverse=True)
            means = np.bincount(inv, weights=r[1]) / np.bincount(inv)
            v.append((means.max() - np.median(r[1]), means.std()))
        v = np.array(v)
        print(f"by {nm}: std of group means {np.median(v[:, 1]):.2f} us; tail if each group's waves ended at their "
              f"mean {np.median(v[:, 0]):.2f} us")
    # by the block's slot on its CU (blocks dealt to CUs breadth-first; waves numbered XCD-major, g // wpb =
    # (b & 7) * per + (b >> 3) for grids of the XCD-contiguous numbering; the fixed kernel numbers b * wpb + w)
    nw = min(len(r[1]) for r in rows)
    per = nw // a.wpb // 8
    if per:
        slot = ((np.arange(nw) // a.wpb) % per) // max(1, a.cus // 8)
        for k in range(int(slot.max()) + 1):
            v = [np.median(r[1][:nw][slot == k]) - np.median(r[1]) for r in rows]
            print(f"slot {k}: waves {int((slot == k).sum())}, median end minus launch median {np.median(v):+.2f} us")
    tails = [r[1].max() - np.median(r[1]) for r in rows]
    spans = [r[1].max() for r in rows]
    print(f"launch span (first start -> last end) us: median {np.median(spans):.2f}; tail (last end - median end) "
          f"{np.median(tails):.2f}")


if __name__ == "__main__":
    main()
