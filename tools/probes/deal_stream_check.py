#!/usr/bin/env python3
"""Which streams get per-stream deal counters (deal_heads in csum_kernels.hip): the HIP queries deal_heads makes on
the null stream, torch's current stream and a created stream, and the library's sets in use after a receive-pass
launch on each.
    python tools/probes/deal_stream_check.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "network-stack_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import nsx  # noqa: E402


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    w = bench.build_workload(bench.WORKLOADS[18], 0, "cuda")
    cs = torch.cuda.current_stream()
    made = torch.cuda.Stream()
    for name, handle in (("null (0)", 0), ("torch current", cs.cuda_stream), ("torch default", torch.cuda.default_stream().cuda_stream),
                         ("created", made.cuda_stream)):
        cap, dev = ctypes.c_int(-1), ctypes.c_int(-1)
        r1 = hip.hipStreamIsCapturing(ctypes.c_void_p(handle), ctypes.byref(cap))
        r2 = hip.hipStreamGetDevice(ctypes.c_void_p(handle), ctypes.byref(dev))
        hip.hipGetLastError()
        print(f"{name:14s} handle {handle:#x}: hipStreamIsCapturing rc {r1} status {cap.value}; "
              f"hipStreamGetDevice rc {r2} device {dev.value}")
    for name, s in (("torch current", cs), ("created", made)):
        before = nsx.deal_sets_in_use()
        with torch.cuda.stream(s):
            w["step"]()
        torch.cuda.synchronize()
        print(f"after a workload-18 step on {name}: deal sets in use {before} -> {nsx.deal_sets_in_use()}")


if __name__ == "__main__":
    main()
