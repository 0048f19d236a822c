#!/usr/bin/env python3
"""Same-process A/B for the f1 build: workload 6 (option-less) launched without an
option array (tcp_build_kernel<..., OPT=false>) and with an all-empty one
(OPT=true, every optlen 0: identical bytes), interleaved rounds, per-launch HIP
events on the launch stream, medians.

    python tools/opt_ab.py [--rounds 10] [--iters 20]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import nsx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    w = bench.build_workload(bench.WORKLOADS[6], 0, torch.device("cuda", 0))
    n = bench.WORKLOADS[6]["n"]
    P = bench.WORKLOADS[6]["payload"]
    f, data, wire, raw = w["fields"], w["data"], w["wire"], w["out"]
    idx = torch.arange(n + 1, dtype=torch.int64, device="cuda")
    data_off, out_off = idx * P, idx * (P + 20)
    opts = torch.zeros(16, dtype=torch.uint8, device="cuda")
    opt_off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    ref = None
    variants = {
        "no_opt_array": lambda: nsx.tcp_build_dev(f, data, data_off, wire, out_off, raw=raw),
        "empty_opt_array": lambda: nsx.tcp_build_dev(f, data, data_off, wire, out_off, opts=opts, opt_off=opt_off,
                                                     raw=raw),
    }
    for name, fn in variants.items():  # identical images and sums
        fn()
        torch.cuda.synchronize()
        got = (wire.sum(dtype=torch.int64).item(), raw.sum(dtype=torch.int64).item())
        ref = ref or got
        assert got == ref, name
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, fn in variants.items():
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.iters)]
            for e0, e1 in evs:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            times[name].append(statistics.median(e0.elapsed_time(e1) for e0, e1 in evs))
    for name, t in times.items():
        print(f"{name:>16} median {statistics.median(t):.4f} ms  min {min(t):.4f}  max {max(t):.4f}", flush=True)


if __name__ == "__main__":
    main()
