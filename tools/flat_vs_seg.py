#!/usr/bin/env python3
"""Same-process A/B on a fixed-stride batch (stride == segment length): the fixed-stride
kernel (per-segment tasks) against the ragged prefix-scan kernel fed offsets i*L (a
flat stream of 128 B-aligned 1 KiB rows, boundaries by scan). Results must agree.

    python tools/flat_vs_seg.py [--segs 16777216] [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import torch  # noqa: E402

import nsx  # noqa: E402

L = 1500


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=1 << 24)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n = a.segs
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(buf, 0x1071)
    offs = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    o1 = torch.empty(n, dtype=torch.int16, device="cuda")
    o2 = torch.empty(n, dtype=torch.int16, device="cuda")
    variants = {"fixed": lambda: nsx.fixed_dev(buf, L, L, n, out=o1),
                "ragged_scan": lambda: nsx.ragged_dev(buf, offs, out=o2)}
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    assert torch.equal(o1, o2), "fixed and ragged results differ"
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
        ms = statistics.median(t)
        print(f"segs={n} {name:>12} median {ms:.4f} ms  {n * L / ms / 1e6:.0f} GB/s (payload)", flush=True)


if __name__ == "__main__":
    main()
