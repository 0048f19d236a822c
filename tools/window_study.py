#!/usr/bin/env python3
"""Why does config 5 (16M x 1500 B = 23.4 GiB per GPU) run ~6% slower per byte than
config 2 (1M x 1500 B)? Times nsx_csum_fixed_dev over the whole config-5 batch and
over windows of it (1M, 4M segments at several offsets) in one process: if every
window runs at config 2's rate, the gap comes from the batch's size (translation,
DRAM page policy), not from where its pages sit.

    python tools/window_study.py [--segs 16777216] [--rounds 3]
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


def time_on(buf, n, out, iters=10):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record()
        nsx.fixed_dev(buf, L, L, n, out=out)
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=1 << 24)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.segs
    buf = torch.empty(N * L, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(buf, 0x1071)
    out = torch.empty(N, dtype=torch.int16, device="cuda")
    cases = [("full", 0, N)]
    for w in (1 << 20, 1 << 22):
        for k in (0, N // (2 * w), N // w - 1):
            cases.append((f"win{w >> 20}M@{k}", k * w, w))
    for _, s0, n in cases:
        time_on(buf[s0 * L:(s0 + n) * L], n, out, 3)
    res = {c[0]: [] for c in cases}
    for _ in range(a.rounds):
        for name, s0, n in cases:
            res[name].append(time_on(buf[s0 * L:(s0 + n) * L], n, out))
    for name, s0, n in cases:
        ms = statistics.median(res[name])
        print(f"{name:>14} segs={n:>9} ms={ms:.4f} GB/s={(n * (L + 2)) / ms / 1e6:.0f}", flush=True)


if __name__ == "__main__":
    main()
