#!/usr/bin/env python3
"""Throughput vs segment shape (fixed stride, ~1.5 GB per batch), steady state.

    python tools/shape_sweep.py [--param kernel=2 ...]
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
    ap.add_argument("--param", action="append", default=[])
    ap.add_argument("--shapes", default="64:64,512:512,1024:1024,1496:1496,1500:1500,1504:1504,1536:1536,2048:2048,"
                                        "3000:3000,4096:4096,8192:8192,65536:65536")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    total = 1_572_864_000
    buf = torch.empty(total + 65536, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(buf, 0x1071)
    shapes = [tuple(int(x) for x in s.split(":")) for s in a.shapes.split(",")]
    variants = [dict()] + [dict(kv.split("=") for kv in p.split(";")) for p in a.param]
    out = torch.empty(total // 64 + 1, dtype=torch.int16, device="cuda")
    # settle clocks
    for _ in range(200):
        nsx.fixed_dev(buf, 1500, 1500, total // 1500, out=out)
    torch.cuda.synchronize()
    for L, S in shapes:
        n = (total - L) // S + 1
        line = []
        for v in variants:
            for p in nsx.ALL_PARAMS:
                nsx.set_param(p, 0)
            for k, val in v.items():
                nsx.set_param(bench.PARAMS[k], int(val))
            ts = []
            for _ in range(3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    nsx.fixed_dev(buf, S, L, n, out=out)
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) / 20)
            ms = statistics.median(ts)
            line.append(f"{n * L / ms / 1e6:7.0f}")
        print(f"L={L:6d} S={S:6d} n={n:9d}  GB/s: " + " ".join(line) + "   variants: default " +
              " | ".join(a.param), flush=True)


if __name__ == "__main__":
    main()
