#!/usr/bin/env python3
"""Steady-state behaviour of the checksum kernel over many back-to-back launches:
per-launch HIP-event durations in buckets, and whole-region averages with and
without per-launch events (does event recording between launches change it?).

    python tools/drift.py [--config 2] [--launches 600]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import nsx  # noqa: E402


def region(w, k):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.record()
    for _ in range(k):
        w["step"]()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / k, (time.perf_counter() - t0) * 1e3 / k


def per_launch(w, k):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    torch.cuda.synchronize()
    for a, b in evs:
        a.record()
        w["step"]()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--launches", type=int, default=600)
    ap.add_argument("--tune", action="append", default=[])
    a = ap.parse_args()
    torch.cuda.set_device(0)
    w = bench.build_workload(bench.WORKLOADS[a.config], 0, torch.device("cuda", 0), bench.parse_tune(a.tune) or None)
    alg = w["alg"]
    for rep in range(2):
        d = per_launch(w, a.launches)
        buckets = [statistics.mean(d[i:i + 50]) for i in range(0, len(d), 50)]
        print(f"rep{rep} per-launch ms by 50s:", " ".join(f"{x:.4f}" for x in buckets), flush=True)
        print(f"rep{rep} per-launch median {statistics.median(d):.4f} min {min(d):.4f} max {max(d):.4f} "
              f"-> {alg / statistics.median(d) / 1e6:.0f} GB/s median", flush=True)
        ev, wall = region(w, a.launches)
        print(f"rep{rep} region (no inner events): {ev:.4f} ms/launch (events), {wall:.4f} ms wall "
              f"-> {alg / ev / 1e6:.0f} GB/s", flush=True)
        time.sleep(2)
        ev, wall = region(w, 20)
        print(f"rep{rep} after 2 s idle, 20 launches: {ev:.4f} ms/launch -> {alg / ev / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
