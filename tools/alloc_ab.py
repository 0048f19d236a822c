#!/usr/bin/env python3
"""Allocation dependence of one bench workload: build it K times in one process
(K sets of device buffers at different physical placements), optionally with
launch overrides, and time every (allocation, variant) pair in interleaved
rounds. A kernel whose speed follows the allocation shows a spread across rows
that the variants do not close.

    python tools/alloc_ab.py --config 6 --allocs 4 --variants "def:;b2:blocks_per_cu=2"
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "network-stack_amd")]


def main():
    import bench
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=6)
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--variants", default="def:")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=30)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    cfg = bench.WORKLOADS[a.config]
    ws = [bench.build_workload(cfg, 0, torch.device("cuda", 0)) for _ in range(a.allocs)]
    variants = []
    for item in a.variants.split(";"):
        name, _, kv = item.partition(":")
        variants.append((name, bench.parse_tune([x for x in kv.split(",") if x]) or None))
    steps = {(i, name): w["step_for"](t) for i, w in enumerate(ws) for name, t in variants}
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:
        for st in steps.values():
            st()
        torch.cuda.synchronize()
    res = {k: [] for k in steps}
    for _ in range(a.rounds):
        for k, st in steps.items():
            for _ in range(3):
                st()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.launches):
                st()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / a.launches)
    alg = ws[0]["alg"]
    for name, _ in variants:
        meds = [statistics.median(res[(i, name)]) for i in range(a.allocs)]
        print(f"ALLOC config{a.config} {name:12s} " + " ".join(f"{m:.4f}" for m in meds) +
              f"  ms/launch  frac {alg / (min(meds) * 1e-3) / 8e12:.3f}..{alg / (max(meds) * 1e-3) / 8e12:.3f}",
              flush=True)


if __name__ == "__main__":
    main()
