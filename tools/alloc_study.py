#!/usr/bin/env python3
"""Does a kernel's speed depend on which allocation backs the batch?

Fresh processes on one box measured 0.221-0.240 ms for the same config-2 launch.
This builds the same bench workload several times in ONE process (separate
allocations), then times each under each launch variant in interleaved rounds
(HIP events, median per buffer). A deal that is fast on every allocation is
robust; one that is fast on some and 8% slow on others depends on where the
driver placed the pages.

    python tools/alloc_study.py --config 2 --buffers 4 --rounds 3 \
        --variants "xcd_map=1;xcd_map=1,xcd_chunk=12"
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import nsx  # noqa: E402


def time_on(step, iters=20):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record()
        step()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def apply(v):
    for p in nsx.ALL_PARAMS:
        nsx.set_param(p, 0)
    for kv in v.split(","):
        if kv:
            k, val = kv.split("=")
            nsx.set_param(bench.PARAMS[k], int(val))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="xcd_map=0",
                    help="';'-separated variants, each a ','-list of bench.PARAMS name=value")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    cfg = bench.WORKLOADS[a.config]
    ws = [bench.build_workload(cfg, 0, torch.device("cuda", 0)) for _ in range(a.buffers)]
    variants = [v for v in a.variants.split(";") if v]
    for v in variants:
        apply(v)
        for w in ws:
            time_on(w["step"], 3)
    res = {(i, v): [] for i in range(len(ws)) for v in variants}
    for r in range(a.rounds):
        for v in variants:
            apply(v)
            for i, w in enumerate(ws):
                res[(i, v)].append(time_on(w["step"], a.iters))
        print(f"round {r} done", flush=True)
    apply("")
    for v in variants:
        meds = [statistics.median(res[(i, v)]) for i in range(len(ws))]
        print(f"config{a.config} {v}: " + " ".join(f"{m:.4f}" for m in meds), flush=True)
        print(f"SUMMARY config{a.config} {v}: worst {max(meds):.4f} ms, mean {statistics.mean(meds):.4f} ms, "
              f"frac(mean) {ws[0]['alg'] / statistics.mean(meds) / 1e6 / 8000:.4f}", flush=True)


if __name__ == "__main__":
    main()
