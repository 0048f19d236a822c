#!/usr/bin/env python3
"""Does the fused TCP build (workload 6) gain from back-to-back windows as the fixed checksum
path does? The batch built in one nsx_tcp_build_dev call and as K calls
over equal segment ranges (offsets are absolute, so a window is a slice of the per-segment
arrays), interleaved rounds, wire images and raw sums compared with the one-call output.

    python tools/build_window_ab.py [--segs 1048576] [--ks 1,2,4] [--rounds 5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=1 << 20)
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n = a.segs
    w = bench.build_workload(dict(bench.WORKLOADS[6], n=n), 0, torch.device("cuda", 0))
    f, raw, wire = w["fields"], w["out"], w["wire"]

    def run(k):
        cuts = [n * i // k for i in range(k + 1)]
        for c0, c1 in zip(cuts, cuts[1:]):
            nsx.tcp_build_dev({key: v[c0:c1] for key, v in f.items()}, w["data"], w["data_off"][c0:c1 + 1], wire,
                              w["out_off"][c0:c1 + 1], partial=w["part"][c0:c1], raw=raw[c0:c1])

    run(1)
    torch.cuda.synchronize()
    ref_wire, ref_raw = wire.clone(), raw.clone()
    ks = [int(x) for x in a.ks.split(",")]
    for k in ks:
        wire.zero_()
        raw.zero_()
        run(k)
        torch.cuda.synchronize()
        assert torch.equal(wire, ref_wire) and torch.equal(raw, ref_raw), k
    res = {k: [] for k in ks}
    for _ in range(a.rounds):
        for k in ks:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.iters)]
            for e0, e1 in evs:
                e0.record()
                run(k)
                e1.record()
            torch.cuda.synchronize()
            res[k].append(statistics.median(e0.elapsed_time(e1) for e0, e1 in evs))
    for k in ks:
        ms = statistics.median(res[k])
        print(f"segs={n} K={k} ms={ms:.4f} GB/s={w['alg'] / ms / 1e6:.0f} "
              f"all={','.join(f'{x:.4f}' for x in res[k])}", flush=True)


if __name__ == "__main__":
    main()
