#!/usr/bin/env python3
"""Does the ragged kernel gain from back-to-back windows as the fixed path does (DESIGN.md §7
step 21)? Config 3's batch checksummed in one nsx_csum_ragged_dev call and as K calls over
equal segment-count slices of the offsets, interleaved rounds, results compared.

    python tools/ragged_window_ab.py [--segs 1048576] [--ks 1,2,3,4,6] [--rounds 5]
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
    ap.add_argument("--ks", default="1,2,3,4,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    cfg = dict(bench.WORKLOADS[3], n=a.segs)
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    buf, out, n = w["buf"], w["out"], a.segs
    d_offs = torch.from_numpy(w["offsets"].view("int64")).cuda()
    ref = nsx.ragged_dev(buf, d_offs).clone()

    def run(k):
        cuts = [n * i // k for i in range(k + 1)]
        for c0, c1 in zip(cuts, cuts[1:]):
            nsx.ragged_dev(buf, d_offs[c0:c1 + 1], out=out[c0:c1])

    ks = [int(x) for x in a.ks.split(",")]
    for k in ks:
        out.zero_()
        run(k)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), k
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
        print(f"segs={n} bytes={w['bytes']} K={k} ms={ms:.4f} GB/s={w['alg'] / ms / 1e6:.0f} "
              f"all={','.join(f'{x:.4f}' for x in res[k])}", flush=True)


if __name__ == "__main__":
    main()
