#!/usr/bin/env python3
"""A/B of NSX_PARAM_WINDOW_BYTES on the fixed-stride path: the same batch checksummed in
one launch and as back-to-back windows of several sizes, interleaved rounds in one process,
results compared with the one-launch output.

    python tools/window_ab.py [--segs 16777216] [--rounds 5] [--windows 768,1536,3072]
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


def time_on(buf, n, out, iters):
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--windows", default="384,768,1536,3072", help="window sizes in MB (1e6 B)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.segs
    buf = torch.empty(N * L, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(buf, 0x1071)
    ref = torch.empty(N, dtype=torch.int16, device="cuda")
    out = torch.empty(N, dtype=torch.int16, device="cuda")
    nsx.set_param(nsx.PARAM_WINDOW_BYTES, -1)
    nsx.fixed_dev(buf, L, L, N, out=ref)
    torch.cuda.synchronize()
    cases = [("one", -1), ("auto", 0)] + [(f"w{w}MB", int(w) * 1000000) for w in a.windows.split(",")]
    for name, w in cases:
        nsx.set_param(nsx.PARAM_WINDOW_BYTES, w)
        out.zero_()
        nsx.fixed_dev(buf, L, L, N, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), name
    res = {c[0]: [] for c in cases}
    for _ in range(a.rounds):
        for name, w in cases:
            nsx.set_param(nsx.PARAM_WINDOW_BYTES, w)
            res[name].append(time_on(buf, N, out, a.iters))
    nsx.set_param(nsx.PARAM_WINDOW_BYTES, 0)
    for name, _ in cases:
        ms = statistics.median(res[name])
        print(f"segs={N} {name:>8} ms={ms:.4f} GB/s={(N * (L + 2)) / ms / 1e6:.0f} "
              f"all={','.join(f'{x:.4f}' for x in res[name])}", flush=True)


if __name__ == "__main__":
    main()
