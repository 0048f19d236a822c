#!/usr/bin/env python3
"""f1 build over layouts the bench does not cover: the bench's packed 1480 B payloads
(fast path), the same payloads shifted by 1 or 2 bytes (general path: realigned
loads), and odd 1481 B payloads (images of 1501 B, ragged image ends). Same process,
interleaved rounds, per-launch HIP events; prints ms and wire GB/s per layout.

    python tools/build_variants.py [--segs 1048576] [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import nsx  # noqa: E402


def layout(n, P, lead, g):
    data = torch.empty(lead + n * P + 8, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(data, 0x77)
    rnd = lambda bits, dt: torch.randint(0, 1 << bits, (n,), generator=g, device="cuda", dtype=torch.int64).to(dt)
    fields = {"src_port": rnd(16, torch.int16), "dst_port": rnd(16, torch.int16), "seq_num": rnd(32, torch.int32),
              "ack_num": rnd(32, torch.int32), "offset": torch.full((n,), 5, dtype=torch.uint8, device="cuda"),
              "control": rnd(8, torch.uint8), "window": rnd(16, torch.int16), "urgent_ptr": rnd(16, torch.int16)}
    d_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(P) + np.uint64(lead)
    o_off = nsx.tcp_layout_host(d_off)
    out = torch.empty(int(o_off[-1]), dtype=torch.uint8, device="cuda")
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    do, oo = torch.from_numpy(d_off.view(np.int64)).cuda(), torch.from_numpy(o_off.view(np.int64)).cuda()
    return (lambda: nsx.tcp_build_dev(fields, data, do, out, oo, raw=raw)), n * (P + 20)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kernels", type=lambda v: [int(x) for x in v.split(",")], default=[])
    a = ap.parse_args()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(5)
    n = a.segs
    variants = {"packed_1480": layout(n, 1480, 0, g), "lead1_1480": layout(n, 1480, 1, g),
                "lead2_1480": layout(n, 1480, 2, g), "odd_1481": layout(n, 1481, 0, g)}
    if a.kernels:  # the same layouts under other NSX_PARAM_KERNEL values (e.g. 3: general pipelined path only)
        base = dict(variants)
        for k in a.kernels:
            for name, (fn, wire) in base.items():
                def run(fn=fn, k=k):
                    nsx.set_param(nsx.PARAM_KERNEL, k)
                    fn()
                    nsx.set_param(nsx.PARAM_KERNEL, 0)
                variants[f"{name}/k{k}"] = (run, wire)
    times = {k: [] for k in variants}
    for fn, _ in variants.values():
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, (fn, _) in variants.items():
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.iters)]
            for e0, e1 in evs:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            times[name].append(statistics.median(e0.elapsed_time(e1) for e0, e1 in evs))
    for name, (_, wire) in variants.items():
        ms = statistics.median(times[name])
        print(f"{name:>12} {ms:.4f} ms  wire {wire / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
