#!/usr/bin/env python3
"""Kernel-variant sweep: interleaved rounds in ONE process (cdna_hip_programming.md
§5.4 rule 24), per-launch HIP-event time on the launch stream, median per variant.

    python tools/sweep.py [--configs 2,3,4] [--rounds 5] [--iters 20]
"""
import argparse
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import nsx  # noqa: E402


def variants(kind):
    out = []
    if kind == "fixed_big":  # config 5: the default buffer kernel's neighbourhood only
        for bpc, spw, xcd in itertools.product((1, 2, 4), (2, 4), (1, 2, 3)):
            out.append(dict(kernel=3, blocks_per_cu=bpc, segs_per_wave=spw, nontemporal=1, xcd_map=xcd))
        return out
    for bpc, rows, nt, xcd in itertools.product((8, 4, 2), (4, 8, 16), (1,), (1, 3)):
        out.append(dict(kernel=1, blocks_per_cu=bpc, stream_rows=rows, nontemporal=nt, xcd_map=xcd))
    for bpc, spw, nt in itertools.product((8, 4, 2), (1, 2, 4), (1,)):
        if kind != "fixed2" and spw != 1:
            continue
        for xcd in (1, 3):
            out.append(dict(kernel=2, blocks_per_cu=bpc, segs_per_wave=spw, nontemporal=nt, xcd_map=xcd))
    if kind == "ragged":
        for bpc, rows, run in itertools.product((8, 4, 2), (4, 8, 16), (4, 8, 16, 32, 63)):
            out.append(dict(kernel=4, blocks_per_cu=bpc, stream_rows=rows, nontemporal=1, xcd_map=1, run_segs=run))
        for bpc, rows in itertools.product((8, 4), (8, 16)):
            out.append(dict(kernel=3, blocks_per_cu=bpc, stream_rows=rows, nontemporal=1, xcd_map=1))
    if kind == "ragged_ab":  # the default scan kernel against its software-pipelined form
        return ([dict(kernel=4, blocks_per_cu=2, stream_rows=8, nontemporal=1, xcd_map=4, run_segs=63)] +
                [dict(kernel=6, blocks_per_cu=b, stream_rows=r, nontemporal=1, xcd_map=4, run_segs=63)
                 for b in (1, 2, 4) for r in (4, 8)])
    if kind == "ipv4_hdr":  # 0 auto (flat for packed 20 B), 1 per-thread, 2 LDS-dense
        return ([dict(kernel=0, blocks_per_cu=b, segs_per_wave=u) for b in (1, 2, 3, 4) for u in (1, 2, 4)] +
                [dict(kernel=2, blocks_per_cu=8)])
    if kind == "tcp_build":  # cache policy (nontemporal knob) x grid
        return ([dict(blocks_per_cu=b, segs_per_wave=ps) for b in (1, 2, 4) for ps in (1, 2)] +
                [dict(blocks_per_cu=b, kernel=2) for b in (4, 8)])
    if kind == "swp_big":  # config 5: the default software-pipelined kernel at more blocks / other depths
        return [dict(kernel=5, blocks_per_cu=b, segs_per_wave=u, nontemporal=1) for b in (1, 2, 3) for u in (4, 8)] + \
               [dict(kernel=5, blocks_per_cu=1, segs_per_wave=8, nontemporal=1, xcd_chunk=c) for c in (8, 12, 16)] + \
               [dict(kernel=5, blocks_per_cu=1, segs_per_wave=8, nontemporal=0)]
    if kind == "ragged_deep":  # deeper in-flight windows: 16-row batches, pipelined, 1-2 blocks/CU
        return ([dict(kernel=4, blocks_per_cu=2, stream_rows=8, nontemporal=1, xcd_map=4, run_segs=63)] +
                [dict(kernel=k, blocks_per_cu=b, stream_rows=r, nontemporal=1, xcd_map=4, run_segs=63)
                 for k in (4, 6) for b in (1, 2, 3) for r in (8, 16)])
    if kind == "ragged_bal":  # scan kernel: XCD deal vs byte-balanced wave ranges
        for bpc, rows, run, xcd in itertools.product((1, 2, 4, 8), (4, 8, 16), (8, 16, 32, 63), (1, 4)):
            out.append(dict(kernel=4, blocks_per_cu=bpc, stream_rows=rows, nontemporal=1, xcd_map=xcd, run_segs=run))
        return out
    if kind == "fixed2":
        for bpc, spw, xcd in itertools.product((8, 4, 2, 1), (1, 2, 4, 8), (1, 3)):
            out.append(dict(kernel=3, blocks_per_cu=bpc, segs_per_wave=spw, nontemporal=1, xcd_map=xcd))
    return out


def apply(v):
    for p in nsx.ALL_PARAMS:
        nsx.set_param(p, 0)
    for k, val in v.items():
        nsx.set_param(bench.PARAMS[k], val)


def time_variant(w, iters):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for i in range(iters):
        evs[i][0].record()
        w["step"]()
        evs[i][1].record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in evs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kind", default="", help="variant family override (e.g. ragged_bal)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.json"))
    a = ap.parse_args()
    torch.cuda.set_device(0)
    results = {}
    for cid in [int(c) for c in a.configs.split(",")]:
        cfg = bench.WORKLOADS[cid]
        w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
        kind = "fixed2" if cfg["kind"] == "fixed" and cfg["seg_len"] <= 4093 else cfg["kind"]
        if cid == 5:
            kind = "fixed_big"
        vs = variants(a.kind or kind)
        if cid in (3, 4):
            vs += [dict(v, block_mode=2) for v in vs if v["kernel"] == 2 and v["blocks_per_cu"] == 8]
        times = {i: [] for i in range(len(vs))}
        for i, v in enumerate(vs):  # warm each once
            apply(v)
            time_variant(w, 3)
        for r in range(a.rounds):
            for i, v in enumerate(vs):
                apply(v)
                times[i].append(time_variant(w, a.iters))
            print(f"config{cid} round {r} done", flush=True)
        rows = []
        for i, v in enumerate(vs):
            med = statistics.median(times[i])
            rows.append(dict(v, ms=round(med, 4), GBps=round(w["alg"] / med / 1e6, 1),
                             frac=round(w["alg"] / med / 1e6 / 8000, 4), ms_min=round(min(times[i]), 4)))
            for p in nsx.ALL_PARAMS:
                nsx.set_param(p, 0)
        rows.sort(key=lambda r: r["ms"])
        results[f"config{cid}"] = rows
        for r in rows[:8]:
            print(f"config{cid}", json.dumps(r), flush=True)
        print(f"config{cid} worst", json.dumps(rows[-1]), flush=True)
        del w
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
