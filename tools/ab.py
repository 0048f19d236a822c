#!/usr/bin/env python3
"""Same-process A/B of launch overrides (variants named x_* are diagnostics: no parity check) (include/nsx_tune.h) on one bench workload.

    python tools/ab.py --config 6 --variants "def:;b3:blocks_per_cu=3;b8:blocks_per_cu=8" [--rounds 7]

For the receive-pass configs, a variant named scan* runs the plain ragged
checksum (nsx_csum_ragged_dev) over the same frames instead: the receive pass's
own cost against the one-pass checksum it is built on; raw* runs the receive pass
also writing its 2 B TCP raw sums (the ragged checksum's output volume). For the ragged
configs, verify* runs the batch verify (nsx_verify_ragged_dev: 1 B ok per segment) over the same segments.

Builds the workload once (bench.build_workload), settles the clocks, then runs
the variants in interleaved rounds (each round: every variant, `--launches`
back-to-back launches bracketed by HIP events on the launch stream) and prints
the median per-launch time and roofline fraction per variant. Box-to-box and
allocation effects cancel because every variant sees the same buffers in the
same process.
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
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variants", required=True, help="name:field=v,field=v;name2:...")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--n", type=int, default=0, help="override the workload's unit count")
    ap.add_argument("--set", action="append", default=[], help="override a workload field, key=int")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    cfg = dict(bench.WORKLOADS[a.config])
    if a.n:
        cfg["n"] = a.n
    for kv in a.set:
        k, _, v = kv.partition("=")
        cfg[k] = float(v) if "." in v else int(v)
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    variants = []
    for item in a.variants.split(";"):
        name, _, kv = item.partition(":")
        tune = bench.parse_tune([x for x in kv.split(",") if x]) or None
        step = w["step_for"](tune)
        if cfg["kind"] == "rx" and name.startswith("raw"):  # the receive pass also writing its 2 B TCP raw sums
            import nsx
            rxf = nsx.rx_ipv6_tcp_verify_dev if cfg.get("ipver") == 6 else nsx.rx_ipv4_tcp_verify_dev
            traw = torch.empty(cfg["n"], dtype=torch.int16, device="cuda")
            step = (lambda t: lambda: rxf(w["buf"], w["d_offs"], mask=w["out"], tcp_raw=traw, tune=t))(tune)
        if cfg["kind"] == "ragged" and name.startswith("verify"):  # the batch verify (1 B ok per segment, no raw)
            import nsx
            vpart = w.get("partial")
            step = (lambda t: lambda: nsx.verify_ragged_dev(w["buf"], w["d_offs"], partial=vpart, tune=t))(tune)
        if cfg["kind"] == "rx" and name.startswith("scan"):
            import nsx
            rout = torch.empty(cfg["n"], dtype=torch.int16, device="cuda")
            step = (lambda t: lambda: nsx.ragged_dev(w["buf"], w["d_offs"], out=rout, tune=t))(tune)
        variants.append((name, step, __import__("nsx").fixed_launch_count(
            cfg["stride"], cfg["seg_len"], cfg["n"], tune) if cfg["kind"] == "fixed" else 1))
    # every variant must give the first one's results on this batch (they differ only in launch shape or code path)
    ref = None
    for name, step, _ in variants:
        if (cfg["kind"] == "rx" and name.startswith("scan")) or name.startswith("x_") or \
                (cfg["kind"] == "ragged" and name.startswith("verify")):
            continue  # another computation / a diagnostic variant whose results are wrong on purpose
        w["out"].zero_()
        step()
        torch.cuda.synchronize()
        got = w["out"].clone()
        if ref is None:
            ref = got
        same = bool(torch.equal(got, ref))
        print(f"parity {name}: {'same as first' if same else 'MISMATCH'}", flush=True)
        if not same:
            raise SystemExit(f"variant {name} differs from the first variant")
    for name, step, _ in variants:  # one synchronised launch each first, so a hang names its variant
        step()
        torch.cuda.synchronize()
        print(f"ran {name}", flush=True)
    t_end = time.perf_counter() + 1.0
    while time.perf_counter() < t_end:  # settle
        for _, step, _ in variants:
            step()
        torch.cuda.synchronize()
    res = {name: [] for name, _, _ in variants}
    for r in range(a.rounds):
        for name, step, launches in variants:
            for _ in range(3):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.launches):
                step()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.launches / launches)
        print(f"round {r}: " + " ".join(f"{k} {v[-1]:.5f}" for k, v in res.items()), flush=True)
    base = None
    for name, _, launches in variants:
        med = statistics.median(res[name])
        frac = w["alg"] / launches / (med * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS
        base = base or med
        print(f"AB config{a.config}{f' n={a.n}' if a.n else ''}{''.join(' ' + x for x in a.set)} {name:16s} median {med:.5f} ms/launch  frac {frac:.4f}  vs first {med / base:.4f}  "
              f"min {min(res[name]):.5f} max {max(res[name]):.5f}", flush=True)


if __name__ == "__main__":
    main()
