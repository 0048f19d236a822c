#!/usr/bin/env python3
"""Markdown results table from a round's committed bench lines (profiles/<tag>_bench_config<W>.json).

    python tools/results_table.py r04 > /tmp/table.md

One row per workload: whole-job rate, kernel mean per launch, kernel rate and roofline fraction, HBM traffic over
the algorithmic bytes (from the line's `roofline.traffic`, i.e. the committed traffic_config<W>.json), and the CPU
baseline (the Go-faithful loop on the box's CPU share and on one thread)."""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def order(path):
    m = re.search(r"config(\d+)(n?)\.json$", path)
    return (int(m.group(1)), m.group(2)) if m else (999, "")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"{tag}_bench_config*.json")), key=order)
    print("| workload | whole-job | kernel mean per launch | kernel rate | roofline frac | HBM traffic / alg "
          "| CPU, all threads | CPU, 1 thread |")
    print("|---|---|---|---|---|---|---|---|")
    for f in files:
        d = json.load(open(f))
        w, suffix = order(f)
        rf = d["roofline"]
        lps = rf.get("launches_per_step", 1)
        kern = f"{d['kernel_ms_mean']:.4f} ms" + (f" (× {lps} per step)" if lps and lps > 1 else "")
        tr = rf.get("traffic")
        ratio = f"{tr / rf['alg_bytes_per_launch']:.3f}" if tr else "—"
        cb = d.get("cpu_baseline") or {}
        cpu = f"{cb['value']:.1f} GiB/s" if cb.get("value") else "—"
        st = (cb.get("single_thread") or {}).get("value")
        cpu1 = f"{st:.2f} GiB/s" if st else "—"
        name = d["config"]["workload"].split(":")[0]
        label = f"{w}{' (no partials)' if suffix else ''}: {d['config']['workload'].split(':', 1)[1].split(',')[0].strip()}" \
            if ":" in d["config"]["workload"] else name
        print(f"| {label} | {d['value']:.0f} GiB/s | {kern} | {rf['achieved'] / 1000:.2f} TB/s | **{rf['frac']:.3f}** "
              f"| {ratio} | {cpu} | {cpu1} |")


if __name__ == "__main__":
    main()
