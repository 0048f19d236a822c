#!/usr/bin/env python3
"""Markdown results table from a round's committed bench lines (profiles/<tag>_bench_config<W>.json).

    python tools/results_table.py r04 > /tmp/table.md

One row per workload: whole-job rate, kernel mean per launch, kernel rate and roofline fraction, HBM traffic over
the algorithmic bytes (this round's profiles/traffic_config<W>.json if there is one, else the line's
`roofline.traffic`), and the CPU
baseline (the Go-faithful loop on the box's CPU share and on one thread)."""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LABELS = {
    "2": "2: 1M × 1500 B, IPv4 pseudo-header partials (headline)", "2n": "2: the same without partials",
    "3": "3: 1M ragged 64-9000 B", "4": "4: 256K × 64 KiB", "5": "5: 16M × 1500 B per GPU (23.4 GiB), partials",
    "6": "6 (f1): 1M TCP builds, 1480 B payloads", "7": "7 (f3): 64M packed 20 B IPv4 headers",
    "8": "8 (f1): 1M builds, 12 B options", "9": "9 (f3+f2): 64M headers into a bitmask",
    "10": "10 (rx): 1M IPv4 datagrams, 40-1500 B", "11": "11 (rx6): 1M IPv6 packets, 60-1500 B",
    "12": "12 (f1): 256K jumbo builds, 8960 B images", "13": "13 (rx): 8M IPv4 datagrams, 40-100 B",
    "14": "14 (rx): 2M frames, half ACK / half 1500 B", "15": "15: 8M ragged 64-128 B",
    "16": "16 (rx6): 8M IPv6 packets, 60-120 B", "17": "17 (rx): 8M frames, 95% ACK / 5% 1500 B",
    "18": "18 (rx): 8M IPv4 datagrams, 40-400 B",
}


def order(path):
    m = re.search(r"config(\d+)(n?)\.json$", path)
    return (int(m.group(1)), m.group(2)) if m else (999, "")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    files = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", f"{tag}_bench_config*.json"))
                    if order(f)[0] != 999), key=order)  # config<W>[n].json only (not e.g. *_unpinned.json)
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
        tf = os.path.join(ROOT, "profiles", f"traffic_config{w}{suffix}.json")
        if os.path.exists(tf) and json.load(open(tf)).get("profile", "").startswith(f"profiles/{tag}_"):
            tr = json.load(open(tf))["bytes_per_launch"]  # this round's PMC pass, taken after the bench line
        ratio = f"{tr / rf['alg_bytes_per_launch']:.3f}" if tr else "—"
        cb = d.get("cpu_baseline") or {}
        cpu = f"{cb['value']:.1f} GiB/s" if cb.get("value") else "—"
        st = (cb.get("single_thread") or {}).get("value")
        cpu1 = f"{st:.2f} GiB/s" if st else "—"
        label = LABELS.get(f"{w}{suffix}", d["config"]["workload"].split(",")[0])
        print(f"| {label} | {d['value']:.0f} GiB/s | {kern} | {rf['achieved'] / 1000:.2f} TB/s | **{rf['frac']:.3f}** "
              f"| {ratio} | {cpu} | {cpu1} |")


if __name__ == "__main__":
    main()
