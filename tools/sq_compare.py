#!/usr/bin/env python3
"""Side-by-side SQ counters of two or more bench workloads' receive kernel (tools/profile.sh groups kt, sq, sq2, lds
under one tag), per launch, per frame and per KiB of frames — VERDICT r5 item 5: where does workload 17 (95% ACKs,
5% 1500 B) lose against workload 13 (40-100 B)?

    python tools/sq_compare.py r06sq 13 17 > profiles/r06_sq_13_17.md
"""
import collections
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "network-stack_amd")]


def per_launch(tag, cfg):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_c{cfg}")
    trace = [r for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))) if "nsx::" in r["Kernel_Name"]]
    kname = collections.Counter(r["Kernel_Name"] for r in trace).most_common(1)[0][0]
    dur = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                            for r in trace if r["Kernel_Name"] == kname)
    c = collections.defaultdict(list)
    for grp in ("sq", "sq2", "lds"):
        path = os.path.join(src, grp, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if r["Kernel_Name"] == kname:
                c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return kname, dur, {n: statistics.median(v) for n, v in c.items()}


def main(tag, *cfgs):
    import bench
    rows = {c: per_launch(tag, c) for c in cfgs}
    frames = {c: bench.WORKLOADS[int(c)]["n"] for c in cfgs}
    kib = {}
    for c in cfgs:  # the workload's frame bytes per launch, from its alg-bytes rule: bytes = alg − 8n − n/8
        w = dict(bench.WORKLOADS[int(c)])
        kib[c] = w.get("mean_bytes", 0)
    names = sorted(set().union(*(r[2] for r in rows.values())))
    print(f"kernel: {rows[cfgs[0]][0]}\n")
    print("| counter | " + " | ".join(f"{c}: per launch | {c}: per frame" for c in cfgs) + " |")
    print("|---|" + "---|---|" * len(cfgs))
    print("| kernel µs (median) | " + " | ".join(f"{rows[c][1]:.1f} | {rows[c][1] * 1e3 / frames[c]:.4f} ns"
                                             for c in cfgs) + " |")
    for n in names:
        cells = []
        for c in cfgs:
            v = rows[c][2].get(n, float("nan"))
            cells.append(f"{v:.4g} | {v / frames[c]:.4g}")
        print(f"| {n} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main(*sys.argv[1:])
