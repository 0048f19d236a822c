#!/usr/bin/env python3
"""Tabulate tools/valu_ab.sh: per-launch SQ counters of one workload's kernel under each library build.

    python tools/valu_ab.py 13 r04 new > profiles/r05_config13_valu.md
"""
import collections
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(cfg, k):
    src = os.path.join(ROOT, "gpurun_out", f"prof_valu_{k}_c{cfg}")
    # the workload's kernel: the library kernel launched most (setup launches — the bench fills and fixes its
    # frames with other library kernels — run once or a few times)
    trace = [r for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))) if "nsx::" in r["Kernel_Name"]]
    kname = collections.Counter(r["Kernel_Name"] for r in trace).most_common(1)[0][0]
    dur = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                            for r in trace if r["Kernel_Name"] == kname)
    c = collections.defaultdict(list)
    for grp in ("sq", "sq2"):
        for r in csv.DictReader(open(os.path.join(src, grp, "run_counter_collection.csv"))):
            if r["Kernel_Name"] == kname:
                c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return kname, dur, {n: statistics.median(v) for n, v in c.items()}


def main(cfg, *libs):
    rows = {k: per_launch(cfg, k) for k in libs}
    names = sorted(set().union(*(r[2] for r in rows.values())))
    print(f"| counter (median per launch), workload {cfg} | " + " | ".join(libs) + " | last/first |")
    print("|---|" + "---|" * (len(libs) + 1))
    print("| kernel µs (kernel trace, median) | " + " | ".join(f"{rows[k][1]:.1f}" for k in libs) +
          f" | {rows[libs[-1]][1] / rows[libs[0]][1]:.3f} |")
    for n in names:
        v = [rows[k][2].get(n, float('nan')) for k in libs]
        print(f"| {n} | " + " | ".join(f"{x:.4g}" for x in v) + f" | {v[-1] / v[0]:.3f} |" if v[0] else
              f"| {n} | " + " | ".join(f"{x:.4g}" for x in v) + " | - |")
    print()
    print("kernel: " + "; ".join(f"{k}: `{rows[k][0][:100]}`" for k in libs))


if __name__ == "__main__":
    main(int(sys.argv[1]), *sys.argv[2:])
