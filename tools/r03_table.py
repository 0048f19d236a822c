#!/usr/bin/env python3
"""Round-3 results table from the evidence pass's bench lines (gpurun_out/r03ev/bench_c<N>.log → markdown rows),
and the saved copies profiles/r03_bench_config<N>.json. usage: tools/r03_table.py [--save]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {2: "2: 1M × 1500 B (headline)", 3: "3: 1M ragged 64-9000 B", 4: "4: 256K × 64 KiB",
         5: "5: 16M × 1500 B per GPU (23.4 GiB)", 6: "6 (f1): 1M TCP builds, 1480 B payloads",
         7: "7 (f3): 64M packed 20 B IPv4 headers", 8: "8 (f1): 1M builds, 12 B options",
         9: "9 (f3+f2): 64M headers into a bitmask", 10: "10 (rx): 1M IPv4 datagrams, 40-1500 B",
         11: "11 (rx6): 1M IPv6 packets, 60-1500 B", 12: "12 (f1): 256K jumbo builds, 8960 B images",
         13: "13 (rx): 8M IPv4 datagrams, 40-100 B", 14: "14 (rx): 2M frames, half ACK / half 1500 B",
         15: "15: 8M ragged 64-128 B", 16: "16 (rx6): 8M IPv6 packets, 60-120 B",
         17: "17 (rx): 8M frames, 95% ACK / 5% 1500 B"}


def line(c):
    p = os.path.join(ROOT, "gpurun_out", "r03ev", f"bench_c{c}.log")
    if not os.path.exists(p):
        return None
    js = [l for l in open(p) if l.startswith("{")]
    return json.loads(js[-1]) if js else None


def main(save):
    print("| workload | whole-job | kernel mean per launch | kernel rate | roofline frac | HBM traffic / alg | "
          "CPU, 16 threads | CPU, 1 thread |")
    print("|---|---|---|---|---|---|---|---|")
    for c in sorted(NAMES):
        d = line(c)
        if d is None:
            continue
        if save:
            json.dump(d, open(os.path.join(ROOT, "profiles", f"r03_bench_config{c}.json"), "w"), indent=1)
        r = d["roofline"]
        lps = r.get("launches_per_step", 1)
        km = d.get("kernel_ms_mean")
        kms = f"{km:.4f} ms" + (f" (× {lps} per step)" if lps > 1 else "") if km else "—"
        tr = f"{r['traffic'] / r['alg_bytes_per_launch']:.3f}" if r.get("traffic") else "—"
        cb = d.get("cpu_baseline") or {}
        cpu = f"{cb['value']:.1f} {cb['unit']}" if cb.get("value") else "—"
        st = cb.get("single_thread") or {}
        cpu1 = f"{st['value']:.2f} {st['unit']}" if st.get("value") else "—"
        print(f"| {NAMES[c]} | {d['value']:.0f} {d['unit']} | {kms} | {r['achieved'] / 1000:.2f} TB/s | "
              f"**{r['frac']:.3f}** | {tr} | {cpu} | {cpu1} |")


def traffic():
    """DESIGN §5 traffic rows: PMC HBM bytes per launch (profiles/traffic_config<N>.json) against the bench line's
    algorithmic bytes, and the profile's mean kernel duration against the bench's HIP-event mean."""
    import re
    print("| workload | HBM bytes per launch | algorithmic | traffic / alg | rocprofv3 mean | bench event mean |")
    print("|---|---|---|---|---|---|")
    for c in sorted(NAMES):
        d = line(c)
        tp = os.path.join(ROOT, "profiles", f"traffic_config{c}.json")
        md = os.path.join(ROOT, "profiles", f"r03_config{c}.md")
        if d is None or not os.path.exists(tp) or not os.path.exists(md):
            continue
        t = json.load(open(tp))
        alg = d["roofline"]["alg_bytes_per_launch"]
        m = re.search(r"per-launch durations \(µs, trace order\): median [0-9.]+, mean ([0-9.]+)", open(md).read())
        print(f"| {c} | {t['bytes_per_launch'] / 1e9:.4f} GB | {alg / 1e9:.4f} GB | {t['bytes_per_launch'] / alg:.4f} | "
              f"{m.group(1) if m else '—'} µs | {d['kernel_ms_mean'] * 1000:.1f} µs |")


if __name__ == "__main__":
    if "--traffic" in sys.argv:
        traffic()
    else:
        main("--save" in sys.argv)
