#!/usr/bin/env python3
"""Where the CPU baseline's threads leg loses time on the packed-header workloads.

bench.py's leg for workloads 7/9 runs the Go-faithful loop (oracle_go_batch_fixed: malloc + copy + serial loop per
20 B header) over 16 contiguous shards on the box's 16-CPU share; round 6's lines show the shards imbalanced (slowest
3.8x the fastest, the fastest at its 1-thread time). This probe repeats that leg on synthetic bytes and records, per
pass and shard index, the call's duration and the CPU it started and ended on (sched_getcpu), in three forms:
  free     — the threads as bench.py runs them (the scheduler places them anywhere in the affinity set)
  pinned   — each worker pinned to its own CPU (first CPU of each distinct physical core in the affinity set)
  1500     — the free form over 1500 B segments (workload 2's unit) for comparison
    python tools/probes/cpu_shards.py [--threads 16] [--passes 40] [--forms free,pinned,1500]
"""
import argparse
import collections
import ctypes
import os
import statistics
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
from oracle import csum_oracle as O  # noqa: E402  (the checker's C restatement: timed here, as in bench.py)

libc = ctypes.CDLL(None)
libc.sched_getcpu.restype = ctypes.c_int


def distinct_cores(cpus):
    """One logical CPU per physical core (sysfs thread_siblings_list), in affinity order."""
    seen, out = set(), []
    for c in sorted(cpus):
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out


def cpu_times():
    """Per-CPU (busy, total) jiffies from /proc/stat (the whole host's CPUs where the container shows them)."""
    t = {}
    try:
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3].isdigit():
                f = line.split()
                v = list(map(int, f[1:9]))
                t[int(f[0][3:])] = (sum(v) - v[3] - v[4], sum(v))
    except OSError:
        pass
    return t


def cur_freq(c):
    """The CPU's current clock in MHz as cpufreq reports it right after the call (None without cpufreq)."""
    try:
        return int(open(f"/sys/devices/system/cpu/cpu{c}/cpufreq/scaling_cur_freq").read()) / 1e3
    except (OSError, ValueError):
        return None


def package(c):
    try:
        return int(open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id").read())
    except OSError:
        return -1


def numa_pages(addr, nbytes):
    """Pages per NUMA node of the mapping holding addr (/proc/self/numa_maps N<k>=<pages>; numpy's large arrays are
    mappings of their own) and of any further mappings inside [addr, addr + nbytes)."""
    nodes = {}
    try:
        maps = [line.split() for line in open("/proc/self/numa_maps")]
    except OSError:
        return nodes
    starts = sorted(int(f[0], 16) for f in maps)
    holder = max((s for s in starts if s <= addr), default=None)
    for f in maps:
        start = int(f[0], 16)
        if start == holder or addr < start < addr + nbytes:
            for x in f[2:]:
                if x.startswith("N") and "=" in x:
                    k, v = x[1:].split("=")
                    nodes[int(k)] = nodes.get(int(k), 0) + int(v)
    return nodes


def run(form, T, passes, lib):
    unit = 1500 if form == "1500" else 20
    m = (256 << 20) // unit // 64 * 64
    buf = np.random.default_rng(7).integers(0, 256, m * unit, dtype=np.uint8)
    out = np.empty(m, np.uint16)
    bounds = [m * t // T // 64 * 64 for t in range(T)] + [m]
    pin = distinct_cores(os.sched_getaffinity(0))[:T] if form == "pinned" else None

    def shard(t):
        c0 = libc.sched_getcpu()
        t0 = time.perf_counter()
        lo, hi = bounds[t], bounds[t + 1]
        lib.oracle_go_batch_fixed(ctypes.c_void_p(buf.ctypes.data + lo * unit), unit, unit, hi - lo, None, 0,
                                  ctypes.c_void_p(out.ctypes.data + lo * 2))
        t1 = time.perf_counter()
        c1 = libc.sched_getcpu()
        return t, t1 - t0, c0, c1, cur_freq(c1)

    rows = []
    with ThreadPoolExecutor(T) as ex:
        if pin:  # give every worker its own CPU once: one task per thread, each waiting until all have started
            gate = threading.Barrier(T)
            cpus = iter(pin)
            lock = threading.Lock()

            def claim(_):
                with lock:
                    c = next(cpus)
                os.sched_setaffinity(0, {c})  # pid 0 = the calling thread only (Linux)
                gate.wait()
            list(ex.map(claim, range(T)))
        list(ex.map(shard, range(T)))  # warm (first touch of out)
        walls = []
        st0 = cpu_times()
        for _ in range(passes):
            p0 = time.perf_counter()
            rows.append(list(ex.map(shard, range(T))))
            walls.append(time.perf_counter() - p0)
        st1 = cpu_times()
    t1 = time.perf_counter()
    lib.oracle_go_batch_fixed(ctypes.c_void_p(buf.ctypes.data), unit, unit, bounds[1], None, 0,
                              ctypes.c_void_p(out.ctypes.data))
    alone = time.perf_counter() - t1
    ratio = [max(r[1] for r in p) / min(r[1] for r in p) for p in rows]
    by_idx = [statistics.median(p[t][1] for p in rows) * 1e3 for t in range(T)]
    slow_idx = [max(p, key=lambda r: r[1])[0] for p in rows]
    migr = sum(r[2] != r[3] for p in rows for r in p)
    # per pass: how many shards ran > 1.5x the fastest, and whether slow shards' CPUs were shared with another shard
    nslow = [sum(r[1] > 1.5 * min(x[1] for x in p) for r in p) for p in rows]
    shared = 0
    for p in rows:
        cpus = [r[2] for r in p]
        shared += sum(cpus.count(r[2]) > 1 for r in p if r[1] > 1.5 * min(x[1] for x in p))
    print(f"form {form}: {T} threads, {passes} passes over {m} units of {unit} B ({m * unit / 2**20:.0f} MiB)")
    print(f"  pass wall median {statistics.median(walls) * 1e3:.2f} ms; one shard alone {alone * 1e3:.2f} ms; "
          f"max/min per pass median {statistics.median(ratio):.2f} (min {min(ratio):.2f}, max {max(ratio):.2f})")
    print(f"  shards > 1.5x the fastest per pass: median {statistics.median(nslow)}; of those, started on a CPU "
          f"another shard of the pass also started on: {shared} of {sum(nslow)}; calls that changed CPU: {migr}")
    print("  median ms by shard index: " + " ".join(f"{x:.1f}" for x in by_idx))
    print("  slowest shard index per pass: " + " ".join(map(str, slow_idx[:40])))
    print("  CPUs of pass 0: " + " ".join(f"{r[2]}" for r in rows[0]))
    slow_pk = [package(r[2]) for p in rows for r in p if r[1] > 1.5 * min(x[1] for x in p)]
    fast_pk = [package(r[2]) for p in rows for r in p if r[1] <= 1.5 * min(x[1] for x in p)]
    print(f"  socket of the CPU each call started on: slow calls {dict(sorted(collections.Counter(slow_pk).items()))}, "
          f"fast calls {dict(sorted(collections.Counter(fast_pk).items()))}; pages of the input per NUMA node "
          f"{numa_pages(buf.ctypes.data, buf.nbytes)}")
    fq = lambda keep: [r[4] for p in rows for r in p if r[4] is not None and keep(r, p)]  # noqa: E731
    slow_f = fq(lambda r, p: r[1] > 1.5 * min(x[1] for x in p))
    fast_f = fq(lambda r, p: r[1] <= 1.5 * min(x[1] for x in p))
    if slow_f or fast_f:
        print(f"  clock right after the call (cpufreq MHz, median): slow calls "
              f"{statistics.median(slow_f) if slow_f else float('nan'):.0f}, fast calls "
              f"{statistics.median(fast_f) if fast_f else float('nan'):.0f}")
    busy = {c: (st1[c][0] - st0[c][0]) / max(st1[c][1] - st0[c][1], 1) for c in st1 if c in st0}
    if busy:
        # CPUs our slow and fast calls ran on, with how busy each CPU and its SMT sibling were over the form's passes
        # (our own shard included: a CPU running only our shard reads ~busy_fraction of the wall)
        def sib(c):
            try:
                s = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
                return [int(x) for x in s.replace("-", ",").split(",") if x and int(x) != c][:1]
            except OSError:
                return []
        slow_c = [r[2] for p in rows for r in p if r[1] > 1.5 * min(x[1] for x in p)]
        fast_c = [r[2] for p in rows for r in p if r[1] <= 1.5 * min(x[1] for x in p)]
        mean = lambda cs, f: statistics.mean(f(c) for c in cs) if cs else float("nan")  # noqa: E731
        sib_busy = lambda c: statistics.mean(busy.get(s, float("nan")) for s in sib(c)) if sib(c) else float("nan")  # noqa: E731
        print(f"  host: {sum(busy.values()):.1f} of {len(busy)} CPUs busy on average over the passes (ours: ≤{T}); "
              f"CPU busy where slow calls ran {mean(slow_c, lambda c: busy.get(c, 0)):.2f}, sibling "
              f"{mean(slow_c, sib_busy):.2f}; where fast calls ran {mean(fast_c, lambda c: busy.get(c, 0)):.2f}, "
              f"sibling {mean(fast_c, sib_busy):.2f}")
    sys.stdout.flush()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(16, len(os.sched_getaffinity(0))))
    ap.add_argument("--passes", type=int, default=40)
    ap.add_argument("--forms", default="free,pinned,1500")
    a = ap.parse_args()
    lib = O.c_oracle()
    print(f"affinity {len(os.sched_getaffinity(0))} CPUs, distinct cores {len(distinct_cores(os.sched_getaffinity(0)))}")
    for f in a.forms.split(","):
        run(f, a.threads, a.passes, lib)


if __name__ == "__main__":
    main()
