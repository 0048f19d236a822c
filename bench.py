#!/usr/bin/env python3
"""bench.py — device-resident Internet checksum throughput (BASELINE.json metric).

One "step" = one pass of the hot path (nsx_csum_fixed_dev → gfx950 kernel) over
one device-resident batch. Default workload = BASELINE.json configs[1]
(config 2): 1,048,576 × 1500 B fixed-stride TCP segments per GPU, splitmix64
bytes (seed 0x1071 + rank) generated on the device. N GPUs = N ranks, one per
GPU (torchrun), each checksumming its own batch: the path shards with no
exchange, so there is no data-path collective and scaling is
weak. value = Σ bytes over all ranks ÷ max over ranks of the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2-18] [--no-pseudo]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N rank
processes itself (a torch.distributed.run child, rendezvous at 127.0.0.1) before
anything touches a GPU, and relays rank 0's line; under a launcher that already
set WORLD_SIZE, a WORLD_SIZE that differs from --gpus is an error (exit 2), as is
more RCCL ranks than visible GPUs. Each rank makes its GPU (LOCAL_RANK) current
before the process group is created; the ranks then exchange their devices' PCI
address and UUID, every line carries `ranks`, `distinct_devices` and the device
list with n_gpus = distinct devices, and RCCL ranks that landed on fewer distinct
GPUs than ranks exit 3 instead of printing a line.

Configs 2-5 are BASELINE.json's device-resident configurations (2 is the
headline and the default). Configs 2 and 5 checksum every segment over its own
IPv4 pseudo-header, given as the N x u32 partials SURVEY.md §8d specifies
(tcp.go:72-73's ipPseudoHeader prefix; generated on the device by
nsx_pseudo_ipv4_partial_dev from random addresses, proto 6, length 1500) and
counted in the algorithmic bytes (+4 B per segment); --no-pseudo measures the
same batch without them. Configs 6 and 7 measure SURVEY.md §8's next rows to
the same bar, each with its own metric string: 6 = the fused sender pass
(nsx_tcp_build_dev: segment.bytes() + computeChecksum + field write,
tcp.go:98-128/:68-71) over 1M 1500 B wire images; 7 = IPv4 header checksum
verify (nsx_ipv4_hdr_csum_dev) over 64M packed 20 B headers; 8 = config 6 with a
12 B option block per segment (the build kernel's option path); 9 =
workload 7 verified straight into a validity bitmask (nsx_ipv4_hdr_verify_mask_dev);
10 / 11 = the fused receive pass over 1M IPv4 datagrams / IPv6 packets
(nsx_rx_ipv4_tcp_verify_dev / nsx_rx_ipv6_tcp_verify_dev); 12 = config 6 with
9000 B MTU segments; 13 / 16 = the receive pass over 8M ACK-sized (40-100 B IPv4 /
60-120 B IPv6) frames; 14 = over a bimodal mix of ACKs and 1500 B data frames;
15 = config 3's small-segment twin (8M ragged 64-128 B segments); 17 / 18 = the
receive pass over 8M frames, 95% ACKs and 5% 1500 B / 40-400 B.

Printed by rank 0: one JSON line with the contract fields plus
  roofline     — dominant kernel: algorithmic bytes per launch ÷ its mean
                 duration (one HIP event pair on the launch stream around
                 the K timed steps, per launch) vs 8 TB/s HBM;
                 traffic = PMC-measured HBM bytes per launch from the committed
                 rocprofv3 summary (profiles/), or null;
  cpu_baseline — the Go-faithful CPU restatement (oracle) timed on a bounded
                 sample of the same workload (rank 0, N=1 only) on every host
                 core this process may use (`cores`), with the 1-thread rate
                 beside it;
  per_gpu      — every rank's own rate (BASELINE config 5: "per-GPU and
                 aggregate GiB/s"): its device, its bytes ÷ its own timed wall,
                 its kernel mean and roofline fraction, so a slow GPU shows in
                 the line itself; value_per_gpu_mean = value / ranks.

The product library is brought up to date (`make -C network-stack_amd`, a no-op
when nothing changed, under a file lock) before it is loaded — by the launching
process, or by each rank an outside launcher started — so a stale pushed binary
never runs.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

METRIC = "GiB/s device-resident Internet checksum, 1M×1500B segments, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md §Chip-level parameters
GIB = float(1 << 30)

# Workloads (BASELINE.json configs; per GPU). "kind" picks the entry point.
WORKLOADS = {
    2: dict(kind="fixed", n=1 << 20, seg_len=1500, stride=1500, seed=0x1071, pseudo=True,
            name="config2: 1M x 1500B fixed-stride TCP segments per GPU, each over its IPv4 pseudo-header "
                 "(N x u32 partials), device-resident"),
    3: dict(kind="ragged", n=1 << 20, lo=64, hi=9000, seed=0x1072,
            name="config3: 1M ragged 64-9000B segments per GPU, densely packed (odd starts), device-resident"),
    4: dict(kind="fixed", n=1 << 18, seg_len=65536, stride=65536, seed=0x1073,
            name="config4: 256K x 64KiB TSO-size segments per GPU, device-resident"),
    5: dict(kind="fixed", n=1 << 24, seg_len=1500, stride=1500, seed=0x1071, pseudo=True,
            name="config5: 16M x 1500B per GPU (128M x 1500B over 8 GPUs), each over its IPv4 pseudo-header "
                 "(N x u32 partials), device-resident"),
    # SURVEY.md §8(f) rows measured to the same bar (not the headline metric):
    6: dict(kind="tcp_build", n=1 << 20, payload=1480, seed=0x1074,
            metric="GiB/s fused TCP segment build (serialize + checksum + field write), wire bytes",
            name="f1: 1M option-less TCP segments per GPU, 1480B payload -> 1500B wire images, IPv4 pseudo-header "
                 "partials, device-resident"),
    # not a BASELINE config: f1 with a 12-byte option block per segment (the size of Linux's NOP NOP timestamps
    # block)
    8: dict(kind="tcp_build", n=1 << 20, payload=1468, opt=12, seed=0x1076,
            metric="GiB/s fused TCP segment build (serialize + checksum + field write), wire bytes",
            name="f1+options: 1M TCP segments per GPU, 12B options (NOP NOP kind-2 len 10), 1468B payload -> 1500B wire images, "
                 "IPv4 pseudo-header partials, device-resident"),
    # not a BASELINE config: f1 with jumbo-frame segments (9000 B MTU: 8960 B TCP segments), images of 9 rows
    12: dict(kind="tcp_build", n=1 << 18, payload=8940, seed=0x107B,
             metric="GiB/s fused TCP segment build (serialize + checksum + field write), wire bytes",
             name="f1 jumbo: 256K option-less TCP segments per GPU, 8940B payload -> 8960B wire images (9000B MTU), "
                  "IPv4 pseudo-header partials, device-resident"),
    # not a BASELINE config: f3's receive side fused with f2's bitmask (1 bit written per header)
    9: dict(kind="ipv4_hdr", mask=True, n=1 << 26, hdr=20, seed=0x1077,
            metric="GiB/s IPv4 header checksum verify into a bitmask, header bytes",
            name="f3+f2: 64M packed 20B IPv4 headers per GPU (header-split ring), verify into a validity bitmask, "
                 "device-resident"),
    7: dict(kind="ipv4_hdr", n=1 << 26, hdr=20, seed=0x1075,
            metric="GiB/s IPv4 header checksum verify, header bytes",
            name="f3: 64M packed 20B IPv4 headers per GPU (header-split ring), verify, device-resident"),
    # not a BASELINE config: the receive side of f2 + f3 fused into one pass over received datagrams
    10: dict(kind="rx", n=1 << 20, lo=40, hi=1500, seed=0x1079,
             metric="GiB/s fused receive verify (IPv4 header + pseudo-header + TCP checksum into a bitmask), frame bytes",
             name="f2+f3 rx: 1M IPv4/TCP datagrams per GPU, 40-1500B (uniform), densely packed (odd starts), "
                  "1 in 1000 corrupted, verified into a validity bitmask, device-resident"),
    # not a BASELINE config: the same receive pass over IPv6 packets (RFC 8200 pseudo-header, no header checksum)
    11: dict(kind="rx", ipver=6, n=1 << 20, lo=60, hi=1500, seed=0x107A,
             metric="GiB/s fused receive verify (IPv6 pseudo-header + TCP checksum into a bitmask), packet bytes",
             name="f2 rx6: 1M IPv6/TCP packets per GPU, 60-1500B (uniform), densely packed (odd starts), "
                  "1 in 1000 corrupted, verified into a validity bitmask, device-resident"),
    # not BASELINE configs: the receiver's common case, ACK-sized frames (a TCP receiver's 40-66 B ACKs;
    # tcp.go:70 receiver rule, tcp.go:56,131 minSegmentLength 20 B): small-frame twins of workloads 10, 11 and 3
    13: dict(kind="rx", n=1 << 23, lo=40, hi=100, seed=0x107C,
             metric="GiB/s fused receive verify (IPv4 header + pseudo-header + TCP checksum into a bitmask), frame bytes",
             name="f2+f3 rx small: 8M IPv4/TCP datagrams per GPU, 40-100B (uniform, ACK-sized), densely packed "
                  "(odd starts), 1 in 1000 corrupted, verified into a validity bitmask, device-resident"),
    14: dict(kind="rx", n=1 << 21, mix="ack_data", seed=0x107D,
             metric="GiB/s fused receive verify (IPv4 header + pseudo-header + TCP checksum into a bitmask), frame bytes",
             name="f2+f3 rx bimodal: 2M IPv4/TCP datagrams per GPU, half 40-66B ACKs and half 1500B data frames "
                  "(random order), densely packed (odd starts), 1 in 1000 corrupted, verified into a validity "
                  "bitmask, device-resident"),
    15: dict(kind="ragged", n=1 << 23, lo=64, hi=128, seed=0x107E,
             metric="GiB/s device-resident Internet checksum, ragged segments",
             name="config3 small-segment twin: 8M ragged 64-128B segments per GPU, densely packed (odd starts), "
                  "device-resident"),
    16: dict(kind="rx", ipver=6, n=1 << 23, lo=60, hi=120, seed=0x107F,
             metric="GiB/s fused receive verify (IPv6 pseudo-header + TCP checksum into a bitmask), packet bytes",
             name="f2 rx6 small: 8M IPv6/TCP packets per GPU, 60-120B (uniform, ACK-sized), densely packed "
                  "(odd starts), 1 in 1000 corrupted, verified into a validity bitmask, device-resident"),
    # not a BASELINE config: ACK-dominated traffic with a few full frames — mean frame 125 B, just under the receive
    # pass's small-frame line (equal-count wave ranges, LDS form), with 5% of the frames 12x the mean
    17: dict(kind="rx", n=1 << 23, mix="ack_data", data_frac=0.05, seed=0x1080,
             metric="GiB/s fused receive verify (IPv4 header + pseudo-header + TCP checksum into a bitmask), frame bytes",
             name="f2+f3 rx ACK-heavy: 8M IPv4/TCP datagrams per GPU, 95% 40-66B ACKs and 5% 1500B data frames "
                  "(random order), densely packed (odd starts), 1 in 1000 corrupted, verified into a validity "
                  "bitmask, device-resident"),
    # not a BASELINE config: frames between the ACK and the full-frame regimes (mean 220 B), the receive pass's
    # 15-row prefix form
    18: dict(kind="rx", n=1 << 23, lo=40, hi=400, seed=0x1081,
             metric="GiB/s fused receive verify (IPv4 header + pseudo-header + TCP checksum into a bitmask), frame bytes",
             name="f2+f3 rx mid: 8M IPv4/TCP datagrams per GPU, 40-400B (uniform), densely packed (odd starts), "
                  "1 in 1000 corrupted, verified into a validity bitmask, device-resident"),
}


def frame_lengths(cfg):
    """Per-unit byte lengths of a ragged / receive workload (the same on every rank; bytes differ by seed):
    uniform on [lo, hi], or the bimodal ACK/data mix (uniform on [40, 66], a fraction data_frac (default half) of
    1500)."""
    import numpy as np
    rng = np.random.default_rng(cfg["seed"])
    n = cfg["n"]
    if cfg.get("mix") == "ack_data":
        return np.where(rng.random(n) < 1.0 - cfg.get("data_frac", 0.5), rng.integers(40, 67, n), 1500).astype(np.uint64)
    return rng.integers(cfg["lo"], cfg["hi"] + 1, n).astype(np.uint64)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=sorted(WORKLOADS),
                    help="2-5: BASELINE configs (2 = headline); 6: f1 fused TCP build; 7: f3 IPv4 header verify; "
                         "8: f1 with 12 B options; 9: f3 verify into a bitmask; 10: fused receive pass (f2+f3); "
                         "11: the receive pass over IPv6; 12: f1 with 9000 B MTU segments; 13 / 16: the receive "
                         "pass over 8M ACK-sized IPv4 / IPv6 frames; 14: over a bimodal ACK/1500 B mix; 15: config 3's "
                         "small-segment twin (8M x 64-128 B); 17: 8M frames, 95% ACKs and 5% 1500 B; 18: 8M "
                         "IPv4 frames of 40-400 B")
    ap.add_argument("--no-pseudo", action="store_true",
                    help="configs 2 and 5: checksum the segments without their pseudo-header partials")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--settle-s", type=float, default=0.5, help="device clock settle time before warmup (setup)")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=V",
                    help="per-call launch override (include/nsx_tune.h nsx_tune field), e.g. blocks_per_cu=2")
    ap.add_argument("--no-build", action="store_true",
                    help="load the library as it is (default: `make -C network-stack_amd` first, a no-op when "
                         "up to date)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: each rank's step is the CPU oracle on a small batch (exercises the launcher, "
                         "rendezvous and the timing/reduction logic; the value is not a measurement)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# rank launch: `--gpus N` without a launcher starts N ranks (before any GPU call)
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nranks: int, argv: list) -> int:
    """Start `nranks` rank processes of this script under torch.distributed.run (one
    process per GPU, rendezvous at 127.0.0.1) and wait for them; rank 0 prints the
    line. The parent has not touched a GPU (no torch.cuda call, library not loaded)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------------------
# distributed plumbing (shared with the gloo CPU tests)
# ---------------------------------------------------------------------------
class Dist:
    def __init__(self, backend: str | None, device_id=None):
        """device_id: this rank's GPU, already made current by the caller (torch.cuda.set_device BEFORE
        init_process_group, so no rank's communicator is created on GPU 0); passed on for nccl so RCCL
        binds the rank to it eagerly."""
        import torch.distributed as dist
        self.dist = dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.on = self.world > 1
        if self.on and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {"device_id": device_id} if backend == "nccl" and device_id is not None else {}
            dist.init_process_group(backend=backend, **kw)

    def gather(self, obj) -> list:
        """Every rank's `obj`, in rank order (one rank: [obj])."""
        if not self.on:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def barrier(self, device=None):
        if self.on:
            if device is not None and self.dist.get_backend() == "nccl":
                self.dist.barrier(device_ids=[device])
            else:
                self.dist.barrier()

    def max(self, x: float, device=None) -> float:
        if not self.on:
            return x
        import torch
        on_dev = device is not None and self.dist.get_backend() == "nccl"
        t = torch.tensor([x], dtype=torch.float64, device=device if on_dev else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float, device=None) -> float:
        if not self.on:
            return x
        import torch
        on_dev = device is not None and self.dist.get_backend() == "nccl"
        t = torch.tensor([x], dtype=torch.float64, device=device if on_dev else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.on and self.dist.is_initialized():
            self.dist.destroy_process_group()


def timed_loop(step, sync, barrier, steps: int, warmup: int, ev_pair=None):
    """W untimed steps; then EXACTLY K steps bracketed by barrier + sync on both
    sides. ev_pair() → (start, end) events recorded on the launch stream around
    the K timed steps (the timed region): the mean step duration on the device,
    inter-launch gaps included, no host synchronisation or barrier inside.
    (Round 1 bracketed single launches; an event between two launches makes the
    next kernel wait for the event's completion and exposes its dispatch
    latency, which read 5-7% above the traced duration for 0.13 ms kernels.)
    Returns (wall_s, [mean_step_ms] ([] without ev_pair), own_s): wall_s closes after the closing barrier, so it
    is the slowest rank's time on every rank (the job's clock); own_s closes at this rank's own sync before that
    barrier (its own clock, for its per-GPU rate — ADVICE r4: a rate from wall_s cannot show a slow GPU)."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    ev = ev_pair() if ev_pair else None
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    for _ in range(steps):
        step()
    if ev:
        ev[1].record()
    sync()
    own = time.perf_counter() - t0
    barrier()
    sync()
    wall = time.perf_counter() - t0
    return wall, ([ev[0].elapsed_time(ev[1]) / steps] if ev else []), own


def device_identity(dev_id: int) -> dict:
    """This rank's GPU as the driver sees it: hostname + PCI domain:bus:device and UUID. Two ranks on one
    physical GPU give the same key, so the line can prove how many distinct GPUs produced it."""
    import torch
    p = torch.cuda.get_device_properties(dev_id)
    pci = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                              getattr(p, "pci_device_id", 0))
    uuid = str(getattr(p, "uuid", "") or "")
    return {"host": socket.gethostname(), "local_device": dev_id, "pci": pci, "uuid": uuid,
            "key": f"{socket.gethostname()}/{pci}/{uuid}"}


def device_fields(idents: list) -> dict:
    """Line fields from every rank's device_identity (rank order): n_gpus = distinct physical devices."""
    distinct = len({d["key"] for d in idents})
    return {"n_gpus": distinct, "ranks": len(idents), "distinct_devices": distinct,
            "devices": [{k: d[k] for k in ("host", "local_device", "pci", "uuid")} for d in idents]}


def per_gpu_entries(rank_stats, *, steps, bytes_per_rank_step, alg_bytes_per_launch, launches=1) -> list:
    """Each rank's own rate from its own clock (rank_stats: every rank's {rank, device, wall_s, own_s, step_ms},
    rank order): bytes ÷ its own timed region (own_s: closed before the closing barrier, so a slow GPU shows;
    wall_s, the barrier-closed job clock, when own_s is absent), its kernel mean per launch (a step of `launches` launches, as config 5's
    windows, split evenly) and that launch's roofline fraction (alg_bytes_per_launch: one launch's bytes)."""
    out = []
    for r in rank_stats:
        k_ms = None if r.get("step_ms") is None else r["step_ms"] / launches
        frac = None if not k_ms else alg_bytes_per_launch / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
        own = r.get("own_s") or r["wall_s"]
        out.append({"rank": r["rank"], "device": r.get("device"),
                    "gib_s": round(bytes_per_rank_step * steps / own / GIB, 3),
                    "own_s": round(own, 6), "wall_s": round(r["wall_s"], 6),
                    "kernel_ms": None if k_ms is None else round(k_ms, 5),
                    "roofline_frac": None if frac is None else round(frac, 4)})
    return out


def result_line(*, world, steps, warmup, wall_max, bytes_per_rank_step, units_total, workload, cfg, launch_ms,
                alg_bytes_per_launch, cpu_baseline, traffic, dtype="u16", metric=METRIC, launches=1,
                n_gpus=None, rank_stats=None) -> dict:
    """world = ranks (each processed bytes_per_rank_step per step); n_gpus = distinct physical GPUs behind
    them (default: one per rank); rank_stats = every rank's own timing (per_gpu_entries)."""
    total_bytes = bytes_per_rank_step * world * steps
    # launch_ms: mean device time of one step over the timed region; a step of `launches` back-to-back
    # launches is reported per launch (alg bytes and duration divided evenly, the gaps between launches
    # included) so that it compares with the rocprofv3 per-launch average and the PMC traffic per launch.
    mean_launch_ms = sum(launch_ms) / len(launch_ms) / launches if launch_ms else None
    alg_bytes_per_launch = alg_bytes_per_launch // launches
    achieved = alg_bytes_per_launch / (mean_launch_ms * 1e-3) / 1e9 if mean_launch_ms else None
    return {
        "metric": metric,
        "value": round(total_bytes / wall_max / GIB, 3),
        "unit": "GiB/s",
        "value_per_gpu_mean": round(total_bytes / wall_max / GIB / world, 3),
        "n_gpus": world if n_gpus is None else n_gpus,
        "ranks": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(wall_max / steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic: splitmix64 bytes (seed %#x + rank) generated on device" % cfg["seed"],
        "config": {"workload": workload, "units_per_gpu": cfg["n"], "bytes_per_gpu": bytes_per_rank_step,
                   "units_per_step_all_gpus": units_total,
                   "parallelism": f"shard{world} (independent per-GPU batches, no collective)"},
        "kernel_ms_mean": None if mean_launch_ms is None else round(mean_launch_ms, 5),
        "roofline": None if achieved is None else {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None if traffic is None else traffic.get("bytes_per_launch"),
            "traffic_source": None if traffic is None else traffic.get("source"),
            "alg_bytes_per_launch": alg_bytes_per_launch, "launches_per_step": launches},
        "per_gpu": None if rank_stats is None else per_gpu_entries(
            rank_stats, steps=steps, bytes_per_rank_step=bytes_per_rank_step,
            alg_bytes_per_launch=alg_bytes_per_launch, launches=launches),
        "cpu_baseline": cpu_baseline,
    }


# ---------------------------------------------------------------------------
# GPU workload
# ---------------------------------------------------------------------------
def parse_tune(items) -> dict:
    import nsx
    tune = {}
    for kv in items:
        k, v = kv.split("=", 1)
        if k not in nsx.TUNE_FIELDS:
            raise SystemExit(f"--tune: unknown nsx_tune field {k!r} (fields: {', '.join(nsx.TUNE_FIELDS)})")
        tune[k] = int(v)
    return tune


def build_workload(cfg, rank, device, tune=None):
    """One rank's device-resident batch and its step (one call of the entry point). cfg["pseudo"]: every
    fixed-stride segment over its own IPv4 pseudo-header (random src/dst, proto 6, TCP length = seg_len),
    passed as the N x u32 partials nsx_pseudo_ipv4_partial_dev makes."""
    import numpy as np
    import torch
    import nsx
    seed = cfg["seed"] + rank
    w = {"seed": seed}
    if cfg["kind"] == "fixed":
        n, L, S = cfg["n"], cfg["seg_len"], cfg["stride"]
        buf = torch.empty((n - 1) * S + L, dtype=torch.uint8, device=device)
        nsx.fill_splitmix64_dev(buf, seed)
        out = torch.empty(n, dtype=torch.int16, device=device)
        part = addrs = None
        if cfg.get("pseudo"):
            g = torch.Generator(device=device).manual_seed(seed)
            addrs = torch.randint(0, 256, (2, n, 4), generator=g, device=device, dtype=torch.int64).to(torch.uint8)
            part = nsx.pseudo_ipv4_partial_dev(addrs[0].reshape(-1), addrs[1].reshape(-1),
                                               torch.full((n,), L, dtype=torch.int32, device=device), 6)
        # launches per step: the library's own count of its back-to-back windows (config 5: 16)
        w.update(buf=buf, out=out, part=part, addrs=addrs, bytes=n * L,
                 alg=n * L + 2 * n + (4 * n if part is not None else 0),
                 launches=nsx.fixed_launch_count(S, L, n, tune),
                 step_for=lambda t: lambda: nsx.fixed_dev(buf, S, L, n, partial=part, out=out, tune=t))
    elif cfg["kind"] == "tcp_build":
        n, P, OL = cfg["n"], cfg["payload"], cfg.get("opt", 0)
        W = P + 20 + OL  # OL ≡ 0 mod 4: tcp.go:118-121 pads nothing
        g = torch.Generator(device=device).manual_seed(seed)
        data = torch.empty(n * P, dtype=torch.uint8, device=device)
        nsx.fill_splitmix64_dev(data, seed)

        def rnd(bits, dtype):
            return torch.randint(0, 1 << bits, (n,), generator=g, device=device, dtype=torch.int64).to(dtype)

        fields = {"src_port": rnd(16, torch.int16), "dst_port": rnd(16, torch.int16),
                  "seq_num": rnd(32, torch.int32), "ack_num": rnd(32, torch.int32),
                  "offset": torch.full((n,), 5 + OL // 4, dtype=torch.uint8, device=device),  # computeOffset
                  "control": rnd(8, torch.uint8), "window": rnd(16, torch.int16), "urgent_ptr": rnd(16, torch.int16)}
        addrs = torch.randint(0, 256, (2, n, 4), generator=g, device=device, dtype=torch.int64).to(torch.uint8)
        wire_len = torch.full((n,), W, dtype=torch.int32, device=device)
        part = nsx.pseudo_ipv4_partial_dev(addrs[0].reshape(-1), addrs[1].reshape(-1), wire_len, 6)
        idx = torch.arange(n + 1, dtype=torch.int64, device=device)
        data_off, out_off = idx * P, idx * W
        out = torch.empty(n * W, dtype=torch.uint8, device=device)
        raw = torch.empty(n, dtype=torch.int16, device=device)
        opts = opt_off = None
        if OL:  # NOP, NOP, a kind-2 option of length 10 with 8 random data bytes (tcp.go:225-231 serialises
            # kind 2 as kind, length, data; every other kind as its kind byte): the layout of a timestamps block
            opts = torch.randint(0, 256, (n, OL), generator=g, device=device, dtype=torch.int64).to(torch.uint8)
            opts[:, :4] = torch.tensor([1, 1, 2, 10], dtype=torch.uint8, device=device)
            opts = opts.reshape(-1)
            opt_off = idx * OL
        # per segment: payload + options + 18 B of header fields + 2 (+2) offsets + partial read; wire image + raw
        # sum written
        w.update(out=raw, wire=out, fields=fields, addrs=addrs, data=data, opts=opts, opt_off=opt_off, part=part,
                 data_off=data_off, out_off=out_off, bytes=n * W,
                 alg=n * (P + OL + 18 + 8 + 8 + (8 if OL else 0) + 4 + W + 2) + 16 + (8 if OL else 0),
                 step_for=lambda t: lambda: nsx.tcp_build_dev(fields, data, data_off, out, out_off, opts=opts,
                                                              opt_off=opt_off, partial=part, raw=raw, tune=t))
    elif cfg["kind"] == "ipv4_hdr":
        n, H = cfg["n"], cfg["hdr"]
        buf = torch.empty(n * H, dtype=torch.uint8, device=device)
        nsx.fill_splitmix64_dev(buf, seed)
        buf.view(n, H)[:, 0] = 0x45  # version 4, IHL 5
        nsx.ipv4_hdr_csum_dev(buf, H, n, mode=1)  # setup: fill valid checksums (RFC 791 §3.1)
        if cfg.get("mask"):
            buf.view(n, H)[::1000, 8] ^= 1  # some invalid headers (TTL flipped after the fill)
            out = torch.empty((n + 63) // 64, dtype=torch.int64, device=device)
            w.update(buf=buf, out=out, bytes=n * H, alg=n * H + (n + 63) // 64 * 8,
                     step_for=lambda t: lambda: nsx.ipv4_hdr_verify_mask_dev(buf, H, n, mask=out, tune=t))
        else:
            out = torch.empty(n, dtype=torch.int16, device=device)
            w.update(buf=buf, out=out, bytes=n * H, alg=n * (H + 2),
                     step_for=lambda t: lambda: nsx.ipv4_hdr_csum_dev(buf, H, n, mode=0, out=out, tune=t))
        # launches per step: the library's count of its back-to-back header windows (64M headers: 2)
        w.update(launches=nsx.ipv4_hdr_launch_count(buf, H, n, tune=tune))
    elif cfg["kind"] == "rx":
        w.update(build_rx_frames(cfg, seed, device))
        n, buf, d_offs, total = cfg["n"], w["buf"], w["d_offs"], w["bytes"]
        out = torch.empty((n + 63) // 64, dtype=torch.int64, device=device)
        rx = nsx.rx_ipv6_tcp_verify_dev if cfg.get("ipver") == 6 else nsx.rx_ipv4_tcp_verify_dev
        w.update(out=out, alg=total + 8 * (n + 1) + (n + 63) // 64 * 8,
                 step_for=lambda t: lambda: rx(buf, d_offs, mask=out, tune=t))
    else:
        n = cfg["n"]
        lens = frame_lengths(cfg)  # same lengths on every rank, bytes differ by seed
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        total = int(offs[-1])
        buf = torch.empty(total, dtype=torch.uint8, device=device)
        nsx.fill_splitmix64_dev(buf, seed)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
        out = torch.empty(n, dtype=torch.int16, device=device)
        w.update(buf=buf, out=out, offsets=offs, d_offs=d_offs, bytes=total, alg=total + 2 * n + 8 * (n + 1),
                 step_for=lambda t: lambda: nsx.ragged_dev(buf, d_offs, out=out, tune=t))
    w["step"] = w["step_for"](tune)  # one pass of the hot path; step_for(t) = the same with other overrides
    return w


def host_cores() -> dict:
    """The host CPU share this process may use for the CPU baseline: its affinity set, capped by a
    cgroup CPU quota and by OMP_NUM_THREADS when the host sets them (the GPU box declares each GPU's
    share of its cores that way; os.cpu_count() there is the whole machine's)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = min(x for x in (aff, quota, omp) if x)
    return {"threads": threads, "affinity_cpus": aff, "cgroup_cpus": quota, "omp_num_threads": omp,
            "host_cpus": os.cpu_count()}


def _ptr(a, lo=0):
    import ctypes
    return ctypes.c_void_p(a.ctypes.data + lo * a.itemsize)


def _run_for(fn, seconds: float):
    t0, reps = time.perf_counter(), 0
    while True:
        fn()
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return reps, time.perf_counter() - t0


def build_rx_frames(cfg, seed, device) -> dict:
    """Workload 10's received datagrams, built on the device: frame lengths uniform on [lo, hi] (same on every
    rank), densely packed; splitmix64 bytes, then per frame an IPv4 header (version 4, IHL 5, total length =
    frame length, DF, protocol 6; the random bytes stay as id / TTL / addresses) and a TCP segment of the
    rest. Both checksum fields are filled with this library's own ragged kernel over the 2n header /
    segment spans (the TCP spans with their pseudo-header partials, RFC 9293 §3.1), then every 1000th frame
    gets one bit flipped in its TCP header (setup; the parity test checks the outcome against the oracle).
    Workload 11 (ipver 6): an IPv6 header instead (version 6, payload length = frame length − 40, Next
    Header 6; the random bytes stay as class / flow / hop limit / addresses), the TCP field filled over the
    RFC 8200 §8.1 pseudo-header."""
    import numpy as np
    import torch
    import nsx
    n = cfg["n"]
    lens = frame_lengths(cfg)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    total = int(offs[-1])
    buf = torch.empty(total, dtype=torch.uint8, device=device)
    nsx.fill_splitmix64_dev(buf, seed)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    st = d_offs[:-1]
    ln = (d_offs[1:] - st)
    put = lambda k, v: buf.index_put_((st + k,), v if torch.is_tensor(v) else torch.full_like(st, v, dtype=torch.uint8))
    if cfg.get("ipver") == 6:
        put(0, ((buf[st] & 0x0F) | 0x60).to(torch.uint8))
        put(4, ((ln - 40) >> 8).to(torch.uint8))
        put(5, ((ln - 40) & 0xFF).to(torch.uint8))
        put(6, 6)
        put(56, 0)
        put(57, 0)
        idx16 = torch.arange(16, device=device)
        src = buf[(st[:, None] + 8 + idx16).reshape(-1)]
        dst = buf[(st[:, None] + 24 + idx16).reshape(-1)]
        pseudo = nsx.pseudo_ipv6_partial_dev(src, dst, (ln - 40).to(torch.int32), 6)
        spans = torch.cat([torch.stack([st, st + 40], 1).reshape(-1), d_offs[-1:]])
        part2 = torch.stack([torch.zeros_like(pseudo), pseudo], 1).reshape(-1)
        tcp_f = (~(nsx.ragged_dev(buf, spans, partial=part2).to(torch.int32) & 0xFFFF))[1::2] & 0xFFFF
        put(56, (tcp_f >> 8).to(torch.uint8))
        put(57, (tcp_f & 0xFF).to(torch.uint8))
        buf[st[::1000] + 50] ^= 1
        torch.cuda.synchronize()
        return {"buf": buf, "d_offs": d_offs, "offsets": offs, "bytes": total}
    put(0, 0x45)
    put(1, 0)
    put(2, (ln >> 8).to(torch.uint8))
    put(3, (ln & 0xFF).to(torch.uint8))
    put(6, 0x40)
    put(7, 0)
    put(9, 6)
    for k in (10, 11, 36, 37):  # checksum fields zero while the sums are taken
        put(k, 0)
    idx4 = torch.arange(4, device=device)
    src = buf[(st[:, None] + 12 + idx4).reshape(-1)]
    dst = buf[(st[:, None] + 16 + idx4).reshape(-1)]
    tcp_len = (ln - 20).to(torch.int32)
    pseudo = nsx.pseudo_ipv4_partial_dev(src, dst, tcp_len, 6)
    spans = torch.stack([st, st + 20], 1).reshape(-1)
    spans = torch.cat([spans, d_offs[-1:]])
    part2 = torch.stack([torch.zeros_like(pseudo), pseudo], 1).reshape(-1)
    raw2 = nsx.ragged_dev(buf, spans, partial=part2).to(torch.int32) & 0xFFFF
    fld = (~raw2) & 0xFFFF
    ip_f, tcp_f = fld[0::2], fld[1::2]
    put(10, (ip_f >> 8).to(torch.uint8))
    put(11, (ip_f & 0xFF).to(torch.uint8))
    put(36, (tcp_f >> 8).to(torch.uint8))
    put(37, (tcp_f & 0xFF).to(torch.uint8))
    bad = st[::1000] + 30
    buf[bad] ^= 1
    torch.cuda.synchronize()
    return {"buf": buf, "d_offs": d_offs, "offsets": offs, "bytes": total}


def cpu_baseline(cfg, w, seconds: float) -> dict:
    """Go-faithful CPU restatement of the workload (allocate + concatenate + serial compare-carry loop
    per segment, tcp.go:72-95; for f1 also segment.bytes(), tcp.go:98-128) over a bounded sample of
    this rank's own batch, timed on every host core this process may use (contiguous shards — byte-
    balanced for ragged batches — one thread each; ctypes releases the GIL) and on one thread. Both
    legs' results are compared with the GPU's for the same segments (the checker role)."""
    from concurrent.futures import ThreadPoolExecutor
    import threading
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from oracle import csum_oracle as O
    lib = O.c_oracle()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    cores = host_cores()
    T = cores["threads"]
    extra = None
    check = {}
    if cfg["kind"] == "fixed":
        n, L, S = cfg["n"], cfg["seg_len"], cfg["stride"]
        m = min(n, max(1, (256 << 20) // S))  # sample: the first m segments (≤ 256 MiB)
        sample = w["buf"][: (m - 1) * S + L].cpu().numpy()
        gpu = w["out"][:m].cpu().numpy().view(np.uint16)
        out = np.empty(m, np.uint16)
        bounds = [m * t // T for t in range(T + 1)]
        part = None
        if w.get("addrs") is not None:  # each segment's own 12 B IPv4 pseudo-header, as a Go caller passes it
            a = w["addrs"][:, :m].cpu().numpy()
            pseudo = np.ascontiguousarray(np.concatenate(
                [a[0], a[1], np.tile(np.array([0, 6, L >> 8, L & 0xFF], np.uint8), (m, 1))], 1))
            part = np.ascontiguousarray(w["part"][:m].cpu().numpy().view(np.uint32))

            def go(lo, hi):
                lib.oracle_go_batch_fixed_pseudo(_ptr(sample, lo * S), S, L, hi - lo, _ptr(pseudo, lo * 12), 12,
                                                 _ptr(out, lo))
        else:
            def go(lo, hi):
                lib.oracle_go_batch_fixed(_ptr(sample, lo * S), S, L, hi - lo, None, 0, _ptr(out, lo))
        nbytes = m * L
        desc = (f"first {m} segments x {L}B of rank 0's batch"
                + (", each over its 12 B IPv4 pseudo-header (computeChecksum(ipPseudoHeader))" if part is not None
                   else ""))
        check["segments"] = lambda: np.array_equal(out, gpu)
    elif cfg["kind"] == "tcp_build":
        n, P, OL = cfg["n"], cfg["payload"], cfg.get("opt", 0)
        W = P + 20 + OL
        m = min(n, max(1, (256 << 20) // W))  # sample: the first segments of ≤ 256 MiB of wire
        cols = [np.ascontiguousarray(w["fields"][k][:m].cpu().numpy().view(dt))
                for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)]
        data = w["data"][: m * P].cpu().numpy()
        a = w["addrs"][:, :m].cpu().numpy()
        pseudo = np.ascontiguousarray(np.concatenate(
            [a[0], a[1], np.tile(np.array([0, 6, W >> 8, W & 0xFF], np.uint8), (m, 1))], 1))
        data_off = np.arange(m + 1, dtype=np.uint64) * np.uint64(P)
        out_off = np.arange(m + 1, dtype=np.uint64) * np.uint64(W)
        gpu = w["out"][:m].cpu().numpy().view(np.uint16)
        gpu_wire = w["wire"][: m * W].cpu().numpy()
        wire = np.zeros(m * W, np.uint8)
        out = np.empty(m, np.uint16)
        bounds = [m * t // T for t in range(T + 1)]
        if OL:
            opts = np.ascontiguousarray(w["opts"][: m * OL].cpu().numpy())
            opt_off = np.arange(m + 1, dtype=np.uint64) * np.uint64(OL)

            def go(lo, hi):
                rc = lib.oracle_go_tcp_build_batch_opts(*[_ptr(c, lo) for c in cols], _ptr(opts), _ptr(opt_off, lo),
                                                        _ptr(data), _ptr(data_off, lo), _ptr(pseudo, lo * 12), 12,
                                                        hi - lo, _ptr(wire), _ptr(out_off, lo), _ptr(out, lo))
                assert rc == 0
        else:
            def go(lo, hi):
                rc = lib.oracle_go_tcp_build_batch(*[_ptr(c, lo) for c in cols], _ptr(data), _ptr(data_off, lo),
                                                   _ptr(pseudo, lo * 12), 12, hi - lo, _ptr(wire), _ptr(out_off, lo),
                                                   _ptr(out, lo))
                assert rc == 0
        nbytes = m * W
        desc = (f"first {m} segments of rank 0's batch: the Go sender loop — bytes()"
                f"{' with ' + str(OL) + ' B of options' if OL else ''} + computeChecksum(12B pseudo-header) + "
                "field store per segment")
        check["segments"] = lambda: np.array_equal(out, gpu)
        check["wire_images"] = lambda: np.array_equal(wire, gpu_wire)
    elif cfg["kind"] == "ipv4_hdr":
        n, H = cfg["n"], cfg["hdr"]
        m = min(n, (256 << 20) // H // 64 * 64)  # sample: ≤ 256 MiB of headers, whole mask words
        sample = w["buf"][: m * H].cpu().numpy()
        mask = cfg.get("mask", False)
        gpu = (w["out"][: m // 64].cpu().numpy().view(np.uint64) if mask
               else w["out"][:m].cpu().numpy().view(np.uint16))
        raw = np.empty(m, np.uint16)
        bounds = [m * t // T // 64 * 64 for t in range(T)] + [m]

        def go(lo, hi):
            lib.oracle_go_batch_fixed(_ptr(sample, lo * H), H, H, hi - lo, None, 0, _ptr(raw, lo))
        nbytes = m * H
        desc = (f"first {m} headers of rank 0's batch, the reference's serial checksum loop per header"
                + (" + bit packing of sum == 0xFFFF" if mask else ""))
        # IHL 5 on every header of this workload, so well-formed; valid iff the sum is 0xFFFF
        whole = m // 64 * 64  # mask words wholly inside the sample
        check["headers"] = (lambda: np.array_equal(
            np.packbits(raw[:whole] == 0xFFFF, bitorder="little").view(np.uint64), gpu)) if mask else (
            lambda: np.array_equal(raw, gpu))
    elif cfg["kind"] == "rx":
        offs_all = w["offsets"]
        m = int(min(len(offs_all) - 1, np.searchsorted(offs_all, 256 << 20))) // 64 * 64  # ≤ 256 MiB, whole words
        hi_b = int(offs_all[m])
        sample = w["buf"][:hi_b].cpu().numpy()
        offs = np.ascontiguousarray(offs_all[: m + 1])
        gpu = w["out"][: m // 64].cpu().numpy().view(np.uint64)
        cmask = np.zeros(m // 64, np.uint64)
        bounds = [int(np.searchsorted(offs, hi_b * t // T)) // 64 * 64 for t in range(T)] + [m]  # byte-balanced

        v6 = cfg.get("ipver") == 6

        def go(lo, hi):
            if v6:
                lib.oracle_go_rx_ipv6_tcp(_ptr(sample), _ptr(offs, lo), hi - lo, _ptr(cmask, lo // 64), None)
            else:
                lib.oracle_go_rx_ipv4_tcp(_ptr(sample), _ptr(offs, lo), hi - lo, _ptr(cmask, lo // 64), None, None)
        nbytes = hi_b
        desc = (f"first {m} frames of rank 0's batch: per frame the reference's checksum loop over "
                + ("pseudo-header ‖ TCP segment (IPv6)" if v6 else
                   "the IPv4 header and over pseudo-header ‖ TCP segment")
                + " (allocate + concatenate + serial loop) + bit packing")
        check["mask"] = lambda: np.array_equal(cmask, gpu)
    else:
        offs_all = w["offsets"]
        m = int(min(len(offs_all) - 1, max(1, np.searchsorted(offs_all, 256 << 20))))  # ≤ 256 MiB of segments
        hi_b = int(offs_all[m])
        sample = w["buf"][:hi_b].cpu().numpy()
        offs = np.ascontiguousarray(offs_all[: m + 1])
        gpu = w["out"][:m].cpu().numpy().view(np.uint16)
        out = np.empty(m, np.uint16)
        bounds = [int(np.searchsorted(offs, hi_b * t // T)) for t in range(T)] + [m]  # byte-balanced

        def go(lo, hi):
            lib.oracle_go_batch_ragged(_ptr(sample), _ptr(offs, lo), hi - lo, None, 0, _ptr(out, lo))
        nbytes, desc = hi_b, f"first {m} ragged segments of rank 0's batch"
        check["segments"] = lambda: np.array_equal(out, gpu)
    busy = []  # seconds of every shard call in the all-threads leg
    passes = []  # per pass: [(shard start − pass start, shard duration)] over its T shard calls

    def timed_go(t):
        t0 = time.perf_counter()
        go(bounds[t], bounds[t + 1])
        t1 = time.perf_counter()
        busy.append(t1 - t0)
        return t0, t1
    # each worker thread pinned to a CPU of its own, on distinct physical cores (round 6): left to
    # the scheduler, the packed-header legs' last two shards of each pass ran 3.3x slower than the rest, each alone on
    # its CPU on a near-idle host, and pinned they ran within 1.2x (tools/probes/cpu_shards.py,
    # profiles/r06_cpu_shards.txt). Pinned to a fixed set of cores, one box's leg still ran 1.9x imbalanced (a core
    # shared with other work), so the cores are the least busy ones at the time (shard_cpus). NSX_BENCH_CPU_PIN=0
    # leaves placement to the scheduler.
    pin = shard_cpus(T) if os.environ.get("NSX_BENCH_CPU_PIN", "1") != "0" else None
    pin_next = iter(pin or ())
    pin_lock = threading.Lock()

    def pin_worker():
        with pin_lock:
            c = next(pin_next, None)
        if c is not None:
            os.sched_setaffinity(0, {c})  # pid 0: the calling thread only (Linux)
    thr0 = cgroup_throttling()
    with ThreadPoolExecutor(T, initializer=pin_worker if pin else None) as ex:
        def all_cores():
            p0 = time.perf_counter()
            passes.append([(a - p0, b - a) for a, b in ex.map(timed_go, range(T))])
        reps_t, dt_t = _run_for(all_cores, seconds / 2)
        ok_t = all(f() for f in check.values())
    thr1 = cgroup_throttling()
    reps_1, dt_1 = _run_for(lambda: go(0, bounds[-1]), seconds / 2)
    ok_1 = all(f() for f in check.values())
    if cfg["kind"] == "fixed":
        extra = cpu_extra_lines(sample, S, L, m, out, max(1.0, seconds / 4), T, part)
    v_t, v_1 = reps_t * nbytes / dt_t / GIB, reps_1 * nbytes / dt_1 / GIB
    eff = v_t / (T * v_1) if v_1 else None
    # why the all-threads leg falls short of T x the 1-thread rate, when it does: the shard calls' busy time against
    # T x the wall time (threads waiting to run) and the per-thread rate inside the calls (threads running slower
    # than alone: allocator or memory contention), plus any CPU-quota throttling the cgroup recorded meanwhile
    busy_frac = sum(busy) / (T * dt_t) if dt_t else None
    in_call = (nbytes * reps_t / T) / (sum(busy) / T) / GIB if busy else None
    # per pass: the shard calls' durations, max / min over the T shards (imbalance: one shard
    # doing more work, or running slower, than the others), the latest shard's start after the pass began (a thread
    # that was not running when its shard was handed out), and the slowest shard's duration against the 1-thread
    # time of its share (every shard running slow: contention); medians over the passes
    shard_max_min = [max(d for _, d in p) / max(min(d for _, d in p), 1e-9) for p in passes]
    late_start_ms = [max(a for a, _ in p) * 1e3 for p in passes]
    slowest_ms = [max(d for _, d in p) * 1e3 for p in passes]
    alone_ms = dt_1 / max(reps_1, 1) / T * 1e3  # one shard's share of the 1-thread pass
    med = (lambda v: round(float(np.median(v)), 3) if v else None)
    diag = {"busy_fraction": None if busy_frac is None else round(busy_frac, 3),
            "per_thread_gib_s_in_call": None if in_call is None else round(in_call, 4),
            "cgroup_throttled_ms": None if thr0 is None or thr1 is None else round((thr1[1] - thr0[1]) / 1e3, 1),
            "cgroup_throttled_periods": None if thr0 is None or thr1 is None else thr1[0] - thr0[0],
            "shard_duration_max_over_min": med(shard_max_min), "shard_latest_start_ms": med(late_start_ms),
            "slowest_shard_ms": med(slowest_ms), "shard_alone_ms": round(alone_ms, 3),
            "pass_wall_ms": round(dt_t / max(reps_t, 1) * 1e3, 3),
            "pinned_cpus": pin}
    why = ""
    if eff is not None and eff < 0.5:
        imbalanced = diag["shard_duration_max_over_min"] is not None and diag["shard_duration_max_over_min"] > 1.5
        late = diag["shard_latest_start_ms"] is not None and diag["shard_latest_start_ms"] > 0.25 * diag["pass_wall_ms"]
        if diag["cgroup_throttled_ms"]:
            why = f"; below 0.5 parallel efficiency: the cgroup's CPU quota throttled the process {diag['cgroup_throttled_ms']} ms"
        elif late:
            why = (f"; below 0.5 parallel efficiency: shards started up to {diag['shard_latest_start_ms']:.1f} ms into a "
                   f"{diag['pass_wall_ms']:.1f} ms pass (threads not running when handed a shard: descheduled)")
        elif imbalanced:
            why = (f"; below 0.5 parallel efficiency: the shards are imbalanced — the slowest call took "
                   f"{diag['shard_duration_max_over_min']:.1f}x the fastest within a pass")
        else:
            why = (f"; below 0.5 parallel efficiency: every shard runs slow — the slowest took {diag['slowest_shard_ms']:.1f} "
                   f"ms against {alone_ms:.1f} ms for its share on one thread alone, {in_call:.2f} GiB/s per thread in "
                   f"the calls against {v_1:.2f} alone (contention in the per-unit allocation or memory system)")
    return {"value": round(v_t, 4), "unit": "GiB/s", "cores": T, "kind": "port",
            "sample": f"{desc} ({nbytes / 2**20:.0f} MiB), {reps_t} pass(es) on {T} threads (Go-faithful loop, "
                      f"contiguous shards, {'each thread pinned to its own core' if pin else 'threads placed by the scheduler'})"
                      f"{why}",
            "seconds": round(dt_t, 2),
            "single_thread": {"value": round(v_1, 4), "unit": "GiB/s", "cores": 1,
                              "passes": reps_1, "seconds": round(dt_1, 2)},
            "parallel_efficiency": None if eff is None else round(eff, 3), "threads_diagnostics": diag,
            "sample_parity_vs_gpu": bool(ok_t and ok_1), "host": cores, "extra": extra}


def shard_cpus(T, probe_s=0.2):
    """T CPUs of this process's affinity set for the CPU leg's worker threads: one per physical core (sysfs
    thread_siblings_list) as far as the set has cores, the least busy cores first — each core's busy fraction over
    `probe_s` seconds (/proc/stat, the busier of its SMT threads, in steps of 5%), so that threads do not land on cores
    that other work on a shared host keeps busy — then those of the calling thread's package; None when there are
    fewer than T CPUs or no topology to read."""
    import ctypes
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < T:
        return None

    def topo(c, leaf):
        with open(f"/sys/devices/system/cpu/cpu{c}/topology/{leaf}") as f:
            return f.read().strip()

    def jiffies():
        t = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = [int(x) for x in line.split()[1:9]]
                    t[int(line.split()[0][3:])] = (sum(v) - v[3] - v[4], sum(v))
        return t
    try:
        here = ctypes.CDLL(None).sched_getcpu()
        pkg_here = topo(here, "physical_package_id") if here >= 0 else None
        j0 = jiffies()
        time.sleep(probe_s)
        j1 = jiffies()
        busy = {c: (j1[c][0] - j0[c][0]) / max(j1[c][1] - j0[c][1], 1) for c in j1 if c in j0}
        groups = {}
        for c in cpus:
            groups.setdefault(topo(c, "thread_siblings_list"), []).append(c)
        cores = []
        for sib, members in groups.items():
            load = max(busy.get(int(x), 0.0) for x in sib.replace("-", ",").split(",") if x)
            cores.append((round(load * 20), topo(members[0], "physical_package_id") != pkg_here, members[0]))
    except (OSError, AttributeError, ValueError):
        return None
    first = [c for _, _, c in sorted(cores)]
    rest = [c for c in cpus if c not in set(first)]
    return (first + rest)[:T]


def cgroup_throttling():
    """(nr_throttled, throttled_usec) of this process's cgroup (cgroup v2 cpu.stat), or None."""
    try:
        st = dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
        return int(st.get("nr_throttled", 0)), int(st.get("throttled_usec", 0))
    except (OSError, ValueError):
        return None


def cpu_extra_lines(sample, S, L, m, want, seconds, threads, part=None):
    """The honest best-CPU line beside the Go-faithful one: a vectorised u64-accumulate
    restatement (oracle/csum_cpu_fast.c) on 1 and `threads` threads, same sample (with the same pseudo-header
    partials as the GPU's when it has them); each result is checked against the Go-faithful output."""
    import numpy as np
    from oracle import csum_oracle as O
    fast = O.c_fast()
    out = np.empty(m, np.uint16)
    ptr = sample.ctypes.data
    pp = None if part is None else part.ctypes.data

    def run(fn):
        reps, dt = _run_for(fn, seconds)
        return {"value": round(reps * m * L / dt / GIB, 3), "unit": "GiB/s", "parity": bool(np.array_equal(out, want))}

    res = {"optimized_1_thread": dict(run(lambda: fast.cpu_fast_batch_fixed(ptr, S, L, m, pp, out.ctypes.data, 1)),
                                      cores=1),
           "optimized_threads": dict(run(lambda: fast.cpu_fast_batch_fixed(ptr, S, L, m, pp, out.ctypes.data,
                                                                           threads)), cores=threads),
           "note": "optimized = oracle/csum_cpu_fast.c (8-byte loads, u64 accumulators, -O3 x86-64-v3): the best-CPU "
                   "line; the baseline value is the reference's algorithm as written"}
    return res


def load_traffic(config_id):
    """The committed PMC traffic of a workload (profiles/traffic_config<id>.json; id 2n = config 2 without its
    pseudo-header partials)."""
    p = os.path.join(ROOT, "profiles", f"traffic_config{config_id}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    d["source"] = os.path.relpath(p, ROOT)
    return d


def dry_run(args) -> int:
    """--dry-run: the rank/launch/timing plumbing with the CPU oracle as each rank's step (no GPU)."""
    sys.path.insert(0, ROOT)
    from oracle import csum_oracle as O
    dist = Dist("gloo")
    n, L = 256, 1500
    buf = O.c_splitmix64(0x1071 + dist.rank, n * L)
    wall, launch_ms, own = timed_loop(lambda: O.c_batch(buf, n, stride=L, seg_len=L, threads=1), lambda: None,
                                      dist.barrier, args.steps, args.warmup)
    wall_max = dist.max(wall)
    idents = dist.gather({"host": socket.gethostname(), "local_device": None, "pci": None, "uuid": None,
                          "key": None})
    stats = dist.gather({"rank": dist.rank, "device": None, "wall_s": wall, "own_s": own, "step_ms": None})
    line = result_line(world=dist.world, steps=args.steps, warmup=args.warmup, wall_max=wall_max,
                       bytes_per_rank_step=n * L, units_total=n * dist.world, workload="dry run", cfg={"n": n, "seed": 0x1071},
                       launch_ms=launch_ms, alg_bytes_per_launch=n * L + 2 * n, cpu_baseline=None, traffic=None,
                       n_gpus=0, rank_stats=stats)
    # no GPU behind any rank: n_gpus 0, the rank count separate
    line.update(dry_run=True, data="dry run: the CPU oracle stands in for the GPU kernel; not a measurement",
                backend="gloo", rehearsal=True, distinct_devices=0,
                devices=[{k: d[k] for k in ("host", "local_device", "pci", "uuid")} for d in idents])
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()
    return 0


def build_library() -> None:
    """Bring libnsx_csum.so up to date before it is loaded (incremental make: a no-op when the pushed binary
    matches its sources; ~35 s for a full rebuild). A failed build is an error, never a stale library."""
    import fcntl
    with open(os.path.join(ROOT, "network-stack_amd", ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-j16", "-C", os.path.join(ROOT, "network-stack_amd")],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise SystemExit(f"bench.py: building network-stack_amd failed:\n{r.stdout[-4000:]}")


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    # bring the library up to date before anything loads it, under a file lock: in the launching process before any
    # rank starts (its ranks inherit NSX_BENCH_BUILT and skip it), and in every rank an outside launcher started
    # (torchrun … bench.py: WORLD_SIZE set, NSX_BENCH_BUILT not) — there the first rank to take the lock builds and
    # the others, waiting on it, find nothing to do, so no rank loads a stale or half-written library
    if not args.dry_run and not args.no_build and os.environ.get("NSX_BENCH_BUILT") != "1":
        build_library()
        os.environ["NSX_BENCH_BUILT"] = "1"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv)  # before anything touches a GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a different GPU count",
              file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args)
    import torch
    import nsx
    # RCCL ("nccl") is the backend; NSX_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a device
    # round-robin, and the line says so), e.g. 2 ranks on a 1-GPU box
    backend = os.environ.get("NSX_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if ndev == 0 or not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU: the checksum path is HIP-only (no CPU fallback)")
    if world > ndev and backend == "nccl":
        print(f"bench.py: {world} ranks but {ndev} visible GPU(s): one rank per GPU is required "
              "(NSX_BENCH_BACKEND=gloo runs a labelled rehearsal)", file=sys.stderr)
        return 2
    # this rank's GPU is made current BEFORE the process group exists (and handed to it), so RCCL never
    # creates a rank's communicator on GPU 0
    dev_id = int(os.environ.get("LOCAL_RANK", "0")) % ndev if world > 1 else 0
    torch.cuda.set_device(dev_id)
    device = torch.device("cuda", dev_id)
    dist = Dist(backend, device_id=device)
    devf = device_fields(dist.gather(device_identity(dev_id)))
    if dist.on and backend == "nccl" and devf["distinct_devices"] < dist.world:
        if dist.rank == 0:
            print(f"bench.py: {dist.world} RCCL ranks ran on {devf['distinct_devices']} distinct GPU(s) "
                  f"({devf['devices']}): refusing to report them as {dist.world} GPUs", file=sys.stderr)
        dist.close()
        return 3
    tune = parse_tune(args.tune) or None

    cfg = dict(WORKLOADS[args.config])
    if args.no_pseudo and cfg.get("pseudo"):
        cfg["pseudo"] = False
        cfg["name"] = cfg["name"].replace(", each over its IPv4 pseudo-header (N x u32 partials)", "") + \
            " (no pseudo-header partials)"
    w = build_workload(cfg, dist.rank, device, tune)
    torch.cuda.synchronize()
    # Setup, not measurement: after data generation the GPU's clocks sit in an
    # idle state and the first ~50 launches run up to 20 % slow (tools/drift.py).
    # Run the workload's own kernel for --settle-s seconds so the W warmup and
    # K timed steps that follow see the steady state a long-running transport
    # loop would.
    settle_until = time.perf_counter() + args.settle_s
    while time.perf_counter() < settle_until:
        for _ in range(10):
            w["step"]()
        torch.cuda.synchronize()

    def ev_pair():
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    wall, launch_ms, own = timed_loop(w["step"], torch.cuda.synchronize, lambda: dist.barrier(dev_id),
                                      args.steps, args.warmup, ev_pair)
    wall_max = dist.max(wall, device)
    stats = dist.gather({"rank": dist.rank, "device": "%s/%s" % (socket.gethostname(), devf["devices"][dist.rank]["pci"]),
                         "wall_s": wall, "own_s": own, "step_ms": launch_ms[0] if launch_ms else None})
    cpu = None
    if dist.world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, w, args.cpu_seconds)
    line = result_line(world=dist.world, steps=args.steps, warmup=args.warmup, wall_max=wall_max,
                       bytes_per_rank_step=w["bytes"], units_total=cfg["n"] * dist.world, workload=cfg["name"],
                       cfg=cfg, launch_ms=launch_ms, alg_bytes_per_launch=w["alg"], cpu_baseline=cpu,
                       # the committed PMC traffic was profiled at the default launch shape
                       traffic=None if tune else load_traffic(
                           f"{args.config}n" if args.no_pseudo and WORKLOADS[args.config].get("pseudo") else args.config), metric=cfg.get("metric", METRIC),
                       launches=w.get("launches", 1), n_gpus=devf["n_gpus"], rank_stats=stats)
    line["backend"] = backend if dist.on else None
    line.update({k: v for k, v in devf.items() if k != "n_gpus"})
    if devf["distinct_devices"] < dist.world:  # gloo rehearsal: ranks share a GPU; n_gpus counts GPUs
        line["rehearsal"] = True
    if tune:
        line["config"]["tune"] = tune
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
