"""bench.py without a GPU: the rank launcher (`--gpus 2` starts two gloo ranks itself
and reports n_gpus 2; a WORLD_SIZE that disagrees with --gpus is an error), the CPU
baseline leg on every host core with its 1-thread rate beside it (checked against
known-correct outputs standing in for the GPU's), the best-CPU extra lines, and
the per-launch reporting of windowed steps."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from conftest import ROOT
from oracle import csum_oracle as O

torch = pytest.importorskip("torch")


def _bench(*args, env_extra=None, timeout=240):
    env = dict(os.environ, **(env_extra or {}))
    env.pop("WORLD_SIZE", None) if not (env_extra and "WORLD_SIZE" in env_extra) else None
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_gpus_2_launches_two_ranks_itself():
    """`bench.py --gpus N` with no launcher must run N ranks, not one rank on GPU 0."""
    r = _bench("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    # two ranks, no GPU behind them: n_gpus counts distinct devices (0), the rank count is separate
    assert line["ranks"] == 2 and line["dry_run"] and line["rehearsal"]
    assert line["n_gpus"] == 0 and line["distinct_devices"] == 0 and len(line["devices"]) == 2
    assert line["config"]["units_per_step_all_gpus"] == 2 * line["config"]["units_per_gpu"]
    # each rank's own rate (BASELINE config 5: per-GPU and aggregate GiB/s): one entry per rank, its own wall
    per = line["per_gpu"]
    assert [p["rank"] for p in per] == [0, 1]
    for p in per:
        assert set(p) == {"rank", "device", "gib_s", "own_s", "wall_s", "kernel_ms", "roofline_frac"}
        assert p["gib_s"] > 0 and 0 < p["own_s"] <= p["wall_s"]
    assert line["value_per_gpu_mean"] == pytest.approx(line["value"] / 2, abs=1e-3)
    assert min(p["gib_s"] for p in per) >= line["value"] / 2 - 1e-3  # the aggregate uses the slowest wall


def test_per_gpu_rate_uses_each_ranks_own_clock():
    """the barrier-closed wall is the slowest rank's time on every rank, so a per-GPU rate from it
    cannot show a slow GPU; per_gpu uses each rank's own clock (own_s, closed before the closing barrier)."""
    stats = [{"rank": r, "device": f"h/{r}", "wall_s": 1.25, "own_s": 1.0 if r != 1 else 1.25, "step_ms": 0.2}
             for r in range(2)]
    line = bench.result_line(world=2, steps=10, warmup=1, wall_max=1.25, bytes_per_rank_step=1 << 30,
                             units_total=2, workload="w", cfg={"n": 1, "seed": 1}, launch_ms=[0.2],
                             alg_bytes_per_launch=1 << 30, cpu_baseline=None, traffic=None, rank_stats=stats)
    assert [p["gib_s"] for p in line["per_gpu"]] == [10.0, 8.0]
    assert line["value"] == pytest.approx(16.0)


def test_per_gpu_entries_show_a_slow_gpu():
    """a SCALE reader must see a slow GPU from the line alone."""
    stats = [{"rank": r, "device": f"h/{r}", "wall_s": 1.0 if r != 2 else 1.25, "step_ms": 0.2 if r != 2 else 0.25}
             for r in range(4)]
    line = bench.result_line(world=4, steps=10, warmup=1, wall_max=1.25, bytes_per_rank_step=1 << 30,
                             units_total=4, workload="w", cfg={"n": 1, "seed": 1}, launch_ms=[0.2],
                             alg_bytes_per_launch=1 << 30, cpu_baseline=None, traffic=None, rank_stats=stats)
    per = line["per_gpu"]
    assert [p["gib_s"] for p in per] == [10.0, 10.0, 8.0, 10.0]
    assert per[2]["roofline_frac"] < per[0]["roofline_frac"]
    assert line["value"] == pytest.approx(32.0)  # 4 GiB x 10 steps / the slowest rank's 1.25 s


def test_per_gpu_roofline_of_a_windowed_step_matches_the_line():
    """Config 5's steps are 16 back-to-back launches: each rank's roofline fraction is per launch, like the line's
    (round 4's first 2-rank rehearsal printed the line's fraction divided by 16 again)."""
    stats = [{"rank": r, "device": f"h/{r}", "wall_s": 0.036, "step_ms": 3.2} for r in range(2)]
    line = bench.result_line(world=2, steps=10, warmup=1, wall_max=0.036, bytes_per_rank_step=16 * 1500,
                             units_total=32, workload="w", cfg={"n": 16, "seed": 1}, launch_ms=[3.2],
                             alg_bytes_per_launch=16 * 1600, cpu_baseline=None, traffic=None, launches=16,
                             rank_stats=stats)
    for p in line["per_gpu"]:
        assert p["kernel_ms"] == pytest.approx(0.2)
        assert p["roofline_frac"] == pytest.approx(line["roofline"]["frac"], abs=1e-4)


def test_device_fields_count_distinct_gpus():
    """a SCALE reader must see from the line alone how many physical GPUs the ranks ran on."""
    a = {"host": "h", "local_device": 0, "pci": "0000:05:00", "uuid": "u0", "key": "h/0000:05:00/u0"}
    b = dict(a, local_device=1, pci="0000:15:00", uuid="u1", key="h/0000:15:00/u1")
    two = bench.device_fields([a, b])
    assert two["n_gpus"] == 2 and two["ranks"] == 2 and [d["pci"] for d in two["devices"]] == [a["pci"], b["pci"]]
    shared = bench.device_fields([a, dict(a)])  # two ranks on one GPU (a rehearsal)
    assert shared["n_gpus"] == 1 and shared["ranks"] == 2 and shared["distinct_devices"] == 1
    line = bench.result_line(world=2, steps=1, warmup=0, wall_max=1.0, bytes_per_rank_step=10, units_total=2,
                             workload="w", cfg={"n": 1, "seed": 1}, launch_ms=[], alg_bytes_per_launch=10,
                             cpu_baseline=None, traffic=None, n_gpus=shared["n_gpus"])
    assert line["n_gpus"] == 1 and line["ranks"] == 2


def test_world_size_disagreeing_with_gpus_is_an_error():
    r = _bench("--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0", env_extra={"WORLD_SIZE": "1"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_host_cores_share():
    c = bench.host_cores()
    assert 1 <= c["threads"] <= c["affinity_cpus"] <= c["host_cpus"]


def _fixed_case(n=4096, L=1500):
    buf = O.c_splitmix64(0x1071, n * L)
    out = O.c_batch(buf, n, stride=L, seg_len=L)
    cfg = dict(kind="fixed", n=n, seg_len=L, stride=L, seed=0x1071)
    return cfg, {"buf": torch.from_numpy(buf), "out": torch.from_numpy(out.view(np.int16))}


def test_cpu_baseline_fixed_all_cores_and_single_thread():
    cfg, w = _fixed_case()
    res = bench.cpu_baseline(cfg, w, 0.2)
    assert res["sample_parity_vs_gpu"] and res["value"] > 0 and res["cores"] == bench.host_cores()["threads"]
    assert res["single_thread"]["cores"] == 1 and res["single_thread"]["value"] > 0
    pin = res["threads_diagnostics"]["pinned_cpus"]  # one CPU per worker, distinct, inside the affinity set
    assert pin is None or (len(pin) == res["cores"] and len(set(pin)) == len(pin)
                           and set(pin) <= os.sched_getaffinity(0))
    for k in ("optimized_1_thread", "optimized_threads"):
        assert res["extra"][k]["parity"] and res["extra"][k]["value"] > 0, k
    w["out"][5] ^= 1  # a wrong "GPU" result is caught
    assert not bench.cpu_baseline(cfg, w, 0.05)["sample_parity_vs_gpu"]


def test_cpu_baseline_ragged_byte_balanced():
    rng = np.random.default_rng(0x1072)
    n = 3000
    lens = rng.integers(64, 9001, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    buf = O.c_splitmix64(0x1072, int(offs[-1]))
    out = O.c_batch(buf, n, offsets=offs)
    cfg = dict(kind="ragged", n=n, seed=0x1072)
    res = bench.cpu_baseline(cfg, {"buf": torch.from_numpy(buf), "out": torch.from_numpy(out.view(np.int16)),
                                   "offsets": offs}, 0.2)
    assert res["sample_parity_vs_gpu"] and res["value"] > 0


@pytest.mark.parametrize("mask", [False, True])
def test_cpu_baseline_ipv4_headers(mask):
    n, H = 64 * 500 + 7, 20
    buf = O.c_splitmix64(0x1075, n * H)
    buf[::H] = 0x45
    raw = O.c_batch(buf, n, stride=H, seg_len=H)
    # make about half valid: any header whose sum is 0xFFFF is valid; force some by setting the field
    if mask:
        valid = raw == 0xFFFF
        out = np.packbits(np.concatenate([valid, np.zeros(-n % 64, bool)]), bitorder="little").view(np.uint64)
        outt = torch.from_numpy(out.view(np.int64))
    else:
        outt = torch.from_numpy(raw.view(np.int16))
    cfg = dict(kind="ipv4_hdr", n=n, hdr=H, mask=mask, seed=0x1075)
    res = bench.cpu_baseline(cfg, {"buf": torch.from_numpy(buf), "out": outt}, 0.1)
    assert res["sample_parity_vs_gpu"] and res["value"] > 0


def test_result_line_per_launch_with_windows():
    line = bench.result_line(world=1, steps=10, warmup=1, wall_max=0.036, bytes_per_rank_step=16 * 1500,
                             units_total=16, workload="w", cfg={"n": 16, "seed": 1}, launch_ms=[3.2, 3.2],
                             alg_bytes_per_launch=16 * 1600, cpu_baseline=None, traffic=None, launches=16)
    assert line["roofline"]["alg_bytes_per_launch"] == 1600
    assert line["roofline"]["launches_per_step"] == 16
    assert abs(line["kernel_ms_mean"] - 0.2) < 1e-9


def test_cpu_baseline_rx_frames():
    """Workload 10's CPU leg: the Go-faithful per-frame receive check on every host core, byte-balanced in
    whole 64-frame mask words, against a known-correct mask standing in for the GPU's."""
    import _rx
    rng = np.random.default_rng(0x10)
    buf, offs, _ = _rx.batch(rng, 64 * 40 + 17, lead=0, max_payload=600)
    mask, _, _ = O.c_rx_ipv4_tcp(buf, offs)
    cfg = dict(kind="rx", n=offs.size - 1, seed=1)
    w = {"buf": torch.from_numpy(buf), "out": torch.from_numpy(mask.view(np.int64)), "offsets": offs}
    res = bench.cpu_baseline(cfg, w, 0.2)
    assert res["sample_parity_vs_gpu"] and res["value"] > 0
    w["out"][3] ^= 1 << 5
    assert not bench.cpu_baseline(cfg, w, 0.05)["sample_parity_vs_gpu"]


def test_config2_pseudo_header_partials_in_the_workload_and_the_line():
    """config 2 (and 5) are measured over N x u32 pseudo-header partials, counted
    in the algorithmic bytes; --no-pseudo names the partial-less line and finds its own traffic profile."""
    for c in (2, 5):
        assert bench.WORKLOADS[c]["pseudo"] and "pseudo-header" in bench.WORKLOADS[c]["name"]
    args = bench.parse_args(["--config", "2", "--no-pseudo"])
    assert args.no_pseudo and not bench.parse_args([]).no_pseudo
    assert bench.load_traffic("2")["bytes_per_launch"] > 0          # with partials (round 4 profile)
    assert bench.load_traffic("2n")["source"].endswith("traffic_config2n.json")
    assert bench.load_traffic("99") is None
