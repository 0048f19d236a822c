"""Multi-rank logic on CPU with gloo, world_size 2: bench.py's barrier-bracketed
timed loop and max-over-ranks reduction, the whole-job value, and the shard plan
(nsx_shard_plan) that splits a batch over GPUs with no exchange step. The
per-rank "step" here is the CPU oracle standing in for the GPU kernel (the
path shards without a collective, so the N>1 logic is independent of the
device)."""
import json
import multiprocessing as mp
import os
import socket
import time

import numpy as np
import pytest

from conftest import ROOT

GIB = float(1 << 30)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import bench
        import nsx
        from oracle import csum_oracle as O
        d = bench.Dist("gloo")
        assert d.on and d.world == world and d.rank == rank
        # Weak scaling: every rank checksums its own batch (seed 0x1071 + rank).
        n, L = 512, 1500
        buf = O.c_splitmix64(0x1071 + rank, n * L)
        res = {}

        def step():
            res["out"] = O.c_batch(buf, n, stride=L, seg_len=L, threads=1)
            if rank == 1:  # a slow GPU: its own rate must show it
                time.sleep(0.05)

        wall, launch_ms, own = bench.timed_loop(step, lambda: None, d.barrier, steps=4, warmup=1)
        wmax = d.max(wall)
        stats = d.gather({"rank": rank, "device": f"cpu{rank}", "wall_s": wall, "own_s": own, "step_ms": 0.5 + rank})
        line = bench.result_line(world=world, steps=4, warmup=1, wall_max=wmax, bytes_per_rank_step=n * L,
                                 units_total=n * world, workload="gloo-test", cfg={"n": n, "seed": 0x1071},
                                 launch_ms=launch_ms, alg_bytes_per_launch=n * L + 2 * n, cpu_baseline=None,
                                 traffic=None, rank_stats=stats)
        # Sharded host batch: a ragged batch split by byte count, each rank does its shard.
        rng = np.random.default_rng(0x1072)
        lens = rng.integers(64, 9001, 3001).astype(np.uint64)
        offs = np.zeros(lens.size + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        rb = O.c_splitmix64(0x1072, int(offs[-1]))
        bounds = nsx.shard_plan(lens.size, world, offs)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        mine = O.c_batch(rb, hi - lo, offsets=np.ascontiguousarray(offs[lo:hi + 1]))
        import torch.distributed as dist
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, mine.tolist()))
        full = O.c_batch(rb, lens.size, offsets=offs)
        stitched = [x for _, _, part in sorted(gathered) for x in part]
        q.put(json.dumps({"rank": rank, "wall": wall, "own": own, "wmax": wmax, "value": line["value"],
                          "value_per_gpu_mean": line["value_per_gpu_mean"], "per_gpu": line["per_gpu"],
                          "n_gpus": line["n_gpus"], "stitched_ok": stitched == full.tolist(),
                          "sizes": [int(offs[b2] - offs[b1]) for b1, b2 in zip(bounds[:-1], bounds[1:])]}))
        d.close()
    except Exception as e:  # surface worker failures to the parent
        q.put(json.dumps({"rank": rank, "error": repr(e)}))
        raise


def test_bench_dist_logic_gloo_ws2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [json.loads(q.get(timeout=240)) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in results:
        assert "error" not in r, r
    by = {r["rank"]: r for r in results}
    wmax = max(r["wall"] for r in results)
    for r in results:
        assert r["wmax"] == pytest.approx(wmax)      # MAX over ranks, identical everywhere
        assert r["n_gpus"] == 2
        assert r["value"] == pytest.approx(round(2 * 512 * 1500 * 4 / wmax / GIB, 3))  # whole-job bytes
        assert r["value_per_gpu_mean"] == pytest.approx(r["value"] / 2, abs=1e-3)      # mean per GPU (3 decimals)
        # every rank's own rate from its own clock, in rank order (BASELINE config 5: per-GPU and aggregate)
        per = r["per_gpu"]
        assert [p["rank"] for p in per] == [0, 1] and [p["device"] for p in per] == ["cpu0", "cpu1"]
        for p in per:
            # (gib_s is rounded to 3 decimals: at ~0.3 GiB/s that is up to 0.2%, so compare absolutely too)
            assert p["gib_s"] == pytest.approx(512 * 1500 * 4 / by[p["rank"]]["own"] / GIB, rel=1e-3, abs=6e-4)
            assert p["gib_s"] >= r["value"] / 2 - 1e-3                               # no rank slower than the max
            assert by[p["rank"]]["own"] <= by[p["rank"]]["wall"] + 1e-9                # own clock closes first
        assert per[1]["gib_s"] < 0.8 * per[0]["gib_s"]  # the slow rank shows in its own rate
        assert per[0]["kernel_ms"] == 0.5 and per[1]["kernel_ms"] == 1.5
        assert per[0]["roofline_frac"] == pytest.approx((512 * 1502) / 0.5e-3 / 1e9 / 8000, abs=1e-4)
        assert r["stitched_ok"]                      # shards cover the batch exactly once
    sizes = by[0]["sizes"]
    assert abs(sizes[0] - sizes[1]) <= 9000          # byte-balanced split
