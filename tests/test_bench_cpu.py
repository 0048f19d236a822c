"""bench.py's CPU reference lines run without a GPU: the multi-thread
Go-faithful and vectorised restatements agree with the 1-thread oracle output
on the same sample (their `parity` flags), and report positive rates."""
import numpy as np

import bench
from oracle import csum_oracle as O


def test_cpu_extra_lines_parity():
    L = S = 1500
    m = 4096
    sample = O.c_splitmix64(0x1071, m * S)
    want = O.c_batch(sample, m, stride=S, seg_len=L)
    res = bench.cpu_extra_lines(O.c_oracle(), sample, S, L, m, want, 0.05)
    for k in ("go_faithful_threads", "optimized_1_thread", "optimized_threads"):
        assert res[k]["parity"] and res[k]["value"] > 0, k


def test_fixed_launches_mirrors_the_auto_window():
    """Config 5's 25 GB batch runs as 16 windows of 1M segments; configs 2 and 4 in one launch."""
    assert bench.fixed_launches(1 << 24, 1500, 1500) == 16
    assert bench.fixed_launches(1 << 20, 1500, 1500) == 1
    assert bench.fixed_launches(1 << 18, 65536, 65536) == 1  # long-segment path: never windowed
    assert bench.fixed_launches(1 << 22, 1500, 1500) == 4


def test_result_line_per_launch_with_windows():
    line = bench.result_line(world=1, steps=10, warmup=1, wall_max=0.036, bytes_per_rank_step=16 * 1500,
                             units_total=16, workload="w", cfg={"n": 16, "seed": 1}, launch_ms=[3.2, 3.2],
                             alg_bytes_per_launch=16 * 1600, cpu_baseline=None, traffic=None, launches=16)
    assert line["roofline"]["alg_bytes_per_launch"] == 1600
    assert line["roofline"]["launches_per_step"] == 16
    assert abs(line["kernel_ms_mean"] - 0.2) < 1e-9


def test_fixed_launches_follows_the_knobs():
    assert bench.fixed_launches(1 << 24, 1500, 1500, window_bytes=-1) == 1
    assert bench.fixed_launches(4096, 1500, 1500, window_bytes=1500 * 1000) == 5
    assert bench.fixed_launches(1 << 24, 1500, 1500, kernel=2) == 1  # per-segment kernel: no windows
    assert bench.fixed_launches(1 << 24, 1501, 1501) == 16  # unaligned batches take the same path
