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
