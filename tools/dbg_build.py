"""Debug helper: reproduce test_fuzz_tcp_build[case] and report the differing images."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import nsx  # noqa: E402
from oracle import csum_oracle as O  # noqa: E402

case = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rng = np.random.default_rng(4000 + case)
n = int(rng.integers(1, 3000))
P = int(rng.choice([int(rng.integers(0, 40)), 1480, int(rng.integers(0, 3000)), int(rng.integers(0, 9000))]))
uniform = case % 2 == 0
lens = np.full(n, P & ~3 if uniform else P, np.uint64) if uniform else rng.integers(0, P + 1, n).astype(np.uint64)
lead = int(rng.choice([0, 1, 20, 24, 33]))
data_off = np.zeros(n + 1, np.uint64)
np.cumsum(lens, out=data_off[1:])
data_off += np.uint64(lead)
data = rng.integers(0, 256, int(data_off[-1]) + 8, dtype=np.uint8)
out_off = nsx.tcp_layout_host(data_off - np.uint64(lead))
fields = {"src_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
          "dst_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
          "seq_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
          "ack_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
          "offset": np.full(n, 5, np.uint8), "control": rng.integers(0, 256, n).astype(np.uint8),
          "window": rng.integers(0, 1 << 16, n).astype(np.uint16),
          "urgent_ptr": rng.integers(0, 1 << 16, n).astype(np.uint16)}
knobs = dict(kernel=int(rng.choice([0, 2, 3])), segs_per_wave=int(rng.choice([0, 1])),
             blocks_per_cu=int(rng.choice([0, 1, 8])))
print("case", case, "n", n, "P", P, "lead", lead, "knobs", knobs)
import bench  # noqa: E402
for k, v in knobs.items():
    nsx.set_param(bench.PARAMS[k], v)
want, wraw = O.c_go_tcp_build(fields, data, data_off, out_off, None)
dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
f = {k: dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
raw = torch.empty(n, dtype=torch.int16, device="cuda")
nsx.tcp_build_dev(f, dev(data), dev(data_off.view(np.int64)), out, dev(out_off.view(np.int64)), raw=raw)
got = out.cpu().numpy()
print("raw ok", np.array_equal(raw.cpu().numpy().view(np.uint16), wraw), "base%16", out.data_ptr() % 16)
bad = 0
for i in range(n):
    a, b = int(out_off[i]), int(out_off[i + 1])
    if not np.array_equal(got[a:b], want[a:b]):
        d = np.nonzero(got[a:b] != want[a:b])[0]
        W = int(lens[i]) + 20
        print(f"seg {i} off {a} q {(a >> 2) & 3} wire {W} db {int(data_off[i])} first_diff {d[:8]} ndiff {d.size} "
              f"got {got[a + d[0]:a + d[0] + 8]} want {want[a + d[0]:a + d[0] + 8]}")
        bad += 1
        if bad > 12:
            break
print("bad", bad)
