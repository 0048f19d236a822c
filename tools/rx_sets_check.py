"""Receive pass: runs of 1 vs 4 frame sets give identical masks (and raw sums) over several frame mixes."""
import sys
import torch
sys.path[:0] = [".", "network-stack_amd"]
import bench as B
torch.cuda.set_device(0)
bad = 0
for c in (10, 11):
    for n, lo, hi in ((1 << 20, 40, 1500), (1000003, 40, 100), (300001, 40, 300), (777, 40, 60), (65, 40, 90)):
        lo, hi = (max(lo, 60), max(hi, 80)) if c == 11 else (lo, hi)  # IPv6 frames hold a 40 B header + 20 B TCP
        cfg = dict(B.WORKLOADS[c]); cfg.update(n=n, lo=lo, hi=hi)
        w = B.build_workload(cfg, 0, torch.device("cuda", 0))
        outs = []
        for sets in (0, 1, 4):
            w["out"].fill_(-1)
            w["step_for"](dict(segs_per_wave=sets))()
            torch.cuda.synchronize()
            outs.append(w["out"].clone())
        ok = torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
        bad += not ok
        print(c, n, lo, hi, ok, flush=True)
sys.exit(1 if bad else 0)
