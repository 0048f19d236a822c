import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "network-stack_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch, nsx, bench
cfg = bench.WORKLOADS[6]
w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
w["step"]()  # 1M wire images of 1500 B
n = cfg["n"]
offs = w["out_off"]
out = nsx.tcp_parse_dev(w["wire"], offs)
for _ in range(20): nsx.tcp_parse_dev(w["wire"], offs, fields=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(100): nsx.tcp_parse_dev(w["wire"], offs, fields=out)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 100
st = out["status"].cpu().numpy()
print(f"parse 1M built images: {ms:.4f} ms/launch, {n / ms / 1e6:.1f} G segments/s, status ok {int((st == 0).sum())}/{n}")
seq = out["seq_num"].cpu().numpy().view(np.uint32)
want = w["fields"]["seq_num"].cpu().numpy().view(np.uint32)
print("seq round trip", bool(np.array_equal(seq, want)))
