"""Device-to-device copy ceiling as a library gives it: torch.Tensor.copy_ of f1's bytes (1M x 1500 B), the
same read + write volume as workload 6's wire images (DESIGN.md §6 "Practical ceilings")."""
import torch, time
n = 1 << 20
W = 1500
a = torch.empty(n * W, dtype=torch.uint8, device="cuda").random_(0, 255)
b = torch.empty_like(a)
a4, b4 = a.view(torch.int32), b.view(torch.int32)
for name, f in (("copy_u8", lambda: b.copy_(a)), ("copy_i32", lambda: b4.copy_(a4))):
    for _ in range(20): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 100
    print(name, f"{ms:.4f} ms", f"{2 * n * W / ms / 1e9:.3f} TB/s (read+write)")
