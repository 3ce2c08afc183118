"""Write-only and copy HBM bandwidth with torch kernels (reference points for store-bound kernels)."""
import torch

n = 256 * 1024 * 1024 // 4
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
for name, fn, nbytes in (("fill", lambda: a.fill_(1.0), 4 * n), ("copy", lambda: b.copy_(a), 8 * n),
                         ("zero", lambda: a.zero_(), 4 * n)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: {ms * 1e3:.1f} us  {nbytes / ms / 1e6:.0f} GB/s")
