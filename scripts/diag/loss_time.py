"""tmvs_entropy_loss (with the logit gradient) at the DTU stage sizes (B=1, 864x1152, 48/32/8),
HIP events, median of 20 after 3 warm-ups; HBM bytes per call = prob read + hyp read + grad write
(+ gt/mask reads, per-pixel outputs)."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from transmvsnet_amd import ops
for d, h, w in ((48, 216, 288), (32, 432, 576), (8, 864, 1152)):
    g = torch.Generator(device="cuda").manual_seed(d)
    prob = torch.softmax(3 * torch.randn(1, d, h, w, device="cuda", generator=g), 1)
    dv = (500 + torch.rand(1, 1, h, w, device="cuda", generator=g) + torch.arange(d, device="cuda").reshape(1, d, 1, 1)).contiguous()
    gt = 500 + d * torch.rand(1, h, w, device="cuda", generator=g)
    mask = (torch.rand(1, h, w, device="cuda", generator=g) > 0.2).float()
    ts = []
    for i in range(23):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.entropy_loss(prob, dv, gt, mask, grad_scale=2.0, want_grad=True)
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    us = float(np.median(ts))
    nbytes = 4 * (3 * d * h * w + 4 * h * w)
    print(f"D={d} {h}x{w}: {us:.1f} us (3 launches + memset), {nbytes / 1e6:.1f} MB -> {nbytes / us / 1e3:.0f} GB/s")
