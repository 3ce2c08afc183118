"""Time tmvs_warp_corr_backward at the three C5 stage shapes (N=4: 3 source views), HIP events.
Usage: python scripts/diag/warp_bwd_time.py   (TMVS_LIB_PATH selects a library variant)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

from transmvsnet_amd import ops, synthetic

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
H, W, V = 576, 768, 3
proj = synthetic.synthetic_cameras(V + 1, H, W, seed=6)
g = torch.Generator().manual_seed(0)
res = []
for s, (c, d, scale) in enumerate(((32, 48, 4), (16, 32, 2), (8, 8, 1))):
    h, w = H // scale, W // scale
    ref = torch.randn(h, w, c, generator=g).to(dev)
    src = torch.randn(V, h, w, c, generator=g).to(dev)
    hyp = (425.0 + 510.0 * torch.rand(d, h, w, generator=g)).sort(0)[0].contiguous().to(dev)
    dsim = torch.randn(V, d, h, w, generator=g).to(dev)
    rows = ops.proj_rows(proj[f"stage{s + 1}"])[0]
    for _ in range(2):
        ops.warp_corr_backward(ref, src, rows, hyp, dsim)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.warp_corr_backward(ref, src, rows, hyp, dsim)
    e1.record()
    torch.cuda.synchronize()
    res.append(round(e0.elapsed_time(e1) / 10, 3))
print(os.environ.get("TMVS_LIB_PATH", "default"), "warp backward ms per stage (C5, N=4):", res)
