"""Time tmvs_warp_corr per stage at DTU size (HIP events, median of 20) for the library in TMVS_LIB_PATH.
    python scripts/diag/warp_time.py"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from transmvsnet_amd import ops, synthetic
DEV = "cuda"

H, W, N = 864, 1152, 5
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
g = torch.Generator().manual_seed(3)
out = []
for s, (c, d, sc) in enumerate(((32, 48, 4), (16, 32, 2), (8, 8, 1))):
    h, w = H // sc, W // sc
    ref = torch.randn(1, h, w, c, generator=g).to(DEV)
    src = torch.randn(1, N - 1, h, w, c, generator=g).to(DEV)
    if s == 0:
        hyp = torch.linspace(425, 902.5, d).view(1, d, 1, 1).expand(1, d, h, w).contiguous().to(DEV)
    else:
        cur = torch.rand(1, 1, h, w, generator=g) * 477 + 425
        hyp = (cur + torch.arange(d).view(1, d, 1, 1) * 2.5 - d * 1.25).contiguous().to(DEV)
    rows = ops.proj_rows(proj[f"stage{s + 1}"])
    kw = dict(pw_params=np.random.rand(201).astype(np.float32)) if s == 0 else dict(
        view_w_in=torch.rand(1, N - 1, h, w).to(DEV), vw_shift=0)
    ts = []
    for it in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.warp_corr(ref, src, rows, hyp, **kw)
        e1.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(e0.elapsed_time(e1))
    out.append(np.median(ts) * 1e3)
print(os.environ.get("TMVS_LIB_PATH", "default"), "us per stage:", [round(x, 1) for x in out])
