"""tmvs_warp_corr at DTU size, stages 2 / 3 (the row-pair kernel), with the source features in the plain
NHWC layout and in the tap-pair layout (TMVS_WARP_SRC_PAIRED, ops.pair_rows): HIP-event medians of 20
launches each, alternating, and the similarity volumes compared bit for bit.
    python scripts/diag/warp_paired.py"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from transmvsnet_amd import ops, synthetic  # noqa: E402

DEV = "cpu" if os.environ.get("TMVS_DRYRUN") else "cuda"
H, W, N = 864, 1152, 5
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
g = torch.Generator().manual_seed(3)
for s, (c, d, sc) in enumerate(((16, 32, 2), (8, 8, 1)), start=1):
    h, w = H // sc, W // sc
    ref = torch.randn(1, h, w, c, generator=g).to(DEV)
    src = torch.randn(1, N - 1, h, w, c, generator=g).to(DEV)
    cur = torch.rand(1, 1, h, w, generator=g) * 477 + 425
    hyp = (cur + torch.arange(d).view(1, d, 1, 1) * 2.5 - d * 1.25).contiguous().to(DEV)
    rows = ops.proj_rows(proj[f"stage{s + 1}"])
    vw = torch.rand(1, N - 1, h, w, generator=g).to(DEV)
    srcp = ops.pair_rows(src[0].contiguous()).unsqueeze(0)
    runs = {"plain": lambda: ops.warp_corr(ref, src, rows, hyp, view_w_in=vw, vw_shift=0)[0],
            "paired": lambda: ops.warp_corr(ref, srcp, rows, hyp, view_w_in=vw, vw_shift=0, src_paired=True)[0]}
    outs, ts = {}, {k: [] for k in runs}
    for it in range(25):
        for k, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            outs[k] = fn()
            e1.record()
            torch.cuda.synchronize()
            if it >= 5:
                ts[k].append(e0.elapsed_time(e1) * 1e3)
    same = torch.equal(outs["plain"], outs["paired"])
    print(f"stage {s + 1}: plain {np.median(ts['plain']):.1f} us, paired {np.median(ts['paired']):.1f} us, "
          f"bitwise {'equal' if same else 'DIFFERENT'}", flush=True)
    if not same:
        print("  max |diff|", float((outs["plain"] - outs["paired"]).abs().max()))
