"""Bitwise A/B of tmvs_dcn_backward between two library builds (run once per build; diagnostic, GPU box).

    TMVS_LIB_PATH=variants/X/libtransmvs_hip.so python scripts/diag/dcn_bwd_bits.py OUT.npz
    python scripts/diag/dcn_bwd_bits.py --compare A.npz B.npz

C5 full-resolution head shape (4 views x 576x768, 32 -> CO), offsets of std 0.3 px (every corner inside
the block windows: the in-window sums are order-independent) and all-zero offsets; dx, d offset/mask, dW.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    worst = 0
    for k in a.files:
        n = int((a[k] != b[k]).sum())
        worst = max(worst, n)
        print(f"{k:16s} differing {n:10d} of {a[k].size:10d}  max|d| {np.abs(a[k].astype(np.float64) - b[k]).max():.3e}")
    print("BITWISE IDENTICAL" if worst == 0 else "DIFFERENT")
    sys.exit(0)
import torch  # noqa: E402

from transmvsnet_amd import ops  # noqa: E402

B, H, W = 4, 576, 768
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(B, H, W, 32, generator=g).cuda()
out = {}
for tag, scale in (("off03", 0.3), ("off0", 0.0)):
    om = (scale * torch.randn(B, 27, H, W, generator=g)).cuda()
    for co in (32, 8):
        w = (0.1 * torch.randn(9, co, 32, generator=g)).cuda()
        dy = torch.randn(B, H, W, co, generator=g).cuda()
        dx = torch.zeros_like(x)
        dom, dw = ops.dcn_backward(x, om, w, dy, dx)
        torch.cuda.synchronize()
        out[f"{tag}_co{co}_dx"] = dx.cpu().numpy()
        out[f"{tag}_co{co}_dom"] = dom.cpu().numpy()
        out[f"{tag}_co{co}_dw"] = dw.cpu().numpy()
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1])
