"""Per-kernel HIP-event timing of tmvs_dcn_backward's launches at the C5 full-resolution head shape
(4 views x 576x768, 32 -> 32): runs the op a few times; use under rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

from transmvsnet_amd import ops

B, H, W = 4, 576, 768
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(B, H, W, 32, generator=g).cuda()
om = (0.3 * torch.randn(B, 27, H, W, generator=g)).cuda()
w = (0.1 * torch.randn(9, 32, 32, generator=g)).cuda()
dy = torch.randn(B, H, W, 32, generator=g).cuda()
dx = torch.zeros_like(x)
for _ in range(5):
    ops.dcn_backward(x, om, w, dy, dx)
torch.cuda.synchronize()
print("done")
