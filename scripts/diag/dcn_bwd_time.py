"""Time tmvs_dcn_backward at the C5 full-resolution head shape (4 views x 576x768, 32 -> CO) with HIP
events; run once per library variant (TMVS_LIB_PATH) for A/B ablations (diagnostic, GPU box)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

from transmvsnet_amd import ops

B, H, W = 4, 576, 768
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(B, H, W, 32, generator=g).cuda()
om = (0.3 * torch.randn(B, 27, H, W, generator=g)).cuda()
for co in (32, 8):
    w = (0.1 * torch.randn(9, co, 32, generator=g)).cuda()
    dy = torch.randn(B, H, W, co, generator=g).cuda()
    dx = torch.zeros_like(x)
    for _ in range(2):
        ops.dcn_backward(x, om, w, dy, dx)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.dcn_backward(x, om, w, dy, dx)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('TMVS_LIB_PATH', 'product')}: CO={co} tmvs_dcn_backward {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
