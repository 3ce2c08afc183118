"""Bitwise A/B of one C5 training step between two library builds (diagnostic, GPU box).

    TMVS_LIB_PATH=variants/X/libtransmvs_hip.so python scripts/diag/train_bits.py OUT.npz
    python scripts/diag/train_bits.py --compare A.npz B.npz

bench.py's C5 setup (768x576, N=4, key-seeded weights, synthetic images / cameras / ground truth);
one eager train_sample step; dumps the flat gradient, the parameters and the BatchNorm running
statistics after the step.
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

import bench  # noqa: E402

torch.cuda.set_device(0)
step, _, m = bench._train_setup(torch.device("cuda", 0))
step()
torch.cuda.synchronize()
out = {"params": torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy(),
       "grads": torch.cat([p.grad.detach().reshape(-1) for p in m.parameters() if p.grad is not None]).cpu().numpy(),
       "running": torch.cat([b.detach().float().reshape(-1) for n, b in m.named_buffers() if "running" in n]).cpu().numpy()}
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1])
