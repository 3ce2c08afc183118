"""CostRegNet training-step timing at the C5 stage shapes (BlendedMVS 768x576, batch 1 per GPU):
HIP train-mode forward + backward (transmvsnet_amd.train) vs the same block through PyTorch-ROCm
autograd (the oracle's functional CostRegNet on GPU tensors: MIOpen conv3d + batch_norm), HIP events,
median of 5 after 2 warm-ups."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch

from oracle import transmvs_ref as oracle
from tests._util import golden_state_dict
from transmvsnet_amd.model import CostRegNet
from transmvsnet_amd.train import costregnet_train

P = "cost_regularization.0."
sd = {k[len(P):]: v for k, v in golden_state_dict().items() if k.startswith(P)}


def timed(fn, n=5, warm=2):
    ts = []
    for i in range(n + warm):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= warm:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


tot_hip = tot_torch = 0.0
for shape in [(1, 48, 144, 192), (1, 32, 288, 384), (1, 8, 576, 768)]:
    cr = CostRegNet(1, 8)
    cr.load_state_dict(sd)
    cr = cr.cuda().train()
    x = torch.randn(shape, device="cuda").requires_grad_()
    gout = torch.randn(shape, device="cuda")

    def hip():
        costregnet_train(cr, x).backward(gout)

    gsd = {k: (v.cuda().clone().requires_grad_() if v.is_floating_point() and "running" not in k else v.cuda().clone())
           for k, v in sd.items()}

    def ref():
        oracle.cost_reg_net(gsd, "", x.unsqueeze(1), training=True)[:, 0].backward(gout)

    th, tr = timed(hip), timed(ref)
    tot_hip += th
    tot_torch += tr
    vox = shape[1] * shape[2] * shape[3]
    print(f"{shape}: HIP fwd+bwd {th:.2f} ms ({3 * 6912 * vox / th / 1e9:.1f} TFLOP/s)   "
          f"PyTorch-ROCm autograd {tr:.2f} ms", flush=True)
print(f"CostRegNet training step, 3 stages: HIP {tot_hip:.2f} ms, PyTorch-ROCm {tot_torch:.2f} ms")
