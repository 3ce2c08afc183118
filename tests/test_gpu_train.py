"""CostRegNet training on the GPU: transmvsnet_amd.train's
train-mode forward + HIP backward against torch autograd through the oracle's CostRegNet in train
mode (models/module.py:447-456 with BatchNorm3d batch statistics), at a small shape and the three
C5 stage shapes (BlendedMVS 768x576: 48 x 144x192, 32 x 288x384, 8 x 576x768).

Tolerances (fp32; the GPU sums in a different order than mkldnn / the CPU batch_norm):
  logits: 1e-4 of max|logits|;  every gradient: 1e-3 of its max magnitude;  running statistics:
  1e-5 of their max magnitude (batch variance from fp64 partial sums here).
"""
import numpy as np
import pytest
import torch

from oracle import transmvs_ref as oracle
from tests._util import golden_state_dict
from transmvsnet_amd.model import CostRegNet
from transmvsnet_amd.train import costregnet_params, costregnet_train

pytestmark = pytest.mark.gpu
DEV = "cuda"
PREFIX = "cost_regularization.0."


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("shape", [(1, 8, 32, 40), (2, 8, 16, 24), (1, 48, 144, 192), (1, 32, 288, 384),
                                   (1, 8, 576, 768)])
def test_costregnet_train_forward_backward(shape):
    sd = {k[len(PREFIX):]: v for k, v in golden_state_dict().items() if k.startswith(PREFIX)}
    cr = CostRegNet(1, 8)
    cr.load_state_dict(sd, strict=True)
    cr = cr.to(DEV).train()
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, generator=g) * 0.5
    gout = torch.randn(shape, generator=g)
    xg = x.to(DEV).requires_grad_()
    out = costregnet_train(cr, xg)
    out.backward(gout.to(DEV))
    torch.cuda.synchronize()
    # reference: torch autograd through the oracle in train mode (CPU)
    ref_sd = {k: (v.clone().requires_grad_() if v.is_floating_point() and "running" not in k else v.clone())
              for k, v in sd.items()}
    xc = x.clone().requires_grad_()
    ref = oracle.cost_reg_net(ref_sd, "", xc.unsqueeze(1), training=True)[:, 0]
    ref.backward(gout)
    rep = {"logits": _rel(out, ref), "dx": _rel(xg.grad, xc.grad)}
    assert rep["logits"] < 1e-4, rep
    assert rep["dx"] < 1e-3, rep
    names = [n for n in sd if n.endswith(("conv.weight", "bn.weight", "bn.bias"))] + ["prob.weight"]
    params = dict(zip([f"{n}.{s}" for n in ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7",
                                             "conv9", "conv11") for s in ("conv.weight", "bn.weight", "bn.bias")]
                      + ["prob.weight"], costregnet_params(cr)))
    assert set(params) == set(names)
    worst = max((_rel(params[n].grad, ref_sd[n].grad), n) for n in names)
    rep["worst_param_grad"] = worst
    assert worst[0] < 1e-3, rep
    for n in sd:
        if "running" in n:
            r = _rel(dict(cr.named_buffers())[n], ref_sd[n])
            assert r < 1e-5, (n, r)
    assert int(cr.conv0.bn.num_batches_tracked) == 1 + int(sd["conv0.bn.num_batches_tracked"])
    print(shape, rep)
