"""CostRegNet training on the GPU: transmvsnet_amd.train's
train-mode forward + HIP backward against torch autograd through the oracle's CostRegNet in train
mode (models/module.py:447-456 with BatchNorm3d batch statistics), at a small shape and the three
C5 stage shapes (BlendedMVS 768x576: 48 x 144x192, 32 x 288x384, 8 x 576x768).

The reference is evaluated twice on the CPU: in fp32 (what the reference computes) and in fp64
(the exact value). At the C5 sizes the fp32 reference's own gradients are 0.5-1.2 % (of their max
magnitude) away from the fp64 ones (BatchNorm's backward subtracts batch means of 1e5-1e6 terms;
measured: dx 4.7e-3 at 48x144x192, 1.2e-2 at 8x576x768), so the gradients are judged against fp64:
  logits: 1e-4 of max|logits| against the fp32 reference;
  every gradient (dx, each weight / gamma / beta): error against fp64 <= max(1e-4, twice the fp32
  reference's own error against fp64), all relative to the quantity's max magnitude (measured:
  the GPU's error is the reference's to within +-30 %, profiles/r05e/pytest_train.log);
  running statistics: 1e-5 of their max magnitude.
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
    # reference: torch autograd through the oracle in train mode (CPU), fp32 and fp64
    refs = {}
    for dt in (torch.float32, torch.float64):
        r_sd = {k: (v.to(dt).clone().requires_grad_() if v.is_floating_point() and "running" not in k
                    else (v.to(dt).clone() if v.is_floating_point() else v.clone())) for k, v in sd.items()}
        xc = x.to(dt).clone().requires_grad_()
        r = oracle.cost_reg_net(r_sd, "", xc.unsqueeze(1), training=True)[:, 0]
        r.backward(gout.to(dt))
        refs[dt] = (r, xc.grad, r_sd)
    ref, ref_dx, ref_sd = refs[torch.float32]
    ex, ex_dx, ex_sd = refs[torch.float64]
    rep = {"logits": _rel(out, ref)}
    assert rep["logits"] < 1e-4, rep
    names = [n for n in sd if n.endswith(("conv.weight", "bn.weight", "bn.bias"))] + ["prob.weight"]
    params = dict(zip([f"{n}.{s}" for n in ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7",
                                             "conv9", "conv11") for s in ("conv.weight", "bn.weight", "bn.bias")]
                      + ["prob.weight"], costregnet_params(cr)))
    assert set(params) == set(names)
    checks = [("dx", xg.grad, ref_dx, ex_dx)] + [(n, params[n].grad, ref_sd[n].grad, ex_sd[n].grad) for n in names]
    worst = (0.0, None, 0.0)
    for n, got, r32, r64 in checks:
        e_gpu, e_ref = _rel(got, r64), _rel(r32, r64)
        assert e_gpu <= max(1e-4, 2.0 * e_ref), (n, e_gpu, e_ref)
        worst = max(worst, (e_gpu, n, e_ref))
    rep["worst_grad_vs_fp64 (gpu, name, fp32 reference)"] = worst
    rep["dx_vs_fp64 (gpu, fp32 reference)"] = (_rel(xg.grad, ex_dx), _rel(ref_dx, ex_dx))
    for n in sd:
        if "running" in n:
            r = _rel(dict(cr.named_buffers())[n], ref_sd[n])
            assert r < 1e-5, (n, r)
    assert int(cr.conv0.bn.num_batches_tracked) == 1 + int(sd["conv0.bn.num_batches_tracked"])
    print(shape, rep)
