"""HIP training losses (csrc/loss.hip via transmvsnet_amd.loss) against the reference's outputs
(tests/golden/loss.npz) and, at DTU size, against torch fp32 on the GPU plus size-independent
properties. Tolerances: loss values rel 2e-6 (fp64 block combine vs torch's reduction order);
gradients |err| <= 2e-6 * max|grad| + rel 1e-5 (closed-form softmax backward vs autograd);
WTA depth / confidence / argmin-argmax indices bit-exact."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "loss.npz")
STAGES = ("stage1", "stage2", "stage3")


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as z:
        return {k: z[k] for k in z.files}


def _inputs(gold, p, dev):
    t = lambda k: torch.from_numpy(gold[f"{p}_{k}"])  # noqa: E731
    inputs, gts, masks = {}, {}, {}
    for s in STAGES:
        prob = t(f"{s}_prob")  # the reference's own softmax output (host softmax differs by ulps across CPUs)
        inputs[s] = {"prob_volume": prob.to(dev), "depth_values": t(f"{s}_dv").to(dev)}
        gts[s] = t(f"{s}_gt").to(dev)
        masks[s] = t(f"{s}_mask").to(dev)
    return inputs, gts, masks


def _grad_close(got, want):
    got = got.cpu().numpy()
    scale = np.abs(want).max()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=2e-6 * scale)


def test_trans_mvsnet_loss_vs_reference(gold):
    from transmvsnet_amd import loss
    inputs, gts, masks = _inputs(gold, "t", "cuda")
    total, depth_loss, total_entropy, depth_entropy, grads = loss.trans_mvsnet_loss(
        inputs, gts, masks, dlossw=[0.5, 1.0, 2.0], return_grad=True)
    np.testing.assert_allclose(total.item(), gold["t_total"], rtol=2e-6)
    np.testing.assert_allclose(total_entropy.item(), gold["t_total_entropy"], rtol=2e-6)
    np.testing.assert_allclose(depth_loss.item(), gold["t_depth_loss"], rtol=2e-6)
    assert np.array_equal(depth_entropy.cpu().numpy(), gold["t_depth_entropy"])
    for s in STAGES:
        _grad_close(grads[s], gold[f"t_{s}_grad"])
    # the empty-mask batch element of stage 1 contributes nothing and gets no gradient
    assert not grads["stage1"][1].any()


def test_entropy_loss_prob_map_vs_reference(gold):
    from transmvsnet_amd import loss
    inputs, gts, masks = _inputs(gold, "t", "cuda")
    l2, wta, conf = loss.entropy_loss(inputs["stage2"]["prob_volume"], gts["stage2"], masks["stage2"] > 0.5,
                                      inputs["stage2"]["depth_values"], return_prob_map=True)
    np.testing.assert_allclose(l2.item(), gold["e_loss"], rtol=2e-6)
    assert np.array_equal(wta.cpu().numpy(), gold["e_wta"])
    assert np.array_equal(conf.cpu().numpy(), gold["e_conf"])


def test_focal_loss_bld_vs_reference(gold):
    from transmvsnet_amd import loss
    inputs, gts, masks = _inputs(gold, "f", "cuda")
    inputs["stage3"]["depth"] = torch.from_numpy(gold["f_depth3"]).cuda()
    res = loss.focal_loss_bld(inputs, gts, masks, torch.from_numpy(gold["f_interval"]), return_grad=True)
    for name, v in zip(("total", "depth_loss", "epe", "less1", "less3"), res[:5]):
        np.testing.assert_allclose(v.item(), gold[f"f_{name}"], rtol=2e-6, err_msg=name)
    for s in STAGES:
        _grad_close(res[5][s], gold[f"f_{s}_grad"])


def test_entropy_loss_dtu_stage3_size():
    """[1, 8, 864, 1152]: loss and gradient against torch fp32 (autograd) on the GPU; per pixel the
    logit gradient sums to ~0 over D (softmax); masked-out pixels get exactly 0."""
    from transmvsnet_amd import ops
    g = torch.Generator(device="cuda").manual_seed(5)
    b, d, h, w = 1, 8, 864, 1152
    logits = 4.0 * torch.randn(b, d, h, w, device="cuda", generator=g)
    dv = 500.0 + torch.rand(b, 1, h, w, device="cuda", generator=g) + 2.0 * torch.arange(d, device="cuda").reshape(
        1, d, 1, 1).float()
    gt = 498.0 + 18.0 * torch.rand(b, h, w, device="cuda", generator=g)
    mask = (torch.rand(b, h, w, device="cuda", generator=g) > 0.25).float()
    prob = torch.softmax(logits, 1)
    lv, dl, wta, conf, grad = ops.entropy_loss(prob, dv.contiguous(), gt, mask, grad_scale=4.0, want_grad=True)
    x = logits.clone().requires_grad_(True)
    p = torch.softmax(x, 1)
    m = mask > 0.5
    idx = torch.round(m * torch.argmin((dv - gt.unsqueeze(1)).abs(), 1).float()).long().unsqueeze(1)
    ce = -torch.log(torch.gather(p, 1, idx) + 1e-6).squeeze(1)
    ref = ((m * ce).sum(dim=[1, 2]) / (m.sum(dim=[1, 2]) + 1e-6)).mean()
    (4.0 * ref).backward()
    np.testing.assert_allclose(lv.item(), ref.item(), rtol=1e-5)
    assert torch.equal(wta, torch.gather(dv, 1, prob.argmax(1, keepdim=True)).squeeze(1))
    assert torch.equal(conf, prob.max(1)[0])
    scale = x.grad.abs().max().item()
    assert (grad - x.grad).abs().max().item() <= 2e-6 * scale + 1e-5 * scale
    assert grad.sum(1).abs().max().item() <= 1e-6 * scale
    assert not grad[(~m).unsqueeze(1).expand_as(grad)].any()
    sl1 = torch.nn.functional.smooth_l1_loss(wta[m], gt[m])
    np.testing.assert_allclose(dl.item(), sl1.item(), rtol=1e-5)


def test_loss_rejects_cpu_and_bad_shapes():
    from transmvsnet_amd import ops
    p = torch.rand(1, 4, 8, 8)
    with pytest.raises(RuntimeError, match="GPU"):
        ops.entropy_loss(p, torch.rand(1, 4), torch.rand(1, 8, 8), torch.ones(1, 8, 8))
    with pytest.raises(ValueError):
        ops.entropy_loss(p.cuda(), torch.rand(1, 5).cuda(), torch.rand(1, 8, 8).cuda(), torch.ones(1, 8, 8).cuda())
