"""Golden vectors for the TRAINING step from the REAL reference (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

Imports /root/reference/models (torchvision's deform_conv2d stubbed by the oracle's restatement, as
make_golden.py does; at the zero-initialised DCN offsets it is exact, and its autograd is the
bilinear adjoint torchvision's backward computes) and runs finetune.py's train_sample body
(finetune.py:144-168) at C1 size (128x160, N=3, ndepths 8/8/8, key-seeded synthetic weights with a
mild logit sharpening, prob.weight x10: the inference fixtures' x100 makes train-mode logits ~1e2,
where the cross entropy's gradient at p_gt ~ 1e-6 turns a 1e-4 relative logit rounding into
percent-level gradient noise for ANY fp32 implementation, the reference's included):

    model.train(); outputs = model(imgs, proj_matrix, depth_values)
    loss, depth_loss, epe, less1, less3 = focal_loss_bld(outputs, depth_gt_ms, mask_ms, depth_interval,
                                                         dlossw=[1.0, 1.0, 1.0])   # finetune.py:42
    loss.backward()

Case "f" (from features): FeatureNet is replaced by seeded leaf tensors (synthetic_features seed 2),
so the gradients w.r.t. the stage features are recorded with every FMT / pathway / PixelwiseNet /
CostRegNet parameter gradient. Case "i" (from images): the whole model including FeatureNet + DCN.
Both store the loss terms, the train-mode outputs (depth, prob volume per stage), every parameter
gradient (.grad of each named parameter) and every BatchNorm running statistic after the step
(momentum 0.1 updates). Writes tests/golden/train_c1.npz: data only.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402
from transmvsnet_amd import synthetic  # noqa: E402

H, W, N, ND = 128, 160, 3, (8, 8, 8)
TRAIN_SHARPEN = 10.0


class _LeafFeatures(torch.nn.Module):
    """TransMVSNet.feature replaced by pre-made per-view leaf pyramids (returned as-is, so their .grad
    is the gradient w.r.t. FeatureNet's outputs)."""

    def __init__(self, feats):
        super().__init__()
        self.feats = feats
        self.i = 0

    def forward(self, img):
        f = self.feats[self.i]
        self.i += 1
        return dict(f)


def ground_truth():
    """Seeded smooth depth maps inside the DTU range + masks, per stage (nearest down-sampling as the
    BlendedMVS loader's depth_ms / mask_ms pyramids)."""
    g = torch.Generator().manual_seed(11)
    coarse = 520.0 + 300.0 * torch.rand(1, 1, 8, 10, generator=g)
    d3 = F.interpolate(coarse, size=(H, W), mode="bilinear", align_corners=False)[:, 0]
    d3 = d3 + 2.0 * torch.randn(1, H, W, generator=g)
    m3 = (torch.rand(1, H, W, generator=g) > 0.2).float()
    gt, mask = {"stage3": d3.contiguous()}, {"stage3": m3}
    for s, f in (("stage2", 2), ("stage1", 4)):
        gt[s] = d3[:, ::f, ::f].contiguous()
        mask[s] = m3[:, ::f, ::f].contiguous()
    return gt, mask


def run_case(TransMVSNet, ref_module, sd, proj, dv, gt, mask, feats=None, imgs=None):
    model = TransMVSNet(ndepths=list(ND))
    model.load_state_dict(sd, strict=True)
    if feats is not None:
        model.feature = _LeafFeatures(feats)
        imgs = torch.zeros(1, N, 3, H, W)
    model.train()
    for p in model.parameters():
        p.grad = None
    outputs = model(imgs, proj, dv)
    interval = torch.tensor([float(dv[0, 1] - dv[0, 0])])
    loss, depth_loss, epe, less1, less3 = ref_module.focal_loss_bld(outputs, gt, mask, interval,
                                                                    dlossw=[1.0, 1.0, 1.0])
    loss.backward()
    d = {"loss": loss.detach().numpy(), "depth_loss": depth_loss.detach().numpy(), "epe": epe.detach().numpy(),
         "less1": less1.detach().numpy(), "less3": less3.detach().numpy(), "interval": interval.numpy()}
    for s in (1, 2, 3):
        o = outputs[f"stage{s}"]
        d[f"stage{s}_depth"] = o["depth"].detach().numpy()
        d[f"stage{s}_prob"] = o["prob_volume"].detach().numpy()
        d[f"stage{s}_hyp"] = o["depth_values"].detach().numpy()
    for n, p in model.named_parameters():
        if p.grad is not None:
            d[f"grad.{n}"] = p.grad.numpy()
    for n, b in model.named_buffers():
        if "running" in n or "num_batches_tracked" in n:
            d[f"buf.{n}"] = b.numpy()
    return d


def main():
    TransMVSNet, ref_module, _ = load_reference()
    torch.manual_seed(0)
    shapes = synthetic.state_dict_shapes(TransMVSNet())
    sd = synthetic.synthetic_state_dict(shapes, seed=0, sharpen=TRAIN_SHARPEN)
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    gt, mask = ground_truth()
    out = {}
    for s in ("stage1", "stage2", "stage3"):
        out[f"gt_{s}"] = gt[s].numpy()
        out[f"mask_{s}"] = mask[s].numpy()
    # case f: from FeatureNet-shaped leaves
    feats = [{k: v.clone().requires_grad_(True) for k, v in f.items()}
             for f in synthetic.synthetic_features(N, H, W, seed=2)]
    d = run_case(TransMVSNet, ref_module, sd, proj, dv, gt, mask, feats=feats)
    out.update({f"f_{k}": v for k, v in d.items()})
    for v, f in enumerate(feats):
        for k, t in f.items():
            out[f"f_featgrad_{v}_{k}"] = t.grad.numpy()
    # case i: from images, FeatureNet + DCN included
    imgs = synthetic.synthetic_images(N, H, W, seed=0)
    d = run_case(TransMVSNet, ref_module, sd, proj, dv, gt, mask, imgs=imgs)
    out.update({f"i_{k}": v for k, v in d.items()})
    np.savez_compressed(os.path.join(HERE, "train_c1.npz"), **out)
    print("wrote train_c1.npz", os.path.getsize(os.path.join(HERE, "train_c1.npz")),
          {k: float(v) for k, v in out.items() if v.ndim == 0 or v.size == 1})
    print("grads f:", sum(1 for k in out if k.startswith("f_grad.")), "i:", sum(1 for k in out if k.startswith("i_grad.")))


if __name__ == "__main__":
    main()
