"""Golden vectors for the training losses from the REAL reference (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_loss.py

Imports models/module.py from /root/reference (via make_golden.load_reference, torchvision stubbed
as there; the losses do not touch it) and runs its trans_mvsnet_loss (dlossw 0.5,1.0,2.0 as
train.py) and focal_loss_bld (dlossw None, B = 1, as finetune.py) on seeded softmax volumes, then
backpropagates the total loss to each stage's logits. Writes inputs, loss values and gradients to
tests/golden/loss.npz. Data only: no reference source is copied.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import load_reference  # noqa: E402

SHAPES = {"stage1": (8, 6, 8), "stage2": (8, 12, 16), "stage3": (4, 24, 32)}  # D, H, W


def make_case(g, batch, per_pixel_stage1):
    logits, dvs, gts, masks = {}, {}, {}, {}
    for k, (d, h, w) in SHAPES.items():
        logits[k] = 3.0 * torch.randn(batch, d, h, w, generator=g)
        base = 500.0 + 10.0 * torch.rand(batch, 1, 1, 1, generator=g)
        step = 4.0 if k == "stage1" else 2.0
        if k == "stage1" and not per_pixel_stage1:
            dvs[k] = (base.reshape(batch, 1) + step * torch.arange(d).float()).contiguous()  # [B,D] (module.py:503)
            lo = dvs[k][:, :1, None]
        else:
            jitter = torch.rand(batch, 1, h, w, generator=g)
            dvs[k] = (base + jitter + step * torch.arange(d).float().reshape(1, d, 1, 1)).contiguous()
            lo = dvs[k][:, 0]
        span = step * (d - 1)
        gt = lo + (span + 6.0) * torch.rand(batch, h, w, generator=g) - 3.0  # some below / above the range
        if k == "stage2":  # exact midpoints between hypotheses: argmin ties -> first index
            dv2 = dvs[k]
            gt[:, 0, :4] = 0.5 * (dv2[:, 2, 0, :4] + dv2[:, 3, 0, :4])
        gts[k] = gt.contiguous()
        masks[k] = (torch.rand(batch, h, w, generator=g) > 0.3).float()
    if batch > 1:
        masks["stage1"][1] = 0.0  # an empty mask in one batch element (valid = 1e-6)
    return logits, dvs, gts, masks


def main():
    _, ref_module, _ = load_reference()
    g = torch.Generator().manual_seed(1234)
    out = {}

    logits, dvs, gts, masks = make_case(g, 2, per_pixel_stage1=False)
    leaves = {k: v.clone().requires_grad_(True) for k, v in logits.items()}
    inputs = {k: {"prob_volume": F.softmax(leaves[k], dim=1), "depth_values": dvs[k]} for k in leaves}
    total, depth_loss, total_entropy, depth_entropy = ref_module.trans_mvsnet_loss(
        inputs, gts, masks, dlossw=[0.5, 1.0, 2.0])
    total.backward()
    for k in SHAPES:
        out[f"t_{k}_logits"] = logits[k].numpy()
        out[f"t_{k}_dv"] = dvs[k].numpy()
        out[f"t_{k}_gt"] = gts[k].numpy()
        out[f"t_{k}_mask"] = masks[k].numpy()
        out[f"t_{k}_grad"] = leaves[k].grad.numpy()
        out[f"t_{k}_prob"] = inputs[k]["prob_volume"].detach().numpy()  # host softmax is not bit-stable across CPUs
    out["t_total"] = total.detach().numpy()
    out["t_depth_loss"] = depth_loss.detach().numpy()
    out["t_total_entropy"] = total_entropy.detach().numpy()
    out["t_depth_entropy"] = depth_entropy.detach().numpy()
    # entropy_loss(return_prob_map=True) on stage 2 alone
    p2 = F.softmax(logits["stage2"], dim=1)
    l2, wta2, conf2 = ref_module.entropy_loss(p2, gts["stage2"], masks["stage2"] > 0.5, dvs["stage2"],
                                              return_prob_map=True)
    out["e_loss"], out["e_wta"], out["e_conf"] = l2.numpy(), wta2.numpy(), conf2.numpy()

    logits, dvs, gts, masks = make_case(g, 1, per_pixel_stage1=True)
    leaves = {k: v.clone().requires_grad_(True) for k, v in logits.items()}
    inputs = {k: {"prob_volume": F.softmax(leaves[k], dim=1), "depth_values": dvs[k]} for k in leaves}
    depth3 = (gts["stage3"] + 8.0 * torch.randn(gts["stage3"].shape, generator=g)).contiguous()
    inputs["stage3"]["depth"] = depth3
    interval = torch.tensor([2.5])
    res = ref_module.focal_loss_bld(inputs, gts, masks, interval)
    res[0].backward()
    for k in SHAPES:
        out[f"f_{k}_logits"] = logits[k].numpy()
        out[f"f_{k}_dv"] = dvs[k].numpy()
        out[f"f_{k}_gt"] = gts[k].numpy()
        out[f"f_{k}_mask"] = masks[k].numpy()
        out[f"f_{k}_grad"] = leaves[k].grad.numpy()
        out[f"f_{k}_prob"] = inputs[k]["prob_volume"].detach().numpy()
    out["f_depth3"] = depth3.numpy()
    out["f_interval"] = interval.numpy()
    for name, v in zip(("total", "depth_loss", "epe", "less1", "less3"), res):
        out[f"f_{name}"] = v.detach().numpy()
    np.savez_compressed(os.path.join(HERE, "loss.npz"), **out)
    print("wrote loss.npz", {k: float(v) for k, v in out.items() if v.ndim == 0})


if __name__ == "__main__":
    main()
