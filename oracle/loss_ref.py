"""CPU oracle for the training losses (TEST INFRASTRUCTURE ONLY: imported by tests/, never by the
product path). A PyTorch-CPU restatement of models/module.py:495-592; the gradient w.r.t. each
stage's logits comes from autograd through F.softmax. Pinned against tests/golden/loss.npz, made by
tests/golden/make_golden_loss.py from the real reference functions.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def entropy_loss(prob_volume, depth_gt, mask, depth_value, return_prob_map=False):
    """module.py:495-531."""
    valid = torch.sum(mask, dim=[1, 2]) + 1e-6                       # :499
    b, h, w = depth_gt.shape
    d = depth_value.shape[1]
    if depth_value.dim() < 3:                                         # :503-506
        dv = depth_value.repeat(h, w, 1, 1).permute(2, 3, 0, 1)
    else:
        dv = depth_value
    gt_idx = torch.argmin(torch.abs(dv - depth_gt.unsqueeze(1)), dim=1)            # :508
    gt_idx = torch.round(torch.mul(mask, gt_idx.float())).long().unsqueeze(1)       # :510-511
    onehot = torch.zeros(b, d, h, w).type(mask.type()).scatter_(1, gt_idx, 1)       # :514
    ce = -torch.sum(onehot * torch.log(prob_volume + 1e-6), dim=1).squeeze(1)       # :517
    masked = torch.sum(torch.mul(mask, ce), dim=[1, 2])                             # :520-521
    loss = torch.mean(masked / valid)                                               # :522
    wta_idx = torch.argmax(prob_volume, dim=1, keepdim=True).long()                 # :524
    wta = torch.gather(dv, 1, wta_idx).squeeze(1)                                   # :525
    if return_prob_map:
        return loss, wta, torch.max(prob_volume, dim=1)[0]
    return loss, wta


def _stages(inputs, depth_gt_ms, mask_ms, dlossw):
    dev = mask_ms["stage1"].device
    total = torch.tensor(0.0, dtype=torch.float32, device=dev)
    total_entropy = torch.tensor(0.0, dtype=torch.float32, device=dev)
    depth_loss = depth_entropy = None
    for key in [k for k in inputs.keys() if "stage" in k]:
        st = inputs[key]
        gt = depth_gt_ms[key]
        mask = mask_ms[key] > 0.5
        entro, depth_entropy = entropy_loss(st["prob_volume"], gt, mask, st["depth_values"])
        entro = entro * 2.0                                                         # :542-544
        depth_loss = F.smooth_l1_loss(depth_entropy[mask], gt[mask], reduction="mean")  # :545
        total_entropy = total_entropy + entro
        if dlossw is not None:
            total = total + dlossw[int(key.replace("stage", "")) - 1] * entro
        else:
            total = total + entro
    return total, depth_loss, total_entropy, depth_entropy


def trans_mvsnet_loss(inputs, depth_gt_ms, mask_ms, dlossw=None):
    """module.py:534-558."""
    return _stages(inputs, depth_gt_ms, mask_ms, dlossw)


def focal_loss_bld(inputs, depth_gt_ms, mask_ms, depth_interval, dlossw=None):
    """module.py:561-592."""
    total, depth_loss, _, _ = _stages(inputs, depth_gt_ms, mask_ms, dlossw)
    err = (depth_gt_ms["stage3"] - inputs["stage3"]["depth"]).abs()
    err = err / (depth_interval * 192. / 128.)
    m = mask_ms["stage3"] > 0.5
    return (total, depth_loss, err[m].mean(), (err[m] < 1.).to(err.dtype).mean(),
            (err[m] < 3.).to(err.dtype).mean())


def loss_and_logit_grads(logits, depth_values, depth_gt_ms, mask_ms, dlossw=None, loss_fn=None):
    """Softmax each stage's logits, run `loss_fn` (default trans_mvsnet_loss) and backpropagate the
    total loss: returns (loss tuple, {stage: d total / d logits})."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in logits.items()}
    inputs = {k: {"prob_volume": F.softmax(leaves[k], dim=1), "depth_values": depth_values[k]} for k in leaves}
    fn = loss_fn or (lambda i: trans_mvsnet_loss(i, depth_gt_ms, mask_ms, dlossw=dlossw))
    out = fn(inputs)
    out[0].backward()
    return out, {k: v.grad.detach() for k, v in leaves.items()}
