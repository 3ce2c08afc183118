"""Training losses, reference names and return values, on the HIP kernels
of csrc/loss.hip. Each stage's gradient of the total loss w.r.t. its CostRegNet logits
(prob_volume = softmax(logits), models/TransMVSNet.py) comes from the same pass as the loss: with
return_grad=True it is returned (the seed of a backward chain), and when the outputs come from a
train-mode TransMVSNet.forward (their prob_volume carries its logits) the returned total loss is
connected to those logits, so ``loss.backward()`` works as in the reference's train_sample.

  entropy_loss      models/module.py:495-531
  trans_mvsnet_loss models/module.py:534-558 (train.py: dlossw default 0.5,1.0,2.0)
  focal_loss_bld    models/module.py:561-592 (finetune.py: dlossw default 1.0,1.0,1.0)
"""
from __future__ import annotations

import torch

from . import ops

ENTROPY_WEIGHT = 2.0  # module.py:542 / :566


def _f32(t):
    return t.float().contiguous()


def entropy_loss(prob_volume, depth_gt, mask, depth_value, return_prob_map=False):
    """module.py:495: (masked cross entropy, wta depth[, photo confidence]). `mask` as passed by the
    reference's callers (bool after `> 0.5`); any dtype, > 0.5 counts as valid."""
    loss, _, wta, conf, _ = ops.entropy_loss(_f32(prob_volume), _f32(depth_value), _f32(depth_gt), _f32(mask))
    if return_prob_map:
        return loss, wta, conf
    return loss, wta


def _stage_keys(inputs):
    return [k for k in inputs.keys() if "stage" in k]


class _AttachLogitGrads(torch.autograd.Function):
    """total (no graph) -> the same value whose backward hands each stage's logits its precomputed
    d total / d logits (scaled by the incoming gradient)."""

    @staticmethod
    def forward(ctx, total, *logits_and_grads):
        n = len(logits_and_grads) // 2
        ctx.n = n
        ctx.save_for_backward(*logits_and_grads[n:])
        return total.clone()

    @staticmethod
    def backward(ctx, g):
        return (None, *[gr * g for gr in ctx.saved_tensors], *([None] * ctx.n))


def _graph_logits(inputs):
    """{stage: logits} when every stage's prob_volume comes from a train-mode forward, else None."""
    if not torch.is_grad_enabled():
        return None
    out = {}
    for key in _stage_keys(inputs):
        lg = getattr(inputs[key]["prob_volume"], "_tmvs_logits", None)
        if lg is None or not lg.requires_grad:
            return None
        out[key] = lg
    return out


def _stage_losses(inputs, depth_gt_ms, mask_ms, dlossw, want_grad):
    logits = _graph_logits(inputs)
    total, depth_loss, total_entropy, depth_entropy, grads = _stage_values(inputs, depth_gt_ms, mask_ms, dlossw,
                                                                           want_grad or logits is not None)
    if logits is not None:
        keys = list(logits)
        total = _AttachLogitGrads.apply(total, *[logits[k] for k in keys], *[grads[k] for k in keys])
    return total, depth_loss, total_entropy, depth_entropy, grads


def _stage_values(inputs, depth_gt_ms, mask_ms, dlossw, want_grad):
    total = torch.zeros((), device=mask_ms["stage1"].device)
    total_entropy = torch.zeros((), device=mask_ms["stage1"].device)
    grads, depth_loss, depth_entropy = {}, None, None
    for key in _stage_keys(inputs):
        st = inputs[key]
        w = 1.0 if dlossw is None else float(dlossw[int(key.replace("stage", "")) - 1])
        loss, depth_loss, depth_entropy, _, g = ops.entropy_loss(
            _f32(st["prob_volume"]), _f32(st["depth_values"]), _f32(depth_gt_ms[key]), _f32(mask_ms[key]),
            grad_scale=ENTROPY_WEIGHT * w, want_grad=want_grad)
        entro = loss * ENTROPY_WEIGHT
        total_entropy = total_entropy + entro
        total = total + w * entro
        if want_grad:
            grads[key] = g
    return total, depth_loss, total_entropy, depth_entropy, grads


def trans_mvsnet_loss(inputs, depth_gt_ms, mask_ms, dlossw=None, return_grad=False):
    """module.py:532: (total_loss, depth_loss, total_entropy, depth_entropy) of the last stage's
    depth_loss / WTA depth, as the reference. return_grad=True appends {stage: d total_loss /
    d logits [B,D,H,W]}."""
    total, depth_loss, total_entropy, depth_entropy, grads = _stage_losses(inputs, depth_gt_ms, mask_ms, dlossw,
                                                                            return_grad)
    out = (total, depth_loss, total_entropy, depth_entropy)
    return out + (grads,) if return_grad else out


def focal_loss_bld(inputs, depth_gt_ms, mask_ms, depth_interval, dlossw=None, return_grad=False):
    """module.py:559: (total_loss, depth_loss, epe, less1, less3). depth_interval: a number or a
    one-element tensor. The reference divides [B,H,W] errors by a [B] tensor, which broadcasts
    along W (an error unless W == B, and then not a per-sample scaling): a depth_interval with more
    than one element is refused here rather than silently reduced to sample 0's."""
    if torch.is_tensor(depth_interval) and depth_interval.numel() != 1:
        raise ValueError(f"focal_loss_bld: depth_interval must be a number or a one-element tensor, got shape "
                         f"{tuple(depth_interval.shape)} (the reference's [B] broadcast is along W)")
    total, depth_loss, _, _, grads = _stage_losses(inputs, depth_gt_ms, mask_ms, dlossw, return_grad)
    di = float(depth_interval.reshape(-1)[0]) if torch.is_tensor(depth_interval) else float(depth_interval)
    m = ops.depth_metrics(_f32(inputs["stage3"]["depth"]), _f32(depth_gt_ms["stage3"]), _f32(mask_ms["stage3"]), di)
    out = (total, depth_loss, m[0], m[1], m[2])
    return out + (grads,) if return_grad else out
