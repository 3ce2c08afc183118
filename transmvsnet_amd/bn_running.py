"""BatchNorm running-statistics updates of a training step, batched.

nn.BatchNorm's train-mode forward updates, per call, running = (1 - m) running + m stat (the variance
unbiased: var * n / (n - 1)), and num_batches_tracked += 1. A module the reference calls once per
view (FeatureNet, PixelwiseNet; models/TransMVSNet.py:151-153, 71-77) is updated G times in view
order. After G calls: running_G = (1 - m)^G running_0 + sum_v m (1 - m)^(G-1-v) stat_v, which this
module evaluates for every BatchNorm of a step with a handful of multi-tensor launches instead of
~8 elementwise launches per BatchNorm and call (400+ per C5 step). The closed form re-associates the
fp32 sums (differences of a few ulps against the sequential updates)."""
from __future__ import annotations

import torch


def update_running_stats(items, momentum):
    """items: [(bn, mean [G, C], var [G, C] (biased, per call, in call order), n elements per call)].
    Multi-tensor launches only (no per-BatchNorm kernels): per group of modules with the same G, one
    scale of the running buffers, then per call v one weighted add of that call's statistics."""
    if not items:
        return
    with torch.no_grad():
        by_g = {}
        for bn, mean, var, n in items:
            by_g.setdefault(int(mean.shape[0]), []).append((bn, mean, var, n))
        m = float(momentum)
        for g, group in by_g.items():
            rms = [bn.running_mean for bn, _, _, _ in group]
            rvs = [bn.running_var for bn, _, _, _ in group]
            torch._foreach_mul_(rms, (1.0 - m) ** g)
            torch._foreach_mul_(rvs, (1.0 - m) ** g)
            for v in range(g):
                c = m * (1.0 - m) ** (g - 1 - v)
                torch._foreach_add_(rms, [mean[v] for _, mean, _, _ in group], alpha=c)
                torch._foreach_add_(rvs, torch._foreach_mul([var[v] for _, _, var, _ in group],
                                                            [c * n / max(n - 1, 1) for _, _, _, n in group]))
            torch._foreach_add_([bn.num_batches_tracked for bn, _, _, _ in group], g)
