"""Depth-parity classification against the oracle -- TEST INFRASTRUCTURE ONLY.

Shared by ``tests/test_gpu_fullsize.py`` (the asserted full-size checks) and ``bench.py``'s
``cpu_baseline`` leg (the reported ``abs_depth_l1_vs_ref``), so the bench line and the tests classify
every differing pixel the same way. The product path never imports it.

The north-star bar (BASELINE.json): mean |depth_gpu - depth_ref| <= 1e-4 mm at stage 3,
argmax identical except near-ties. Rules:

* near tie: the reference's top-2 log-probability margin at that pixel is < MARGIN (1e-4). The
  reference's own fp32 result moves such pixels with its thread count. Where both sides
  share the hypotheses (fed / gpu-seeded runs) the margin is the larger of 1e-4 and the measured top-2
  spread (classify), capped at 2e-3;
* cascade-explained (the plain cascade only): an upstream near-tie flip moves the next stage's
  hypotheses (models/TransMVSNet.py:174-190, bilinear x2: the pixels within 2 of it) and CostRegNet's
  3-D convolutions carry the moved cost values RF_RADIUS pixels further;
* gpu-seeded: the reference cascade continued from the GPU's own previous-stage depths
  (``transmvs_ref.forward_from_features(seed_depth=...)``) has identical hypotheses, so there the
  near-tie rule alone applies -- the stage's own arithmetic, with no footprint rule;
* anything else is a failure, unless listed as an exact-arithmetic pick (float64 evaluation of the
  stage picks the GPU's index with a larger margin than the reference's).
"""
from __future__ import annotations

import numpy as np
import torch

MARGIN = 1e-4  # near-tie margin
TOP2_CAP = 2e-3  # bound on the measured top-2 spread that may widen it (runs with shared hypotheses)
# CostRegNet's receptive field in pixels of its own stage: 3 stride-2 levels of 3x3x3 convs (conv1-6),
# the 3 transposed convs back up, conv0 and prob: 1 + 2(1+1) + 4(1+1) + 8(1+1) + 4 + 2 + 1 = 36 < 40.
RF_RADIUS = 40


def raw_depth(stage_out):
    """Unclamped WTA depth (models/TransMVSNet.py:217-218) of a stage dict (prob_volume, depth_values)."""
    idx = torch.argmax(stage_out["prob_volume"], dim=1, keepdim=True)
    return torch.gather(stage_out["depth_values"], 1, idx).squeeze(1)


def dilate(mask, r):
    """Chebyshev dilation of a [H, W] bool mask by r pixels (separable running max)."""
    out = mask.copy()
    for axis in (0, 1):
        acc = out.copy()
        for k in range(1, r + 1):
            acc |= np.roll(out, k, axis) | np.roll(out, -k, axis)  # wrap-around only widens the footprint
        out = acc
    return out


def classify(depth_gpu, ref_stage, allowed=frozenset(), explained=None, prob_gpu=None):
    """Per-pixel classification of one stage's depth against the reference's.

    explained: [H, W] bool, the cascade footprint of moved hypotheses (None where both sides share the
    hypotheses). prob_gpu (those runs, where both sides share the hypotheses): besides the log-probability
    spread over live cells (reported), the TOP-2 spread -- the largest change the GPU's fp32 rounding makes
    to a pixel's top-2 log-probability difference, over the pixels whose argmax agrees (so no flip enters
    it) -- is measured; a flip whose reference margin is below max(MARGIN, that spread) is a near tie (the
    GPU's rounding moves margins that far elsewhere in the same volume). The spread must stay below
    TOP2_CAP."""
    g = depth_gpu.detach().float().cpu().numpy().astype(np.float64)
    r = ref_stage["depth"].numpy().astype(np.float64)
    pr = ref_stage["prob_volume"].numpy().astype(np.float64)
    lpr = np.log(np.maximum(pr, 1e-30))
    order = np.argsort(-pr, axis=1, kind="stable")
    i1, i2 = order[:, :1], order[:, 1:2]
    marg = (np.take_along_axis(lpr, i1, 1) - np.take_along_axis(lpr, i2, 1))[:, 0]
    spread, top2 = 0.0, 0.0
    if prob_gpu is not None:
        lpg = np.log(np.maximum(prob_gpu.detach().float().cpu().numpy().astype(np.float64), 1e-30))
        live = pr > 1e-6
        spread = float(np.abs(lpg - lpr)[live].max()) if live.any() else 0.0
        mg = (np.take_along_axis(lpg, i1, 1) - np.take_along_axis(lpg, i2, 1))[:, 0]
        same = np.argmax(lpg, axis=1) == i1[:, 0]
        if explained is not None:  # only where both sides have the same hypotheses
            same = same & ~np.broadcast_to(explained, same.shape)
        top2 = float(np.abs(mg - marg)[same].max()) if same.any() else 0.0
    margin = max(MARGIN, min(top2, TOP2_CAP))
    near = marg < margin
    diff = np.abs(g - r) > 1e-3
    casc = np.zeros_like(diff) if explained is None else np.broadcast_to(explained, diff.shape)
    other = [(int(y), int(x)) for _, y, x in np.argwhere(diff & ~near & ~casc)]
    absd = np.abs(g - r)
    outside = ~casc
    return {"mean_abs_mm": float(absd.mean()), "max_abs_mm": float(absd.max()), "differing": int(diff.sum()),
            "differing_pixels": [(int(y), int(x)) for _, y, x in np.argwhere(diff)[:64]],
            "footprint_pixels": int(casc[0].sum()),
            "mean_abs_mm_outside_footprint": float(absd[outside].mean()) if outside.any() else 0.0,
            "near_tie_flips": int((diff & near).sum()), "cascade_explained": int((diff & ~near & casc).sum()),
            "logprob_spread": spread, "top2_spread": top2, "near_tie_margin": margin,
            "other_flips": len(other), "max_flip_margin": float(marg[diff].max()) if diff.any() else 0.0,
            "flip_margins": sorted(float(m) for m in marg[diff][:64]),
            "unexplained": [p for p in other if p not in allowed], "exact_arithmetic_picks": [p for p in other if p in allowed],
            "_diff": diff[0]}


def moved(out_stage, ref_stage):
    """[H, W] bool: pixels whose GPU hypotheses differ from the reference's (an upstream flip)."""
    hg = out_stage["depth_values"].float().cpu().numpy()
    return (np.abs(hg - ref_stage["depth_values"].numpy()) > 1e-3).any(axis=1)[0]


def cascade_report(out, ref, allowed=None, spread=False):
    """Per-stage classification of the plain cascaded forward; asserts that every moved hypothesis lies
    within the up-sampling footprint (2 pixels) of a differing pixel of the previous stage. spread: widen
    the near-tie margin by the measured top-2 spread outside the footprint (GPU against GPU, e.g. the
    view-sharded forward against the single-rank one); the oracle cascade keeps the fixed 1e-4."""
    allowed = allowed or {}
    report, prev_diff = {}, None
    for s in (1, 2, 3):
        mv = moved(out[f"stage{s}"], ref[f"stage{s}"])
        if prev_diff is None:
            assert not mv.any(), "stage-1 hypotheses differ"
        else:
            up = np.kron(dilate(prev_diff, 1), np.ones((2, 2), dtype=bool))[:mv.shape[0], :mv.shape[1]]
            stray = mv & ~up
            assert not stray.any(), (s, np.argwhere(stray)[:10].tolist())
        rep = classify(out[f"stage{s}"]["depth"], ref[f"stage{s}"], allowed.get(s, frozenset()),
                       explained=dilate(mv, RF_RADIUS) if mv.any() else None,
                       prob_gpu=out[f"stage{s}"]["prob_volume"] if spread else None)
        rep["moved_hypotheses"] = int(mv.sum())
        prev_diff = rep.pop("_diff")
        report[f"cascade_stage{s}"] = rep
    return report


def gpu_seeded_report(out, sref, allowed=None):
    """Stages 2/3 of the GPU cascade against the reference cascade continued from the GPU's previous-stage
    depths (sref): identical hypotheses (asserted), near-tie rule only."""
    allowed = allowed or {}
    report = {}
    for s in (2, 3):
        np.testing.assert_array_equal(out[f"stage{s}"]["depth_values"].cpu().numpy(),
                                      sref[f"stage{s}"]["depth_values"].numpy())
        rep = classify(out[f"stage{s}"]["depth"], sref[f"stage{s}"], allowed.get(s, frozenset()),
                       prob_gpu=out[f"stage{s}"]["prob_volume"])
        rep.pop("_diff")
        report[f"gpu_seeded_stage{s}"] = rep
    return report


def seed_depths(out):
    """{stage2, stage3: the GPU's unclamped previous-stage WTA depth (CPU)} for forward_from_features."""
    return {f"stage{s + 1}": raw_depth({k: v.cpu() for k, v in out[f"stage{s}"].items()}) for s in (1, 2)}
