"""Shared test helpers: golden fixtures, synthetic weights, parity metrics."""
import json
import os

import numpy as np
import torch

from transmvsnet_amd import synthetic

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# The fixtures were generated (tests/golden/make_golden.py) by the reference on this build
# container's AVX-512 Xeon, whose MKL rounds homo_warping's rot·(x, y, 1) as an FMA chain;
# comparisons against them pin that rounding (ops.host_rot_order explains the two forms).
GOLDEN_ROT_ORDER = "fma"


class golden_rot:
    """with golden_rot(model): forward passes reproduce the fixtures' host rounding."""

    def __init__(self, model):
        self.model = model

    def __enter__(self):
        self.prev = self.model.warp_rot_order
        self.model.warp_rot_order = GOLDEN_ROT_ORDER
        return self.model

    def __exit__(self, *a):
        self.model.warp_rot_order = self.prev


def golden(name):
    return dict(np.load(os.path.join(GOLD, name)))


def golden_shapes():
    with open(os.path.join(GOLD, "state_dict_keys.json")) as f:
        keys = json.load(f)
    return {k: (tuple(v[0]), v[1]) for k, v in keys.items()}


def golden_state_dict(seed=0, sharpen=100.0):
    return synthetic.synthetic_state_dict(golden_shapes(), seed=seed, sharpen=sharpen)


def depth_parity(depth, ref_depth, prob_ref, margin=1e-4):
    """(mean |Δdepth|, fraction of pixels whose argmax may legitimately flip, flips outside them)."""
    d = np.abs(np.asarray(depth, np.float64) - np.asarray(ref_depth, np.float64))
    srt = np.sort(np.asarray(prob_ref, np.float64), axis=1)
    lp = np.log(np.maximum(srt[:, -1], 1e-30)) - np.log(np.maximum(srt[:, -2], 1e-30))
    near_tie = lp < margin
    return float(d.mean()), float(near_tie.mean()), int(((d > 1e-3) & ~near_tie).sum())


def to_np(t):
    return t.detach().float().cpu().numpy()
