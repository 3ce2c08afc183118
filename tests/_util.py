"""Shared test helpers: golden fixtures, synthetic weights, parity metrics."""
import json
import os

import numpy as np
import torch

from transmvsnet_amd import synthetic

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


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
