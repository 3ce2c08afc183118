"""Deterministic synthetic inputs and weights for the TransMVSNet hot path.

There is no network here (no DTU download, no Google-Drive checkpoint), so every
benchmark, smoke run and parity test feeds the same seeded data:

* ``synthetic_state_dict`` -- key-name-seeded weights for the reference state_dict
  layout (465 keys, ``models/TransMVSNet.py:112-139``), randomised BN statistics and
  an optional sharpening factor on ``cost_regularization.{s}.prob.weight`` so that the
  probability volumes are peaked (random-init volumes are nearly uniform, which
  makes winner-take-all parity meaningless).
* ``synthetic_cameras`` -- DTU-like ``proj_matrix`` dict (``datasets/general_eval.py:
  182-210``): extrinsic in ``[:, :, 0]``, 1/4-resolution intrinsics in
  ``[:, :, 1, :3, :3]``, scaled x2 / x4 for stages 2 / 3.
* ``synthetic_depth_values`` -- ``np.arange(425, 2.5*(192-0.5)+425, 2.5)``
  (``datasets/general_eval.py:190-192``).
* ``synthetic_features`` -- stand-in for FeatureNet's per-view pyramid
  (``models/module.py:399-422``): stage1 [B,32,H/4,W/4], stage2 [B,16,H/2,W/2],
  stage3 [B,8,H,W].
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

DTU_DEPTH_MIN = 425.0
DTU_DEPTH_INTERVAL = 2.5
DTU_NDEPTH = 192


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng([int(seed) & 0xFFFFFFFF, zlib.crc32(key.encode("utf-8"))])


def synthetic_state_dict(shapes, seed: int = 0, sharpen: float = 100.0):
    """Fill every key of ``shapes`` ({key: (shape, dtype)}) deterministically.

    The generator depends only on (seed, key name, shape), so the reference model,
    the CPU oracle and the HIP model all receive bit-identical weights.
    """
    out = {}
    for key, (shape, dtype) in shapes.items():
        rng = _rng(seed, key)
        leaf = key.rsplit(".", 1)[-1]
        shape = tuple(int(s) for s in shape)
        if leaf == "num_batches_tracked":
            out[key] = torch.zeros(shape, dtype=torch.long)
            continue
        if "conv_offset_mask" in key:
            # the reference zero-initialises the DCN offset/mask conv (models/dcn.py:62-64)
            arr = np.zeros(shape, np.float32)
        elif leaf == "running_mean":
            arr = rng.uniform(-0.1, 0.1, shape)
        elif leaf == "running_var":
            arr = rng.uniform(0.5, 1.5, shape)
        elif len(shape) == 1 and leaf == "weight":  # BatchNorm / LayerNorm affine
            arr = rng.uniform(0.8, 1.2, shape)
        elif len(shape) == 1:  # biases
            arr = rng.uniform(-0.1, 0.1, shape)
        else:
            fan_in = int(np.prod(shape[1:]))
            b = math.sqrt(3.0 / fan_in)
            arr = rng.uniform(-b, b, shape)
            if sharpen != 1.0 and key.startswith("cost_regularization.") and key.endswith("prob.weight"):
                arr = arr * sharpen
        out[key] = torch.from_numpy(np.asarray(arr, dtype=np.float32))
    return out


def state_dict_shapes(module: torch.nn.Module):
    return {k: (tuple(v.shape), v.dtype) for k, v in module.state_dict().items()}


def synthetic_depth_values(batch: int = 1) -> torch.Tensor:
    dv = np.arange(DTU_DEPTH_MIN, DTU_DEPTH_INTERVAL * (DTU_NDEPTH - 0.5) + DTU_DEPTH_MIN,
                   DTU_DEPTH_INTERVAL, dtype=np.float32)
    return torch.from_numpy(np.tile(dv[None], (batch, 1)))


def _rodrigues(axis, angle):
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + math.sin(angle) * k + (1 - math.cos(angle)) * (k @ k)


def _look_at(center, target, up_jitter):
    z = target - center
    z = z / np.linalg.norm(z)
    up = np.array([0.0, 1.0, 0.0]) + up_jitter
    x = np.cross(up, z)
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])  # rows: camera axes in world frame -> R (world->cam)


def synthetic_cameras(n_views: int, height: int, width: int, batch: int = 1, seed: int = 1):
    """DTU-like multi-view rig looking at a scene centred ~650 mm in front of the ref camera.

    Returns {"stage1","stage2","stage3": float32 tensor [B, N, 2, 4, 4]} in the layout
    of ``datasets/general_eval.py:182-210``.
    """
    rng = np.random.default_rng(seed)
    # 1/4-resolution intrinsics: DTU 2892.33/2883.18/823.205/619.071 /4 x0.72 at 864x1152
    sx = (width / 4.0) / 288.0
    sy = (height / 4.0) / 216.0
    K = np.array([[520.6 * sx, 0.0, 148.2 * sx], [0.0, 519.0 * sy, 111.4 * sy], [0.0, 0.0, 1.0]])
    target = np.array([0.0, 0.0, 650.0])
    mats = np.zeros((batch, n_views, 2, 4, 4), np.float32)
    for b in range(batch):
        for v in range(n_views):
            if v == 0:
                R = np.eye(3)
                C = np.zeros(3)
            else:
                ang = rng.uniform(0, 2 * math.pi)
                rad = rng.uniform(50.0, 150.0)
                C = np.array([rad * math.cos(ang), rad * math.sin(ang), rng.uniform(-20.0, 20.0)])
                R = _look_at(C, target + rng.uniform(-15, 15, 3), rng.uniform(-0.03, 0.03, 3))
                R = _rodrigues(rng.normal(size=3), math.radians(rng.uniform(0, 1.5))) @ R
            t = -R @ C
            E = np.eye(4)
            E[:3, :3] = R
            E[:3, 3] = t
            mats[b, v, 0] = E.astype(np.float32)
            mats[b, v, 1, :3, :3] = K.astype(np.float32)
    s2 = mats.copy()
    s2[:, :, 1, :2, :] = mats[:, :, 1, :2, :] * 2
    s3 = mats.copy()
    s3[:, :, 1, :2, :] = mats[:, :, 1, :2, :] * 4
    return {"stage1": torch.from_numpy(mats), "stage2": torch.from_numpy(s2), "stage3": torch.from_numpy(s3)}


def synthetic_images(n_views: int, height: int, width: int, batch: int = 1, seed: int = 0):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.random((batch, n_views, 3, height, width), dtype=np.float32))


def synthetic_features(n_views: int, height: int, width: int, batch: int = 1, seed: int = 2):
    """Per-view FeatureNet-shaped pyramids, ~N(0,1), NCHW float32 (CPU)."""
    rng = np.random.default_rng(seed)
    feats = []
    for _ in range(n_views):
        f = {}
        for name, c, s in (("stage1", 32, 4), ("stage2", 16, 2), ("stage3", 8, 1)):
            f[name] = torch.from_numpy(rng.standard_normal((batch, c, height // s, width // s), dtype=np.float32))
        feats.append(f)
    return feats


def stacked_features(n_views: int, height: int, width: int, seed: int = 2):
    """FeatureNet-shaped pyramids already stacked as forward_features takes them:
    {stage: [1, N, C, h, w]} ~N(0,1) from torch's CPU generator (bench.py's inputs)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    return {name: torch.randn(1, n_views, c, height // s, width // s, generator=g)
            for name, c, s in (("stage1", 32, 4), ("stage2", 16, 2), ("stage3", 8, 1))}
