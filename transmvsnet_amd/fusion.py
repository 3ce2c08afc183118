"""Output side of the reference's test.py: depth/camera/image writers (test.py:40-66, 119-158,
utils.py:11-22) and the gipuma depth-map fusion (gipuma/fusibile, run by gipuma.py:7-21) with its
fusion kernel as the HIP kernel ``tmvs_fusibile`` (csrc/fusion.hip) -- SURVEY.md 8f rank 4.

The reference hands depth maps to fusibile through files: per view an RGBA PNG whose alpha is the
clamped depth as uint8((d - 425) / 510 * 255) (utils.depth_normal), decoded by fusibile as
425 + 512 * alpha / 255 (main.cpp:136) -- the 510-vs-512 mismatch is the reference's and is kept
(``depth_decode``) -- and a 3x4 projection matrix P = K [R | t] (test.write_cam). ``fuse`` takes
those arrays (or device tensors) directly; ``save_point_cloud`` writes fusibile's PLY
(displayUtils.h:10-55). Camera parameters follow cameraGeometryUtils.h:100-162 on the host.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from ._lib import check, load

CAM_FLOATS = 32  # csrc/fusion.hip fz::CAM: P[12], RK_inv[9], C4[3], fx, pad


def depth_normal(depth, depth_min=425.0, depth_max=935.0):
    """utils.depth_normal (utils.py:11-22): clamp, scale to [0, 1], uint8 (truncation)."""
    d = np.clip(np.asarray(depth, np.float32), depth_min, depth_max)
    return ((d - depth_min) / (depth_max - depth_min) * 255).astype(np.uint8)


def depth_decode(alpha_u8):
    """fusibile's decoding (main.cpp:131-137): convertTo(1/255) then 425 + 512 * a, float32."""
    a = (np.asarray(alpha_u8, np.float64) * (1.0 / 255.0)).astype(np.float32)
    return (425.0 + 512.0 * a.astype(np.float64)).astype(np.float32)


def projection_matrix(cam):
    """test.write_cam (test.py:40-66): cam [2, 4, 4] (extrinsic, intrinsic) -> P = K E [3, 4]."""
    cam = np.asarray(cam)
    k = np.zeros((4, 4))
    k[:3, :3] = cam[1][:3, :3]
    return np.matmul(k, cam[0])[:3]


def write_cam(filename, cam):
    """test.write_cam: the 3x4 projection matrix as text, one row per line, then a blank line."""
    p = projection_matrix(cam)
    with open(filename, "w") as f:
        for i in range(3):
            for j in range(4):
                f.write(str(p[i][j]) + " ")
            f.write("\n")
        f.write("\n")


def read_cam(filename):
    """fusibile's read_camera_parameters (cameraGeometryUtils.h:77-98): up to 3 x 4 floats."""
    p = np.zeros((3, 4), np.float32)
    p[:, :3] = np.eye(3)
    with open(filename) as f:
        rows = [ln.split() for ln in f.read().splitlines() if ln.strip() and "CONTOUR" not in ln]
    for i, vals in enumerate(rows[:3]):
        for j, v in enumerate(vals[:4]):
            p[i, j] = np.float32(float(v))
    return p


def _rq3(m):
    """RQ decomposition m = K R, K upper triangular with positive diagonal (OpenCV RQDecomp3x3's
    convention for a camera with det(R) = +1)."""
    q, r = np.linalg.qr(np.flipud(m).T)
    k = np.flipud(np.fliplr(r.T))
    rot = np.flipud(q.T)
    s = np.diag(np.sign(np.diag(k)))
    return k @ s, s @ rot


def camera_params(p):
    """get_camera_parameters (cameraGeometryUtils.h:100-162) for one P [3, 4]: K (its fx is the
    focal length of depth_convert_cu), the camera centre C4 from P's 3x3 minors (getCameraCenter),
    RK_inv = inv(P[:, :3]). Returns the packed float32[32] the kernel reads and a dict for tests."""
    p = np.asarray(p, np.float64)
    k, _ = _rq3(p[:, :3])
    c = np.array([np.linalg.det(p[:, [1, 2, 3]]), -np.linalg.det(p[:, [0, 2, 3]]),
                  np.linalg.det(p[:, [0, 1, 3]]), -np.linalg.det(p[:, [0, 1, 2]])])
    c = c / c[3]
    rk_inv = np.linalg.inv(p[:, :3])
    d = {"P": p.astype(np.float32), "RK_inv": rk_inv.astype(np.float32), "C4": c[:3].astype(np.float32),
         "fx": np.float32(k[0, 0])}
    pk = np.zeros(CAM_FLOATS, np.float32)
    pk[0:12] = d["P"].reshape(-1)
    pk[12:21] = d["RK_inv"].reshape(-1)
    pk[21:24] = d["C4"]
    pk[24] = d["fx"]
    return pk, d


def rgbd_from_images(bgr_u8, depth_u8):
    """fusibile's texture images (main.cpp:126-138): [V, H, W, 4] float32 (B, G, R, depth) from the
    BGR uint8 images and the uint8 depth alphas test.py wrote."""
    bgr = np.asarray(bgr_u8, np.float64) * (1.0 / 255.0)
    out = np.empty(bgr.shape[:-1] + (4,), np.float32)
    out[..., :3] = bgr.astype(np.float32)
    out[..., 3] = depth_decode(depth_u8)
    return out


def fuse(rgbd, cams_packed, consistent_threshold=3, depth_threshold=0.25):
    """fusibile_cu (fusibile.cu:231-286) on the GPU: one tmvs_fusibile launch per reference camera
    into ONE persistent point buffer (as the reference), each followed by copy_pc_to_host's
    compaction (pixels whose x, y and z are all nonzero, in pixel order).

    rgbd: [V, H, W, 4] float32 (device tensor or array); cams_packed: [V, 32] (camera_params).
    Returns (coords [N, 3], textures [N, 3]) as device tensors."""
    lib = load()
    if not isinstance(rgbd, torch.Tensor) or not rgbd.is_cuda:
        raise RuntimeError("fuse: rgbd must be a CUDA tensor (HIP kernel; no CPU fallback)")
    rgbd = rgbd.contiguous().float()
    v, h, w, c = rgbd.shape
    if c != 4:
        raise ValueError("fuse: rgbd must be [V, H, W, 4]")
    cams = torch.as_tensor(np.ascontiguousarray(cams_packed, np.float32)).reshape(v, CAM_FLOATS).to(rgbd.device)
    coord = torch.zeros(h, w, 4, device=rgbd.device)
    tex = torch.zeros(h, w, 4, device=rgbd.device)
    xs, ts = [], []
    for ref in range(v):
        with ops._Span("tmvs_fusibile"):
            check(lib.tmvs_fusibile(rgbd.data_ptr(), cams.data_ptr(), v, h, w, ref, int(consistent_threshold),
                                    float(depth_threshold), coord.data_ptr(), tex.data_ptr(), ops._stream()),
                  "tmvs_fusibile")
        keep = (coord[..., 0] != 0) & (coord[..., 1] != 0) & (coord[..., 2] != 0)
        xs.append(coord[..., :3][keep])
        ts.append(tex[..., :3][keep])
    return torch.cat(xs), torch.cat(ts)


def save_point_cloud(filename, coords, textures):
    """save_point_cloud (displayUtils.h:10-55): binary little-endian PLY, float x y z and uchar
    red green blue = int(texture[2|1|0] * 255); non-finite coordinates are written as 0."""
    x = np.asarray(coords, np.float32).reshape(-1, 3).copy()
    t = np.asarray(textures, np.float32).reshape(-1, 3)
    bad = ~np.isfinite(x).all(axis=1) | (np.abs(x) >= np.finfo(np.float32).max).any(axis=1)
    x[bad] = 0.0
    rgb = (t[:, [2, 1, 0]] * 255.0).astype(np.int64).astype(np.uint8)
    rec = np.empty(len(x), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("g", "u1"), ("b", "u1")])
    rec["x"], rec["y"], rec["z"] = x[:, 0], x[:, 1], x[:, 2]
    rec["r"], rec["g"], rec["b"] = rgb[:, 0], rgb[:, 1], rgb[:, 2]
    with open(filename, "wb") as f:
        f.write(("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
                 "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n"
                 % len(x)).encode("ascii"))
        f.write(rec.tobytes())
